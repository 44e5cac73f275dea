// Shared pieces of the LDS-DMA MFMA GEMM pipelines (wgrad.hip, tokennorm.hip): raw barrier,
// counted vmcnt waits, one LDS-DMA instruction and the transposing LDS read.
//
// The ring's LDS-DMA is inline asm on purpose: the compiler's waitcnt pass would otherwise see
// an LDS write behind every DMA and wait vmcnt(0) for the whole ring before each LDS read; the
// stage waits are counted by hand (gemm_vm_wait), and the "memory" clobbers keep every LDS read
// of a slot on its side of the barriers.
#pragma once
#include "common.h"

namespace dcr {

// raw barrier: __syncthreads()' release fence would wait vmcnt(0) for the in-flight ring
__device__ __forceinline__ void gemm_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void gemm_vm_wait(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
  }
}

// one LDS-DMA instruction: 16 B per lane to LDS address lds + 16 lane (M0 = lds)
__device__ __forceinline__ void gemm_dma(__amdgpu_buffer_rsrc_t r, unsigned lds, unsigned voff,
                                         unsigned soff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(lds), "v"(voff), "s"(r), "s"(soff) : "memory");
}

// transposed 64-bit LDS read: 4 bf16 of 4 consecutive rows for this lane's column
typedef short gemm_s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x2 gemm_rd_tr(unsigned addr) {
  return __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                       (__attribute__((address_space(3))) gemm_s16x4*)(size_t)addr));
}

// plain 128-bit LDS read at a byte address (compiler-visible)
__device__ __forceinline__ u32x4 gemm_rd128(unsigned addr) {
  return *(const __attribute__((address_space(3))) u32x4*)(size_t)addr;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t gemm_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7FFFFFF0, 0x00020000);
}

}  // namespace dcr
