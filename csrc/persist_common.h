// Shared pieces of the persistent recurrent kernels (lstm_persist.hip, gru_persist.hip): the
// cross-workgroup hand-off protocol of cdna_hip_programming.md §6 Guideline 16 ("Valid forms"
// row 1: sc1 write-through payload stores drained before an agent-scope counter add; consumers
// poll the counter with sc1 loads, a workgroup barrier releases the other waves, and every load
// of handed-off bytes is a `buffer_load ... sc1`), plus the block -> tile mapping.
#pragma once
#include "common.h"

namespace dcr {

constexpr int kAuxSc1 = 16;  // buffer-op cache-policy bits: sc1 (bypass L1, write-through)
#ifndef XCD_GROUPING
#define XCD_GROUPING 1
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, size_t bytes) {
  const unsigned n = bytes > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (unsigned)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, n, 0x00020000);
}
__device__ __forceinline__ bf16x8 ld8_sc1(__amdgpu_buffer_rsrc_t r, unsigned byte_off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, kAuxSc1);
  return __builtin_bit_cast(bf16x8, v);
}
// The same with the address split into a per-lane VGPR part and a wave-uniform part passed as
// the instruction's SGPR offset: a loop that loads many fragments then keeps ONE offset VGPR
// instead of one per fragment (the KS = 16 BPTT had spilled its hoisted offsets to scratch,
// each reload a serialising vmcnt(0) in the payload loop).
__device__ __forceinline__ bf16x8 ld8_sc1(__amdgpu_buffer_rsrc_t r, unsigned lane_off,
                                          unsigned uniform_off) {
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, lane_off, uniform_off, kAuxSc1);
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ void st4bf_sc1(bf16* p, float a, float b, float c, float d) {
  bf16x4 v;
  v[0] = f2bf(a); v[1] = f2bf(b); v[2] = f2bf(c); v[3] = f2bf(d);
  __hip_atomic_store(reinterpret_cast<uint64_t*>(p), __builtin_bit_cast(uint64_t, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st4bf(bf16* p, float a, float b, float c, float d) {
  bf16x4 v;
  v[0] = f2bf(a); v[1] = f2bf(b); v[2] = f2bf(c); v[3] = f2bf(d);
  *reinterpret_cast<bf16x4*>(p) = v;
}

// ---- XCD-resident hand-offs ------------------------------------------------------------------
// A batch column's hand-off (its producers and consumers are the same workgroup set) can keep its
// lines in ONE XCD's L2 when every workgroup of the column runs on that XCD: the payload is then
// stored PLAIN (the line stays in the producer XCD's L2; an sc1 store writes through and DROPS
// it, so a same-XCD reader pays the fabric round trip: MI355X_MICROARCH.md, "stores of each
// flavour"), still drained with vmcnt(0) before the counter add; consumers keep sc1 loads (L1
// bypass, L2-served) after the poll.  HIP promises no placement, so it is checked in-kernel: each
// workgroup adds 1 << (8 XCC_ID) to its column's 8-B exchange word (zeroed with the counters)
// and waits until all nwg (<= 255) have; the column runs local only if one byte holds them all,
// otherwise it keeps the write-through protocol above.  Every workgroup of a column reads the
// same final word, so producers and consumers agree.  Validated by scripts/micro/handoff_xcd.hip
// (tagged lines, uneven load) and bitwise against the write-through protocol
// (tests/test_handoff_local.py).
__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7u;
}
__device__ __forceinline__ void xcd_publish(unsigned long long* word) {
  __hip_atomic_fetch_add(word, 1ull << (8 * xcc_id()), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// (one lane) 1: all nwg workgroups of the column share one XCD; 0: not, or timed out (error
// word set, the caller keeps going so the grid drains)
__device__ __forceinline__ int xcd_decide(unsigned long long* word, unsigned nwg, unsigned limit,
                                          unsigned* err, unsigned code) {
  unsigned spins = 0;
  for (;;) {
    const unsigned long long m = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned tot = 0;
    int one = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const unsigned c = (unsigned)(m >> (8 * i)) & 0xFFu;
      tot += c;
      one |= c == nwg;
    }
    if (tot >= nwg) return one;
    if (++spins > limit) {
      __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return 0;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
// The local form's signal is not an atomic counter (agent-scope atomics are performed at the
// memory side and drop the line: ~1.5 us of a 3.1 us tick in scripts/micro/handoff_xcd.hip) but
// one flag dword per producing workgroup and layer, stored plain (L2-resident) by the LAST of the
// workgroup's storing waves (LDS counter, every storing wave drained first): value = producing
// tick + 1, monotonic.  One consumer wave polls all flags of both layers with ONE sc1 dword
// load per lane (lanes [0, n): layer l, [32, 32 + n): layer l+1) and a wave vote: 1.35 vs 3.11 us
// per tick in the micro-benchmark, no stale tag over 48k checked column-ticks.  The flags live
// in the (then unused) counter slots 1-8 of each layer's column region (needs T >= 8, n <= 32).
__device__ __forceinline__ void wg_arrive_flag(unsigned* lds_cnt, unsigned nwaves, unsigned* flag,
                                               unsigned value) {
  const unsigned old = __hip_atomic_fetch_add(lds_cnt, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
  if (old == nwaves - 1) {
    __hip_atomic_store(lds_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_store(flag, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // plain
  }
}
// (a whole wave) wait until the n flags of each needed layer are >= target; false on timeout
// (error word set)
__device__ __forceinline__ bool poll_flags2(const unsigned* f0, bool need0, const unsigned* f1,
                                            bool need1, int n, unsigned target, unsigned limit,
                                            unsigned* err, unsigned code) {
  const int lane = threadIdx.x & 63, i = lane & 31;
  const bool hi = lane >= 32;
  const bool watch = i < n && (hi ? need1 : need0);
  const unsigned* p = (hi ? f1 : f0) + (i < n ? i : 0);
  unsigned spins = 0;
  for (;;) {
    const unsigned v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__all(!watch || v >= target)) return true;
    if (++spins > limit) {
      if (lane == 0) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
// (a whole wave) the same for one set of n <= 64 flags (lane i watches flag i)
__device__ __forceinline__ bool poll_flags1(const unsigned* f, int n, unsigned target,
                                            unsigned limit, unsigned* err, unsigned code) {
  const int lane = threadIdx.x & 63;
  const bool watch = lane < n;
  const unsigned* p = f + (watch ? lane : 0);
  unsigned spins = 0;
  for (;;) {
    const unsigned v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__all(!watch || v >= target)) return true;
    if (++spins > limit) {
      if (lane == 0) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
// a hand-off payload store: plain when the column is XCD-local, write-through (sc1) otherwise
__device__ __forceinline__ void st4bf_ho(bool local, bf16* p, float a, float b, float c, float d) {
  if (local)
    st4bf(p, a, b, c, d);
  else
    st4bf_sc1(p, a, b, c, d);
}
__device__ __forceinline__ void ld4bf(const bf16* p, float (&o)[4]) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  o[0] = (float)v[0]; o[1] = (float)v[1]; o[2] = (float)v[2]; o[3] = (float)v[3];
}
__device__ __forceinline__ void ld4f(const float* p, float (&o)[4]) {
  const float4 v = *reinterpret_cast<const float4*>(p);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}

// Hand-off protocol (MI355X_MICROARCH.md "Valid forms", third row, matched in every cell):
//   producer: every handed-off byte stored sc1 (global_store_dwordx2 sc1; every 128-B line
//             written whole by one store instruction of one wave: the fragment-order rings
//             below), the storing wave's s_waitcnt vmcnt(0), then ONE lane of that wave adds 1
//             to the (batch group, step) counter (agent-scope atomic);
//   consumer: ONE lane polls that counter with global_load_dword sc1 (+ s_sleep), a workgroup
//             barrier, then every load of the bytes is buffer_load_dwordx4 sc1.
// One unsharded counter per (batch group, step): a single dword poll per iteration (polling
// four quarter shards with four dword loads cost 13 % on the GRU).  Returns false on timeout
// after setting the error word; the caller keeps going so the grid always drains.
__device__ __forceinline__ bool poll_counter(unsigned* cnt, unsigned target, unsigned limit,
                                             unsigned* err, unsigned code) {
  unsigned spins = 0;
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    if (++spins > limit) {
      __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// Sharded form (the same table's FIRST row): ONE lane of each storing workgroup signals for ALL
// that workgroup's stores -- every epilogue wave drains (vmcnt(0)) and then adds to an LDS
// counter, and the wave whose add comes last does the agent-scope add -- on one of four shards
// (the workgroup's K quarter); the consumer polls every shard with one 16-B sc1 load.  Used by
// the GRU, whose H/16 = 64 epilogue waves per counter (H = 1024) made a single counter's atomics
// the bottleneck (21.7 vs 14.4 ms per step).
__device__ __forceinline__ bool poll_shards4(unsigned* cnt4, unsigned target, unsigned limit,
                                             unsigned* err, unsigned code) {
  const __amdgpu_buffer_rsrc_t r = make_rsrc(cnt4, 16);
  unsigned spins = 0;
  for (;;) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, kAuxSc1);
    if (v[0] >= target && v[1] >= target && v[2] >= target && v[3] >= target) return true;
    if (++spins > limit) {
      __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Workgroup-level arrival (first-row form): call from lane 0 of each of the `nwaves` storing
// waves AFTER that wave's s_waitcnt vmcnt(0); the last of them adds 1 to `shard`.
__device__ __forceinline__ void wg_arrive(unsigned* lds_cnt, unsigned nwaves, unsigned* shard) {
  if (nwaves == 1) {  // the workgroup's only storing wave signals for itself
    __hip_atomic_fetch_add(shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const unsigned old = __hip_atomic_fetch_add(lds_cnt, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
  if (old == nwaves - 1) {
    __hip_atomic_store(lds_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_add(shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Two counters polled together (both dword loads in flight per iteration): the two-layer
// wavefront waits for both layers' previous tick without a second round trip.
__device__ __forceinline__ bool poll_counter2(unsigned* c0, unsigned t0, unsigned* c1,
                                              unsigned t1, unsigned limit, unsigned* err,
                                              unsigned code) {
  unsigned spins = 0;
  for (;;) {
    const unsigned v0 = __hip_atomic_load(c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned v1 = __hip_atomic_load(c1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v0 >= t0 && v1 >= t1) return true;
    if (++spins > limit) {
      __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Index helpers below are __host__ __device__ so tests/native/layout_check.hip can verify them
// on the host under ASan/UBSan (tests/test_native_host.py).
// Fragment-tiled hand-off layout.  Element (b, k) of a [B, K] bf16 slab lives at
//   ((b/16 * K/32 + k/32) * 64 + ((k%32)/8)*16 + b%16) * 8 + k%8        (bf16 elements)
// i.e. exactly where mfma_f32_16x16x32_bf16's B fragment of (batch tile b/16, k-step k/32)
// wants it: a consumer wave's load of one k-step is ONE contiguous 1 KB buffer_load (lane l at
// byte 16*l), instead of 16 rows x 64 B of a row-major slab.  Measured with sc1 loads, 64 KB per
// workgroup, 256 workgroups: 0.60 vs 1.74 us (half the L2 requests;
// scripts/micro/payload_pattern.hip).  Producers' 4-unit (8 B) stores land 8-B aligned.
__host__ __device__ __forceinline__ size_t frag_index(int b, int k, int K) {
  return ((size_t)((b >> 4) * (K >> 5) + (k >> 5)) * 64 + ((k & 31) >> 3) * 16 + (b & 15)) * 8 +
         (k & 7);
}
__host__ __device__ __forceinline__ unsigned frag_load_off(int bg, int kstep, int K, int lane) {
  return (unsigned)((((size_t)bg * (K >> 5) + kstep) * 64 + lane) * 16);
}
// A copy of `x` the compiler cannot see through: offsets built from it inside a loop stay in
// the loop (base + constant, the constant folded into the load's immediate offset where it
// fits) instead of being hoisted as one register per fragment.
__device__ __forceinline__ unsigned opaque_vgpr(unsigned x) {
  unsigned r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// frag_load_off = lane * 16 + frag_tile_off (the wave-uniform part)
__host__ __device__ __forceinline__ unsigned frag_tile_off(int bg, int kstep, int K) {
  return (unsigned)(((size_t)bg * (K >> 5) + kstep) * 1024);
}

// Block -> (unit block, batch group).  Place the unit-block workgroups of one batch group on the
// same XCD under the observed round-robin dispatch (blocks b, b+8, ... share an XCD;
// MI355X_MICROARCH.md "Workgroup dispatch"), so the batch group's hand-off payload stays in one
// L2.  Correctness never depends on the placement: the kernel checks it at run time (xcd_decide
// above) and a column takes the XCD-local form (plain stores + per-workgroup flags) only when
// all its workgroups were found on one XCD, otherwise the write-through form (sc1 stores +
// arrival counters).
__host__ __device__ __forceinline__ void map_block(int bid, int nwg_u, int nbg, int& ubk,
                                                    int& bg) {
  if (nbg % 8 == 0 && XCD_GROUPING) {
    const int xcd = bid % 8, j = bid / 8;  // j in [0, nwg_u * nbg / 8)
    bg = xcd + 8 * (j / nwg_u);
    ubk = j % nwg_u;
  } else {
    ubk = bid % nwg_u;
    bg = bid / nwg_u;
  }
}

// Grid of a column-mapped persistent launch padded to whole XCD groups: 8 x nwg_u workgroups per
// 8 columns.  Under round-robin dispatch blocks b, b + 8, ... share an XCD, so with this grid
// every column's nwg_u workgroups can sit on ONE XCD even when there are fewer than 8
// (or not a multiple of 8) columns -- the XCD-resident hand-off form then applies to the small
// shapes too (the reference default B = 50 has 2 forward columns).  Blocks of the padding
// columns exit at once.  The launcher uses it only when the padded grid is still co-resident;
// with a multiple of 8 columns it equals the plain grid.
__host__ __device__ __forceinline__ int xcd_grid(int nwg_u, int ncol) {
  return 8 * nwg_u * ((ncol + 7) / 8);
}
// map_block for a launch of `grid` workgroups: the XCD-grouped map when grid == xcd_grid (false
// for a padding block, which must exit), otherwise the plain column-major map
__host__ __device__ __forceinline__ bool map_block_grid(int bid, int grid, int nwg_u, int ncol,
                                                        int& ubk, int& col) {
  if (XCD_GROUPING && grid == xcd_grid(nwg_u, ncol)) {
    const int x = bid % 8, j = bid / 8;
    col = x + 8 * (j / nwg_u);
    ubk = j % nwg_u;
    return col < ncol;
  }
  ubk = bid % nwg_u;
  col = bid / nwg_u;
  return true;
}

// Hand-off poller.  GRU kernels poll from lane 0 of wave 3, which never runs a cell epilogue
// (UB * NT <= 3), so polling overlaps the epilogue waves' drain and post-arrival work: 3-layer
// GRU-1024 16.8 -> 15.3 ms/step.  The LSTM kernels keep the poller on wave 0 (an epilogue wave):
// the same change measured 2.74 -> 3.18 ms/step there (forward 420 -> 508 us per layer).
constexpr int kPollerThread = 192;
constexpr int kLstmPollerThread = 0;

__device__ __forceinline__ void arrive(unsigned* cnt) {
  // every store of this wave must be complete (write-through) before the counter moves
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace dcr
