// Microbenchmark: per-step hand-off payload read, 64 KB per workgroup, sc1 buffer loads.
//   pattern 0: MFMA B-fragment order over row-major rows (what the persistent BPTT does):
//              lane -> row (lane & 15) x 4 KB stride, 16 B at column 16*(lane>>4) + 64*s
//   pattern 1: fragment-tiled: the same 16 B per lane, but the 64 lanes' fragments of one
//              k-step are contiguous (1 KB per instruction)
// Each of R rounds: 4 waves x 16 loads (64 KB) -> sum into a register; workgroup barrier.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int PAT>
__global__ void __launch_bounds__(256) payload(const unsigned* buf, unsigned* out, int rounds) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int grp = blockIdx.x % 16;  // 16 "batch groups", each 64 KB x rounds
  const char* base = reinterpret_cast<const char*>(buf) + (size_t)grp * 64 * 1024;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, 64 * 1024, 0x00020000);
  unsigned acc = 0;
  for (int it = 0; it < rounds; ++it) {
    u32x4 v[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      unsigned off;
      if (PAT == 0) off = (lane & 15) * 4096 + 16 * (lane >> 4) + 64 * (w * 16 + s);
      else off = ((w * 16 + s) * 64 + lane) * 16;
      v[s] = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16 /* sc1 */);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) acc += v[s][0] ^ v[s][3];
    __syncthreads();
  }
  if (acc == 0x12345678) out[0] = acc;
}

int main() {
  unsigned *buf, *out;
  hipMalloc(&buf, 16 * 64 * 1024);
  hipMalloc(&out, 16);
  hipMemset(buf, 1, 16 * 64 * 1024);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int R = 2000;
  for (int pat = 0; pat < 2; ++pat) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(a);
      if (pat == 0) payload<0><<<256, 256>>>(buf, out, R);
      else payload<1><<<256, 256>>>(buf, out, R);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (rep == 2) printf("pattern %d: %.3f us per 64 KB round per workgroup\n", pat, ms * 1e3 / R);
    }
  }
  return 0;
}
