// Standalone lab for the token-reduction weight-gradient GEMM (C_s = A_sᵀ B_s over split-K
// slabs, both operands token-major): variants of csrc/wgrad.hip's pipeline timed on the
// headline's shapes in ONE process (interleaved rounds, median), checked against an fp32
// reference.  Build here, run on the GPU box:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I csrc scripts/micro/gemm_lab.hip -o build/gemm_lab
//   ./build/gemm_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.h"

using namespace dcr;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

struct Prob {
  const bf16* A; long lda;
  const bf16* B; long ldb;
  float* C; long ldc; long slab;
  int M, N, S, tiles, tile0;  // tile0: first work item of this problem
};
struct LabArgs {
  Prob p[4];
  int np, K, items;
};

constexpr int kTile = 256, kK = 32, kWaves = 8;
constexpr int kStageB = 2 * kK * kTile * 2;
constexpr int kDmaPerWave = 32 / kWaves;

__device__ __forceinline__ int swz(int r) { return 2 * (r & 7) + ((r >> 4) & 1); }
__device__ __forceinline__ void barrier_raw() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void vm_wait(int n) {
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
typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x2 rd_tr(unsigned addr) {
  return __builtin_bit_cast(u32x2, __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                                       (__attribute__((address_space(3))) s16x4*)(size_t)addr));
}
__device__ __forceinline__ void dma(__amdgpu_buffer_rsrc_t r, unsigned lds, unsigned voff, unsigned soff) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(lds), "v"(voff), "s"(r), "s"(soff) : "memory");
}

// VAR: bits 0-1 priority (0 none, 1 static waves 4-7, 2 per MFMA cluster), bit 2: 5 stages,
// bit 3: XCD map "per-problem block" (items of a problem spread over XCDs slab-major)
template <int VAR>
__global__ void __launch_bounds__(512, 2) lab_kernel(LabArgs a) {
  constexpr int ST = (VAR & 4) ? 5 : 4;
  constexpr int PRIO = VAR & 3;
  extern __shared__ __attribute__((aligned(1024))) unsigned char lds[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nb = gridDim.x;
  const int lin = (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8;
  if (lin >= a.items) return;
  int pi = 0;
  while (pi + 1 < a.np && lin >= a.p[pi + 1].tile0) ++pi;
  const Prob& P = a.p[pi];
  const int loc = lin - P.tile0;
  const int s = loc / P.tiles, tile = loc % P.tiles;
  const int tn = P.N / kTile;
  const int m0 = (tile / tn) * kTile, n0 = (tile % tn) * kTile;
  const int ksteps = a.K / kK;
  const int kt0 = (int)((long)ksteps * s / P.S), kt1 = (int)((long)ksteps * (s + 1) / P.S);
  const int nk = kt1 - kt0;
  if constexpr (PRIO == 1) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  }

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(P.A), (short)0, 0x7FFFFFF0, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(P.B), (short)0, 0x7FFFFFF0, 0x00020000);
  unsigned offa[kDmaPerWave / 2], offb[kDmaPerWave / 2];
#pragma unroll
  for (int j = 0; j < kDmaPerWave / 2; ++j) {
    const int r = kDmaPerWave * w + 2 * j + (lane >> 5);
    const int c = (lane & 31) ^ swz(r);
    offa[j] = (unsigned)(((size_t)r * P.lda + m0 + 8 * c) * sizeof(bf16));
    offb[j] = (unsigned)(((size_t)r * P.ldb + n0 + 8 * c) * sizeof(bf16));
  }
  const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)lds;
  auto issue = [&](int kt) {
    const unsigned st = lds0 + ((kt - kt0) % ST) * kStageB;
    const unsigned sa = (unsigned)((size_t)kt * kK * P.lda * sizeof(bf16));
    const unsigned sb = (unsigned)((size_t)kt * kK * P.ldb * sizeof(bf16));
#pragma unroll
    for (int j = 0; j < kDmaPerWave / 2; ++j) {
      const unsigned r = (unsigned)(kDmaPerWave * w + 2 * j);
      dma(ra, st + r * 512, offa[j], sa);
      dma(rb, st + kK * 512 + r * 512, offb[j], sb);
    }
  };
  const int q = lane >> 4, ta = (lane & 15) >> 2, tp = lane & 3;
  const int bq = 4 * q + 8 * (q >> 1);
  const int wm = 128 * (w >> 2), wn = 64 * (w & 3);
  const int cb_a = (wm >> 3) + (tp >> 1), cb_b = (wn >> 3) + (tp >> 1);
  unsigned rowb[2], xa[2], xb[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = bq + ta + 8 * h;
    rowb[h] = (unsigned)(row * 512 + ((tp & 1) << 3));
    xa[h] = (unsigned)(cb_a ^ swz(row));
    xb[h] = (unsigned)(cb_b ^ swz(row));
  }
  auto read_frags = [&](int kt, u32x4 (&fa)[8], u32x4 (&fb)[4]) {
    const unsigned base = lds0 + ((kt - kt0) % ST) * kStageB;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const u32x2 lo = rd_tr(base + rowb[0] + ((xa[0] ^ (2u * i)) << 4));
      const u32x2 hi = rd_tr(base + rowb[1] + ((xa[1] ^ (2u * i)) << 4));
      fa[i] = u32x4{lo[0], lo[1], hi[0], hi[1]};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32x2 lo = rd_tr(base + kK * 512 + rowb[0] + ((xb[0] ^ (2u * j)) << 4));
      const u32x2 hi = rd_tr(base + kK * 512 + rowb[1] + ((xb[1] ^ (2u * j)) << 4));
      fb[j] = u32x4{lo[0], lo[1], hi[0], hi[1]};
    }
  };
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 fa0[8], fb0[4], fa1[8], fb1[4];
  if (nk > 0) {
    const int pro = nk < ST ? nk : ST;
    for (int j = 0; j < pro; ++j) issue(kt0 + j);
    vm_wait((pro - 1) * kDmaPerWave);
    barrier_raw();
    read_frags(kt0, fa0, fb0);
  }
  constexpr bool IL = (VAR & 16) != 0;
  auto mf = [&](int g, u32x4 (&fa)[8], u32x4 (&fb)[4]) {  // MFMA group g: rows 2g, 2g+1
#pragma unroll
    for (int ii = 2 * g; ii < 2 * g + 2; ++ii)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        acc[ii][jj] = mfma16(__builtin_bit_cast(bf16x8, fa[ii]), __builtin_bit_cast(bf16x8, fb[jj]), acc[ii][jj]);
  };
  auto rd_a = [&](int kt, u32x4 (&fa)[8], int i0, int i1) {
    const unsigned base = lds0 + ((kt - kt0) % ST) * kStageB;
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const u32x2 lo = rd_tr(base + rowb[0] + ((xa[0] ^ (2u * i)) << 4));
      const u32x2 hi = rd_tr(base + rowb[1] + ((xa[1] ^ (2u * i)) << 4));
      fa[i] = u32x4{lo[0], lo[1], hi[0], hi[1]};
    }
  };
  auto rd_b = [&](int kt, u32x4 (&fb)[4]) {
    const unsigned base = lds0 + ((kt - kt0) % ST) * kStageB;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32x2 lo = rd_tr(base + kK * 512 + rowb[0] + ((xb[0] ^ (2u * j)) << 4));
      const u32x2 hi = rd_tr(base + kK * 512 + rowb[1] + ((xb[1] ^ (2u * j)) << 4));
      fb[j] = u32x4{lo[0], lo[1], hi[0], hi[1]};
    }
  };
  auto kstep_il = [&](int i, u32x4 (&fa)[8], u32x4 (&fb)[4], u32x4 (&na)[8], u32x4 (&nb_)[4]) {
    const int kt = kt0 + i;
    const bool more = i + 1 < nk;
    if (more) {
      const int later = nk - 2 - i < ST - 2 ? nk - 2 - i : ST - 2;
      vm_wait(later * kDmaPerWave);
      barrier_raw();
    }
    __builtin_amdgcn_sched_barrier(0);
    mf(0, fa, fb);
    __builtin_amdgcn_sched_barrier(0);
    if (more && i + ST < nk) issue(kt + ST);
    __builtin_amdgcn_sched_barrier(0);
    mf(1, fa, fb);
    __builtin_amdgcn_sched_barrier(0);
    if (more) { rd_b(kt + 1, nb_); rd_a(kt + 1, na, 0, 2); }
    __builtin_amdgcn_sched_barrier(0);
    mf(2, fa, fb);
    __builtin_amdgcn_sched_barrier(0);
    if (more) rd_a(kt + 1, na, 2, 8);
    __builtin_amdgcn_sched_barrier(0);
    mf(3, fa, fb);
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr bool IL2 = (VAR & 32) != 0;
  auto issue_part = [&](int kt, int j) {  // this wave's DMA pair j of stage kt
    const unsigned st = lds0 + ((kt - kt0) % ST) * kStageB;
    const unsigned sa = (unsigned)((size_t)kt * kK * P.lda * sizeof(bf16));
    const unsigned sb = (unsigned)((size_t)kt * kK * P.ldb * sizeof(bf16));
    const unsigned r = (unsigned)(kDmaPerWave * w + 2 * j);
    dma(ra, st + r * 512, offa[j], sa);
    dma(rb, st + kK * 512 + r * 512, offb[j], sb);
  };
  auto kstep_il2 = [&](int i, u32x4 (&fa)[8], u32x4 (&fb)[4], u32x4 (&na)[8], u32x4 (&nb_)[4]) {
    const int kt = kt0 + i;
    const bool more = i + 1 < nk;
    const bool pf = more && i + ST < nk;
    if (more) {
      const int later = nk - 2 - i < ST - 2 ? nk - 2 - i : ST - 2;
      vm_wait(later * kDmaPerWave);
      barrier_raw();
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(1);
    mf(0, fa, fb);
    __builtin_amdgcn_sched_barrier(0);
    if (pf) issue_part(kt + ST, 0);
    if (more) rd_b(kt + 1, nb_);
    __builtin_amdgcn_sched_barrier(0);
    mf(1, fa, fb);
    __builtin_amdgcn_sched_barrier(0);
    if (pf) issue_part(kt + ST, 1);
    if (more) rd_a(kt + 1, na, 0, 3);
    __builtin_amdgcn_sched_barrier(0);
    mf(2, fa, fb);
    __builtin_amdgcn_sched_barrier(0);
    if (more) rd_a(kt + 1, na, 3, 8);
    __builtin_amdgcn_sched_barrier(0);
    mf(3, fa, fb);
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto kstep = [&](int i, u32x4 (&fa)[8], u32x4 (&fb)[4], u32x4 (&na)[8], u32x4 (&nb_)[4]) {
    if constexpr (IL2) { kstep_il2(i, fa, fb, na, nb_); return; }
    if constexpr (IL) { kstep_il(i, fa, fb, na, nb_); return; }
    const int kt = kt0 + i;
    if (i + 1 < nk) {
      const int later = nk - 2 - i < ST - 2 ? nk - 2 - i : ST - 2;
      vm_wait(later * kDmaPerWave);
      barrier_raw();
      if (i + ST < nk) issue(kt + ST);
      read_frags(kt + 1, na, nb_);
    }
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ii = 0; ii < 8; ++ii)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        acc[ii][jj] = mfma16(__builtin_bit_cast(bf16x8, fa[ii]), __builtin_bit_cast(bf16x8, fb[jj]), acc[ii][jj]);
    if constexpr (PRIO == 2) __builtin_amdgcn_s_setprio(0);
  };
  for (int i = 0; i < nk; i += 2) {
    kstep(i, fa0, fb0, fa1, fb1);
    if (i + 1 < nk) kstep(i + 1, fa1, fb1, fa0, fb0);
  }
  float* c = P.C + (size_t)s * P.slab + (size_t)(m0 + wm + 4 * q) * P.ldc + n0 + wn + (lane & 15);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) c[(size_t)(16 * i + r) * P.ldc + 16 * j] = acc[i][j][r];
}

// fp32 reference C[m][n] = sum_k A[k][m] B[k][n]
__global__ void ref_kernel(const bf16* A, long lda, const bf16* B, long ldb, int K, int M, int N,
                           float* C) {
  const int m = blockIdx.y * 16 + threadIdx.y, n = blockIdx.x * 16 + threadIdx.x;
  if (m >= M || n >= N) return;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) acc += (float)A[(size_t)k * lda + m] * (float)B[(size_t)k * ldb + n];
  C[(size_t)m * N + n] = acc;
}
__global__ void fill_kernel(bf16* x, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    x[i] = (bf16)(uniform01(seed, 7, i) * 2.f - 1.f);
}
__global__ void slabsum_kernel(const float* part, int S, size_t mn, float* out) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < mn; i += (size_t)gridDim.x * blockDim.x) {
    float t = 0.f;
    for (int s = 0; s < S; ++s) t += part[s * mn + i];
    out[i] = t;
  }
}

typedef void (*KFn)(LabArgs);
struct Variant { const char* name; KFn fn; int stages; };

int main() {
  const int K = 32768;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  printf("%s, %d CUs\n", prop.gcnArchName, prop.multiProcessorCount);
  // operands like the headline: C = [T+2, B, 2H] pair buffer (A1 = rows 1..T, A2 = rows 0..T-1
  // first H columns), dZ1, dZ0 [N, 4H]
  const int H = 512, B = 256, T = 128;
  bf16 *Cp, *dz1, *dz0;
  CK(hipMalloc(&Cp, (size_t)(T + 2) * B * 2 * H * 2));
  CK(hipMalloc(&dz1, (size_t)K * 4 * H * 2));
  CK(hipMalloc(&dz0, (size_t)K * 4 * H * 2));
  fill_kernel<<<1024, 256>>>(Cp, (size_t)(T + 2) * B * 2 * H, 1);
  fill_kernel<<<1024, 256>>>(dz1, (size_t)K * 4 * H, 2);
  fill_kernel<<<1024, 256>>>(dz0, (size_t)K * 4 * H, 3);
  const bf16* A1 = Cp + (size_t)B * 2 * H;  // rows 1..T, [K, 2H]
  const bf16* A2 = Cp;                       // rows 0..T-1, first H columns, lda 2H
  float* part;
  CK(hipMalloc(&part, (size_t)16 * 1536 * 2048 * 4));
  float *ref1, *ref2, *sum;
  CK(hipMalloc(&ref1, (size_t)1024 * 2048 * 4));
  CK(hipMalloc(&ref2, (size_t)512 * 2048 * 4));
  CK(hipMalloc(&sum, (size_t)1024 * 2048 * 4));
  ref_kernel<<<dim3(2048 / 16, 1024 / 16), dim3(16, 16)>>>(A1, 2 * H, dz1, 4 * H, K, 1024, 2048, ref1);
  ref_kernel<<<dim3(2048 / 16, 512 / 16), dim3(16, 16)>>>(A2, 2 * H, dz0, 4 * H, K, 512, 2048, ref2);
  CK(hipDeviceSynchronize());

  Variant vars[] = {
      {"v2", lab_kernel<0>, 4},         {"prio-static", lab_kernel<1>, 4},
      {"prio-cluster", lab_kernel<2>, 4},
      {"interleave", lab_kernel<16>, 4},  {"interleave2", lab_kernel<32>, 4},
      {"interleave2+prio-static", lab_kernel<33>, 4}, {"interleave2+prio-cluster", lab_kernel<34>, 4},
  };
  const int nv = sizeof(vars) / sizeof(vars[0]);
  for (auto& v : vars)
    CK(hipFuncSetAttribute((const void*)v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, v.stages * kStageB));

  struct Shape { const char* name; int np; int S1, S2; };
  Shape shapes[] = {{"P1 [1024x2048] S=8", 1, 8, 0}, {"P2 [512x2048] S=16", 2, 0, 16},
                    {"P1+P2 S=5", 3, 5, 5}, {"P1+P2 S=8/8 (384 WG)", 3, 8, 8}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& sh : shapes) {
    LabArgs a{};
    int items = 0;
    float* cp = part;
    double flops = 0;
    if (sh.np & 1) {
      Prob& p = a.p[a.np++];
      p = Prob{A1, 2 * H, dz1, 4 * H, cp, 2048, 1024L * 2048, 1024, 2048, sh.S1, 32, items};
      items += 32 * sh.S1;
      cp += (size_t)sh.S1 * 1024 * 2048;
      flops += 2.0 * K * 1024 * 2048;
    }
    if (sh.np & 2) {
      Prob& p = a.p[a.np++];
      p = Prob{A2, 2 * H, dz0, 4 * H, cp, 2048, 512L * 2048, 512, 2048, sh.S2, 16, items};
      items += 16 * sh.S2;
      flops += 2.0 * K * 512 * 2048;
    }
    a.K = K;
    a.items = items;
    const int grid = (items + 7) / 8 * 8;
    // correctness (each variant once)
    for (int vi = 0; vi < nv; ++vi) {
      hipLaunchKernelGGL(vars[vi].fn, dim3(grid), dim3(512), vars[vi].stages * kStageB, 0, a);
      CK(hipGetLastError());
      double maxrel = 0;
      for (int pi = 0; pi < a.np; ++pi) {
        const Prob& p = a.p[pi];
        const size_t mn = (size_t)p.M * p.N;
        slabsum_kernel<<<1024, 256>>>(p.C, p.S, mn, sum);
        std::vector<float> h(mn), r(mn);
        CK(hipMemcpy(h.data(), sum, mn * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r.data(), p.M == 1024 ? ref1 : ref2, mn * 4, hipMemcpyDeviceToHost));
        double num = 0, den = 0;
        for (size_t i = 0; i < mn; ++i) {
          num += (h[i] - r[i]) * (double)(h[i] - r[i]);
          den += (double)r[i] * r[i];
        }
        maxrel = std::max(maxrel, sqrt(num / den));
      }
      if (maxrel > 1e-4) printf("  !! %s %s rel err %.2e\n", sh.name, vars[vi].name, maxrel);
    }
    // timing: interleaved rounds
    const int R = 7, reps = 10;
    std::vector<std::vector<float>> t(nv);
    for (int r = 0; r < R; ++r)
      for (int vi = 0; vi < nv; ++vi) {
        hipLaunchKernelGGL(vars[vi].fn, dim3(grid), dim3(512), vars[vi].stages * kStageB, 0, a);
        CK(hipEventRecord(e0));
        for (int k = 0; k < reps; ++k)
          hipLaunchKernelGGL(vars[vi].fn, dim3(grid), dim3(512), vars[vi].stages * kStageB, 0, a);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t[vi].push_back(ms * 1e3f / reps);
      }
    printf("%s (%d WG):\n", sh.name, items);
    for (int vi = 0; vi < nv; ++vi) {
      std::sort(t[vi].begin(), t[vi].end());
      printf("  %-22s median %7.1f us  min %7.1f us  %6.0f TF/s\n", vars[vi].name, t[vi][R / 2],
             t[vi][0], flops / (t[vi][R / 2] * 1e-6) / 1e12);
    }
    fflush(stdout);
  }
  return 0;
}
