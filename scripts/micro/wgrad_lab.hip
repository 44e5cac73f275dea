// Where does csrc/wgrad.hip's time go?  Its measurement variants (template V, see the kernel)
// timed on the headline step's launch (layer-1 [1024 x 2048] + layer-0 [512 x 2048], K = 32768,
// 5 slabs, 240 workgroups) in ONE process, interleaved rounds, median; V = 0 and the 5-stage
// ring are checked against an fp32 reference.  Build here, run on the GPU box:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I csrc scripts/micro/wgrad_lab.hip -o build/wgrad_lab
//   ./build/wgrad_lab
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../csrc/wgrad.hip"

using namespace dcr;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

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

typedef void (*KFn)(WgradArgs);
struct Variant { const char* name; KFn fn; bool check; };

int main() {
  const int H = 512, B = 256, T = 128, K = T * B;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  printf("%s, %d CUs\n", prop.gcnArchName, prop.multiProcessorCount);
  bf16 *Cp, *dz1, *dz0;
  CK(hipMalloc(&Cp, (size_t)(T + 2) * B * 2 * H * 2));
  CK(hipMalloc(&dz1, (size_t)K * 4 * H * 2));
  CK(hipMalloc(&dz0, (size_t)K * 4 * H * 2));
  fill_kernel<<<1024, 256>>>(Cp, (size_t)(T + 2) * B * 2 * H, 1);
  fill_kernel<<<1024, 256>>>(dz1, (size_t)K * 4 * H, 2);
  fill_kernel<<<1024, 256>>>(dz0, (size_t)K * 4 * H, 3);
  const bf16* A1 = Cp + (size_t)B * 2 * H;  // [x_t ; h_{t-1}] rows of layer 1, [K, 2H]
  const bf16* A2 = Cp;                       // h0_{t-1}: first H columns, lda 2H
  float *part, *ref1, *ref2, *sum;
  CK(hipMalloc(&part, (size_t)8 * 1536 * 2048 * 4));
  CK(hipMalloc(&ref1, (size_t)1024 * 2048 * 4));
  CK(hipMalloc(&ref2, (size_t)512 * 2048 * 4));
  CK(hipMalloc(&sum, (size_t)1024 * 2048 * 4));
  ref_kernel<<<dim3(2048 / 16, 1024 / 16), dim3(16, 16)>>>(A1, 2 * H, dz1, 4 * H, K, 1024, 2048, ref1);
  ref_kernel<<<dim3(2048 / 16, 512 / 16), dim3(16, 16)>>>(A2, 2 * H, dz0, 4 * H, K, 512, 2048, ref2);
  CK(hipDeviceSynchronize());

  Variant vars[] = {
      {"step (V=0)", wgrad_kernel<0>, true},
      {"runtime waits (r5)", wgrad_kernel<128>, true},
      {"prio over MFMA groups", wgrad_kernel<256>, true},
      {"DMA after groups 1, 2", wgrad_kernel<512>, true},
      {"prio + late DMA", wgrad_kernel<768>, true},
      {"5-stage ring", wgrad_kernel<8>, true},
      {"L2-hot operands", wgrad_kernel<1>, false},
      {"no DMA", wgrad_kernel<2>, false},
      {"no DMA, no barrier", wgrad_kernel<6>, false},
      {"A panel DMA only", wgrad_kernel<16>, false},
      {"DMA never waited", wgrad_kernel<32>, false},
      {"hot, never waited", wgrad_kernel<33>, false},
      {"barrier w/o lgkmcnt(0)", wgrad_kernel<64>, true},
      {"no DMA, bar w/o lgkm", wgrad_kernel<66>, false},
  };
  const int nv = sizeof(vars) / sizeof(vars[0]);
  const int S = wgrad_splits_tiles(48, K, prop.multiProcessorCount);
  WgradArgs a{};
  a.np = 2;
  a.K = K;
  a.p[0] = WgradProblem{A1, 2 * H, dz1, 4 * H, part, 2048, 1024L * 2048, 1024, 2048, S, 0, 0};
  a.p[1] = WgradProblem{A2, 2 * H, dz0, 4 * H, part + (size_t)S * 1024 * 2048, 2048, 512L * 2048,
                        512, 2048, S, 0, 0};
  int items = 0;
  for (int i = 0; i < a.np; ++i) {
    a.p[i].tiles = (a.p[i].M / kWgTile) * (a.p[i].N / kWgTile);
    a.p[i].item0 = items;
    items += a.p[i].tiles * a.p[i].S;
  }
  a.items = items;
  const int grid = (items + 7) / 8 * 8;
  const double flops = 2.0 * K * (1024 + 512) * 2048;
  printf("S = %d, %d workgroups\n", S, items);
  for (int vi = 0; vi < nv; ++vi) {
    hipLaunchKernelGGL(vars[vi].fn, dim3(grid), dim3(64 * kWgWaves), 0, 0, a);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    if (!vars[vi].check) continue;
    double maxrel = 0;
    for (int pi = 0; pi < a.np; ++pi) {
      const WgradProblem& p = a.p[pi];
      const size_t mn = (size_t)p.M * p.N;
      slabsum_kernel<<<1024, 256>>>(p.C, p.S, mn, sum);
      std::vector<float> h(mn), r(mn);
      CK(hipMemcpy(h.data(), sum, mn * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r.data(), pi == 0 ? ref1 : ref2, mn * 4, hipMemcpyDeviceToHost));
      double num = 0, den = 0;
      for (size_t i = 0; i < mn; ++i) {
        num += (h[i] - r[i]) * (double)(h[i] - r[i]);
        den += (double)r[i] * r[i];
      }
      maxrel = std::max(maxrel, std::sqrt(num / den));
    }
    printf("  %-22s rel err %.2e%s\n", vars[vi].name, maxrel, maxrel > 1e-4 ? "  !! WRONG" : "");
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int R = 7, reps = 10;
  std::vector<std::vector<float>> t(nv);
  for (int r = 0; r < R; ++r)
    for (int vi = 0; vi < nv; ++vi) {
      hipLaunchKernelGGL(vars[vi].fn, dim3(grid), dim3(64 * kWgWaves), 0, 0, a);
      CK(hipEventRecord(e0));
      for (int k = 0; k < reps; ++k)
        hipLaunchKernelGGL(vars[vi].fn, dim3(grid), dim3(64 * kWgWaves), 0, 0, a);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[vi].push_back(ms * 1e3f / reps);
    }
  for (int vi = 0; vi < nv; ++vi) {
    std::sort(t[vi].begin(), t[vi].end());
    printf("  %-22s median %7.1f us  min %7.1f us  %6.0f TF/s\n", vars[vi].name, t[vi][R / 2],
           t[vi][0], flops / (t[vi][R / 2] * 1e-6) / 1e12);
  }
  return 0;
}
