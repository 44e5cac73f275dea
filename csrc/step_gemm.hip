// Split-K "step GEMM" of the large-H recurrent layers (native_backend._lstm_*_lib):
//   partial[z][b][n] = sum_{k in split z} X[b][k] * W[n][k]
// X = [B, K] bf16 rows (h_{t-1} forward, dZ_{t+1} BPTT), W = [N, K] bf16 rows, K contiguous for
// both (W_hᵀ [4H, H] forward, W_h [H, 4H] BPTT: the persistent layouts the backend keeps), fp32
// partial slabs summed by the epilogue-only cell kernel (rnn_step.hip, zrec / partial with
// nsplit).  One step's W_h (32 MB at H = 2048) is read exactly once per step and the payload X
// once per 32*NTW output rows; split-K over z fills the 256 CUs although M = B is small.
//
// Workgroup = 64 batch rows x 32*NTW weight rows x K/S.  4 waves: token half th = w&1 (32 rows =
// 2 tiles), row half ch = w>>1 (16*NTW rows = NTW tiles): acc[NTW][2] fp32 fragments per lane.
// K streams in 32-wide stages through a 3-stage LDS ring filled by LDS-DMA
// (global_load_lds_dwordx4) in MFMA fragment order (lane-linear, bank-conflict-free), two stages
// in flight across raw barriers -- the structure of optim.hip's tok_norm kernel.
#include "common.h"
#include "kernels.h"

namespace dcr {

constexpr int kSgTok = 64;  // batch rows per workgroup

static constexpr unsigned sg_waitcnt_vm(unsigned n) {
  return (n & 15u) | ((n >> 4) << 14) | (7u << 4) | (15u << 8);
}

template <int NTW>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2)))
step_gemm_kernel(const bf16* __restrict__ X, const bf16* __restrict__ W, int B, int N, int K,
                 int kc, float* __restrict__ part) {
  constexpr int kWTiles = 2 * NTW;
  constexpr int kTiles = kWTiles + kSgTok / 16;
  constexpr int kPer = kTiles / 4;
  constexpr int kStage = kTiles * 512;
  constexpr int kRing = 3;
  static_assert(kTiles % 4 == 0, "NTW must be even");
  __shared__ __attribute__((aligned(16))) bf16 lds[kRing * kStage];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int th = wv & 1, ch = wv >> 1;
  const int n0 = blockIdx.x * (32 * NTW), b0 = blockIdx.y * kSgTok, z = blockIdx.z;
  const int k0 = z * kc;

  // DMA instruction i of wave wv moves tile 4 i + wv: lane l loads row 64 i + 16 wv + (l & 15),
  // 16-B k-chunk l >> 4; rows < 32*NTW are weight rows (i < NTW/2), the rest batch rows
  const int rr = 16 * wv + (lane & 15), cc = lane >> 4;
  const bf16* wsrc = W + (size_t)(n0 + rr) * K + k0 + 8 * cc;
  const bf16* xsrc = X + (size_t)(b0 + rr) * K + k0 + 8 * cc;
  auto issue = [&](int s, int buf) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const bf16* g = (i < NTW / 2 ? wsrc + (size_t)(64 * i) * K
                                   : xsrc + (size_t)(64 * (i - NTW / 2)) * K) + 32 * s;
      __builtin_amdgcn_global_load_lds(
          reinterpret_cast<const void*>(g),
          reinterpret_cast<__attribute__((address_space(3))) void*>(
              (__attribute__((address_space(3))) bf16*)&lds[buf * kStage + (4 * i + wv) * 512]),
          16, 0, 0);
    }
  };

  f32x4 acc[NTW][2];
#pragma unroll
  for (int a = 0; a < NTW; ++a)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[a][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const bf16* base = &lds[buf * kStage + lane * 8];
    bf16x8 bt[2], at[NTW];
#pragma unroll
    for (int j = 0; j < 2; ++j)
      bt[j] = *reinterpret_cast<const bf16x8*>(base + (kWTiles + 2 * th + j) * 512);
#pragma unroll
    for (int a = 0; a < NTW; ++a)
      at[a] = *reinterpret_cast<const bf16x8*>(base + (ch * NTW + a) * 512);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int a = 0; a < NTW; ++a)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        // AGPR-pinned accumulators (see optim.hip tok_norm_kernel)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                     : "+a"(acc[a][j]) : "v"(at[a]), "v"(bt[j]));
  };

  const int S = kc / 32;
  issue(0, 0);
  issue(S > 1 ? 1 : 0, 1);
  int q0 = 0, q1 = 1, q2 = 2;
  for (int s = 0; s < S; ++s) {
    __builtin_amdgcn_s_waitcnt(sg_waitcnt_vm(kPer));
    __builtin_amdgcn_s_barrier();
    issue(min(s + 2, S - 1), q2);
    compute(q0);
    const int t = q0;
    q0 = q1;
    q1 = q2;
    q2 = t;
  }
  __builtin_amdgcn_s_waitcnt(sg_waitcnt_vm(0));
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  // C tile (a, j): lane l holds C[n = 4 (l >> 4) + r][b = l & 15] -> 4 consecutive n of one b
  float* pz = part + (size_t)z * B * N;
#pragma unroll
  for (int a = 0; a < NTW; ++a)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 16 * (ch * NTW + a) + 4 * (lane >> 4);
      const int b = b0 + 16 * (2 * th + j) + (lane & 15);
      *reinterpret_cast<float4*>(pz + (size_t)b * N + n) =
          make_float4(acc[a][j][0], acc[a][j][1], acc[a][j][2], acc[a][j][3]);
    }
}

static int sg_ntw(int N) { return N % 256 == 0 ? 8 : N % 128 == 0 ? 4 : 2; }

bool step_gemm_supported(int B, int N, int K) {
  return B > 0 && B % kSgTok == 0 && N % 64 == 0 && K % 32 == 0 && K > 0;
}

// split count so that the grid reaches ~256 workgroups with >= 256-deep K slices
int step_gemm_splits(int B, int N, int K) {
  const int blocks = (N / (32 * sg_ntw(N))) * (B / kSgTok);
  int s = 1;
  while (blocks * s * 2 <= 256 && K % (32 * s * 2) == 0 && K / (s * 2) >= 256) s *= 2;
  return s;
}

void launch_step_gemm(const bf16* X, const bf16* W, int B, int N, int K, int splits, float* part,
                      hipStream_t stream) {
  const int ntw = sg_ntw(N);
  const dim3 grid((unsigned)(N / (32 * ntw)), (unsigned)(B / kSgTok), (unsigned)splits);
  const int kc = K / splits;
  switch (ntw) {
    case 8: step_gemm_kernel<8><<<grid, 256, 0, stream>>>(X, W, B, N, K, kc, part); break;
    case 4: step_gemm_kernel<4><<<grid, 256, 0, stream>>>(X, W, B, N, K, kc, part); break;
    default: step_gemm_kernel<2><<<grid, 256, 0, stream>>>(X, W, B, N, K, kc, part); break;
  }
}

}  // namespace dcr
