// Fused global-norm clip + TF-variant Adam over ONE flat fp32 parameter buffer (K13 + K14 of
// SURVEY.md §2.3).  The reference runs `clip_by_global_norm` (model.py:91-92) and
// `AdamOptimizer(lr).apply_gradients` (model.py:94-98) as ~2×#vars small TF kernels on the PS
// CPU; here all parameters, gradients and Adam slots live in flat buffers so the whole
// optimizer is two launches regardless of the number of variables:
//   1. sumsq_partials: grid-stride float4 sum of g^2, one partial per block (fixed grid =>
//      deterministic order).
//   2. adam_apply: every block re-reduces the (<=1024) partials in LDS, derives
//      scale = clip / max(||g||, clip) (g optionally pre-scaled by 1/world) and applies
//        m = b1 m + (1-b1) g s ;  v = b2 v + (1-b2) (g s)^2 ;  p -= lr_t m / (sqrt(v) + eps)
//      with TF's lr_t = lr * sqrt(1-b2^t) / (1-b1^t) computed on the host (TF "epsilon-hat").
//      Optionally refreshes a bf16 mirror of the parameters in the same pass.
// The norm covers g[0, n_norm) plus an optional extra sum of squares read from device memory:
// TF's global norm sees the embedding gradient as IndexedSlices, i.e. the per-token values
// before the segment sum (model.py:55,91-92), so the trainer excludes the dense embedding
// gradient from the sum and supplies sum_tokens ||dx_token||^2 instead (see sumsq below).
#include "common.h"
#include "kernels.h"

namespace dcr {

constexpr int kOptThreads = 256;

// sum of squares of the i-th 16-byte vector (4 fp32 or 8 bf16 elements)
__device__ __forceinline__ float sqv(const float* g, int64_t i) {
  const float4 x = reinterpret_cast<const float4*>(g)[i];
  return x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
}
__device__ __forceinline__ float sqv(const bf16* g, int64_t i) {
  const bf16x8 x = reinterpret_cast<const bf16x8*>(g)[i];
  float a = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float f = bf2f(x[k]);
    a += f * f;
  }
  return a;
}
__device__ __forceinline__ float sq1(const float* g, int64_t i) { return g[i] * g[i]; }
__device__ __forceinline__ float sq1(const bf16* g, int64_t i) {
  const float f = bf2f(g[i]);
  return f * f;
}

template <typename T>
__global__ void __launch_bounds__(kOptThreads) sumsq_partials_kernel(
    const T* __restrict__ g, int64_t n, float* __restrict__ partials,
    const float* __restrict__ extra) {
  __shared__ float red[kOptThreads / 64];
  constexpr int kVec = 16 / (int)sizeof(T);
  float acc = 0.f;
  const int64_t nv = n / kVec;
  for (int64_t i = blockIdx.x * (int64_t)kOptThreads + threadIdx.x; i < nv;
       i += (int64_t)gridDim.x * kOptThreads)
    acc += sqv(g, i);
  if (blockIdx.x == 0) {  // tail (+ the extra term, once)
    for (int64_t i = nv * kVec + threadIdx.x; i < n; i += kOptThreads) acc += sq1(g, i);
    if (extra && threadIdx.x == 0) acc += extra[0];
  }
  const float t = block_sum<kOptThreads>(acc, red);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float s, float lr_t,
                                         float b1, float b2, float eps) {
  g *= s;
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  p -= lr_t * m / (sqrtf(v) + eps);
}

__global__ void __launch_bounds__(kOptThreads) adam_apply_kernel(
    float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
    bf16* __restrict__ pbf, int64_t n, const float* __restrict__ partials, int nparts,
    float* __restrict__ norm_out, float lr_t, float b1, float b2, float eps, float clip,
    float gscale, const unsigned* __restrict__ skip_if) {
  __shared__ float red[kOptThreads / 64];
  // a persistent recurrent kernel that hit its spin timeout leaves garbage gradients and sets
  // its error word: the update is skipped on device (weights and slots stay unchanged) and the
  // host raises when it reads the word
  if (skip_if && __hip_atomic_load(skip_if, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
    return;
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += kOptThreads) acc += partials[i];
  const float sumsq = block_sum<kOptThreads>(acc, red);
  // gscale folds the data-parallel 1/world average into this pass (the gradient buffer holds
  // the all-reduced SUM): the norm and the update see g * gscale
  const float norm = sqrtf(sumsq) * gscale;
  // TF clip_by_global_norm: t * clip / max(norm, clip); clip <= 0 disables clipping.
  const float s = ((clip > 0.f) ? clip / fmaxf(norm, clip) : 1.f) * gscale;
  if (blockIdx.x == 0 && threadIdx.x == 0 && norm_out) norm_out[0] = norm;

  const int64_t n4 = n >> 2;
  float4* p4 = reinterpret_cast<float4*>(p);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  for (int64_t i = blockIdx.x * (int64_t)kOptThreads + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * kOptThreads) {
    float4 pp = p4[i], mm = m4[i], vv = v4[i];
    const float4 gg = g4[i];
    adam_one(pp.x, gg.x, mm.x, vv.x, s, lr_t, b1, b2, eps);
    adam_one(pp.y, gg.y, mm.y, vv.y, s, lr_t, b1, b2, eps);
    adam_one(pp.z, gg.z, mm.z, vv.z, s, lr_t, b1, b2, eps);
    adam_one(pp.w, gg.w, mm.w, vv.w, s, lr_t, b1, b2, eps);
    p4[i] = pp;
    m4[i] = mm;
    v4[i] = vv;
    if (pbf) {
      bf16x4 o;
      o[0] = f2bf(pp.x); o[1] = f2bf(pp.y); o[2] = f2bf(pp.z); o[3] = f2bf(pp.w);
      *reinterpret_cast<bf16x4*>(pbf + 4 * i) = o;
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += kOptThreads) {
      float pp = p[i], mm = m[i], vv = v[i];
      adam_one(pp, g[i], mm, vv, s, lr_t, b1, b2, eps);
      p[i] = pp; m[i] = mm; v[i] = vv;
      if (pbf) pbf[i] = f2bf(pp);
    }
  }
}

__global__ void __launch_bounds__(kOptThreads) norm_only_kernel(const float* __restrict__ partials,
                                                                int nparts, float* __restrict__ out,
                                                                int take_sqrt) {
  __shared__ float red[kOptThreads / 64];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nparts; i += kOptThreads) acc += partials[i];
  const float t = block_sum<kOptThreads>(acc, red);
  if (threadIdx.x == 0) out[0] = take_sqrt ? sqrtf(t) : t;
}

// ------------------------------------------------------------------------------------------
// TF clip-norm term of the embedding: sum over tokens of ||dx_tok||^2 with dx = dZ0 · W_x0ᵀ
// ([N, K] x [K, H], K = gate width), fused: the [N, H] product is never written.
//
// Workgroup = 128 tokens x 32*NTW weight rows (grid.y splits H when H/32 > 16; the sum of
// squares is separable over columns).  4 waves: token half th = w&1, row half ch = w>>1, so a
// wave owns 64 tokens x 16*NTW columns = 4 x NTW accumulator tiles (AGPRs, pinned by inline
// asm).  K streams in 32-wide stages through a 3-stage LDS ring filled by LDS-DMA
// (global_load_lds_dwordx4) in MFMA fragment order, two stages in flight across raw barriers.
// One fp32 partial per workgroup (deterministic reduction).
//
// Status (scripts/bench_tok_norm.py, N = 32768): H = 512 92 us (745 TFLOP/s) vs 66 us for the
// library GEMM + sumsq route; H = 256 29.6 vs 30.7 us.  The backend therefore keeps the
// library route unless DCR_TOK_NORM=fused.  The ladder so far: register-staged 1-deep 97-119
// us -> accumulators pinned to AGPRs (the builtin form rotated them through VGPRs) -> bank-
// conflict-free lane-linear staging -> LDS-DMA ring 92 us.  PMC: no LDS conflicts, 85 % L2 hit,
// waves mostly stalled on MFMA issue + the per-stage barrier; a 40 KB stage leaves room for
// only 3 ring slots, so the DMA latency is only two stages deep.
// ------------------------------------------------------------------------------------------
constexpr int kTokTile = 128;

// s_waitcnt immediate that waits for vmcnt <= n only (expcnt / lgkmcnt at their maxima)
constexpr unsigned waitcnt_vm(unsigned n) { return (n & 15u) | ((n >> 4) << 14) | (7u << 4) | (15u << 8); }

template <int NTW>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
tok_norm_kernel(const bf16* __restrict__ dz, const bf16* __restrict__ w, int K,
                float* __restrict__ partials) {
  constexpr int kWTiles = 2 * NTW;              // weight row tiles of this workgroup
  constexpr int kTiles = kWTiles + kTokTile / 16;
  constexpr int kPer = kTiles / 4;              // LDS-DMA instructions per wave and stage
  constexpr int kStage = kTiles * 512;          // bf16 elements per stage (1 KB per tile)
  constexpr int kRing = 3;
  static_assert(kTiles % 4 == 0, "H must be a multiple of 64");
  // ONE __shared__ object (a second one can make hipcc drain the DMA queue before every
  // ds_read): the 3-stage ring + 4 floats of reduction scratch at the end
  __shared__ __attribute__((aligned(16))) bf16 lds[kRing * kStage + 8];
  float* red = reinterpret_cast<float*>(&lds[kRing * kStage]);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int th = wv & 1, ch = wv >> 1;
  const int64_t tok0 = (int64_t)blockIdx.x * kTokTile;
  w += (int64_t)blockIdx.y * (32 * NTW) * K;  // this workgroup's 32*NTW weight rows

  // Stage copy by LDS-DMA (global_load_lds_dwordx4: per-lane source, lane-linear destination):
  // instruction i of wave wv moves tile 4 i + wv, lane l loading row 64 i + 16 wv + (l & 15),
  // 16-B k-chunk l >> 4 -- the tile lands in MFMA fragment order (lane l's 16 B at l*16), read
  // back conflict-free by ds_read_b128.  Rows < 32*NTW are weight rows (i < NTW/2, static).
  const int rr = 16 * wv + (lane & 15), cc = lane >> 4;
  const int64_t off = (int64_t)rr * K + 8 * cc;
  const bf16* wsrc = w + off;
  const bf16* zsrc = dz + tok0 * K + off;
  auto issue = [&](int s, int buf) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const bf16* g = (i < NTW / 2 ? wsrc + (int64_t)(64 * i) * K
                                   : zsrc + (int64_t)(64 * (i - NTW / 2)) * K) + 32 * s;
      __builtin_amdgcn_global_load_lds(
          reinterpret_cast<const void*>(g),
          reinterpret_cast<__attribute__((address_space(3))) void*>(
              (__attribute__((address_space(3))) bf16*)&lds[buf * kStage + (4 * i + wv) * 512]),
          16, 0, 0);
    }
  };

  f32x4 acc[NTW][4];
#pragma unroll
  for (int a = 0; a < NTW; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const bf16* base = &lds[buf * kStage + lane * 8];
    bf16x8 bt[4], at[NTW];
#pragma unroll
    for (int b = 0; b < 4; ++b)
      bt[b] = *reinterpret_cast<const bf16x8*>(base + (kWTiles + 4 * th + b) * 512);
#pragma unroll
    for (int a = 0; a < NTW; ++a)
      at[a] = *reinterpret_cast<const bf16x8*>(base + (ch * NTW + a) * 512);
    // all fragment reads ahead of the MFMAs (left alone, the scheduler reused one fragment
    // register and waited out a full LDS latency per weight tile)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int a = 0; a < NTW; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
        // inline asm pins the accumulators to AGPRs: the builtin form made the register
        // allocator rotate them through VGPRs (80-192 v_accvgpr moves per 32-64 MFMAs, each
        // waiting on an MFMA result).  Hazards: a given acc is re-read 4*NTW MFMAs later.
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                     : "+a"(acc[a][b]) : "v"(at[a]), "v"(bt[b]));
  };

  // 3-stage ring, two stages in flight: at stage s wait for stage s (vmcnt <= kPer leaves
  // stage s+1 outstanding), raw barrier (no __syncthreads: its fence would drain the DMA
  // queue), refill the buffer every wave finished reading at stage s-1, compute.  Past the
  // end the refill re-reads the last stage into a buffer nobody reads again (branch-free).
  const int S = K / 32;
  issue(0, 0);
  issue(S > 1 ? 1 : 0, 1);
  int b0 = 0, b1 = 1, b2 = 2;  // buffers of stages s, s+1, s+2
  for (int s = 0; s < S; ++s) {
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(kPer));
    __builtin_amdgcn_s_barrier();
    issue(min(s + 2, S - 1), b2);
    compute(b0);
    const int t = b0;
    b0 = b1;
    b1 = b2;
    b2 = t;
  }
  __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));  // no DMA may still target LDS at exit
  // MFMA result -> VALU read of the same AGPRs: cover the 16x16x32 latency explicitly (the
  // hazard recognizer does not look inside the inline asm above)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  float sq = 0.f;
#pragma unroll
  for (int a = 0; a < NTW; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int j = 0; j < 4; ++j) sq += acc[a][b][j] * acc[a][b][j];
  __syncthreads();
  const float t = block_sum<256>(sq, red);
  if (tid == 0) partials[blockIdx.y * gridDim.x + blockIdx.x] = t;
}

bool tok_norm_supported(int64_t N, int H, int K) {
  return N > 0 && N % kTokTile == 0 && K % 64 == 0 && K > 0 &&
         H > 0 && H % 64 == 0;
}

// weight-row tiles per wave: the largest of 16, 8, 6, 4, 2 dividing H/32 (16 = the whole of
// H = 512 per workgroup, 256 fp32 accumulators per lane in AGPRs: dZ is read exactly once)
static int tok_norm_ntw(int H) {
  const int t = H / 32;
  return t % 16 == 0 ? 16 : t % 8 == 0 ? 8 : t % 6 == 0 ? 6 : t % 4 == 0 ? 4 : 2;
}

int tok_norm_num_partials(int64_t N, int H) {
  return (int)(N / kTokTile) * (H / (32 * tok_norm_ntw(H)));
}

void launch_tok_norm(const bf16* dz, const bf16* w, int64_t N, int H, int K, float* partials,
                     float* out, hipStream_t stream) {
  const int ntw = tok_norm_ntw(H);
  const dim3 grid((unsigned)(N / kTokTile), (unsigned)(H / (32 * ntw)));
  switch (ntw) {
    case 2: tok_norm_kernel<2><<<grid, 256, 0, stream>>>(dz, w, K, partials); break;
    case 4: tok_norm_kernel<4><<<grid, 256, 0, stream>>>(dz, w, K, partials); break;
    case 6: tok_norm_kernel<6><<<grid, 256, 0, stream>>>(dz, w, K, partials); break;
    case 8: tok_norm_kernel<8><<<grid, 256, 0, stream>>>(dz, w, K, partials); break;
    default: tok_norm_kernel<16><<<grid, 256, 0, stream>>>(dz, w, K, partials); break;
  }
  const int nb = (int)(grid.x * grid.y);
  norm_only_kernel<<<1, kOptThreads, 0, stream>>>(partials, nb, out, 0);
}

int opt_num_partials(int64_t n) {
  // 4 blocks per CU-ish cap; enough to stream a few-MB buffer at HBM rate.
  int64_t blocks = (n / 4 + kOptThreads - 1) / kOptThreads;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

void launch_global_norm(const float* g, int64_t n, float* partials, float* norm_out,
                        hipStream_t stream) {
  const int nb = opt_num_partials(n);
  sumsq_partials_kernel<float><<<nb, kOptThreads, 0, stream>>>(g, n, partials, nullptr);
  norm_only_kernel<<<1, kOptThreads, 0, stream>>>(partials, nb, norm_out, 1);
}

void launch_sumsq(const void* x, bool is_bf16, int64_t n, float* partials, float* out,
                  hipStream_t stream) {
  const int nb = opt_num_partials(n);
  if (is_bf16)
    sumsq_partials_kernel<bf16><<<nb, kOptThreads, 0, stream>>>(
        static_cast<const bf16*>(x), n, partials, nullptr);
  else
    sumsq_partials_kernel<float><<<nb, kOptThreads, 0, stream>>>(
        static_cast<const float*>(x), n, partials, nullptr);
  norm_only_kernel<<<1, kOptThreads, 0, stream>>>(partials, nb, out, 0);
}

void launch_adam_clip(float* p, const float* g, float* m, float* v, bf16* pbf, int64_t n,
                      float* partials, float* norm_out, float lr_t, float b1, float b2, float eps,
                      float clip, float gscale, int64_t n_norm, const float* extra_sq,
                      const unsigned* skip_if, hipStream_t stream) {
  const int nb = opt_num_partials(n);
  sumsq_partials_kernel<float><<<nb, kOptThreads, 0, stream>>>(g, n_norm, partials, extra_sq);
  adam_apply_kernel<<<nb, kOptThreads, 0, stream>>>(p, g, m, v, pbf, n, partials, nb, norm_out,
                                                    lr_t, b1, b2, eps, clip, gscale, skip_if);
}

}  // namespace dcr
