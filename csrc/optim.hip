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

__device__ __forceinline__ float sq4(const float* g, int64_t i) {
  const float4 x = reinterpret_cast<const float4*>(g)[i];
  return x.x * x.x + x.y * x.y + x.z * x.z + x.w * x.w;
}
__device__ __forceinline__ float sq4(const bf16* g, int64_t i) {
  const bf16x4 x = reinterpret_cast<const bf16x4*>(g)[i];
  float a = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
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
  float acc = 0.f;
  const int64_t n4 = n >> 2;
  for (int64_t i = blockIdx.x * (int64_t)kOptThreads + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * kOptThreads)
    acc += sq4(g, i);
  if (blockIdx.x == 0) {  // tail (+ the extra term, once)
    for (int64_t i = (n4 << 2) + threadIdx.x; i < n; i += kOptThreads) acc += sq1(g, i);
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
    float gscale) {
  __shared__ float red[kOptThreads / 64];
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
// Workgroup = 128 tokens x 32*NTW weight rows (grid.y splits H; the sum of squares is
// separable over columns).  4 waves: token half th = w&1, row half ch = w>>1, so a wave owns
// 64 tokens x 16*NTW columns = 4 x NTW accumulator tiles (AGPRs, pinned by inline asm).  K
// streams in 32-wide stages through double-buffered LDS in MFMA fragment order (lane-linear,
// bank-conflict-free both ways); two register prefetch sets keep stages s+1 and s+2 in flight.
// One fp32 partial per workgroup (deterministic reduction).
//
// Status (scripts/bench_tok_norm.py, N = 32768, H = 512): correct, 128-145 us = 470-530
// TFLOP/s, behind the library GEMM + sumsq route (66 us), so the backend uses the library
// route unless DCR_TOK_NORM=fused.  Measured on the way: plain fragment-order stores were
// 4-way bank conflicted (60 % of LDS cycles); the builtin MFMA form rotated the accumulators
// through VGPRs (up to 192 v_accvgpr moves per 64 MFMAs); what remains is the latency of the
// fragment-shaped global loads (16 rows x 64 B per wave instruction).  Next: LDS-DMA
// (global_load_lds_dwordx4, lane-linear destination = this layout) with a 3-4 stage ring.
// ------------------------------------------------------------------------------------------
constexpr int kTokTile = 128;

template <int NTW>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
tok_norm_kernel(const bf16* __restrict__ dz,
                                                       const bf16* __restrict__ w, int K,
                                                       float* __restrict__ partials) {
  constexpr int kWTiles = 2 * NTW;            // H / 16 weight row tiles
  constexpr int kTiles = kWTiles + kTokTile / 16;
  constexpr int kChunks = kTiles * 64;        // 16-B chunks per stage
  constexpr int kPer = kChunks / 256;         // per thread
  static_assert(kChunks % 256 == 0, "H must be a multiple of 64");
  __shared__ __attribute__((aligned(16))) bf16 lds[2][kTiles * 512];
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int th = wv & 1, ch = wv >> 1;
  const int64_t tok0 = (int64_t)blockIdx.x * kTokTile;
  w += (int64_t)blockIdx.y * (32 * NTW) * K;  // this workgroup's 32*NTW weight rows

  // Stage copy, chunk i of every thread: wave wv, lane l loads row 64 i + 16 wv + (l & 15),
  // 16-B k-chunk l >> 4, and stores it at lane-linear LDS slot l of tile 4 i + wv -- which is
  // exactly the MFMA fragment order (lane l: row l & 15, chunk l >> 4).  Lane-linear stores
  // and reads are bank-conflict-free for ds_write_b128 (8-lane groups) and ds_read_b128
  // (16-lane groups); the coalesced 4-threads-per-row form made the writes 4-way conflicted.
  // Rows < 32*NTW are weight rows (i < NTW/2, static), the rest the workgroup's tokens.
  const int rr = 16 * wv + (lane & 15), cc = lane >> 4;
  const int64_t off = (int64_t)rr * K + 8 * cc;
  const bf16* wsrc = w + off;
  const bf16* zsrc = dz + tok0 * K + off;
  const int dst0 = wv * 512 + lane * 8;  // element offset; + 4 i tiles per chunk i
  const int frag = lane * 8;
  auto chunk = [&](int i, int s) -> const bf16* {
    return (i < NTW / 2 ? wsrc + (int64_t)(64 * i) * K : zsrc + (int64_t)(64 * (i - NTW / 2)) * K) +
           32 * s;
  };
  // two register prefetch sets: stages s+1 and s+2 are in flight while stage s computes (one
  // set, i.e. one stage of ~1 us of L2 latency hidden behind ~0.4 us of MFMAs, measured 97 us)
  bf16x8 p0[kPer], p1[kPer];
  auto load = [&](bf16x8 (&p)[kPer], int s) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      // dZ is streamed once per workgroup: non-temporal, so it does not evict the weight
      // rows every workgroup of the XCD re-reads from L2
      if (i < NTW / 2)
        p[i] = ld8(chunk(i, s));
      else
        p[i] = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(chunk(i, s)));
    }
  };
  auto store = [&](const bf16x8 (&p)[kPer], int buf) {
#pragma unroll
    for (int i = 0; i < kPer; ++i)
      *reinterpret_cast<bf16x8*>(&lds[buf][dst0 + 4 * i * 512]) = p[i];
  };

  f32x4 acc[NTW][4];
#pragma unroll
  for (int a = 0; a < NTW; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    // all fragments of the stage are read before the first MFMA (64 + 16 VGPRs): one LDS
    // round trip per stage instead of one per weight tile
    bf16x8 bt[4], at[NTW];
#pragma unroll
    for (int b = 0; b < 4; ++b)
      bt[b] = *reinterpret_cast<const bf16x8*>(&lds[buf][(kWTiles + 4 * th + b) * 512 + frag]);
#pragma unroll
    for (int a = 0; a < NTW; ++a)
      at[a] = *reinterpret_cast<const bf16x8*>(&lds[buf][(ch * NTW + a) * 512 + frag]);
    // keep the reads ahead of the MFMAs (left alone, the scheduler reuses one fragment
    // register and waits out a full LDS latency per weight tile: measured 119 us)
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

  // S = K/32 stages, S even (K % 64 == 0).  Branch-free body: past the end the prefetch
  // re-reads the last stage (clamped) and the store fills a buffer nobody reads again.
  const int S = K / 32;
  load(p0, 0);
  load(p1, S > 1 ? 1 : 0);
  store(p0, 0);
  load(p0, S > 2 ? 2 : S - 1);
  __syncthreads();
  for (int s = 0; s < S; s += 2) {
    compute(0);                       // stage s; p1 = s+1, p0 = s+2 in flight
    store(p1, 1);
    load(p1, min(s + 3, S - 1));
    __syncthreads();
    compute(1);                       // stage s+1; p0 = s+2, p1 = s+3 in flight
    store(p0, 0);
    load(p0, min(s + 4, S - 1));
    __syncthreads();
  }
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
  const float t = block_sum<256>(sq, red);
  if (tid == 0) partials[blockIdx.y * gridDim.x + blockIdx.x] = t;
}

bool tok_norm_supported(int64_t N, int H, int K) {
  return N > 0 && N % kTokTile == 0 && K % 64 == 0 && K > 0 &&
         H > 0 && H % 64 == 0;
}

// weight-row tiles per wave: the largest of 8, 6, 4, 2 dividing H/32 (8 keeps the 128 fp32
// accumulators per lane in AGPRs with both prefetch sets in VGPRs; 16 spilled)
static int tok_norm_ntw(int H) {
  const int t = H / 32;
  return t % 8 == 0 ? 8 : t % 6 == 0 ? 6 : t % 4 == 0 ? 4 : 2;
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
    default: tok_norm_kernel<8><<<grid, 256, 0, stream>>>(dz, w, K, partials); break;
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
                      hipStream_t stream) {
  const int nb = opt_num_partials(n);
  sumsq_partials_kernel<float><<<nb, kOptThreads, 0, stream>>>(g, n_norm, partials, extra_sq);
  adam_apply_kernel<<<nb, kOptThreads, 0, stream>>>(p, g, m, v, pbf, n, partials, nb, norm_out,
                                                    lr_t, b1, b2, eps, clip, gscale);
}

}  // namespace dcr
