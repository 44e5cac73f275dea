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
    float gscale, const unsigned* __restrict__ skip_if, const float* __restrict__ lr_dev) {
  __shared__ float red[kOptThreads / 64];
  // a persistent recurrent kernel that hit its spin timeout leaves garbage gradients and sets
  // its error word: the update is skipped on device (weights and slots stay unchanged) and the
  // host raises when it reads the word
  if (skip_if && __hip_atomic_load(skip_if, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
    return;
  // a step replayed from a hipGraph reads its (per-step) lr_t from device memory
  if (lr_dev) lr_t = *lr_dev;
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

// sumsq_partials + the final sum in ONE launch: each block stores its partial, then takes a
// ticket; the block that draws the last ticket sums all partials in block order (the same
// fixed order as norm_only_kernel: bitwise equal results) and resets the ticket counter for
// the next launch (it must start zeroed: a torch.zeros buffer owned by the caller).  The
// cross-block hand-off is the sc1 form of the in-launch split-K recipe of
// cdna_hip_programming.md ("Projection GEMM at M = 256", item 2): write-through partial stores
// drained (vmcnt(0)) before the agent-scope ticket add, sc1 loads of them in the last block.
// 256 blocks (not 1024): the tickets are same-address atomics.
template <typename T>
__global__ void __launch_bounds__(kOptThreads) sumsq_final_kernel(
    const T* __restrict__ g, int64_t n, float* __restrict__ partials, unsigned* __restrict__ ticket,
    float* __restrict__ out, const float* __restrict__ extra, const int* __restrict__ guard) {
  __shared__ float red[kOptThreads / 64];
  __shared__ unsigned last;
  constexpr int kVec = 16 / (int)sizeof(T);
  float acc = 0.f;
  const int64_t nv = n / kVec;
  // 4 vectors in flight per trip (a 256-block grid streams 32 MB: one load per trip would be
  // latency-bound)
  const int64_t stride = (int64_t)gridDim.x * kOptThreads;
  int64_t i = blockIdx.x * (int64_t)kOptThreads + threadIdx.x;
  for (; i + 3 * stride < nv; i += 4 * stride) {
    const float a0 = sqv(g, i), a1 = sqv(g, i + stride), a2 = sqv(g, i + 2 * stride),
                a3 = sqv(g, i + 3 * stride);
    acc += (a0 + a1) + (a2 + a3);
  }
  for (; i < nv; i += stride) acc += sqv(g, i);
  if (blockIdx.x == 0)
    for (int64_t j = nv * kVec + threadIdx.x; j < n; j += kOptThreads) acc += sq1(g, j);
  const float t = block_sum<kOptThreads>(acc, red);
  if (threadIdx.x == 0) {
    // write-through (sc1) partial store drained before the ticket: no release fence (an
    // agent-scope release writes back the L2 -- per block, that made this launch 32 us)
    __hip_atomic_store(partials + blockIdx.x, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned k = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = k == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  float s = 0.f;
  for (int i = threadIdx.x; i < (int)gridDim.x; i += kOptThreads)
    s += __hip_atomic_load(partials + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float total = block_sum<kOptThreads>(s, red);
  if (threadIdx.x == 0) {
    // (extra: one more norm term, e.g. the TF token-norm slot; guard: an error word, copied as a
    // float value into out[1] so that one all-reduce carries both)
    out[0] = extra ? total + extra[0] : total;
    if (guard) out[1] = (float)guard[0];
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
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
                  unsigned* ticket, hipStream_t stream, const float* extra, const int* guard) {
  const int nb = opt_num_partials(n);
  if (ticket) {
    const int nb = opt_num_partials(n) < 256 ? opt_num_partials(n) : 256;
    if (is_bf16)
      sumsq_final_kernel<bf16><<<nb, kOptThreads, 0, stream>>>(static_cast<const bf16*>(x), n,
                                                                partials, ticket, out, extra, guard);
    else
      sumsq_final_kernel<float><<<nb, kOptThreads, 0, stream>>>(static_cast<const float*>(x), n,
                                                                 partials, ticket, out, extra, guard);
    return;
  }
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
                      const unsigned* skip_if, const float* lr_dev, hipStream_t stream) {
  const int nb = opt_num_partials(n);
  // no norm terms in g (the sharded step's packed chunks: the reduced sum of squares comes in
  // as extra_sq): the update reads that one value, no partials launch
  const bool only_extra = n_norm == 0 && extra_sq;
  if (!only_extra)
    sumsq_partials_kernel<float><<<nb, kOptThreads, 0, stream>>>(g, n_norm, partials, extra_sq);
  adam_apply_kernel<<<nb, kOptThreads, 0, stream>>>(
      p, g, m, v, pbf, n, only_extra ? extra_sq : partials, only_extra ? 1 : nb, norm_out, lr_t,
      b1, b2, eps, clip, gscale, skip_if, lr_dev);
}

}  // namespace dcr
