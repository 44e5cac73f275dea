// On-device autoregressive sampling step for gfx950: softmax head + categorical draw.
//
// Reference: Model.sample (model.py:105-140) runs one Session.run per generated character to
// fetch `probs = softmax(h·W_s + b_s)` (model.py:76-77, K11 of SURVEY.md §2.3) and then picks
// on the host (model.py:113-135, K16): argmax (sampling_type 0), inverse-CDF weighted pick
// `searchsorted(cumsum(p), rand * sum(p))` (1), or the weighted pick only when the previous
// character is a space, else argmax (2).
//
// Here the pick happens on the device and feeds the next step's input id directly, so the
// whole generation loop is a replayed hipGraph of [recurrent step kernels, this kernel] with no
// host round trip until the end (engine/native_backend.py: sample_sequence).  One workgroup per
// sample stream: each wave computes logits of whole vocabulary rows from the transposed
// [V, H] softmax weight (one 16-B load per lane per 512 hidden units, wave-reduced), the
// workgroup reduces max / sum, and a chunked block scan of exp(l - max) gives the CDF.  The
// uniform draw is counter-based (mix64 of seed, stream, per-stream counter), so a replay is
// deterministic for a given seed.
#include "common.h"
#include "kernels.h"

namespace dcr {

constexpr int kSampleThreads = 256;
constexpr int kSampleMaxV = 8192;
constexpr int kSampleMaxH = 4096;

__global__ void __launch_bounds__(kSampleThreads) sample_step_kernel(SampleArgs a) {
  __shared__ float logit[kSampleMaxV];
  __shared__ float red[kSampleThreads / 64];
  __shared__ float chunk_sum[kSampleThreads];
  __shared__ int pick_sh;
  const int s = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int H = a.H, V = a.V;
  constexpr int NW = kSampleThreads / 64;

  // ---- logits: wave w takes rows v = w, w + NW, ...; lanes split H in 8-element pieces
  const bf16* o = a.O + (size_t)s * H;
  for (int v = w; v < V; v += NW) {
    const bf16* wr = a.WsT + (size_t)v * H;
    float acc = 0.f;
    for (int k = lane * 8; k < H; k += 64 * 8) {
      const bf16x8 x = ld8(o + k), y = ld8(wr + k);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += (float)x[j] * (float)y[j];
    }
    acc = wave_sum(acc);
    if (lane == 0) logit[v] = acc + a.bs[v];
  }
  __syncthreads();
  if (a.logits_out)
    for (int v = tid; v < V; v += kSampleThreads) a.logits_out[(size_t)s * V + v] = logit[v];

  // ---- max (and its first index for argmax)
  float m = -INFINITY;
  for (int v = tid; v < V; v += kSampleThreads) m = fmaxf(m, logit[v]);
  m = wave_max(m);
  if (lane == 0) red[w] = m;
  __syncthreads();
  m = red[0];
#pragma unroll
  for (int i = 1; i < NW; ++i) m = fmaxf(m, red[i]);
  __syncthreads();
  if (tid == 0) pick_sh = V;
  __syncthreads();
  for (int v = tid; v < V; v += kSampleThreads)
    if (logit[v] == m) atomicMin(&pick_sh, v);
  __syncthreads();
  const int amax = pick_sh;

  const int prev = a.cur[s];
  const bool weighted = a.mode == 1 || (a.mode == 2 && prev == a.space_id);
  int pick = amax;
  if (weighted) {
    // ---- CDF of exp(l - max): thread t owns the contiguous chunk [t*C, (t+1)*C)
    const int C = (V + kSampleThreads - 1) / kSampleThreads;
    const int lo = tid * C, hi = min(lo + C, V);
    float cs = 0.f;
    for (int v = lo; v < hi; ++v) {
      const float p = __expf(logit[v] - m);
      logit[v] = p;
      cs += p;
    }
    chunk_sum[tid] = cs;
    __syncthreads();
    // inclusive scan of the chunk sums (Hillis-Steele in LDS; 8 rounds for 256 threads)
    for (int off = 1; off < kSampleThreads; off <<= 1) {
      const float add = tid >= off ? chunk_sum[tid - off] : 0.f;
      __syncthreads();
      chunk_sum[tid] += add;
      __syncthreads();
    }
    const float total = chunk_sum[kSampleThreads - 1];
    const float u = a.u ? a.u[s] : uniform01(a.seed, (uint64_t)s, (uint64_t)a.ctr[s]);
    const float r = u * total;
    if (tid == 0) pick_sh = V - 1;  // r beyond the last bucket by rounding: clamp like the host
    __syncthreads();
    const float before = tid ? chunk_sum[tid - 1] : 0.f;
    if (lo < hi && r <= chunk_sum[tid] && (tid == 0 || r > before)) {
      // searchsorted(cdf, r, side='left'): first v with cdf[v] >= r
      float c = before;
      int hit = hi - 1;
      for (int v = lo; v < hi; ++v) {
        c += logit[v];
        if (c >= r) { hit = v; break; }
      }
      pick_sh = hit;
    }
    __syncthreads();
    pick = pick_sh;
  }
  if (tid == 0) {
    a.cur[s] = pick;
    const int p = a.pos[s];
    a.out[(size_t)s * a.ld + p] = pick;
    a.pos[s] = p + 1;
    a.ctr[s] = a.ctr[s] + 1;
  }
}

int sample_supported(int V, int H) {
  return (V >= 1 && V <= kSampleMaxV && H % 8 == 0 && H <= kSampleMaxH) ? 1 : 0;
}

void launch_sample_step(const SampleArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(sample_step_kernel, dim3(a.S), dim3(kSampleThreads), 0, s, a);
}

}  // namespace dcr
