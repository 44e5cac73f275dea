// Sparse softmax cross-entropy, forward + backward in one pass (K10 of SURVEY.md §2.3).
//
// Reference: `sequence_loss_by_example([logits], [targets], [ones])` then
// `cost = reduce_sum(loss) / batch_size / seq_length` (model.py:79-85), i.e. TF's
// SparseSoftmaxCrossEntropyWithLogits + Sum + RealDiv.  Here one wave owns a row: it reads the
// fp32 logits row once (online max / sum-exp over V in 64-lane strips), writes the per-row CE,
// and writes dlogits = (softmax - onehot) * scale in bf16 directly (the training path never
// materialises probabilities).  Rows are time-major (n = t*B + b); the loss is a mean so the
// order is irrelevant.  A deterministic two-level reduction produces the summed loss.
#include "common.h"
#include "kernels.h"

namespace dcr {

constexpr int kXentThreads = 256;
constexpr int kXentRowsPerWave = 4;

__global__ void __launch_bounds__(kXentThreads) xent_kernel(
    const float* __restrict__ logits, const int* __restrict__ targets, int N, int V,
    float scale, float* __restrict__ row_loss, bf16* __restrict__ dlogits,
    float* __restrict__ partial) {
  __shared__ float red[kXentThreads / 64];
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * (kXentThreads / 64) + (threadIdx.x >> 6);
  float acc = 0.f;
  for (int rr = 0; rr < kXentRowsPerWave; ++rr) {
    const int n = wave * kXentRowsPerWave + rr;
    if (n >= N) break;
    const float* x = logits + (size_t)n * V;
    float m = -INFINITY;
    for (int v = lane; v < V; v += 64) m = fmaxf(m, x[v]);
    m = wave_max(m);
    float s = 0.f;
    for (int v = lane; v < V; v += 64) s += __expf(x[v] - m);
    s = wave_sum(s);
    const float lse = m + __logf(s);
    const int y = targets[n];
    const float loss = lse - x[y];
    if (lane == 0) {
      if (row_loss) row_loss[n] = loss;
      acc += loss;
    }
    if (dlogits) {
      const float inv = 1.f / s;
      bf16* d = dlogits + (size_t)n * V;
      for (int v = lane; v < V; v += 64) {
        const float p = __expf(x[v] - m) * inv;
        d[v] = f2bf((p - (v == y ? 1.f : 0.f)) * scale);
      }
    }
  }
  const float t = block_sum<kXentThreads>(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = t;
}

__global__ void __launch_bounds__(kXentThreads) sum_partials_kernel(const float* __restrict__ p,
                                                                   int n, float scale,
                                                                   float* __restrict__ out) {
  __shared__ float red[kXentThreads / 64];
  float a = 0.f;
  for (int i = threadIdx.x; i < n; i += kXentThreads) a += p[i];
  const float t = block_sum<kXentThreads>(a, red);
  if (threadIdx.x == 0) out[0] = t * scale;
}

int xent_num_partials(int N) {
  const int rows_per_block = (kXentThreads / 64) * kXentRowsPerWave;
  return (N + rows_per_block - 1) / rows_per_block;
}

void launch_xent(const float* logits, const int* targets, int N, int V, float grad_scale,
                 float* row_loss, bf16* dlogits, float* partial, float* loss_out,
                 hipStream_t s) {
  const int nb = xent_num_partials(N);
  xent_kernel<<<nb, kXentThreads, 0, s>>>(logits, targets, N, V, grad_scale, row_loss, dlogits,
                                          partial);
  sum_partials_kernel<<<1, kXentThreads, 0, s>>>(partial, nb, 1.0f / (float)N, loss_out);
}

}  // namespace dcr
