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


// ------------------------------------------------------------------------------------------
// Wide vocabularies (BASELINE.json's 8k-token config).  The row-per-wave kernel above reads a
// V = 8192 fp32 row three times, d softmax_b needed a separate column sum over the bf16
// dlogits, and the logits GEMM's bias broadcast cost a 1 GB copy (864 + 255 + 155 us per step
// at N = 32768).  Here a wave owns kWideRPW rows and holds ONE row at a time in registers
// (NC float4 per lane), so the logits are read exactly once:
//   online (max, sum-exp) over the row's registers -> lse, row loss
//   dlogits = (softmax - onehot) * scale written as bf16x4, and the bf16-rounded values
//   accumulated per column in registers (d softmax_b, exactly what the weight GEMM sees);
// the softmax bias is added here (the GEMM runs without it).  The 4 waves' column partials are
// reduced through LDS in 1 KB chunks -> one [V] partial per block -> xent_colsum_kernel.
// ------------------------------------------------------------------------------------------
constexpr int kWideRPW = 32;  // rows per wave

template <int NC>
__global__ void __launch_bounds__(256) xent_wide_kernel(
    const float* __restrict__ logits, const float* __restrict__ bias,
    const int* __restrict__ targets, int N, int V, float scale, float* __restrict__ row_loss,
    bf16* __restrict__ dlogits, float* __restrict__ colpart, float* __restrict__ partial) {
  __shared__ float4 red[3][64];
  __shared__ float lred[4];
  __shared__ float4 bz[64 * NC];  // the softmax bias, staged once (registers hold the row)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = (blockIdx.x * 4 + w) * kWideRPW;
  const int V4 = V / 4;
  for (int f = threadIdx.x; f < 64 * NC; f += 256)
    bz[f] = (bias && f < V4) ? reinterpret_cast<const float4*>(bias)[f] : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  float acc[NC][4];
#pragma unroll
  for (int j = 0; j < NC; ++j) acc[j][0] = acc[j][1] = acc[j][2] = acc[j][3] = 0.f;
  float lacc = 0.f;
  for (int i = 0; i < kWideRPW; ++i) {
    const int n = r0 + i;
    if (n >= N) break;
    const float4* xr = reinterpret_cast<const float4*>(logits + (size_t)n * V);
    float x[NC][4];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int f = lane + 64 * j;
      const float4 v = f < V4 ? xr[f] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
      const float4 bb = bz[f];
      x[j][0] = v.x + bb.x; x[j][1] = v.y + bb.y; x[j][2] = v.z + bb.z; x[j][3] = v.w + bb.w;
    }
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) m = fmaxf(m, x[j][q]);
    m = wave_max(m);
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) sm += __expf(x[j][q] - m);
    sm = wave_sum(sm);
    const int y = targets[n];
    if (lane == 0) {
      const float loss = m + __logf(sm) - (logits[(size_t)n * V + y] + (bias ? bias[y] : 0.f));
      if (row_loss) row_loss[n] = loss;
      lacc += loss;
    }
    if (dlogits) {
      const float inv = 1.f / sm;
      bf16x4* d = reinterpret_cast<bf16x4*>(dlogits + (size_t)n * V);
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int f = lane + 64 * j;
        if (f < V4) {
          bf16x4 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            o[q] = f2bf((__expf(x[j][q] - m) * inv - (4 * f + q == y ? 1.f : 0.f)) * scale);
            acc[j][q] += (float)o[q];
          }
          d[f] = o;
        }
      }
    }
  }
  lacc = wave_sum(lacc);
  if (lane == 0) lred[w] = lacc;
  if (dlogits && colpart) {
    float4* out = reinterpret_cast<float4*>(colpart + (size_t)blockIdx.x * V);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      if (w > 0) red[w - 1][lane] = make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
      __syncthreads();
      const int f = lane + 64 * j;
      if (w == 0 && f < V4) {
        float4 t = make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          t.x += red[k][lane].x; t.y += red[k][lane].y; t.z += red[k][lane].z; t.w += red[k][lane].w;
        }
        out[f] = t;
      }
      __syncthreads();
    }
  } else {
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = lred[0] + lred[1] + lred[2] + lred[3];
}

// d softmax_b[v] = sum of the per-block partial rows: 64 columns x 4 row-interleaved groups per
// block, fixed order per thread and a fixed LDS combine (deterministic)
__global__ void __launch_bounds__(256) xent_colsum_kernel(const float* __restrict__ colpart,
                                                          int nrows, int V,
                                                          float* __restrict__ out) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  float s = 0.f;
  if (c < V)
    for (int k = rg; k < nrows; k += 4) s += colpart[(size_t)k * V + c];
  red[rg][threadIdx.x & 63] = s;
  __syncthreads();
  if (rg == 0 && c < V) out[c] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

int xent_wide_blocks(int N) { return ((N + kWideRPW - 1) / kWideRPW + 3) / 4; }
int xent_wide_waves(int N) { return xent_wide_blocks(N); }  // partial rows: one per block
int xent_wide_supported(int V) { return V % 4 == 0 && V <= 64 * 4 * 32 ? 1 : 0; }

void launch_xent_wide(const float* logits, const float* bias, const int* targets, int N, int V,
                      float grad_scale, float* row_loss, bf16* dlogits, float* colpart, float* db,
                      float* partial, float* loss_out, hipStream_t s) {
  const int nb = xent_wide_blocks(N);
  const int nc = (V / 4 + 63) / 64;
#define XW(K)                                                                                \
  if (nc <= K) {                                                                             \
    xent_wide_kernel<K><<<nb, 256, 0, s>>>(logits, bias, targets, N, V, grad_scale, row_loss, \
                                           dlogits, colpart, partial);                       \
  } else
  XW(1) XW(2) XW(4) XW(8) XW(16) XW(32) {}
#undef XW
  sum_partials_kernel<<<1, kXentThreads, 0, s>>>(partial, nb, 1.0f / (float)N, loss_out);
  if (dlogits && colpart && db)
    xent_colsum_kernel<<<(V + 63) / 64, 256, 0, s>>>(colpart, nb, V, db);
}

}  // namespace dcr
