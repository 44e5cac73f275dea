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
// Wide vocabularies (BASELINE.json's 8k-token config).  A row-per-wave kernel reads a V = 8192
// fp32 row three times, d softmax_b needed a separate column sum over the bf16 dlogits, and
// the logits GEMM's bias broadcast cost a 1 GB copy (864 + 255 + 155 us per step at
// N = 32768).  Here the logits are read exactly once:
//   a WORKGROUP owns kWideRPB consecutive rows and holds one row at a time in registers,
//   thread t holding float4 columns t, t + 256, ... (NC of them, so NC float4 per lane and
//   every load / store of a wave is one contiguous 1 KB / 512 B segment);
//   row max and sum-exp: wave reduction + a 4-entry LDS exchange (2 barriers per row);
//   dlogits = (softmax - onehot) * scale written as bf16x4, and the bf16-rounded values
//   accumulated per column in registers (d softmax_b, exactly what the weight GEMM sees);
//   the row loss comes from the thread that owns column y (no dependent global load).
// The softmax bias is added here (the GEMM runs without it).  Each thread's column sums are
// the block's [V] partial directly -> xent_colsum_kernel.
// (The previous row-per-wave layout held 2 x 128 fp32 per lane at V = 8192: 256 VGPRs + 226
// AGPRs, one wave per SIMD, 456-465 us per step = 3.5 TB/s.)
// ------------------------------------------------------------------------------------------
constexpr int kWideRPB = 32;  // rows per workgroup

template <int NC>
__global__ void __launch_bounds__(256) xent_wide_kernel(
    const float* __restrict__ logits, const float* __restrict__ bias,
    const int* __restrict__ targets, int N, int V, float scale, float* __restrict__ row_loss,
    bf16* __restrict__ dlogits, float* __restrict__ colpart, float* __restrict__ partial) {
  __shared__ float red[2][4];
  __shared__ float lred[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int V4 = V / 4;
  const int r0 = blockIdx.x * kWideRPB;
  __shared__ float4 bb[NC][256];  // the softmax bias (each thread reads only its own columns)
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int f = tid + 256 * j;
    bb[j][tid] = (bias && f < V4) ? reinterpret_cast<const float4*>(bias)[f]
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float acc[NC][4];
#pragma unroll
  for (int j = 0; j < NC; ++j) acc[j][0] = acc[j][1] = acc[j][2] = acc[j][3] = 0.f;
  float lacc = 0.f;
  for (int i = 0; i < kWideRPB; ++i) {
    const int n = r0 + i;
    if (n >= N) break;  // uniform across the workgroup
    const int y = targets[n];
    const int fy = y >> 2, qy = y & 3;
    const float4* xr = reinterpret_cast<const float4*>(logits + (size_t)n * V);
    float x[NC][4];
    float zy = 0.f;
    bool own = false;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int f = tid + 256 * j;
      const float4 v = f < V4 ? xr[f] : make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
      const float4 bv = bb[j][tid];
      x[j][0] = v.x + bv.x; x[j][1] = v.y + bv.y; x[j][2] = v.z + bv.z; x[j][3] = v.w + bv.w;
      if (f == fy) {
        own = true;
        zy = qy == 0 ? x[j][0] : qy == 1 ? x[j][1] : qy == 2 ? x[j][2] : x[j][3];
      }
    }
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) m = fmaxf(m, x[j][q]);
    m = wave_max(m);
    if (lane == 0) red[0][w] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    float sm = 0.f;  // x becomes exp(x - m): reused for dlogits (one exp per element)
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        x[j][q] = __expf(x[j][q] - m);
        sm += x[j][q];
      }
    sm = wave_sum(sm);
    if (lane == 0) red[1][w] = sm;
    __syncthreads();
    sm = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    if (own) {
      const float loss = m + __logf(sm) - zy;
      if (row_loss) row_loss[n] = loss;
      lacc += loss;
    }
    if (dlogits) {
      const float inv = 1.f / sm;
      bf16x4* d = reinterpret_cast<bf16x4*>(dlogits + (size_t)n * V);
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const int f = tid + 256 * j;
        if (f < V4) {
          bf16x4 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            o[q] = f2bf((x[j][q] * inv - (f == fy && q == qy ? 1.f : 0.f)) * scale);
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
      const int f = tid + 256 * j;
      if (f < V4) out[f] = make_float4(acc[j][0], acc[j][1], acc[j][2], acc[j][3]);
    }
  }
  __syncthreads();
  if (tid == 0) partial[blockIdx.x] = lred[0] + lred[1] + lred[2] + lred[3];
}

// d softmax_b = column sums of the per-block partials [nrows, V].  A workgroup owns 4 float4
// columns x 64 row groups (16 independent float4 loads per thread at nrows = 1024, all in flight;
// 512 workgroups at V = 8192), reduced in a fixed order through LDS (bitwise reproducible).
// (One column per thread over 256 serial rows took 62 us at V = 8192 with 1024 partials.)
// The last workgroup also sums the loss partials (lpart[0, nlp) x lscale -> loss_out): one
// launch instead of a separate one-workgroup sum_partials_kernel.
__global__ void __launch_bounds__(256) xent_colsum_kernel(const float* __restrict__ colpart,
                                                          int nrows, int V,
                                                          float* __restrict__ out,
                                                          const float* __restrict__ lpart, int nlp,
                                                          float lscale,
                                                          float* __restrict__ loss_out) {
  __shared__ float4 red[64][4];
  if (lpart && blockIdx.x == gridDim.x - 1) {
    __shared__ float lred[256 / 64];
    float a = 0.f;
    for (int i = threadIdx.x; i < nlp; i += 256) a += lpart[i];
    const float t = block_sum<256>(a, lred);
    if (threadIdx.x == 0) loss_out[0] = t * lscale;
  }
  const int cl = threadIdx.x & 3, rg = threadIdx.x >> 2;
  const int f = blockIdx.x * 4 + cl, V4 = V / 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (f < V4) {
    const float4* p = reinterpret_cast<const float4*>(colpart) + f;
#pragma unroll 16
    for (int k = rg; k < nrows; k += 64) {
      const float4 v = p[(size_t)k * V4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[rg][cl] = s;
  __syncthreads();
#pragma unroll
  for (int h = 32; h > 0; h >>= 1) {
    if (rg < h) {
      const float4 o = red[rg + h][cl];
      s.x += o.x; s.y += o.y; s.z += o.z; s.w += o.w;
      red[rg][cl] = s;
    }
    __syncthreads();
  }
  if (rg == 0 && f < V4) {  // scalar stores: out is a gradient view of unknown alignment
    out[4 * f] = s.x; out[4 * f + 1] = s.y; out[4 * f + 2] = s.z; out[4 * f + 3] = s.w;
  }
}

void launch_xent_finalize(const float* partial, int nb, int N, float* loss_out,
                          const float* colpart, int ncp, int V, float* db, hipStream_t s) {
  if (colpart && db)
    xent_colsum_kernel<<<(V / 4 + 3) / 4, 256, 0, s>>>(colpart, ncp, V, db, partial, nb,
                                                       1.0f / (float)N, loss_out);
  else
    sum_partials_kernel<<<1, kXentThreads, 0, s>>>(partial, nb, 1.0f / (float)N, loss_out);
}

int xent_wide_blocks(int N) { return (N + kWideRPB - 1) / kWideRPB; }
int xent_wide_waves(int N) { return xent_wide_blocks(N); }  // partial rows: one per block
int xent_wide_supported(int V) { return V % 4 == 0 && V <= 256 * 4 * 16 ? 1 : 0; }

void launch_xent_wide(const float* logits, const float* bias, const int* targets, int N, int V,
                      float grad_scale, float* row_loss, bf16* dlogits, float* colpart, float* db,
                      float* partial, float* loss_out, hipStream_t s) {
  const int nb = xent_wide_blocks(N);
  const int nc = (V / 4 + 255) / 256;
#define XW(K)                                                                                \
  if (nc <= K) {                                                                             \
    xent_wide_kernel<K><<<nb, 256, 0, s>>>(logits, bias, targets, N, V, grad_scale, row_loss, \
                                           dlogits, colpart, partial);                       \
  } else
  XW(1) XW(2) XW(4) XW(8) XW(16) {}
#undef XW
  if (dlogits && colpart && db)
    xent_colsum_kernel<<<(V / 4 + 3) / 4, 256, 0, s>>>(colpart, nb, V, db, partial, nb,
                                                       1.0f / (float)N, loss_out);
  else
    sum_partials_kernel<<<1, kXentThreads, 0, s>>>(partial, nb, 1.0f / (float)N, loss_out);
}

}  // namespace dcr
