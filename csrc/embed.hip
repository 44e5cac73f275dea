// Segmented (by token id) row sums: out[v][c] = sum_{n : ids[n] == v} X[n][c].
//
// Reference: the embedding gradient of `tf.nn.embedding_lookup` is an IndexedSlices
// ([B*T, H] values + ids) that TF densifies with UnsortedSegmentSum before Adam (model.py:55,
// 91-98; K2 of SURVEY.md §2.3).  With V = 65 every id repeats ~500x per batch, so global atomics
// would serialise on 65 hot rows.  Here each workgroup owns a (row chunk, 128-column strip),
// accumulates into an LDS-resident [V x 128] fp32 tile with LDS atomics, and writes one partial
// per row chunk; a second pass sums the partials in a fixed order (bitwise reproducible).
//
// Uses in the native backend:
//  * layer-0 fusion: Zx0 = (E·W_x0 + b0)[ids], so the backward needs dEW = segsum(dZ0, ids)
//    [V, G·H] and then dE = dEW·W_x0ᵀ, dW_x0 = Eᵀ·dEW, db0 = colsum(dEW) -- all tiny;
//  * dropout path: dE = segsum(dX0, ids);
//  * bias gradients: ids == nullptr puts every row in bucket 0 (a column sum).
// Large vocabularies (V > kSegLdsMaxV) use fp32 global atomics into a zeroed output instead.
#include "common.h"
#include "kernels.h"

namespace dcr {

constexpr int kSegThreads = 256;
constexpr int kSegCols = 128;
constexpr int kSegLdsMaxV = 96;

template <typename T>
__global__ void __launch_bounds__(kSegThreads) segsum_lds_kernel(
    const T* __restrict__ X, int ldx, const int* __restrict__ ids, int N, int W, int V,
    int rows_per_chunk, float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float acc[];  // [V][kSegCols]
  const int c0 = blockIdx.x * kSegCols;
  const int chunk = blockIdx.y;
  for (int i = threadIdx.x; i < V * kSegCols; i += kSegThreads) acc[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // each lane owns columns c0+lane and c0+64+lane: a wave reads 64 consecutive elements per
  // row per access (coalesced for any width/stride, odd vocabularies included)
  const int ca = c0 + lane, cb = c0 + 64 + lane;
  const bool va = ca < W, vb = cb < W;
  const int r0 = chunk * rows_per_chunk;
  const int r1 = min(N, r0 + rows_per_chunk);
  constexpr int U = 8;  // rows in flight per wave (the loop is load-latency bound otherwise)
  constexpr int WS = kSegThreads / 64;
  for (int n = r0 + wave; n < r1; n += WS * U) {
    int vv[U];
    float xa[U], xb[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int nn = n + WS * j;
      const bool ok = nn < r1;
      vv[j] = ok ? (ids ? ids[nn] : 0) : -1;
      const T* row = X + (size_t)(ok ? nn : r0) * ldx;
      xa[j] = (ok && va) ? (float)row[ca] : 0.f;
      xb[j] = (ok && vb) ? (float)row[cb] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (vv[j] < 0) continue;
      if (va) atomicAdd(&acc[vv[j] * kSegCols + lane], xa[j]);
      if (vb) atomicAdd(&acc[vv[j] * kSegCols + 64 + lane], xb[j]);
    }
  }
  __syncthreads();
  float* out = partial + (size_t)chunk * V * W;
  for (int i = threadIdx.x; i < V * kSegCols; i += kSegThreads) {
    const int v = i / kSegCols, cc = c0 + (i % kSegCols);
    if (cc < W) out[(size_t)v * W + cc] = acc[i];
  }
}

template <typename T>
__global__ void __launch_bounds__(kSegThreads) colsum_kernel(const T* __restrict__ X, int ldx, int N,
                                                            int W, int rows_per_chunk,
                                                            float* __restrict__ partial) {
  __shared__ float red[kSegThreads / 64][kSegCols];
  const int c0 = blockIdx.x * kSegCols, chunk = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ca = c0 + lane, cb = c0 + 64 + lane;
  const bool va = ca < W, vb = cb < W;
  const int r0 = chunk * rows_per_chunk, r1 = min(N, r0 + rows_per_chunk);
  constexpr int U = 8, WS = kSegThreads / 64;
  float sa = 0.f, sb = 0.f;
  for (int n = r0 + wave; n < r1; n += WS * U) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int nn = n + WS * j;
      if (nn < r1) {
        const T* row = X + (size_t)nn * ldx;
        if (va) sa += (float)row[ca];
        if (vb) sb += (float)row[cb];
      }
    }
  }
  red[wave][lane] = sa;
  red[wave][64 + lane] = sb;
  __syncthreads();
  if (wave == 0) {
    float ta = 0.f, tb = 0.f;
#pragma unroll
    for (int k = 0; k < WS; ++k) { ta += red[k][lane]; tb += red[k][64 + lane]; }
    if (va) partial[(size_t)chunk * W + ca] = ta;
    if (vb) partial[(size_t)chunk * W + cb] = tb;
  }
}

// Column sums (bias gradients) of a bf16 [N, W] matrix with 16-byte rows: each lane reads 8
// consecutive columns (one 1 KB access per wave and row instead of 128 B), 8 rows in flight
// per wave; a workgroup owns 512 columns x one row chunk.  (The scalar colsum_kernel read the
// GRU-1024 [32768, 3072] dZ at 1.7 TB/s: 122 us.)
constexpr int kVecCols = 512;

__global__ void __launch_bounds__(kSegThreads) colsum_vec_kernel(const bf16* __restrict__ X, int ldx,
                                                                int N, int W, int rows_per_chunk,
                                                                float* __restrict__ partial) {
  __shared__ float red[kSegThreads / 64][kVecCols];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * kVecCols + lane * 8, chunk = blockIdx.y;
  const bool ok = c < W;  // W % 8 == 0: a lane's 8 columns are all in or all out
  const int r0 = chunk * rows_per_chunk, r1 = min(N, r0 + rows_per_chunk);
  constexpr int U = 8, WS = kSegThreads / 64;
  float acc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) acc[q] = 0.f;
  if (ok) {
    for (int n = r0 + wave; n < r1; n += WS * U) {
      bf16x8 v[U];
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const int nn = n + WS * j;
        if (nn < r1) {
          v[j] = *reinterpret_cast<const bf16x8*>(X + (size_t)nn * ldx + c);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) v[j][q] = f2bf(0.f);
        }
      }
#pragma unroll
      for (int j = 0; j < U; ++j)
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] += bf2f(v[j][q]);
    }
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) red[wave][lane * 8 + q] = acc[q];
  __syncthreads();
  for (int i = threadIdx.x; i < kVecCols; i += kSegThreads) {
    const int cc = blockIdx.x * kVecCols + i;
    if (cc < W) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < WS; ++k) t += red[k][i];
      partial[(size_t)chunk * W + cc] = t;
    }
  }
}

__global__ void __launch_bounds__(kSegThreads) segsum_reduce_kernel(const float* __restrict__ partial,
                                                                   int nchunks, int64_t VW,
                                                                   float* __restrict__ out,
                                                                   int accumulate) {
  for (int64_t i = blockIdx.x * (int64_t)kSegThreads + threadIdx.x; i < VW;
       i += (int64_t)gridDim.x * kSegThreads) {
    float s = 0.f;
    for (int k = 0; k < nchunks; ++k) s += partial[(size_t)k * VW + i];
    out[i] = accumulate ? out[i] + s : s;
  }
}

// Wide vocabularies: each workgroup owns kAtomicRows consecutive rows x one 256-column strip
// (one workgroup per row was dispatch-bound: 65536 one-atomic-per-thread workgroups took
// 141 us at N = 32768, W = 512); runs of equal ids inside the chunk are summed in registers
// and flushed with one fp32 atomic.  With ``perm`` the caller passes the ids sorted and perm[n]
// = source row of sorted position n: a frequent id then costs one atomic per chunk instead of
// one per occurrence (hot rows serialise the atomics; the synthetic 8k stream is unigram-skewed).
constexpr int kAtomicRows = 32;

template <typename T>
__global__ void __launch_bounds__(kSegThreads) segsum_atomic_kernel(const T* __restrict__ X, int ldx,
                                                                   const int* __restrict__ ids,
                                                                   const int* __restrict__ perm,
                                                                   int N, int W,
                                                                   float* __restrict__ out) {
  const int c = blockIdx.x * kSegThreads + threadIdx.x;
  const int n0 = blockIdx.y * kAtomicRows;
  const int n1 = n0 + kAtomicRows < N ? n0 + kAtomicRows : N;
  if (c >= W) return;
  float x[kAtomicRows];
#pragma unroll
  for (int i = 0; i < kAtomicRows; ++i)  // all loads in flight before the first atomic
    x[i] = n0 + i < n1 ? (float)X[(size_t)(perm ? perm[n0 + i] : n0 + i) * ldx + c] : 0.f;
  int cur = ids ? ids[n0] : 0;
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < kAtomicRows; ++i) {
    if (n0 + i >= n1) break;
    const int v = ids ? ids[n0 + i] : 0;
    if (v != cur) {
      atomicAdd(out + (size_t)cur * W + c, acc);
      acc = 0.f;
      cur = v;
    }
    acc += x[i];
  }
  atomicAdd(out + (size_t)cur * W + c, acc);
}

int segsum_rows_per_chunk(int N) {
  // ~64 chunks for large N: with the column strips this gives hundreds of workgroups, each
  // keeping 8 rows of loads in flight per wave, while the partials stay a few MB
  int r = (N + 63) / 64;
  r = ((r + 255) / 256) * 256;
  return r < 256 ? 256 : r;
}

size_t segsum_workspace_floats(int N, int W, int V) {
  if (V > kSegLdsMaxV) return 0;
  const int rpc = segsum_rows_per_chunk(N);
  const int nchunks = (N + rpc - 1) / rpc;
  return (size_t)nchunks * V * W;
}

template <typename T>
static void launch_segsum_t(const T* X, int ldx, const int* ids, int N, int W, int V, float* out,
                            float* workspace, int accumulate, const int* perm, hipStream_t s) {
  if (V > kSegLdsMaxV || perm) {
    if (!accumulate) (void)hipMemsetAsync(out, 0, sizeof(float) * (size_t)V * W, s);
    dim3 grid((W + kSegThreads - 1) / kSegThreads, (N + kAtomicRows - 1) / kAtomicRows);
    segsum_atomic_kernel<T><<<grid, kSegThreads, 0, s>>>(X, ldx, ids, perm, N, W, out);
    return;
  }
  const int rpc = segsum_rows_per_chunk(N);
  const int nchunks = (N + rpc - 1) / rpc;
  dim3 grid((W + kSegCols - 1) / kSegCols, nchunks);
  if (ids == nullptr && V == 1 && sizeof(T) == 2 && W % 8 == 0 && ldx % 8 == 0 &&
      (reinterpret_cast<uintptr_t>(X) & 15) == 0) {
    dim3 vgrid((W + kVecCols - 1) / kVecCols, nchunks);
    colsum_vec_kernel<<<vgrid, kSegThreads, 0, s>>>(reinterpret_cast<const bf16*>(X), ldx, N, W,
                                                    rpc, workspace);
  } else if (ids == nullptr && V == 1) {
    colsum_kernel<T><<<grid, kSegThreads, 0, s>>>(X, ldx, N, W, rpc, workspace);
  } else {
    const size_t lds = sizeof(float) * V * kSegCols;
    segsum_lds_kernel<T><<<grid, kSegThreads, lds, s>>>(X, ldx, ids, N, W, V, rpc, workspace);
  }
  const int64_t VW = (int64_t)V * W;
  int nb = (int)((VW + kSegThreads - 1) / kSegThreads);
  if (nb > 2048) nb = 2048;
  segsum_reduce_kernel<<<nb, kSegThreads, 0, s>>>(workspace, nchunks, VW, out, accumulate);
}

void launch_segsum_bf16(const bf16* X, int ldx, const int* ids, int N, int W, int V, float* out,
                        float* workspace, int accumulate, hipStream_t s, const int* perm) {
  launch_segsum_t<bf16>(X, ldx, ids, N, W, V, out, workspace, accumulate, perm, s);
}
void launch_segsum_f32(const float* X, int ldx, const int* ids, int N, int W, int V, float* out,
                       float* workspace, int accumulate, hipStream_t s, const int* perm) {
  launch_segsum_t<float>(X, ldx, ids, N, W, V, out, workspace, accumulate, perm, s);
}

}  // namespace dcr
