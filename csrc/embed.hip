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

// bf16 rows (16-byte aligned, ldx % 8 == 0) and V <= 128: the segment sum as a one-hot MFMA
// product, out[v][w] = sum_n onehot(ids[n])[v] * X[n][w] -- no atomics.  (LDS fp32 atomics
// measured ~190 G adds/s chip-wide on gfx950: 339 us for the [32768, 2048] dEW, 89 us for
// the [32768, 512] dropout dE -- far below the HBM bound of the read.)
//
// mfma_f32_16x16x32_bf16 with A = onehotᵀ (rows v, k = tokens) built in registers from the
// ids and B = the X tile (k = tokens, columns w).  B wants 8 consecutive TOKENS per lane, i.e.
// a column of the row-major X tile: the tile is staged in LDS as it lies in memory and read
// back with ds_read_b64_tr_b16 (gfx950's transposing LDS read: a 16-lane group reads a 4-row x
// 16-column block and lane i receives column i).  Workgroup = 64 columns x one row chunk,
// wave = one 16-column n-tile x all VT v-tiles; partials [chunk][V][W] are summed by
// segsum_reduce_kernel in a fixed order (bitwise reproducible).
constexpr int kOhCols = 64;               // columns per workgroup (4 waves x 16)
constexpr int kOhRows = 128;              // rows staged per LDS fill (4 MFMA k-steps)
constexpr int kOhLd = kOhCols + 8;        // LDS row stride (bf16): 144 B, fewer bank conflicts

typedef short s16x4 __attribute__((ext_vector_type(4)));

template <int VT>
__global__ void __launch_bounds__(kSegThreads) onehot_segsum_kernel(
    const bf16* __restrict__ X, int ldx, const int* __restrict__ ids, int N, int W, int V,
    int rows_per_chunk, float* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) bf16 tile[kOhRows][kOhLd];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, m = lane & 15;
  const int c0 = blockIdx.x * kOhCols, chunk = blockIdx.y;
  const int r0 = chunk * rows_per_chunk, r1 = min(N, r0 + rows_per_chunk);
  // rows >= r1 read as zero through the buffer range check (a NaN there would survive the
  // one-hot zero; onehot_ok keeps the buffer below 2 GB)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16*>(X), (short)0,
      (unsigned)min((size_t)0xFFFFFFF0ull, sizeof(bf16) * (size_t)N * ldx), 0x00020000);
  // staging: thread t -> rows (t >> 3) + 32 s, 8 columns at 8 (t & 7)
  const int srow = threadIdx.x >> 3, scol = 8 * (threadIdx.x & 7);
  f32x4 acc[VT];
#pragma unroll
  for (int vt = 0; vt < VT; ++vt) acc[vt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // transposing-read addresses: lane 4a + p of a 16-lane group names row a of its 4-row block,
  // columns 4p .. 4p+3 of the wave's 16-column tile
  const int ta = (lane & 15) >> 2, tp = lane & 3;
  // software pipeline: the next fill's rows are loaded into registers while this one computes
  auto fill = [&](int n0, bf16x8 (&st)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      // a row outside [n0, r1) gets an offset past the buffer: the range check returns zero
      // (a select on the loaded value would wait for the load right here)
      const int row = n0 + srow + 32 * s;
      const unsigned off = row < r1 ? (unsigned)(((size_t)row * ldx + c0 + scol) * sizeof(bf16))
                                    : 0x80000000u;
      st[s] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
    }
  };
  bf16x8 st[4];
  fill(r0, st);
  for (int n0 = r0; n0 < r1; n0 += kOhRows) {
    __syncthreads();  // the previous fill has been read
#pragma unroll
    for (int s = 0; s < 4; ++s) *reinterpret_cast<bf16x8*>(&tile[srow + 32 * s][scol]) = st[s];
    __syncthreads();
    if (n0 + kOhRows < r1) fill(n0 + kOhRows, st);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      // the 8 tokens of this lane's k-slice: rows n0 + 32 s + 8 q + j
      const int nb = n0 + 32 * s + 8 * q;
      int id[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) id[j] = nb + j < r1 ? ids[nb + j] : -1;
      const int rb = 32 * s + 8 * q + ta;
      const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)&tile[rb][16 * wave + 4 * tp]);
      const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)&tile[rb + 4][16 * wave + 4 * tp]);
      u32x4 bu;
      bu[0] = (unsigned)(unsigned short)lo[0] | ((unsigned)(unsigned short)lo[1] << 16);
      bu[1] = (unsigned)(unsigned short)lo[2] | ((unsigned)(unsigned short)lo[3] << 16);
      bu[2] = (unsigned)(unsigned short)hi[0] | ((unsigned)(unsigned short)hi[1] << 16);
      bu[3] = (unsigned)(unsigned short)hi[2] | ((unsigned)(unsigned short)hi[3] << 16);
      const bf16x8 b = __builtin_bit_cast(bf16x8, bu);
#pragma unroll
      for (int vt = 0; vt < VT; ++vt) {
        const int v = 16 * vt + m;  // this lane's A row
        u32x4 au;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          au[i] = (id[2 * i] == v ? 0x3F80u : 0u) | (id[2 * i + 1] == v ? 0x3F800000u : 0u);
        acc[vt] = mfma16(__builtin_bit_cast(bf16x8, au), b, acc[vt]);
      }
    }
  }
  // D[v = 16 vt + 4 q + i][w = c0 + 16 wave + m]
  const int w = c0 + 16 * wave + m;
  if (w < W) {
    float* out = partial + (size_t)chunk * V * W + w;
#pragma unroll
    for (int vt = 0; vt < VT; ++vt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int v = 16 * vt + 4 * q + i;
        if (v < V) out[(size_t)v * W] = acc[vt][i];
      }
  }
}

static bool onehot_ok(const void* X, int ldx, const int* ids, int V) {
  return ids != nullptr && V >= 1 && V <= 128 && ldx % 8 == 0 &&
         (reinterpret_cast<uintptr_t>(X) & 15) == 0;
}
static bool onehot_fits(int N, int ldx) {
  return (size_t)N * ldx * sizeof(bf16) < 0x80000000ull;
}

// ~1024 workgroups (4 per CU) without making the partials larger than the data
static int onehot_rows_per_chunk(int N, int W) {
  const int strips = (W + kOhCols - 1) / kOhCols;
  int chunks = (1024 + strips - 1) / strips;
  chunks = chunks < 1 ? 1 : (chunks > 128 ? 128 : chunks);
  int r = (N + chunks - 1) / chunks;
  r = ((r + kOhRows - 1) / kOhRows) * kOhRows;
  return r < kOhRows ? kOhRows : r;
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

// out = sum over chunks of partial[chunk][VW], in a fixed order (bitwise reproducible).  A
// workgroup reduces 32 consecutive elements with 8 chunk lanes each (one thread per element
// looped over all chunks serially: 31 us for 128 x [65 x 512]).
__global__ void __launch_bounds__(kSegThreads) segsum_reduce_kernel(const float* __restrict__ partial,
                                                                   int nchunks, int64_t VW,
                                                                   float* __restrict__ out,
                                                                   int accumulate) {
  __shared__ float red[kSegThreads / 32][32];
  const int e = threadIdx.x & 31, c = threadIdx.x >> 5;
  for (int64_t base = (int64_t)blockIdx.x * 32; base < VW; base += (int64_t)gridDim.x * 32) {
    const int64_t i = base + e;
    float s = 0.f;
    if (i < VW) {
#pragma unroll 4
      for (int k = c; k < nchunks; k += kSegThreads / 32) s += partial[(size_t)k * VW + i];
    }
    red[c][e] = s;
    __syncthreads();
    if (c == 0 && i < VW) {
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < kSegThreads / 32; ++k) t += red[k][e];
      out[i] = accumulate ? out[i] + t : t;
    }
    __syncthreads();
  }
}

static void launch_reduce(const float* partial, int nchunks, int64_t VW, float* out,
                          int accumulate, hipStream_t s) {
  const int64_t nb = (VW + 31) / 32;
  segsum_reduce_kernel<<<(int)(nb < 8192 ? nb : 8192), kSegThreads, 0, s>>>(partial, nchunks, VW,
                                                                            out, accumulate);
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
  // the larger of the LDS route's and the one-hot route's partials (the caller does not know
  // which one a launch takes)
  const int rpc = segsum_rows_per_chunk(N), rpo = onehot_rows_per_chunk(N, W);
  const size_t a = (size_t)((N + rpc - 1) / rpc), b = (size_t)((N + rpo - 1) / rpo);
  return (a > b ? a : b) * V * W;
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
  if (sizeof(T) == 2 && onehot_ok(X, ldx, ids, V) && onehot_fits(N, ldx)) {
    const int rpc = onehot_rows_per_chunk(N, W);
    const int nchunks = (N + rpc - 1) / rpc;
    dim3 grid((W + kOhCols - 1) / kOhCols, nchunks);
    const bf16* Xb = reinterpret_cast<const bf16*>(X);
    switch ((V + 15) / 16) {
#define OH(VT) \
  case VT: onehot_segsum_kernel<VT><<<grid, kSegThreads, 0, s>>>(Xb, ldx, ids, N, W, V, rpc, workspace); break;
      OH(1) OH(2) OH(3) OH(4) OH(5) OH(6) OH(7) OH(8)
#undef OH
    }
    launch_reduce(workspace, nchunks, (int64_t)V * W, out, accumulate, s);
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
  launch_reduce(workspace, nchunks, (int64_t)V * W, out, accumulate, s);
}

// ---- stable id sort for the wide-vocabulary segment sum (a V-bucketed counting sort) --------
// The atomic route above wants the ids sorted (sid) with their source rows (perm).  Instead of a
// general radix / merge sort (~10 small library launches) the ids are bucketed by value in three
// launches over kSortChunk-id chunks:
//   hist     chunk b counts its ids per value (LDS, two 16-bit counts per word) -> cnt[b][v]
//   colscan  one thread per value: cnt[b][v] <- sum_{b' < b} cnt[b'][v] (in place), tot[v]
//   scatter  chunk b: start(v) = exclusive scan of tot (every chunk scans the V totals itself),
//            offs[v] = start(v) + cnt[b][v] (16-bit, LDS); then one wave places the chunk's ids
//            in 64-id rounds: lanes holding the same value are found with one ballot per value
//            bit, ranked by lane and written at offs[v] + rank; the value's lowest lane advances
//            offs[v] by their count.
// Positions within a value follow the id order: the result is torch.sort(ids, stable=True).
// The LDS tables hold 16-bit words (N <= 65535, V <= 16384: at most 16 KB).
constexpr int kSortChunk = 1024, kSortThreads = 256;

__device__ __forceinline__ void lds_add16(unsigned* w, int v, unsigned x) {
  atomicAdd(w + (v >> 1), x << ((v & 1) * 16));
}
__device__ __forceinline__ unsigned lds_get16(const unsigned* w, int v) {
  return (w[v >> 1] >> ((v & 1) * 16)) & 0xFFFFu;
}

// (zero, nz4): an fp32 buffer of nz4 float4s to clear on the side -- the segment sum's atomic
// output (the embedding gradient), which then needs no separate fill launch
__global__ void __launch_bounds__(kSortThreads) id_hist_kernel(const int* __restrict__ ids, int N,
                                                               int V4, int* __restrict__ cnt,
                                                               float4* __restrict__ zero,
                                                               long nz4) {
  extern __shared__ unsigned hist[];  // [V4 / 2] packed 16-bit counts
  for (int i = threadIdx.x; i < V4 / 2; i += kSortThreads) hist[i] = 0u;
  __syncthreads();
  const int n0 = blockIdx.x * kSortChunk;
  int id[kSortChunk / kSortThreads];
#pragma unroll
  for (int i = 0; i < kSortChunk / kSortThreads; ++i) {  // every load before the first atomic
    const int n = n0 + i * kSortThreads + threadIdx.x;
    id[i] = ids[n < N ? n : N - 1];
  }
#pragma unroll
  for (int i = 0; i < kSortChunk / kSortThreads; ++i)
    if (n0 + i * kSortThreads + (int)threadIdx.x < N) lds_add16(hist, id[i], 1u);
  __syncthreads();
  int4* const o = reinterpret_cast<int4*>(cnt + (size_t)blockIdx.x * V4);
  for (int q = threadIdx.x; q < V4 / 4; q += kSortThreads) {
    const unsigned a = hist[2 * q], b = hist[2 * q + 1];
    o[q] = int4{(int)(a & 0xFFFFu), (int)(a >> 16), (int)(b & 0xFFFFu), (int)(b >> 16)};
  }
  if (zero) {
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    for (long i = (long)blockIdx.x * kSortThreads + threadIdx.x; i < nz4;
         i += (long)gridDim.x * kSortThreads)
      zero[i] = z;
  }
}

constexpr int kSortRows = 8;  // count rows in flight per thread

__global__ void __launch_bounds__(kSortThreads) id_colscan_kernel(int V4, int nblk, int* __restrict__ cnt,
                                                                  int* __restrict__ tot) {
  const int v = blockIdx.x * kSortThreads + threadIdx.x;
  if (v >= V4) return;
  int run = 0;
  for (int b0 = 0; b0 < nblk; b0 += kSortRows) {
    int x[kSortRows];
#pragma unroll
    for (int j = 0; j < kSortRows; ++j)  // clamped rows: all loads unconditional
      x[j] = cnt[(size_t)(b0 + j < nblk ? b0 + j : nblk - 1) * V4 + v];
#pragma unroll
    for (int j = 0; j < kSortRows; ++j)
      if (b0 + j < nblk) {
        cnt[(size_t)(b0 + j) * V4 + v] = run;
        run += x[j];
      }
  }
  tot[v] = run;
}

// Q: value quads per thread (V <= 4 Q kSortThreads; Q = 8 at V = 8192)
template <int Q>
__global__ void __launch_bounds__(kSortThreads) id_scatter_kernel(const int* __restrict__ ids, int N,
                                                                  int V4, int nbits,
                                                                  const int* __restrict__ cnt,
                                                                  const int* __restrict__ tot,
                                                                  int* __restrict__ sid,
                                                                  int* __restrict__ perm) {
  extern __shared__ unsigned offs[];  // [V4 / 2] packed 16-bit first positions
  __shared__ int wsum[kSortThreads / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int b = blockIdx.x;
  const int nq = V4 / 4;  // value quads; segment k covers quads [k kSortThreads, (k + 1) kSortThreads)
  const int4* const t4 = reinterpret_cast<const int4*>(tot);
  const int4* const r4 = reinterpret_cast<const int4*>(cnt + (size_t)b * V4);
  int4 tq[Q], rq[Q];
#pragma unroll
  for (int k = 0; k < Q; ++k) {  // clamped quads: all loads unconditional
    const int q = k * kSortThreads + t < nq ? k * kSortThreads + t : nq - 1;
    tq[k] = t4[q];
    rq[k] = r4[q];
  }
  int carry = 0;
#pragma unroll
  for (int k = 0; k < Q; ++k) {
    if (k * kSortThreads >= nq) break;  // (uniform)
    const int q = k * kSortThreads + t;
    const int4 c = q < nq ? tq[k] : int4{0, 0, 0, 0};
    const int mine = c.x + c.y + c.z + c.w;
    int inc = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int o = __shfl_up(inc, d, 64);
      if (lane >= d) inc += o;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int before = carry, seg = 0;
#pragma unroll
    for (int i = 0; i < kSortThreads / 64; ++i) {
      before += i < w ? wsum[i] : 0;
      seg += wsum[i];
    }
    __syncthreads();  // (wsum is reused by the next segment)
    carry += seg;
    if (q < nq) {
      const int e = before + inc - mine;  // start of value 4 q
      const int4 r = rq[k];
      offs[2 * q] = (unsigned)(e + r.x) | ((unsigned)(e + c.x + r.y) << 16);
      offs[2 * q + 1] =
          (unsigned)(e + c.x + c.y + r.z) | ((unsigned)(e + c.x + c.y + c.z + r.w) << 16);
    }
  }
  __syncthreads();
  if (w != 0) return;
  // one wave: 64-id rounds in id order (all ids loaded first)
  const int n0 = b * kSortChunk;
  int idv[kSortChunk / 64];
#pragma unroll
  for (int r = 0; r < kSortChunk / 64; ++r) {
    const int n = n0 + r * 64 + lane;
    idv[r] = ids[n < N ? n : N - 1];
  }
  const unsigned long long lt = (1ull << lane) - 1ull;
  for (int r = 0; r < kSortChunk / 64; ++r) {
    const int n = n0 + r * 64 + lane;
    const bool ok = n < N;
    const int id = idv[r];
    unsigned long long m = __ballot(ok);
    for (int bit = 0; bit < nbits; ++bit) {
      const bool on = (id >> bit) & 1;
      const unsigned long long bal = __ballot(on);
      m &= on ? bal : ~bal;
    }
    const int base = (int)lds_get16(offs, id);
    const int pos = base + __popcll(m & lt);
    if (ok) {
      sid[pos] = id;
      perm[pos] = n;
      if ((m & lt) == 0ull) lds_add16(offs, id, (unsigned)__popcll(m));  // the value's lowest lane
    }
    // (one wave: its LDS operations complete in order, so the next round reads the updates)
  }
}

int id_sort_blocks(int N) { return (N + kSortChunk - 1) / kSortChunk; }
int id_sort_cols(int V) { return (V + 3) / 4 * 4; }
size_t id_sort_workspace(int N, int V) {
  return (size_t)(id_sort_blocks(N) + 1) * id_sort_cols(V);  // counts + totals
}

int launch_id_sort(const int* ids, int N, int V, int* ws, int* sid, int* perm, hipStream_t s,
                   float* zero, size_t zero_n) {
  if (N <= 0 || N > 65535 || V <= 0 || V > 16384) return -1;
  const int nblk = id_sort_blocks(N), V4 = id_sort_cols(V);
  int nbits = 0;
  while ((1 << nbits) < V) ++nbits;
  int* const tot = ws + (size_t)nblk * V4;
  const size_t lds = sizeof(unsigned) * (size_t)V4 / 2;
  // (zero: 16-B aligned, a whole number of float4s -- the caller checks)
  id_hist_kernel<<<nblk, kSortThreads, lds, s>>>(ids, N, V4, ws, reinterpret_cast<float4*>(zero),
                                                 zero ? (long)(zero_n / 4) : 0L);
  id_colscan_kernel<<<(V4 + kSortThreads - 1) / kSortThreads, kSortThreads, 0, s>>>(V4, nblk, ws, tot);
  const int q = (V4 / 4 + kSortThreads - 1) / kSortThreads;
#define SCAT(Q) id_scatter_kernel<Q><<<nblk, kSortThreads, lds, s>>>(ids, N, V4, nbits, ws, tot, sid, perm)
  if (q <= 1) SCAT(1);
  else if (q <= 2) SCAT(2);
  else if (q <= 4) SCAT(4);
  else if (q <= 8) SCAT(8);
  else SCAT(16);
#undef SCAT
  return 0;
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
