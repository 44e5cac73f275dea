// One launch for the per-step data movement around the persistent kernels.
//
// After every optimizer step the recurrent kernels need bf16 copies of the fp32 master weights in
// several layouts (W_h, W_hᵀ, W_x, W_xᵀ, the padded head matrices) and the layer-0 table
// E·W_x0 + b0; before each forward the initial state goes into slot 0 of the h/c sequence
// buffers, the hand-off counters are zeroed, the batch's token ids are transposed to time-major
// order and (gather route) expanded into the one-hot matrix of the embedding-table gradient.
// After the weight-gradient GEMMs their split-K slabs and the BPTT kernels' bias partials are
// summed into the flat gradient buffer.  Done with torch ops that was ~30 small kernels per step
// (~5 us each on MI355X: profiles/r1_v6_exclusive_fused_head.md, profiles/r2_tail_*.md).  Here
// the host builds a table of tasks over arbitrary row-strided 2-D views and ONE kernel executes
// it: each workgroup takes one 64x64 tile of one task.
//
//   COPY       dst[r, c] = convert(src[r, c])            (fp32 -> bf16 / fp32, or raw 32-bit)
//   TRANSPOSE  dst[c, r] = convert(src[r, c])            64x64 tile staged through LDS
//   ZERO       dst[r, c] = 0                             (4-byte elements; counters)
//   SUM        dst[r, c] = sum_s src[s][r, c]            split-K slabs, fixed order s = 0..S-1
//   COLSUM     dst[0, c] = sum_r src[r, c]               bias partials, fixed order
//   ONEHOT     dst[n, v] = (ids[n % B][n / B] == v)      bf16 one-hot of the time-major ids
//   TABLE      dst[v, c] = bias[c] + sum_k E[v, k] W[k, c]   fp32 FMA (layer-0 gather table)
//   GATHER     dst[n, c] = bf16(E[ids[n % B][n / B], c])    time-major embedding rows (the wide-
//              vocabulary dW_x0 = X0ᵀ·dZ0 operand: no separate gather launch mid-backward)
// Every output element is written by exactly one thread with a fixed summation order, so the
// results are bitwise reproducible.
#include "common.h"
#include "kernels.h"

namespace dcr {

constexpr int kPrepTile = 64;

// Rows per tile: 64, except the long-reduction modes, whose per-element work is K (TABLE) or
// S (scalar SUM) dependent loads/FMAs: 16-row tiles give them 4x the workgroups.
__host__ __device__ __forceinline__ int prep_tile_rows(int mode, int vec4) {
  return (mode == PREP_TABLE || (mode == PREP_SUM && !vec4)) ? 16 : kPrepTile;
}
// (ONEHOT vec4: a tile spans the whole row, up to 256 columns, in 16-B chunks)
__host__ __device__ __forceinline__ int prep_tile_cols(int mode, int vec4) {
  return mode == PREP_TABLE ? 16 : (mode == PREP_ONEHOT && vec4) ? 256 : kPrepTile;
}

__device__ __forceinline__ void prep_put(const PrepTask& T, size_t idx, float v) {
  if (T.kind == PREP_BF16) reinterpret_cast<bf16*>(T.dst)[idx] = f2bf(v);
  else reinterpret_cast<float*>(T.dst)[idx] = v;
}

// 4 consecutive destination elements (16-B aligned fp32 / 8-B aligned bf16: vec4 tasks)
__device__ __forceinline__ void prep_put4(const PrepTask& T, size_t idx, float4 v) {
  if (T.kind == PREP_BF16) {
    bf16x4 b;
    b[0] = f2bf(v.x); b[1] = f2bf(v.y); b[2] = f2bf(v.z); b[3] = f2bf(v.w);
    *reinterpret_cast<bf16x4*>(reinterpret_cast<bf16*>(T.dst) + idx) = b;
  } else {
    *reinterpret_cast<float4*>(reinterpret_cast<float*>(T.dst) + idx) = v;
  }
}

__global__ void __launch_bounds__(256) prep_kernel(PrepTable tab) {
  __shared__ float tile[kPrepTile][kPrepTile + 1];
  int bid = blockIdx.x, k = 0;
  while (k + 1 < tab.n && bid >= tab.t[k + 1].tile0) ++k;
  const PrepTask& T = tab.t[k];
  const int local = bid - T.tile0;
  const int tcw = prep_tile_cols(T.mode, T.vec4);
  const int tiles_c = (T.cols + tcw - 1) / tcw;
  const int tr = prep_tile_rows(T.mode, T.vec4);
  const int r0 = (local / tiles_c) * tr, c0 = (local % tiles_c) * tcw;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4
  const int r1 = min(r0 + tr, T.rows);
  const float* src = static_cast<const float*>(T.src);
  switch (T.mode) {
    case PREP_ZERO:
      for (int r = r0 + ty; r < r1; r += 4)
        if (c0 + tx < T.cols) reinterpret_cast<float*>(T.dst)[(size_t)r * T.dst_ld + c0 + tx] = 0.f;
      return;
    case PREP_COPY:
      if (T.kind == PREP_RAW32) {
        const unsigned* s = static_cast<const unsigned*>(T.src);
        const int cc = min(c0 + tx, T.cols - 1);
        unsigned v[kPrepTile / 4];  // (all loads before the first store)
#pragma unroll
        for (int i = 0; i < kPrepTile / 4; ++i)
          v[i] = s[(size_t)min(r0 + ty + 4 * i, T.rows - 1) * T.src_ld + cc];
        if (c0 + tx < T.cols)
#pragma unroll
          for (int i = 0; i < kPrepTile / 4; ++i)
            if (r0 + ty + 4 * i < r1)
              reinterpret_cast<unsigned*>(T.dst)[(size_t)(r0 + ty + 4 * i) * T.dst_ld + c0 + tx] = v[i];
        return;
      }
      if (T.vec4) {  // 16 lanes x float4 per 64-column row, 16 rows per pass
        const int c = c0 + 4 * (threadIdx.x & 15);
        if (c >= T.cols) return;
        float4 v[kPrepTile / 16];  // (all loads before the first store)
#pragma unroll
        for (int i = 0; i < kPrepTile / 16; ++i)
          v[i] = *reinterpret_cast<const float4*>(
              src + (size_t)min(r0 + (threadIdx.x >> 4) + 16 * i, T.rows - 1) * T.src_ld + c);
#pragma unroll
        for (int i = 0; i < kPrepTile / 16; ++i) {
          const int r = r0 + (threadIdx.x >> 4) + 16 * i;
          if (r < r1) prep_put4(T, (size_t)r * T.dst_ld + c, v[i]);
        }
        return;
      }
      {
        const int cc = min(c0 + tx, T.cols - 1);
        float v[kPrepTile / 4];  // (all loads before the first store)
#pragma unroll
        for (int i = 0; i < kPrepTile / 4; ++i)
          v[i] = src[(size_t)min(r0 + ty + 4 * i, T.rows - 1) * T.src_ld + cc];
        if (c0 + tx < T.cols)
#pragma unroll
          for (int i = 0; i < kPrepTile / 4; ++i)
            if (r0 + ty + 4 * i < r1) prep_put(T, (size_t)(r0 + ty + 4 * i) * T.dst_ld + c0 + tx, v[i]);
      }
      return;
    case PREP_SUM: {
      if (T.vec4) {
        // 16 lanes x float4 cover the tile's 64 columns; each thread owns 4 rows (16 apart) and
        // issues its loads for 4 rows x up to 4 slabs together before summing (the slab loop
        // with one dependent load per trip was latency-bound: 1 TB/s)
        const int c = c0 + 4 * (threadIdx.x & 15);
        const int rr = r0 + (threadIdx.x >> 4);
        if (c >= T.cols) return;
        float4 acc[4];
        const float* p[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          // rows past the tile end re-read the tile's first row r0 (< r1; never stored)
          const int r = rr + 16 * i < r1 ? rr + 16 * i : r0;
          p[i] = src + (size_t)r * T.src_ld + c;
          acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        int s = 0;
        for (; s + 4 <= T.nslab; s += 4) {
          float4 v[4][4];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              v[i][j] = *reinterpret_cast<const float4*>(p[i] + (size_t)(s + j) * T.slab);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              acc[i].x += v[i][j].x; acc[i].y += v[i][j].y;
              acc[i].z += v[i][j].z; acc[i].w += v[i][j].w;
            }
        }
        for (; s < T.nslab; ++s) {
          float4 v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = *reinterpret_cast<const float4*>(p[i] + (size_t)s * T.slab);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            acc[i].x += v[i].x; acc[i].y += v[i].y; acc[i].z += v[i].z; acc[i].w += v[i].w;
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (rr + 16 * i < r1)
            *reinterpret_cast<float4*>(static_cast<float*>(T.dst) + (size_t)(rr + 16 * i) * T.dst_ld + c) = acc[i];
        return;
      }
      {
        // scalar path (16-row tile): thread (tx, ty) owns rows ty + 4 i, i < 4; loads of 4 rows
        // x 4 slabs in flight per batch
        const int c = c0 + tx;
        if (c >= T.cols) return;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        const float* p[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = r0 + ty + 4 * i < r1 ? r0 + ty + 4 * i : r0;
          p[i] = src + (size_t)r * T.src_ld + c;
        }
        int s = 0;
        for (; s + 4 <= T.nslab; s += 4) {
          float v[4][4];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) v[i][j] = p[i][(size_t)(s + j) * T.slab];
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] += v[i][0] + v[i][1] + v[i][2] + v[i][3];
        }
        for (; s < T.nslab; ++s)
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i] += p[i][(size_t)s * T.slab];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (r0 + ty + 4 * i < r1)
            reinterpret_cast<float*>(T.dst)[(size_t)(r0 + ty + 4 * i) * T.dst_ld + c] = acc[i];
      }
      return;
    }
    case PREP_COLSUM: {
      // one tile row spans every source row; 4 row phases (ty), combined
      // in LDS in a fixed order
      float acc = 0.f;
      if (c0 + tx < T.cols)
        for (int r = ty; r < T.rows; r += 4) acc += src[(size_t)r * T.src_ld + c0 + tx];
      tile[ty][tx] = acc;
      __syncthreads();
      if (ty == 0 && c0 + tx < T.cols)
        reinterpret_cast<float*>(T.dst)[c0 + tx] = tile[0][tx] + tile[1][tx] + tile[2][tx] + tile[3][tx];
      return;
    }
    case PREP_ONEHOT: {
      // dst row n = t*B + b (time-major) <- ids[b][t] of the batch-major source view
      // (the 16 ids of a thread's rows loaded together, unconditionally at clamped rows: a
      // guarded load in the row loop is one serialised round trip per row)
      const int* ids = static_cast<const int*>(T.src);
      const int B = T.kdim;
      if (T.vec4) {
        // whole rows in 16-B chunks of 8 columns: 4 threads per row, chunks j = t % 4 + 4 i
        // (2-byte stores of 64-column tiles wrote the 72-column rows at 0.9 TB/s)
        const int r = r0 + (threadIdx.x >> 2);
        if (r >= r1) return;
        const int id = ids[(size_t)(r % B) * T.src_ld + r / B];
        bf16* row = reinterpret_cast<bf16*>(T.dst) + (size_t)r * T.dst_ld;
        for (int j = threadIdx.x & 3; 8 * j < T.cols; j += 4) {
          const int k = id - 8 * j;  // the one's position in this chunk (outside: none)
          const unsigned one = (k >= 0 && k < 8) ? 0x3F80u << (16 * (k & 1)) : 0u;  // bf16 1.0
          const int wd = k >> 1;
          uint4 v;
          v.x = wd == 0 ? one : 0u;
          v.y = wd == 1 ? one : 0u;
          v.z = wd == 2 ? one : 0u;
          v.w = wd == 3 ? one : 0u;
          *reinterpret_cast<uint4*>(row + 8 * j) = v;
        }
        return;
      }
      int idv[kPrepTile / 4];
#pragma unroll
      for (int i = 0; i < kPrepTile / 4; ++i) {
        const int n = min(r0 + ty + 4 * i, T.rows - 1);
        idv[i] = ids[(size_t)(n % B) * T.src_ld + n / B];
      }
      if (c0 + tx < T.cols)
#pragma unroll
        for (int i = 0; i < kPrepTile / 4; ++i) {
          const int n = r0 + ty + 4 * i;
          if (n < r1)
            reinterpret_cast<bf16*>(T.dst)[(size_t)n * T.dst_ld + c0 + tx] =
                f2bf(idv[i] == c0 + tx ? 1.f : 0.f);
        }
      return;
    }
    case PREP_GATHER: {
      // as ONEHOT: dst row n = t*B + b <- E row ids[b][t]; every load of the tile (the 16 ids,
      // then the 16 E values at clamped rows / columns) before the first store
      const int* ids = static_cast<const int*>(T.src);
      const int B = T.kdim;
      if (T.vec4) {  // 16 lanes x float4 per 64-column row, 16 rows per pass (as COPY)
        const int c = c0 + 4 * (threadIdx.x & 15);
        if (c >= T.cols) return;
        int idv[kPrepTile / 16];
#pragma unroll
        for (int i = 0; i < kPrepTile / 16; ++i) {
          const int n = min(r0 + (int)(threadIdx.x >> 4) + 16 * i, T.rows - 1);
          idv[i] = ids[(size_t)(n % B) * T.src_ld + n / B];
        }
        float4 v[kPrepTile / 16];
#pragma unroll
        for (int i = 0; i < kPrepTile / 16; ++i)
          v[i] = *reinterpret_cast<const float4*>(T.src2 + (size_t)idv[i] * T.src2_ld + c);
#pragma unroll
        for (int i = 0; i < kPrepTile / 16; ++i) {
          const int n = r0 + (threadIdx.x >> 4) + 16 * i;
          if (n < r1) prep_put4(T, (size_t)n * T.dst_ld + c, v[i]);
        }
        return;
      }
      int idv[kPrepTile / 4];
#pragma unroll
      for (int i = 0; i < kPrepTile / 4; ++i) {
        const int n = min(r0 + ty + 4 * i, T.rows - 1);
        idv[i] = ids[(size_t)(n % B) * T.src_ld + n / B];
      }
      const int cc = min(c0 + tx, T.cols - 1);
      float v[kPrepTile / 4];
#pragma unroll
      for (int i = 0; i < kPrepTile / 4; ++i) v[i] = T.src2[(size_t)idv[i] * T.src2_ld + cc];
      if (c0 + tx < T.cols)
#pragma unroll
        for (int i = 0; i < kPrepTile / 4; ++i) {
          const int n = r0 + ty + 4 * i;
          if (n < r1) reinterpret_cast<bf16*>(T.dst)[(size_t)n * T.dst_ld + c0 + tx] = f2bf(v[i]);
        }
      return;
    }
    case PREP_TABLE: {
      // 16 x 16 tile of E·W + b on fp32 MFMA (v_mfma_f32_16x16x4_f32: fp32 operands and
      // accumulation, the precision of the fp32 library GEMM it replaces).  The 4 waves split K
      // in quarters; each lane issues all its operand loads of the quarter at once (straight
      // from L2/HBM: 64 loads in flight) and the quarters' tiles are summed through LDS in a
      // fixed order.  Lane l: A = E[l & 15][k + (l >> 4)], B = W[k + (l >> 4)][l & 15],
      // D[4 (l >> 4) + i][l & 15].  (64 x 64 tiles staged through LDS k-block by k-block were
      // latency-bound: 33-53 us for the 65 x 2048 table.)
      const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
      const int kq = (((T.kdim + 3) / 4) + 15) & ~15;      // k per wave, a multiple of 16
      const int ka = w * kq, kz = min(T.kdim, ka + kq);
      const int ar = r0 + (lane & 15), bc = c0 + (lane & 15);
      const float* Ep = src + (size_t)min(ar, T.rows - 1) * T.src_ld;
      const float* Wp = T.src2 + min(bc, T.cols - 1);
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int k0 = ka; k0 < kz; k0 += 64) {
        float av[16], bv[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {  // (unconditional loads at a clamped k, then a select)
          const int k = k0 + 4 * j + (lane >> 4);
          const int kc = min(k, kz - 1);
          const float a_ = Ep[kc], b_ = Wp[(size_t)kc * T.src2_ld];
          av[j] = k < kz ? a_ : 0.f;
          bv[j] = k < kz ? b_ : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[j], acc, 0, 0, 0);
      }
      // rows >= rows / cols >= cols computed on clamped operands: never stored
      float* red = &tile[0][0];  // [4 waves][64 lanes][4]
      *reinterpret_cast<float4*>(red + (w * 64 + lane) * 4) = make_float4(acc[0], acc[1], acc[2], acc[3]);
      __syncthreads();
      if (w == 0) {
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          o[i] = red[lane * 4 + i] + red[(64 + lane) * 4 + i] + red[(128 + lane) * 4 + i] +
                 red[(192 + lane) * 4 + i];
        if (bc < T.cols) {
          const float b = T.aux ? T.aux[bc] : 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = r0 + 4 * (lane >> 4) + i;
            if (r < T.rows) reinterpret_cast<float*>(T.dst)[(size_t)r * T.dst_ld + bc] = o[i] + b;
          }
        }
      }
      return;
    }
    default:
      break;
  }
  // TRANSPOSE: coalesced read of rows r, coalesced write of dst rows c
  if (T.kind == PREP_RAW32) {
    // (every load of the tile issued before the LDS stores, unconditionally at clamped
    // coordinates: guarded loads in the row loop serialise one round trip per row)
    const unsigned* s = static_cast<const unsigned*>(T.src);
    const int cc = min(c0 + tx, T.cols - 1);
    unsigned v[kPrepTile / 4];
#pragma unroll
    for (int i = 0; i < kPrepTile / 4; ++i)
      v[i] = s[(size_t)min(r0 + ty + 4 * i, T.rows - 1) * T.src_ld + cc];
#pragma unroll
    for (int i = 0; i < kPrepTile / 4; ++i) tile[ty + 4 * i][tx] = __builtin_bit_cast(float, v[i]);
    __syncthreads();
    for (int c = ty; c < kPrepTile; c += 4)
      if (c0 + c < T.cols && r0 + tx < T.rows)
        reinterpret_cast<unsigned*>(T.dst)[(size_t)(c0 + c) * T.dst_ld + r0 + tx] =
            __builtin_bit_cast(unsigned, tile[tx][c]);
    return;
  }
  if (T.vec4) {
    // float4 row reads into the tile; each thread then writes 4 consecutive destination
    // elements (source rows r..r+3 of one column) as one 8-B (bf16) / 16-B (fp32) store
    const int cq = 4 * (threadIdx.x & 15);
    const int cqc = min(c0 + cq, T.cols - 4);  // (vec4: cols % 4 == 0)
    float4 v[kPrepTile / 16];
#pragma unroll
    for (int i = 0; i < kPrepTile / 16; ++i)
      v[i] = *reinterpret_cast<const float4*>(
          src + (size_t)min(r0 + (threadIdx.x >> 4) + 16 * i, T.rows - 1) * T.src_ld + cqc);
#pragma unroll
    for (int i = 0; i < kPrepTile / 16; ++i) {
      const int r = (threadIdx.x >> 4) + 16 * i;
      tile[r][cq] = v[i].x; tile[r][cq + 1] = v[i].y; tile[r][cq + 2] = v[i].z; tile[r][cq + 3] = v[i].w;
    }
    __syncthreads();
    const int rq = 4 * (threadIdx.x & 15);
    for (int c = threadIdx.x >> 4; c < kPrepTile; c += 16)
      if (c0 + c < T.cols && r0 + rq < T.rows)
        prep_put4(T, (size_t)(c0 + c) * T.dst_ld + r0 + rq,
                  make_float4(tile[rq][c], tile[rq + 1][c], tile[rq + 2][c], tile[rq + 3][c]));
    return;
  }
  {
    const int cc = min(c0 + tx, T.cols - 1);
    float v[kPrepTile / 4];
#pragma unroll
    for (int i = 0; i < kPrepTile / 4; ++i)
      v[i] = src[(size_t)min(r0 + ty + 4 * i, T.rows - 1) * T.src_ld + cc];
#pragma unroll
    for (int i = 0; i < kPrepTile / 4; ++i) tile[ty + 4 * i][tx] = v[i];
  }
  __syncthreads();
  for (int c = ty; c < kPrepTile; c += 4)
    if (c0 + c < T.cols && r0 + tx < T.rows) prep_put(T, (size_t)(c0 + c) * T.dst_ld + r0 + tx, tile[tx][c]);
}

int prep_tiles(const PrepTask& t) {
  const int tcw = prep_tile_cols(t.mode, t.vec4);
  const int tc = (t.cols + tcw - 1) / tcw;
  if (t.mode == PREP_COLSUM) return tc;  // one tile row spans every source row
  const int tr = prep_tile_rows(t.mode, t.vec4);
  return ((t.rows + tr - 1) / tr) * tc;
}

void launch_prep(PrepTable& tab, hipStream_t s) {
  int tiles = 0;
  for (int i = 0; i < tab.n; ++i) {
    tab.t[i].tile0 = tiles;
    tiles += prep_tiles(tab.t[i]);
  }
  if (tiles > 0) prep_kernel<<<tiles, 256, 0, s>>>(tab);
}

}  // namespace dcr
