// The training step's tail as two persistent launches (gfx950): gradient FINALIZE after the
// weight-gradient GEMMs, and the fused ADAM update that also writes every bf16 kernel layout.
//
// Reference: clip_by_global_norm(tf.gradients(cost, tvars), grad_clip) and
// AdamOptimizer(lr).apply_gradients (model.py:88-98); SURVEY.md K13 + K14.
//
// What it replaces (profiles/r4_headline_trace.txt, one headline step): the split-K slab flush
// (prep SUM / COLSUM tasks), two fp32 library GEMMs of the layer-0 gather route (dW_x0 = Eᵀ·dEW,
// dE = dEW·W_x0ᵀ), the sum-of-squares pass of the global norm, the Adam pass and, at the next
// step's start, the prep pass that rebuilt W_hᵀ / W_xᵀ / the padded head matrices and the
// E·W_x0 + b0 gather table from the fp32 masters -- six launches that each streamed
// parameter-sized buffers, now two.
//
// One kernel, a table of tasks, a persistent grid (two workgroups per CU) that takes the
// tasks' tiles in list order from an atomic queue head:
//
//   FINALIZE (phase 0)
//     SUM      dst[r, c] = sum_s src[s][r, c]            split-K slabs, fixed order s = 0..S-1
//     COLSUM   dst[c] = sum_r src[r, c]                  bias partials of the BPTT kernels
//     SUMSQ    (no output)                               a gradient finished elsewhere (head)
//     MM       dst[r, c] = sum_k A(r, k) B(k, c)         fp32; strided operands (dW_x0, dE)
//   Every output of a task flagged `norm` is squared into the workgroup's partial; the last
//   workgroup to finish (ticket) adds the partials in workgroup order plus one extra term (the
//   TF per-token embedding norm slot) and writes the global sum of squares.  Single-GPU steps
//   hand it to the ADAM launch, so the update needs no norm pass of its own.
//
//   ADAM (phase 1)
//     (the global sum of squares comes from FINALIZE, or -- data parallelism: the gradients
//     changed in the all-reduce -- from a sum-of-squares launch in front of this one)
//     ADAM     64 x 64 tiles of a parameter region: TF-Adam (clipped by the global norm), the
//              fp32 master, both slots, the bf16 mirror of the flat buffer (whose slices ARE the
//              W_h / W_x / softmax_w operand layouts) and up to two more bf16 layouts of the tile
//              (copies with another row stride, or transposes staged through LDS)
//     MM+bias  the E·W_x0 + b0 gather table, once E, W_x0 and b0 are updated
//
// Dependencies inside a launch (dE / dW_x0 on the dEW slab sum; the table on the updated E, W_x0
// and b0) are counters: producer tiles write their outputs with write-through (sc1) stores,
// drain them (vmcnt(0)), pass a workgroup barrier and add 1 to the counter; the consumer's one
// polling lane waits (bounded spin) until the counter reaches the producer tile count, then
// issues one agent-scope acquire before the workgroup's plain loads (MI355X_MICROARCH.md
// "Consumer, always"), once per workgroup and dependency.
// Producers precede their consumers in the tile list and tiles are taken in list order by
// running workgroups, so every producer of a waiting tile is done or in progress.  The last
// workgroup of the launch resets the counters, the queue head and the ticket.  Every output element is written by one thread with a fixed
// summation order: results are bitwise reproducible.
#include "common.h"
#include "kernels.h"
#include "debug_env.h"

namespace dcr {

constexpr int kTailThreads = 256;

__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 ld4(const float* p, bool sc1) {
  if (sc1) return make_float4(ld_sc1(p), ld_sc1(p + 1), ld_sc1(p + 2), ld_sc1(p + 3));
  return *reinterpret_cast<const float4*>(p);
}
__device__ __forceinline__ void st4(float* p, float4 v, bool sc1) {
  if (sc1) {
    st_sc1(p, v.x); st_sc1(p + 1, v.y); st_sc1(p + 2, v.z); st_sc1(p + 3, v.w);
  } else {
    *reinterpret_cast<float4*>(p) = v;
  }
}
__device__ __forceinline__ float sq4(float4 v) { return v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w; }

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float s, float lr_t,
                                      float b1, float b2, float eps) {
  g *= s;
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  p -= lr_t * m / (sqrtf(v) + eps);
}

// bounded spin of one lane until *cnt >= need; false (and the error word set) on timeout
__device__ bool tail_wait(unsigned* cnt, unsigned need, unsigned limit, unsigned* err) {
  unsigned n = 0;
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
    __builtin_amdgcn_s_sleep(2);
    if (++n > limit) {
      if (err) atomicOr(err, 0x20u);
      return false;
    }
  }
  return true;
}

// a producer tile is done: its sc1 stores drained by every wave, then one add
__device__ __forceinline__ void tail_signal(unsigned* cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- FINALIZE tiles ---------------------------------------------------------------------------

// SUM: 64 x 64 tile, 16 lanes x float4 per row, 4 rows per thread (loads of 4 slabs in flight)
__device__ float tail_sum(const TailTask& T, int local, bool sc1) {
  const int tiles_c = (T.cols + 63) / 64;
  const int r0 = (local / tiles_c) * 64, c0 = (local % tiles_c) * 64;
  const int r1 = min(r0 + 64, T.rows);
  float sq = 0.f;
  if (T.vec4) {
    const int c = c0 + 4 * (threadIdx.x & 15);
    const int rr = r0 + (threadIdx.x >> 4);
    if (c >= T.cols) return 0.f;
    float4 acc[4];
    const float* p[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = rr + 16 * i < r1 ? rr + 16 * i : r0;
      p[i] = T.a + (size_t)r * T.ar + c;
      acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    int s = 0;
    for (; s + 4 <= T.nslab; s += 4) {
      float4 v[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] = *reinterpret_cast<const float4*>(p[i] + (size_t)(s + j) * T.ak);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[i].x += v[i][j].x; acc[i].y += v[i][j].y; acc[i].z += v[i][j].z; acc[i].w += v[i][j].w;
        }
    }
    for (; s < T.nslab; ++s) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float4 v = *reinterpret_cast<const float4*>(p[i] + (size_t)s * T.ak);
        acc[i].x += v.x; acc[i].y += v.y; acc[i].z += v.z; acc[i].w += v.w;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (rr + 16 * i < r1) {
        st4(T.dst + (size_t)(rr + 16 * i) * T.dst_ld + c, acc[i], sc1);
        sq += sq4(acc[i]);
      }
    return sq;
  }
  // scalar path (odd widths): 4 rows x 4 slabs of loads in flight per batch
  const int c = c0 + (threadIdx.x & 63);
  if (c >= T.cols) return 0.f;
  for (int rb = r0 + (threadIdx.x >> 6); rb < r1; rb += 16) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const float* p[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) p[i] = T.a + (size_t)min(rb + 4 * i, r1 - 1) * T.ar + c;
    int s = 0;
    for (; s + 4 <= T.nslab; s += 4) {
      float v[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[i][j] = p[i][(size_t)(s + j) * T.ak];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] += ((v[i][0] + v[i][1]) + v[i][2]) + v[i][3];
    }
    for (; s < T.nslab; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] += p[i][(size_t)s * T.ak];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = rb + 4 * i;
      if (r >= r1) continue;
      float* d = T.dst + (size_t)r * T.dst_ld + c;
      if (sc1) st_sc1(d, acc[i]); else *d = acc[i];
      sq += acc[i] * acc[i];
    }
  }
  return sq;
}

// COLSUM: 64 columns per tile, 4 row phases combined in LDS in a fixed order
__device__ float tail_colsum(const TailTask& T, int local, float* lds) {
  const int c0 = local * 64, tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  float acc = 0.f;
  if (c0 + tx < T.cols)
    for (int r = ty; r < T.k; r += 4) acc += T.a[(size_t)r * T.ar + c0 + tx];
  lds[ty * 64 + tx] = acc;
  __syncthreads();
  float sq = 0.f;
  if (ty == 0 && c0 + tx < T.cols) {
    const float v = lds[tx] + lds[64 + tx] + lds[128 + tx] + lds[192 + tx];
    T.dst[c0 + tx] = v;
    sq = v * v;
  }
  __syncthreads();
  return sq;
}

// SUMSQ: 4096 contiguous elements per tile
__device__ float tail_sumsq(const TailTask& T, int local) {
  const long n = (long)T.rows * T.cols, base = (long)local * 4096;
  float v[4096 / kTailThreads];
#pragma unroll
  for (int j = 0; j < 4096 / kTailThreads; ++j) {  // unconditional loads, clamped
    const long i = base + threadIdx.x + (long)kTailThreads * j;
    v[j] = T.a[i < n ? i : n - 1];
  }
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < 4096 / kTailThreads; ++j)
    if (base + threadIdx.x + (long)kTailThreads * j < n) sq += v[j] * v[j];
  return sq;
}

// MM with a short reduction (K <= 128: dW_x0 = Eᵀ·dEW over the vocabulary): 64 x 64 tile on fp32
// MFMA (v_mfma_f32_16x16x4_f32), each wave a 32 x 32 quarter.  The whole reduction is staged
// through LDS at once (every load of the tile in flight together: one round trip), each operand
// loaded along whichever of its dimensions is contiguous.  Row strides 132 (A) and 80 (B) words
// put the 64 lanes of an operand read (16 rows / columns x 4 k) on 64 different banks.
constexpr int kMmShortK = 128;
constexpr int kMmAS = 132, kMmBS = 80;
constexpr int kTailLds = 64 * kMmAS + kMmShortK * kMmBS;  // floats (>= the Adam tile [64][65])
// Stage NCH 16-deep chunks of both operand tiles (64 rows / columns each) into LDS: every load
// unconditional at a clamped address (a guarded load becomes its own branch with a vmcnt(0)
// wait: one round trip per element), out-of-range elements zeroed by a select afterwards.
template <int NCH>
__device__ __forceinline__ void mm_fill(const TailTask& T, int r0, int c0, float* As, float* Bs) {
  float va[NCH * 4], vb[NCH * 4];
  const int tid = threadIdx.x;
  // element e = tid + 256 j of chunk e >> 10: (row / column, k) along the contiguous dimension
  auto ra = [&](int j, int& r, int& kk) {
    const int e = tid + kTailThreads * j, ch = e >> 10, ei = e & 1023;
    if (T.ar == 1) { r = ei & 63; kk = 16 * ch + (ei >> 6); } else { kk = 16 * ch + (ei & 15); r = ei >> 4; }
  };
  auto rb = [&](int j, int& cc, int& kb) {
    const int e = tid + kTailThreads * j, ch = e >> 10, ei = e & 1023;
    if (T.bc == 1) { cc = ei & 63; kb = 16 * ch + (ei >> 6); } else { kb = 16 * ch + (ei & 15); cc = ei >> 4; }
  };
#pragma unroll
  for (int j = 0; j < NCH * 4; ++j) {
    int r, kk, cc, kb;
    ra(j, r, kk);
    rb(j, cc, kb);
    const int gr = r0 + r, gc = c0 + cc;
    va[j] = T.a[(size_t)min(gr, T.rows - 1) * T.ar + (size_t)min(kk, T.k - 1) * T.ak];
    vb[j] = T.b[(size_t)min(kb, T.k - 1) * T.bk + (size_t)min(gc, T.cols - 1) * T.bc];
  }
#pragma unroll
  for (int j = 0; j < NCH * 4; ++j) {
    int r, kk, cc, kb;
    ra(j, r, kk);
    rb(j, cc, kb);
    As[r * kMmAS + kk] = (r0 + r < T.rows && kk < T.k) ? va[j] : 0.f;
    Bs[kb * kMmBS + cc] = (c0 + cc < T.cols && kb < T.k) ? vb[j] : 0.f;
  }
}

__device__ float tail_mm_short(const TailTask& T, int local, float* lds) {
  const int tiles_c = (T.cols + 63) / 64;
  const int r0 = (local / tiles_c) * 64, c0 = (local % tiles_c) * 64;
  const int tid = threadIdx.x;
  float* As = lds;                 // [64][kMmAS]: A(r0 + r, k)
  float* Bs = lds + 64 * kMmAS;    // [kMmShortK][kMmBS]: B(k, c0 + c)
  const int KP = (T.k + 15) & ~15;
  const int nch = KP >> 4;  // 16-deep chunks (1024 elements of each operand)
  if (nch <= 2) mm_fill<2>(T, r0, c0, As, Bs);
  else if (nch <= 4) mm_fill<4>(T, r0, c0, As, Bs);
  else mm_fill<8>(T, r0, c0, As, Bs);
  __syncthreads();
  const int lane = tid & 63, w = tid >> 6;
  const int wr = 32 * (w >> 1), wc = 32 * (w & 1);
  const int m = lane & 15, q = lane >> 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int k0 = 0; k0 < KP; k0 += 4) {
    const float a0 = As[(wr + m) * kMmAS + k0 + q], a1 = As[(wr + 16 + m) * kMmAS + k0 + q];
    const float b0 = Bs[(k0 + q) * kMmBS + wc + m], b1 = Bs[(k0 + q) * kMmBS + wc + 16 + m];
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
  }
  __syncthreads();  // (the LDS is the next tile's)
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = c0 + wc + 16 * j + m;
      if (c >= T.cols) continue;
      const float bias = T.bias ? T.bias[c] : 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = r0 + wr + 16 * i + 4 * q + t;  // D[4 q + t][m]
        if (r >= T.rows) continue;
        const float v = acc[i][j][t] + bias;
        if (T.sig >= 0) st_sc1(T.dst + (size_t)r * T.dst_ld + c, v);
        else T.dst[(size_t)r * T.dst_ld + c] = v;
        sq += v * v;
      }
    }
  return sq;
}

// MM with a long reduction (dE = dEW·W_x0ᵀ, the E·W_x0 + b0 table: few rows, long k): a tile is
// up to 80 rows (5 MFMA row blocks: every vocabulary row, so the big operand B is read once per
// column block) x 16 columns of one k-slab, on fp32 MFMA (v_mfma_f32_16x16x4_f32: fp32 operands
// and accumulation).  The 4 waves split the slab's k range in quarters and meet in LDS in a
// fixed order.  A must be k-contiguous (ak == 1: float4 loads); B k-contiguous (B4) or
// column-contiguous (one dword per k).  With nslab > 1 the task covers nslab k-slabs x the tiles
// (slab-major) and writes slab s to dst + s * off (a SUM task of the same table adds the slabs
// in order); the bias goes into slab 0.
// Lane l = (m, q): MFMA t of a 16-deep k group g takes k = g + 4 q + t (a fixed permutation of
// the reduction order: 4 consecutive k per lane, one float4); A(r0 + 16 i + m, k),
// B(k, c0 + m); D[16 i + 4 q + t][m].  Loads of the next 16-deep group are issued before the
// current group's MFMAs; every load is unconditional at a clamped k (k % 4 == 0: a lane's 4 k
// are all in range or all out), zeroed by a select.
constexpr int kMmRows = 80;  // rows per long-MM tile (5 blocks)
template <bool B4>
__device__ float tail_mm_long_t(const TailTask& T, int local, float* lds) {
  const int tiles_c = (T.cols + 15) / 16, tiles = tiles_c * ((T.rows + kMmRows - 1) / kMmRows);
  const int ns = T.nslab > 1 ? T.nslab : 1;
  const int slab = local / tiles;
  local -= slab * tiles;
  const int r0 = (local / tiles_c) * kMmRows, c0 = (local % tiles_c) * 16;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ks = ((T.k + ns - 1) / ns + 63) & ~63;  // slab length: the wave quarters are 16-aligned
  const int sb = slab * ks, se = min(T.k, sb + ks);
  const int ka = min(se, sb + w * (ks / 4)), kz = min(se, ka + ks / 4);
  const int m = lane & 15, q = lane >> 4;
  const float* Ap[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) Ap[i] = T.a + (size_t)min(r0 + 16 * i + m, T.rows - 1) * T.ar;
  const float* Bp = T.b + (size_t)min(c0 + m, T.cols - 1) * T.bc;
  f32x4 acc[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 av[2][5], bv[2];
  auto load = [&](int k0, float4 (&a)[5], float4& b) {
    const int k = k0 + 4 * q, kc = min(k, kz - 4);
    const bool in = k < kz;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const float4 v = *reinterpret_cast<const float4*>(Ap[i] + kc);
      a[i] = in ? v : z;
    }
    float4 v;
    if (B4) v = *reinterpret_cast<const float4*>(Bp + kc);
    else v = make_float4(Bp[(size_t)kc * T.bk], Bp[(size_t)(kc + 1) * T.bk],
                         Bp[(size_t)(kc + 2) * T.bk], Bp[(size_t)(kc + 3) * T.bk]);
    b = in ? v : z;
  };
  auto mma = [&](float4 (&a)[5], float4& b) {
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, b.x, acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, b.y, acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, b.z, acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, b.w, acc[i], 0, 0, 0);
    }
  };
  // 16-deep groups, the next group's loads issued before this group's MFMAs
  if (ka < kz) {
    load(ka, av[0], bv[0]);
    for (int k0 = ka; k0 < kz; k0 += 32) {
      if (k0 + 16 < kz) load(k0 + 16, av[1], bv[1]);
      mma(av[0], bv[0]);
      if (k0 + 16 >= kz) break;
      if (k0 + 32 < kz) load(k0 + 32, av[0], bv[0]);
      mma(av[1], bv[1]);
    }
  }
  // the 4 waves' partials meet in LDS ([wave][block][lane] float4), added in wave order
#pragma unroll
  for (int i = 0; i < 5; ++i)
    *reinterpret_cast<float4*>(lds + ((w * 5 + i) * 64 + lane) * 4) = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
  __syncthreads();
  float sq = 0.f;
  // thread (wv, lane) finishes blocks wv, wv + 4 (5 blocks over 4 waves)
  const int c = c0 + m;
  float* dst = T.dst + (size_t)slab * T.off;
  for (int i = w; i < 5; i += 4) {
    float4 o = *reinterpret_cast<const float4*>(lds + ((0 * 5 + i) * 64 + lane) * 4);
#pragma unroll
    for (int v = 1; v < 4; ++v) {
      const float4 p = *reinterpret_cast<const float4*>(lds + ((v * 5 + i) * 64 + lane) * 4);
      o.x += p.x; o.y += p.y; o.z += p.z; o.w += p.w;
    }
    const float ov[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int r = r0 + 16 * i + 4 * q + t;
      if (r < T.rows && c < T.cols) {
        const float val = ov[t] + ((T.bias && slab == 0) ? T.bias[c] : 0.f);
        if (T.sig >= 0) st_sc1(dst + (size_t)r * T.dst_ld + c, val);  // (a producer: write-through)
        else dst[(size_t)r * T.dst_ld + c] = val;
        sq += val * val;
      }
    }
  }
  __syncthreads();
  return sq;
}
__device__ float tail_mm_long(const TailTask& T, int local, float* lds) {
  return T.bk == 1 ? tail_mm_long_t<true>(T, local, lds) : tail_mm_long_t<false>(T, local, lds);
}

// ---- ADAM tile --------------------------------------------------------------------------------
struct AdamCtx {
  float s, lr_t, b1, b2, eps;
};

__device__ __forceinline__ void put_bf4(bf16* d, float4 v) {
  bf16x4 b;
  b[0] = f2bf(v.x); b[1] = f2bf(v.y); b[2] = f2bf(v.z); b[3] = f2bf(v.w);
  *reinterpret_cast<bf16x4*>(d) = b;
}

__device__ void tail_adam(const TailArgs& a, const TailTask& T, int local, const AdamCtx& A,
                          bool sc1_out, float (*tile)[65]) {
  // 64 x 64 tiles (float4 path) or 16 x 64 (scalar path: odd widths, e.g. softmax_w [H, 65],
  // 4 rows per thread in one batch of loads instead of 16 in four)
  const int TR = T.vec4 ? 64 : 16;
  const int tiles_c = (T.cols + 63) / 64;
  const int r0 = (local / tiles_c) * TR, c0 = (local % tiles_c) * 64;
  const bool tr = (T.o1 && T.o1_t) || (T.o2 && T.o2_t);
  // every load of the tile's rows is issued before the first store (the stores could alias the
  // next row's loads for all the compiler knows, which would serialise the rows' round trips)
  if (T.vec4) {
    const int cq = 4 * (threadIdx.x & 15), c = c0 + cq;
    float4 P[4], Gv[4], M[4], Vv[4];
    bool ok[4];
    size_t idx[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = r0 + (threadIdx.x >> 4) + 16 * i;
      ok[i] = r < T.rows && c < T.cols;
      idx[i] = (size_t)T.off + (size_t)(ok[i] ? r : r0) * T.ld + (c < T.cols ? c : c0);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      P[i] = *reinterpret_cast<const float4*>(a.p + idx[i]);
      Gv[i] = *reinterpret_cast<const float4*>(a.g + idx[i]);
      M[i] = *reinterpret_cast<const float4*>(a.m + idx[i]);
      Vv[i] = *reinterpret_cast<const float4*>(a.v + idx[i]);
    }
    // (the update is computed for every row, clamped ones included, and only the stores are
    // guarded: a guarded use lets the compiler sink each row's loads into its own branch,
    // one serialised round trip per row)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float4 p = P[i], m = M[i], v = Vv[i];
      const float4 g = Gv[i];
      adam1(p.x, g.x, m.x, v.x, A.s, A.lr_t, A.b1, A.b2, A.eps);
      adam1(p.y, g.y, m.y, v.y, A.s, A.lr_t, A.b1, A.b2, A.eps);
      adam1(p.z, g.z, m.z, v.z, A.s, A.lr_t, A.b1, A.b2, A.eps);
      adam1(p.w, g.w, m.w, v.w, A.s, A.lr_t, A.b1, A.b2, A.eps);
      P[i] = p; M[i] = m; Vv[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ri = (threadIdx.x >> 4) + 16 * i, r = r0 + ri;
      if (!ok[i]) continue;
      const float4 p = P[i], m = M[i], v = Vv[i];
      st4(a.p + idx[i], p, sc1_out);
      *reinterpret_cast<float4*>(a.m + idx[i]) = m;
      *reinterpret_cast<float4*>(a.v + idx[i]) = v;
      if (a.mirror) put_bf4(a.mirror + idx[i], p);
      if (T.o1 && !T.o1_t) put_bf4(T.o1 + (size_t)r * T.o1_ld + c, p);
      if (T.o2 && !T.o2_t) put_bf4(T.o2 + (size_t)r * T.o2_ld + c, p);
      if (tr) {
        tile[ri][cq] = p.x; tile[ri][cq + 1] = p.y; tile[ri][cq + 2] = p.z; tile[ri][cq + 3] = p.w;
      }
    }
  } else {
    // 16 rows per thread in 4 batches of 4 (loads of a batch in flight together)
    const int tx = threadIdx.x & 63, c = c0 + tx;
    if (c < T.cols) {
      for (int rb = threadIdx.x >> 6; rb < 16; rb += 16) {
        float P[4], Gv[4], M[4], Vv[4];
        size_t idx[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = r0 + rb + 4 * i;
          idx[i] = (size_t)T.off + (size_t)(r < T.rows ? r : r0) * T.ld + c;
          P[i] = a.p[idx[i]]; Gv[i] = a.g[idx[i]]; M[i] = a.m[idx[i]]; Vv[i] = a.v[idx[i]];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) adam1(P[i], Gv[i], M[i], Vv[i], A.s, A.lr_t, A.b1, A.b2, A.eps);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ri = rb + 4 * i, r = r0 + ri;
          if (r >= T.rows) continue;
          const float p = P[i], m = M[i], v = Vv[i];
          if (sc1_out) st_sc1(a.p + idx[i], p); else a.p[idx[i]] = p;
          a.m[idx[i]] = m;
          a.v[idx[i]] = v;
          if (a.mirror) a.mirror[idx[i]] = f2bf(p);
          if (T.o1 && !T.o1_t) T.o1[(size_t)r * T.o1_ld + c] = f2bf(p);
          if (T.o2 && !T.o2_t) T.o2[(size_t)r * T.o2_ld + c] = f2bf(p);
          if (tr) tile[ri][tx] = p;
        }
      }
    }
  }
  if (!tr) return;
  __syncthreads();
  // transposed layouts: destination row c holds source column c; each thread writes 4
  // consecutive destination elements (source rows rq..rq+3 of one column) when they are whole
  for (int o = 0; o < 2; ++o) {
    bf16* d = o ? T.o2 : T.o1;
    const long ld = o ? T.o2_ld : T.o1_ld;
    if (!d || !(o ? T.o2_t : T.o1_t)) continue;
    const int rq = 4 * (threadIdx.x & 15);
    for (int cc = threadIdx.x >> 4; cc < 64; cc += 16) {
      const int c = c0 + cc;
      if (c >= T.cols) continue;
      bf16* row = d + (size_t)c * ld + r0;
      if (rq >= TR) continue;
      if (r0 + rq + 3 < T.rows && (ld & 3) == 0 && (r0 & 3) == 0) {
        put_bf4(row + rq, make_float4(tile[rq][cc], tile[rq + 1][cc], tile[rq + 2][cc], tile[rq + 3][cc]));
      } else {
        for (int j = 0; j < 4; ++j)
          if (r0 + rq + j < T.rows) row[rq + j] = f2bf(tile[rq + j][cc]);
      }
    }
  }
  __syncthreads();
}

// ---- the kernel -------------------------------------------------------------------------------
__global__ void __launch_bounds__(kTailThreads, 2) tail_kernel(TailArgs a) {
  __shared__ float lds_buf[kTailLds];  // the Adam tile [64][65] / MM operand tiles
  __shared__ float red[kTailThreads / 64];
  __shared__ unsigned flag;
  float* lds = lds_buf;
  float (*tile)[65] = reinterpret_cast<float (*)[65]>(lds_buf);
  const int G = gridDim.x;
  (void)G;
  AdamCtx A{};
  if (a.phase == 1) {
    // the global sum of squares: from this step's FINALIZE launch, or (data parallelism: the
    // gradients changed in the exchange) from a sum-of-squares launch in front of this one
    const float total = ld_sc1(a.total_in);
    const float lr_t = a.lr_dev ? *a.lr_dev : a.lr_t;
    const float norm = sqrtf(total) * a.gscale;
    const float s = ((a.clip > 0.f) ? a.clip / fmaxf(norm, a.clip) : 1.f) * a.gscale;
    // (the pre-clip norm is reported for a guarded step too, as the plain adam_clip does)
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.norm_out) a.norm_out[0] = norm;
    // a step whose persistent kernels timed out: no update (weights and slots stay unchanged;
    // the host raises when it reads the word).  FINALIZE still runs (its sums are harmless).
    if (a.skip_if &&
        __hip_atomic_load(a.skip_if, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
      return;
    A = AdamCtx{s, lr_t, a.b1, a.b2, a.eps};
  }

  // Tile assignment.  Static (a.dynamic == 0; the launcher's choice when the GPU is this
  // process's alone, as for the persistent recurrence): workgroup b takes tiles b, b + G, ... in
  // order.  With every workgroup co-resident, the smallest unfinished tile's owner is working on
  // it and it waits only on smaller (finished) tiles, so every wait ends.  Dynamic (the GPU may
  // be shared, DCR_RECURRENCE=step): tiles are handed out in list order by an atomic queue head
  // (sync line kTailQueue), so a tile that waits on a dependency can only have been taken after
  // every producer tile was taken, by workgroups that are running -- every wait ends even when
  // the grid is not co-resident.  Either way the norm partial of a tile goes to part[tile]: the
  // sum runs over tiles in order whichever workgroup took them (bitwise reproducible).
  __shared__ int cur;
  int k = 0;
  unsigned acquired = 0u;  // dependencies this workgroup has acquired
  // dynamic: the first tile of every workgroup is its own when it lies before the first waiting
  // tile (one atomic word serves ~90 takes per us); the queue hands out the rest from qbase on
  const int qbase = a.dynamic ? (a.static_tiles < G ? a.static_tiles : G) : G;
  const bool queue = a.dynamic && qbase < a.ntiles;
  auto take = [&](int prev) -> int {
    if (!a.dynamic) return prev + G;
    return queue ? qbase + (int)__hip_atomic_fetch_add(a.sync + kTailLine * kTailQueue, 1u, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                 : a.ntiles;
  };
  if (threadIdx.x == 0) cur = (int)blockIdx.x < qbase ? (int)blockIdx.x : take(0);
  for (;;) {
    __syncthreads();
    const int tl = cur;
    if (tl >= a.ntiles) break;
    // the next take is issued now, its latency hidden behind this tile (thread 0 only)
    int nxt = 0;
    if (threadIdx.x == 0) nxt = take(tl);
    while (k + 1 < a.n && tl >= a.t[k + 1].tile0) ++k;
    const TailTask& T = a.t[k];
    const int local = tl - T.tile0;
    if (T.wait >= 0 && !(acquired & (1u << T.wait))) {
      // the producers' bytes: one poll, ONE agent-scope acquire (this CU's L1 invalidated),
      // then plain loads -- once per workgroup and dependency (every later load is fresh)
      if (threadIdx.x == 0) {
        flag = tail_wait(a.dep + kTailLine * T.wait, (unsigned)T.need, a.spin_limit, a.err);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();
      acquired |= 1u << T.wait;
    }
    const bool sc1_out = T.sig >= 0;
    float q = 0.f;
    switch (T.op) {
      case TAIL_SUM: q = tail_sum(T, local, sc1_out); break;
      case TAIL_COLSUM: q = tail_colsum(T, local, lds); break;
      case TAIL_SUMSQ: q = tail_sumsq(T, local); break;
      case TAIL_MM: q = T.k <= kMmShortK ? tail_mm_short(T, local, lds) : tail_mm_long(T, local, lds); break;
      case TAIL_ADAM: tail_adam(a, T, local, A, sc1_out, tile); break;
      default: break;
    }
    if (a.phase == 0 && a.total_out) {
      const float t = block_sum<kTailThreads>(T.norm ? q : 0.f, red);
      if (threadIdx.x == 0) st_sc1(a.part + tl, t);
    }
    if (T.sig >= 0) tail_signal(a.dep + kTailLine * T.sig);
    __syncthreads();  // (every thread has read cur)
    if (threadIdx.x == 0) cur = nxt;
  }

  // end of the launch: ticket; the last workgroup adds the tile partials in tile order and
  // resets the counters for the next launch.  Two levels: 8 group tickets (workgroups b with
  // b % 8 == g), then the groups' last arrivals on the top ticket; every word on its own line
  // (512 atomics to one line cost ~6 us).  Static assignment: only the workgroups that had a
  // tile (b < ntiles) take part; dynamic: all of them.
  const int nw = a.dynamic ? G : (a.ntiles < G ? a.ntiles : G);
  if ((int)blockIdx.x >= nw) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int grp = blockIdx.x & 7;
    const int members = (nw - 1 - grp) / 8 + 1;  // workgroups b < nw with b % 8 == grp
    const int groups = nw < 8 ? nw : 8;
    const unsigned k2 = __hip_atomic_fetch_add(a.sync + kTailLine * (kTailGroup0 + grp), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool last = false;
    if (k2 == (unsigned)members - 1) {
      const unsigned k3 = __hip_atomic_fetch_add(a.sync + kTailLine * kTailTop, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = k3 == (unsigned)groups - 1;
    }
    flag = last ? 1u : 0u;
  }
  __syncthreads();
  if (!flag) return;
  if (a.phase == 0 && a.total_out) {
    float s = 0.f;
    for (int i = threadIdx.x; i < a.ntiles; i += kTailThreads) s += ld_sc1(a.part + i);
    const float total = block_sum<kTailThreads>(s, red);
    if (threadIdx.x == 0) st_sc1(a.total_out, a.extra ? total + ld_sc1(a.extra) : total);
  }
  if (threadIdx.x < kTailMaxDeps)
    __hip_atomic_store(a.dep + kTailLine * threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < kTailGroup0 + 8)
    __hip_atomic_store(a.sync + kTailLine * threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int tail_tiles(const TailTask& t) {
  switch (t.op) {
    case TAIL_SUM: return ((t.rows + 63) / 64) * ((t.cols + 63) / 64);
    case TAIL_ADAM: return ((t.rows + (t.vec4 ? 63 : 15)) / (t.vec4 ? 64 : 16)) * ((t.cols + 63) / 64);
    case TAIL_COLSUM: return (t.cols + 63) / 64;
    case TAIL_SUMSQ: return (int)(((long)t.rows * t.cols + 4095) / 4096);
    case TAIL_MM:
      return t.k <= kMmShortK ? ((t.rows + 63) / 64) * ((t.cols + 63) / 64)
                              : (t.nslab > 1 ? t.nslab : 1) * ((t.rows + kMmRows - 1) / kMmRows) * ((t.cols + 15) / 16);
  }
  return 0;
}

// the persistent grid: every workgroup co-resident (grid barrier, dependency waits)
int tail_grid(int cus) {
  static int occ = -1;  // (the kernel's occupancy never changes: queried once per process)
  if (occ < 0) {
    int o = 0;
    occ = hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, (const void*)tail_kernel, kTailThreads, 0) ==
                  hipSuccess ? o : 0;
  }
  const int o = occ;
  if (o < 1) return 0;
  const int want = debug_int("tail_per", 2);  // workgroups per CU (speed only)
  const int per = o < want ? o : want;
  const int g = per * cus < kTailMaxGrid ? per * cus : kTailMaxGrid;
  return g;
}

int launch_tail(TailArgs& a, int cus, hipStream_t s) {
  int tiles = 0;
  for (int i = 0; i < a.n; ++i) {
    a.t[i].tile0 = tiles;
    tiles += tail_tiles(a.t[i]);
  }
  a.ntiles = tiles;
  // tiles before the first waiting task's may be assigned statically (see the tile loop)
  a.static_tiles = tiles;
  for (int i = 0; i < a.n; ++i)
    if (a.t[i].wait >= 0) {
      a.static_tiles = a.t[i].tile0;
      break;
    }
  if (tiles > kTailMaxTiles) return -4;
  const int grid = tail_grid(cus);
  if (grid <= 0) return -1;
  hipLaunchKernelGGL(tail_kernel, dim3(grid), dim3(kTailThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace dcr
