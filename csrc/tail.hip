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
// One kernel, a table of tasks, a persistent grid (a few workgroups per CU, all co-resident:
// the launcher checks the occupancy) that walks the tasks' tiles in list order:
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
//     [norm]   without a total from FINALIZE (data parallelism: the gradients changed in the
//              all-reduce): sum of squares of g[0, n_norm) (+ the slot), one grid barrier
//     ADAM     64 x 64 tiles of a parameter region: TF-Adam (clipped by the global norm), the
//              fp32 master, both slots, the bf16 mirror of the flat buffer (whose slices ARE the
//              W_h / W_x / softmax_w operand layouts) and up to two more bf16 layouts of the tile
//              (copies with another row stride, or transposes staged through LDS)
//     MM+bias  the E·W_x0 + b0 gather table, once E, W_x0 and b0 are updated
//
// Dependencies inside a launch (dE / dW_x0 on the dEW slab sum; the table on the updated E, W_x0
// and b0) are counters: producer tiles write their outputs with write-through (sc1) stores,
// drain them (vmcnt(0)), pass a workgroup barrier and add 1 to the counter; the consumer's one
// polling lane waits (bounded spin) until the counter reaches the producer tile count and every
// load of the produced bytes is an sc1 load (MI355X_MICROARCH.md "Valid forms", first row).
// Producers precede their consumers in the tile list and every workgroup walks its tiles in
// list order, so no wait can block a producer.  The last workgroup of the launch resets the
// counters and the ticket.  Every output element is written by one thread with a fixed
// summation order: results are bitwise reproducible.
#include "common.h"
#include "kernels.h"

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
  const int c = c0 + (threadIdx.x & 63);
  if (c >= T.cols) return 0.f;
  for (int r = r0 + (threadIdx.x >> 6); r < r1; r += 4) {
    float a = 0.f;
    const float* p = T.a + (size_t)r * T.ar + c;
    for (int s = 0; s < T.nslab; ++s) a += p[(size_t)s * T.ak];
    float* d = T.dst + (size_t)r * T.dst_ld + c;
    if (sc1) st_sc1(d, a); else *d = a;
    sq += a * a;
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
  float sq = 0.f;
  for (long i = base + threadIdx.x; i < n && i < base + 4096; i += kTailThreads) {
    const float v = T.a[i];
    sq += v * v;
  }
  return sq;
}

// MM with a short reduction (K <= 128: dW_x0 = Eᵀ·dEW over the vocabulary): 64 x 64 tile on
// the vector ALU, 4 rows x 4 columns per thread
__device__ float tail_mm_short(const TailTask& T, int local, bool sc1_in) {
  const int tiles_c = (T.cols + 63) / 64;
  const int r0 = (local / tiles_c) * 64, c0 = (local % tiles_c) * 64;
  const int c = c0 + 4 * (threadIdx.x & 15);
  const int rr = r0 + (threadIdx.x >> 4);
  float acc[4][4] = {};
  if (c < T.cols) {
    for (int k = 0; k < T.k; ++k) {
      float b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float* bp = T.b + (size_t)k * T.bk + (size_t)min(c + j, T.cols - 1) * T.bc;
        b[j] = sc1_in ? ld_sc1(bp) : *bp;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float* ap = T.a + (size_t)min(rr + 16 * i, T.rows - 1) * T.ar + (size_t)k * T.ak;
        const float a = sc1_in ? ld_sc1(ap) : *ap;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] += a * b[j];
      }
    }
  }
  float sq = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = rr + 16 * i;
    if (r >= T.rows || c >= T.cols) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (c + j >= T.cols) continue;
      const float v = acc[i][j] + (T.bias ? (sc1_in ? ld_sc1(T.bias + c + j) : T.bias[c + j]) : 0.f);
      T.dst[(size_t)r * T.dst_ld + c + j] = v;
      sq += v * v;
    }
  }
  return sq;
}

// MM with a long reduction (dE = dEW·W_x0ᵀ, the E·W_x0 + b0 table): one 16 x 16 tile on fp32
// MFMA (v_mfma_f32_16x16x4_f32: fp32 operands and accumulation), the 4 waves splitting K in
// quarters and meeting in LDS in a fixed order.  Lane l: A(r0 + (l & 15), k + (l >> 4)),
// B(k + (l >> 4), c0 + (l & 15)); D[4 (l >> 4) + i][l & 15].
__device__ float tail_mm_long(const TailTask& T, int local, bool sc1_in, float* lds) {
  const int tiles_c = (T.cols + 15) / 16;
  const int r0 = (local / tiles_c) * 16, c0 = (local % tiles_c) * 16;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kq = (((T.k + 3) / 4) + 15) & ~15;
  const int ka = w * kq, kz = min(T.k, ka + kq);
  const int ar = min(r0 + (lane & 15), T.rows - 1), bc = min(c0 + (lane & 15), T.cols - 1);
  const float* Ap = T.a + (size_t)ar * T.ar;
  const float* Bp = T.b + (size_t)bc * T.bc;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = ka; k0 < kz; k0 += 64) {
    float av[16], bv[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int k = k0 + 4 * j + (lane >> 4);
      const bool ok = k < kz;
      const float* ap = Ap + (size_t)(ok ? k : 0) * T.ak;
      const float* bp = Bp + (size_t)(ok ? k : 0) * T.bk;
      av[j] = ok ? (sc1_in ? ld_sc1(ap) : *ap) : 0.f;
      bv[j] = ok ? (sc1_in ? ld_sc1(bp) : *bp) : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], bv[j], acc, 0, 0, 0);
  }
  *reinterpret_cast<float4*>(lds + (w * 64 + lane) * 4) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  __syncthreads();
  float sq = 0.f;
  if (w == 0) {
    const int c = c0 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float o = lds[lane * 4 + i] + lds[(64 + lane) * 4 + i] + lds[(128 + lane) * 4 + i] +
                      lds[(192 + lane) * 4 + i];
      const int r = r0 + 4 * (lane >> 4) + i;
      if (r < T.rows && c < T.cols) {
        const float v = o + (T.bias ? (sc1_in ? ld_sc1(T.bias + c) : T.bias[c]) : 0.f);
        T.dst[(size_t)r * T.dst_ld + c] = v;
        sq += v * v;
      }
    }
  }
  __syncthreads();
  return sq;
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
  const int tiles_c = (T.cols + 63) / 64;
  const int r0 = (local / tiles_c) * 64, c0 = (local % tiles_c) * 64;
  const bool tr = (T.o1 && T.o1_t) || (T.o2 && T.o2_t);
  if (T.vec4) {
    const int cq = 4 * (threadIdx.x & 15), c = c0 + cq;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ri = (threadIdx.x >> 4) + 16 * i, r = r0 + ri;
      if (r < T.rows && c < T.cols) {
        const size_t idx = (size_t)T.off + (size_t)r * T.ld + c;
        float4 p = *reinterpret_cast<const float4*>(a.p + idx);
        const float4 g = *reinterpret_cast<const float4*>(a.g + idx);
        float4 m = *reinterpret_cast<const float4*>(a.m + idx);
        float4 v = *reinterpret_cast<const float4*>(a.v + idx);
        adam1(p.x, g.x, m.x, v.x, A.s, A.lr_t, A.b1, A.b2, A.eps);
        adam1(p.y, g.y, m.y, v.y, A.s, A.lr_t, A.b1, A.b2, A.eps);
        adam1(p.z, g.z, m.z, v.z, A.s, A.lr_t, A.b1, A.b2, A.eps);
        adam1(p.w, g.w, m.w, v.w, A.s, A.lr_t, A.b1, A.b2, A.eps);
        st4(a.p + idx, p, sc1_out);
        *reinterpret_cast<float4*>(a.m + idx) = m;
        *reinterpret_cast<float4*>(a.v + idx) = v;
        if (a.mirror) put_bf4(a.mirror + idx, p);
        if (T.o1 && !T.o1_t) put_bf4(T.o1 + (size_t)r * T.o1_ld + c, p);
        if (T.o2 && !T.o2_t) put_bf4(T.o2 + (size_t)r * T.o2_ld + c, p);
        if (tr) {
          tile[ri][cq] = p.x; tile[ri][cq + 1] = p.y; tile[ri][cq + 2] = p.z; tile[ri][cq + 3] = p.w;
        }
      }
    }
  } else {
    const int tx = threadIdx.x & 63, c = c0 + tx;
    for (int ri = threadIdx.x >> 6; ri < 64; ri += 4) {
      const int r = r0 + ri;
      if (r >= T.rows || c >= T.cols) continue;
      const size_t idx = (size_t)T.off + (size_t)r * T.ld + c;
      float p = a.p[idx], m = a.m[idx], v = a.v[idx];
      adam1(p, a.g[idx], m, v, A.s, A.lr_t, A.b1, A.b2, A.eps);
      if (sc1_out) st_sc1(a.p + idx, p); else a.p[idx] = p;
      a.m[idx] = m;
      a.v[idx] = v;
      if (a.mirror) a.mirror[idx] = f2bf(p);
      if (T.o1 && !T.o1_t) T.o1[(size_t)r * T.o1_ld + c] = f2bf(p);
      if (T.o2 && !T.o2_t) T.o2[(size_t)r * T.o2_ld + c] = f2bf(p);
      if (tr) tile[ri][tx] = p;
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
__global__ void __launch_bounds__(kTailThreads) tail_kernel(TailArgs a) {
  __shared__ float tile[64][65];
  __shared__ float red[kTailThreads / 64];
  __shared__ unsigned flag;
  float* lds = &tile[0][0];
  const int G = gridDim.x;
  // a step whose persistent kernels timed out: no update (weights and slots stay unchanged; the
  // host raises when it reads the word).  FINALIZE still runs (its sums are harmless).
  if (a.phase == 1 && a.skip_if &&
      __hip_atomic_load(a.skip_if, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
    return;
  AdamCtx A{};
  if (a.phase == 1) {
    float total;
    if (a.total_in) {
      total = ld_sc1(a.total_in);
    } else {
      // global sum of squares of g[0, n_norm) + the slot: per-workgroup partials, one barrier
      float acc = 0.f;
      const long nv = a.n_norm / 4;
      for (long i = blockIdx.x * (long)kTailThreads + threadIdx.x; i < nv; i += (long)G * kTailThreads)
        acc += sq4(reinterpret_cast<const float4*>(a.g)[i]);
      if (blockIdx.x == 0)
        for (long i = nv * 4 + threadIdx.x; i < a.n_norm; i += kTailThreads) acc += a.g[i] * a.g[i];
      const float t = block_sum<kTailThreads>(acc, red);
      if (threadIdx.x == 0) {
        st_sc1(a.part + blockIdx.x, t);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // grid barrier (all workgroups co-resident): arrive, wait for the last arrival
        const unsigned k = __hip_atomic_fetch_add(a.sync + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        (void)k;
        flag = tail_wait(a.sync + 2, (unsigned)G, a.spin_limit, a.err) ? 1u : 0u;
      }
      __syncthreads();
      float s = 0.f;
      for (int i = threadIdx.x; i < G; i += kTailThreads) s += ld_sc1(a.part + i);
      total = block_sum<kTailThreads>(s, red);
      if (a.extra) total += ld_sc1(a.extra);
    }
    const float lr_t = a.lr_dev ? *a.lr_dev : a.lr_t;
    const float norm = sqrtf(total) * a.gscale;
    const float s = ((a.clip > 0.f) ? a.clip / fmaxf(norm, a.clip) : 1.f) * a.gscale;
    if (blockIdx.x == 0 && threadIdx.x == 0 && a.norm_out) a.norm_out[0] = norm;
    A = AdamCtx{s, lr_t, a.b1, a.b2, a.eps};
  }

  float sq = 0.f;  // FINALIZE: this workgroup's share of the norm
  int k = 0;
  for (int tl = blockIdx.x; tl < a.ntiles; tl += G) {
    while (k + 1 < a.n && tl >= a.t[k + 1].tile0) ++k;
    const TailTask& T = a.t[k];
    const int local = tl - T.tile0;
    if (T.wait >= 0) {
      // (uniform per task: every tile of a waiting task waits once; the counter only grows)
      if (threadIdx.x == 0) flag = tail_wait(a.dep + T.wait, (unsigned)T.need, a.spin_limit, a.err);
      __syncthreads();
    }
    const bool sc1_in = T.wait >= 0, sc1_out = T.sig >= 0;
    float q = 0.f;
    switch (T.op) {
      case TAIL_SUM: q = tail_sum(T, local, sc1_out); break;
      case TAIL_COLSUM: q = tail_colsum(T, local, lds); break;
      case TAIL_SUMSQ: q = tail_sumsq(T, local); break;
      case TAIL_MM: q = T.k <= 128 ? tail_mm_short(T, local, sc1_in) : tail_mm_long(T, local, sc1_in, lds); break;
      case TAIL_ADAM: tail_adam(a, T, local, A, sc1_out, tile); break;
      default: break;
    }
    if (T.norm) sq += q;
    if (T.sig >= 0) tail_signal(a.dep + T.sig);
  }

  // end of the launch: ticket; the last workgroup adds the norm partials in workgroup order and
  // resets the counters for the next launch
  if (a.phase == 0) {
    const float t = block_sum<kTailThreads>(sq, red);
    if (threadIdx.x == 0) st_sc1(a.part + blockIdx.x, t);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned k2 = __hip_atomic_fetch_add(a.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = k2 == (unsigned)G - 1;
  }
  __syncthreads();
  if (!flag) return;
  if (a.phase == 0 && a.total_out) {
    float s = 0.f;
    for (int i = threadIdx.x; i < G; i += kTailThreads) s += ld_sc1(a.part + i);
    const float total = block_sum<kTailThreads>(s, red);
    if (threadIdx.x == 0) st_sc1(a.total_out, a.extra ? total + ld_sc1(a.extra) : total);
  }
  if (threadIdx.x < kTailMaxDeps)
    __hip_atomic_store(a.dep + threadIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x == 0) {
    __hip_atomic_store(a.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(a.sync + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

int tail_tiles(const TailTask& t) {
  switch (t.op) {
    case TAIL_SUM:
    case TAIL_ADAM: return ((t.rows + 63) / 64) * ((t.cols + 63) / 64);
    case TAIL_COLSUM: return (t.cols + 63) / 64;
    case TAIL_SUMSQ: return (int)(((long)t.rows * t.cols + 4095) / 4096);
    case TAIL_MM:
      return t.k <= 128 ? ((t.rows + 63) / 64) * ((t.cols + 63) / 64)
                        : ((t.rows + 15) / 16) * ((t.cols + 15) / 16);
  }
  return 0;
}

// the persistent grid: every workgroup co-resident (grid barrier, dependency waits)
int tail_grid(int cus) {
  int o = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, (const void*)tail_kernel, kTailThreads, 0) != hipSuccess || o < 1)
    return 0;
  const int per = o < 2 ? o : 2;
  return per * cus < kTailMaxGrid ? per * cus : kTailMaxGrid;
}

int launch_tail(TailArgs& a, int cus, hipStream_t s) {
  int tiles = 0;
  for (int i = 0; i < a.n; ++i) {
    a.t[i].tile0 = tiles;
    tiles += tail_tiles(a.t[i]);
  }
  a.ntiles = tiles;
  const int grid = tail_grid(cus);
  if (grid <= 0) return -1;
  hipLaunchKernelGGL(tail_kernel, dim3(grid), dim3(kTailThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace dcr
