// Per-time-step recurrent cell kernels (LSTM / GRU / BasicRNN / NAS), gfx950 MFMA.
//
// Reference: the static T x L unroll of TF cells in `legacy_seq2seq.rnn_decoder`
// (model.py:61-73) -- per step and layer a ConcatV2 + MatMul + BiasAdd + ~11 pointwise kernels
// (K4/K5/K6/K7/K8 of SURVEY.md §2.3) -- and their tf.gradients BPTT (K12).
//
// Design (MI355X-first):
//  * The input projection X·W_x (+bias) of all T steps is hoisted out of the recurrence into
//    one big GEMM (or, for layer 0, a gather from the tiny E·W_x table), so a step only runs the
//    recurrent product h_{t-1}·W_h plus the cell epilogue.
//  * Swapped-operand MFMA (mfma_f32_16x16x32_bf16): A = weight rows (gate columns of W_h, k
//    contiguous), B = batch rows of h_{t-1}.  With A-tile `g` = the 16 units [ub, ub+16) of
//    gate g, each lane ends up holding ALL G gate pre-activations of the same 4 consecutive
//    units (rows 4(lane>>4)+reg) for one batch column (lane&15): the whole cell update is
//    lane-local -- no LDS round trip, no shuffles -- and the lane's 4 units are contiguous, so
//    the epilogue's loads/stores are 8-16 B vectors.
//  * State (c) and the backward carry (dc) stay fp32; MFMA operands bf16 with fp32 accumulate.
//  * Backward: dh_rec = dZ_{t+1}·W_hᵀ uses W_h in its TF layout [H, G·H] (k contiguous) as the
//    A operand; the epilogue fuses the cell's pointwise backward and emits dZ_t (bf16).
// Each workgroup owns one 16-unit x 16-batch output tile; its 4 waves split the K reduction
// (interleaved 32-wide k-steps, next step's fragments prefetched) and combine through LDS.
// The time loop runs in C++ (ops.cpp) so one op call launches all T steps of a layer without
// touching Python; the whole sequence is hipGraph-capturable.  The persistent (weights-resident)
// LSTM kernels in lstm_persist.hip replace these for the flagship config.
#include "common.h"
#include "kernels.h"
#include "debug_env.h"
#include <stdlib.h>

namespace dcr {

template <int CELL> struct CellG;
template <> struct CellG<CELL_LSTM> { static constexpr int G = 4; };
template <> struct CellG<CELL_GRU_A> { static constexpr int G = 2; };
template <> struct CellG<CELL_GRU_B> { static constexpr int G = 1; };
template <> struct CellG<CELL_RNN> { static constexpr int G = 1; };
template <> struct CellG<CELL_NAS> { static constexpr int G = 8; };

// Block-cooperative tile GEMM over NBT batch tiles:
//   acc_j[t] = sum_k A[arow_t][k] * Bm[brow_j][k]   over k in [0, K), j < NBT.
// The 4 waves take interleaved 32-wide k-steps (wave w: s = w, w+4, ...) and meet in LDS; each
// A fragment feeds NBT MFMAs, so a workgroup reads its weight slice once per NBT x 16 batch rows.
// At large H these kernels stream their weight slice from L2/MALL every step and are bound by
// loads in flight (one 256-workgroup grid, one workgroup per CU: ~23 GB/s per CU with two stages
// in flight at H = 2048), so the k loop is software-pipelined PD stages deep: PD-1 k-steps of
// fragments (~24 16-B loads per lane) are in flight while the MFMAs of the current one run.
// On return wave w < NBT holds the full sums of batch tile w; the other waves return garbage and
// must not use them.
template <int NT, int NBT>
__device__ __forceinline__ void tile_gemm(f32x4 (&acc)[NT], const bf16* __restrict__ A,
                                          const int (&arow)[NT], int lda,
                                          const bf16* __restrict__ Bm, const int (&brow)[NBT],
                                          int ldb, int K, int lane, int w,
                                          float* part /* [4][NT][NBT][64][4] */) {
  constexpr int PD = (24 / (NT + NBT)) < 2 ? 2 : ((24 / (NT + NBT)) > 8 ? 8 : 24 / (NT + NBT));
  const int kq = 8 * (lane >> 4);
  const bf16* bp[NBT];
#pragma unroll
  for (int j = 0; j < NBT; ++j) bp[j] = Bm + (size_t)brow[j] * ldb + kq;
  const bf16* ap[NT];
  f32x4 c[NT][NBT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    ap[t] = A + (size_t)arow[t] * lda + kq;
#pragma unroll
    for (int j = 0; j < NBT; ++j) c[t][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int KS = K / 32;
  const int n = w < KS ? (KS - w + 3) / 4 : 0;  // this wave's k-steps: s = w + 4 i, i < n
  bf16x8 ra[PD][NT], rb[PD][NBT];
#pragma unroll
  for (int p = 0; p < PD - 1; ++p)
    if (p < n) {
      const int s = w + 4 * p;
#pragma unroll
      for (int j = 0; j < NBT; ++j) rb[p][j] = ld8(bp[j] + s * 32);
#pragma unroll
      for (int t = 0; t < NT; ++t) ra[p][t] = ld8(ap[t] + s * 32);
    }
  for (int i0 = 0; i0 < n; i0 += PD) {
#pragma unroll
    for (int q = 0; q < PD; ++q) {
      const int i = i0 + q;
      if (i < n) {
        if (i + PD - 1 < n) {  // refill the slot freed one step ago
          const int s = w + 4 * (i + PD - 1);
          const int slot = (q + PD - 1) % PD;
#pragma unroll
          for (int j = 0; j < NBT; ++j) rb[slot][j] = ld8(bp[j] + s * 32);
#pragma unroll
          for (int t = 0; t < NT; ++t) ra[slot][t] = ld8(ap[t] + s * 32);
        }
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int j = 0; j < NBT; ++j) c[t][j] = mfma16(ra[q][t], rb[q][j], c[t][j]);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int j = 0; j < NBT; ++j)
      *reinterpret_cast<f32x4*>(part + (((size_t)(w * NT + t) * NBT + j) * 64 + lane) * 4) = c[t][j];
  __syncthreads();
  if (w < NBT) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ww = 0; ww < 4; ++ww)
        acc[t] += *reinterpret_cast<const f32x4*>(part + (((size_t)(ww * NT + t) * NBT + w) * 64 + lane) * 4);
    }
  }
}

__device__ __forceinline__ float4 ld4f(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4f(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
__device__ __forceinline__ void ld4bf(const bf16* p, float (&o)[4]) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  o[0] = (float)v[0]; o[1] = (float)v[1]; o[2] = (float)v[2]; o[3] = (float)v[3];
}
__device__ __forceinline__ void st4bf(bf16* p, float a, float b, float c, float d) {
  bf16x4 v;
  v[0] = f2bf(a); v[1] = f2bf(b); v[2] = f2bf(c); v[3] = f2bf(d);
  *reinterpret_cast<bf16x4*>(p) = v;
}
__device__ __forceinline__ void f4arr(const float4 v, float (&o)[4]) {
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}

// ------------------------------------------------------------------------------------------
// forward step
// ------------------------------------------------------------------------------------------
template <int CELL, int NBT>
__global__ void __launch_bounds__(256) fwd_step_kernel(FwdStepArgs a) {
  constexpr int G = CellG<CELL>::G;
  static_assert(G * NBT <= 16, "partials must fit in 64 KB of LDS");
  __shared__ __attribute__((aligned(16))) float part[4 * G * NBT * 64 * 4];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B;
  const int nub = H / 16;
  const int ub = (blockIdx.x % nub) * 16, bgrp = (blockIdx.x / nub) * 16 * NBT;

  f32x4 acc[G];
  int arow[G], brow[NBT];
#pragma unroll
  for (int g = 0; g < G; ++g) arow[g] = g * H + ub + (lane & 15);
#pragma unroll
  for (int j = 0; j < NBT; ++j) brow[j] = min(bgrp + 16 * j + (lane & 15), B - 1);
  if (a.WT) tile_gemm<G, NBT>(acc, a.WT, arow, H, a.hop, brow, H, H, lane, w, part);
  if (w >= NBT) return;
  const int b0 = bgrp + 16 * w;

  const int b = b0 + (lane & 15);
  if (b >= B) return;
  const int u0 = ub + 4 * (lane >> 4);
  const size_t bh = (size_t)b * H + u0;
  if (!a.WT) {  // epilogue-only step: the recurrent GEMM ran elsewhere (split-K slabs)
    const int ns = a.nsplit > 0 ? a.nsplit : 1;
#pragma unroll
    for (int g = 0; g < G; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < ns; ++sp) {
      const float* zr = a.zrec + (size_t)sp * B * a.zrec_ld + (size_t)b * a.zrec_ld + u0;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float4 v = ld4f(zr + (size_t)g * H);
        acc[g] += f32x4{v.x, v.y, v.z, v.w};
      }
    }
  }
  const float* zrow = (a.ids ? a.zx + (size_t)a.ids[b] * a.zx_ld : a.zx + (size_t)b * a.zx_ld) +
                      a.zx_off + u0;
  float zx[G][4];
#pragma unroll
  for (int g = 0; g < G; ++g) f4arr(ld4f(zrow + (size_t)g * H), zx[g]);

  if constexpr (CELL == CELL_LSTM) {
    float cp[4], hc[4], cn[4], gi[4], gj[4], gf[4], go[4];
    f4arr(ld4f(a.cprev + bh), cp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      gi[r] = sigmoidf_(acc[0][r] + zx[0][r]);
      gj[r] = tanhf_(acc[1][r] + zx[1][r]);
      gf[r] = sigmoidf_(acc[2][r] + zx[2][r] + a.forget_bias);
      go[r] = sigmoidf_(acc[3][r] + zx[3][r]);
      cn[r] = gf[r] * cp[r] + gi[r] * gj[r];
      hc[r] = go[r] * tanhf_(cn[r]);
    }
    st4f(a.cout + bh, cn[0], cn[1], cn[2], cn[3]);
    st4bf(a.hout + bh, hc[0], hc[1], hc[2], hc[3]);
    if (a.hout32) st4f(a.hout32 + bh, hc[0], hc[1], hc[2], hc[3]);
    if (a.gates) {
      bf16* gp = a.gates + (size_t)b * a.gates_ld + u0;
      st4bf(gp, gi[0], gi[1], gi[2], gi[3]);
      st4bf(gp + H, gj[0], gj[1], gj[2], gj[3]);
      st4bf(gp + 2 * H, gf[0], gf[1], gf[2], gf[3]);
      st4bf(gp + 3 * H, go[0], go[1], go[2], go[3]);
    }
  } else if constexpr (CELL == CELL_GRU_A) {
    float hp[4], rr[4], uu[4];
    f4arr(ld4f(a.hprev32 + bh), hp);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      rr[r] = sigmoidf_(acc[0][r] + zx[0][r]);
      uu[r] = sigmoidf_(acc[1][r] + zx[1][r]);
    }
    st4bf(a.rh + bh, rr[0] * hp[0], rr[1] * hp[1], rr[2] * hp[2], rr[3] * hp[3]);
    bf16* gp = a.gates + (size_t)b * a.gates_ld + u0;
    st4bf(gp, rr[0], rr[1], rr[2], rr[3]);
    st4bf(gp + H, uu[0], uu[1], uu[2], uu[3]);
  } else if constexpr (CELL == CELL_GRU_B) {
    float hp[4], uu[4], cc[4], hn[4];
    f4arr(ld4f(a.hprev32 + bh), hp);
    bf16* gp = a.gates + (size_t)b * a.gates_ld + u0;
    ld4bf(gp + H, uu);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      cc[r] = tanhf_(acc[0][r] + zx[0][r]);
      hn[r] = uu[r] * hp[r] + (1.f - uu[r]) * cc[r];
    }
    st4bf(gp + 2 * H, cc[0], cc[1], cc[2], cc[3]);
    st4bf(a.hout + bh, hn[0], hn[1], hn[2], hn[3]);
    st4f(a.hout32 + bh, hn[0], hn[1], hn[2], hn[3]);
  } else if constexpr (CELL == CELL_RNN) {
    float hn[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) hn[r] = tanhf_(acc[0][r] + zx[0][r]);
    st4bf(a.hout + bh, hn[0], hn[1], hn[2], hn[3]);
    if (a.hout32) st4f(a.hout32 + bh, hn[0], hn[1], hn[2], hn[3]);
  } else {  // NAS
    float cp[4], cn[4], mn[4];
    f4arr(ld4f(a.cprev + bh), cp);
    float* pre = a.pre + (size_t)b * a.gates_ld + u0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float p[8];
#pragma unroll
      for (int g = 0; g < 8; ++g) p[g] = (g == 3) ? zx[g][r] * acc[g][r] : zx[g][r] + acc[g][r];
      const float a0 = sigmoidf_(p[0]), a1 = reluf_(p[1]), a2 = sigmoidf_(p[2]);
      const float a3 = reluf_(p[3]), a4 = tanhf_(p[4]), a5 = sigmoidf_(p[5]);
      const float a6 = tanhf_(p[6]), a7 = sigmoidf_(p[7]);
      const float l20 = tanhf_(a0 * a1), l21 = tanhf_(a2 + a3), l22 = tanhf_(a4 * a5);
      const float l23 = sigmoidf_(a6 + a7);
      const float c0 = tanhf_(l20 + cp[r]);
      cn[r] = c0 * l21;
      mn[r] = tanhf_(cn[r] * tanhf_(l22 + l23));
#pragma unroll
      for (int g = 0; g < 8; ++g) pre[(size_t)g * H + r] = p[g];
    }
    st4f(a.aux + bh, acc[3][0], acc[3][1], acc[3][2], acc[3][3]);  // zm3 for d(zx3)
    st4f(a.cout + bh, cn[0], cn[1], cn[2], cn[3]);
    st4bf(a.hout + bh, mn[0], mn[1], mn[2], mn[3]);
    if (a.hout32) st4f(a.hout32 + bh, mn[0], mn[1], mn[2], mn[3]);
  }
}

// ------------------------------------------------------------------------------------------
// backward step:  acc[u][b] = sum_k W[u][k] * dz_next[b][k]   (K = a.K), then cell backward
// ------------------------------------------------------------------------------------------
template <int CELL, int NBT>
__global__ void __launch_bounds__(256) bwd_step_kernel(BwdStepArgs a) {
  __shared__ __attribute__((aligned(16))) float part[4 * NBT * 64 * 4];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B;
  const int nub = H / 16;
  const int ub = (blockIdx.x % nub) * 16, bgrp = (blockIdx.x / nub) * 16 * NBT;
  f32x4 acc[1] = {f32x4{0.f, 0.f, 0.f, 0.f}};
  if (a.dz_next) {
    const int arow[1] = {ub + (lane & 15)};
    int brow[NBT];
#pragma unroll
    for (int j = 0; j < NBT; ++j) brow[j] = min(bgrp + 16 * j + (lane & 15), B - 1);
    tile_gemm<1, NBT>(acc, a.W, arow, a.K, a.dz_next, brow, a.dz_ld, a.K, lane, w, part);
  }
  if (w >= NBT) return;
  const int b0 = bgrp + 16 * w;
  const int b = b0 + (lane & 15);
  if (b >= B) return;
  const int u0 = ub + 4 * (lane >> 4);
  const size_t bh = (size_t)b * H + u0;
  float dtop[4] = {0.f, 0.f, 0.f, 0.f};
  if (a.dtop) f4arr(ld4f(a.dtop + bh), dtop);

  if constexpr (CELL == CELL_LSTM) {
    if (!a.dz_next && a.partial) {  // epilogue-only step: recurrent dh (split-K slabs)
      const int ns = a.nsplit > 0 ? a.nsplit : 1;
      for (int sp = 0; sp < ns; ++sp) {
        const float4 v = ld4f(a.partial + (size_t)sp * B * H + bh);
        acc[0] += f32x4{v.x, v.y, v.z, v.w};
      }
    }
    float gi[4], gj[4], gf[4], go[4], c[4], cp[4], dc[4];
    const bf16* gp = a.gates + (size_t)b * a.gates_ld + u0;
    ld4bf(gp, gi); ld4bf(gp + H, gj); ld4bf(gp + 2 * H, gf); ld4bf(gp + 3 * H, go);
    f4arr(ld4f(a.c + bh), c);
    f4arr(ld4f(a.cprev + bh), cp);
    f4arr(ld4f(a.dc + bh), dc);
    float di[4], dj[4], df[4], dO[4], dcp[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float dh = acc[0][r] + dtop[r];
      const float th = tanhf_(c[r]);
      const float dcv = dc[r] + dh * go[r] * (1.f - th * th);
      dO[r] = dh * th * go[r] * (1.f - go[r]);
      di[r] = dcv * gj[r] * gi[r] * (1.f - gi[r]);
      dj[r] = dcv * gi[r] * (1.f - gj[r] * gj[r]);
      df[r] = dcv * cp[r] * gf[r] * (1.f - gf[r]);
      dcp[r] = dcv * gf[r];
    }
    bf16* dz = a.dz_out + (size_t)b * a.dz_out_ld + u0;
    st4bf(dz, di[0], di[1], di[2], di[3]);
    st4bf(dz + H, dj[0], dj[1], dj[2], dj[3]);
    st4bf(dz + 2 * H, df[0], df[1], df[2], df[3]);
    st4bf(dz + 3 * H, dO[0], dO[1], dO[2], dO[3]);
    st4f(a.dc + bh, dcp[0], dcp[1], dcp[2], dcp[3]);
  } else if constexpr (CELL == CELL_RNN) {
    float h[4];
    ld4bf(a.hcur + bh, h);
    bf16* dz = a.dz_out + (size_t)b * a.dz_out_ld + u0;
    float d[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) d[r] = (acc[0][r] + dtop[r]) * (1.f - h[r] * h[r]);
    st4bf(dz, d[0], d[1], d[2], d[3]);
  } else if constexpr (CELL == CELL_GRU_A) {
    // acc = d(r*h) = dZc_t . Wc_h^T ; dhp = dh'_t (fp32 buffer a.dc)
    float rr[4], uu[4], cc[4], hp[4], dhp[4];
    const bf16* gp = a.gates + (size_t)b * a.gates_ld + u0;
    ld4bf(gp, rr); ld4bf(gp + H, uu); ld4bf(gp + 2 * H, cc);
    f4arr(ld4f(a.hprev32 + bh), hp);
    f4arr(ld4f(a.dc + bh), dhp);
    float dzr[4], dzu[4], P[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float drh = acc[0][r];
      const float du = dhp[r] * (hp[r] - cc[r]);
      dzu[r] = du * uu[r] * (1.f - uu[r]);
      dzr[r] = drh * hp[r] * rr[r] * (1.f - rr[r]);
      P[r] = dhp[r] * uu[r] + drh * rr[r];
    }
    bf16* dz = a.dz_out + (size_t)b * a.dz_out_ld + u0;
    st4bf(dz, dzr[0], dzr[1], dzr[2], dzr[3]);
    st4bf(dz + H, dzu[0], dzu[1], dzu[2], dzu[3]);
    st4f(a.partial + bh, P[0], P[1], P[2], P[3]);
  } else if constexpr (CELL == CELL_GRU_B) {
    // acc = dZg_t . Wg_h^T ; produce dh'_{t-1} (into a.dc) and dZc_{t-1} (for step t-1)
    float P[4] = {0.f, 0.f, 0.f, 0.f}, uu[4], cc[4], dhp[4], dzc[4];
    if (a.partial) f4arr(ld4f(a.partial + bh), P);
    const bf16* gp = a.gates + (size_t)b * a.gates_ld + u0;  // gates of step t-1
    ld4bf(gp + H, uu); ld4bf(gp + 2 * H, cc);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dhp[r] = dtop[r] + P[r] + acc[0][r];
      dzc[r] = dhp[r] * (1.f - uu[r]) * (1.f - cc[r] * cc[r]);
    }
    st4f(a.dc + bh, dhp[0], dhp[1], dhp[2], dhp[3]);
    bf16* dz = a.dz_out + (size_t)b * a.dz_out_ld + u0;
    st4bf(dz, dzc[0], dzc[1], dzc[2], dzc[3]);
  } else {  // NAS
    const float* pre = a.pre + (size_t)b * a.gates_ld + u0;
    const float* zx3 = a.zx3 + (size_t)b * a.zx3_ld + u0;
    float cp[4], dcn[4], zm3[4], zx3v[4];
    f4arr(ld4f(a.cprev + bh), cp);
    f4arr(ld4f(a.dc + bh), dcn);
    f4arr(ld4f(a.aux + bh), zm3);
    f4arr(ld4f(zx3), zx3v);
    float dzm[8][4], dzx3[4], dcp[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float p[8];
#pragma unroll
      for (int g = 0; g < 8; ++g) p[g] = pre[(size_t)g * H + r];
      const float a0 = sigmoidf_(p[0]), a1 = reluf_(p[1]), a2 = sigmoidf_(p[2]);
      const float a3 = reluf_(p[3]), a4 = tanhf_(p[4]), a5 = sigmoidf_(p[5]);
      const float a6 = tanhf_(p[6]), a7 = sigmoidf_(p[7]);
      const float b0v = tanhf_(a0 * a1), b1 = tanhf_(a2 + a3), b2 = tanhf_(a4 * a5);
      const float b3 = sigmoidf_(a6 + a7);
      const float c0 = tanhf_(b0v + cp[r]);
      const float nc = c0 * b1;
      const float l31 = tanhf_(b2 + b3);
      const float m = tanhf_(nc * l31);
      const float dm = acc[0][r] + dtop[r];
      const float dpm = dm * (1.f - m * m);
      const float dnc = dcn[r] + dpm * l31;
      const float dl31 = dpm * nc * (1.f - l31 * l31);
      const float dc0 = dnc * b1 * (1.f - c0 * c0);
      const float db1 = dnc * c0 * (1.f - b1 * b1);
      const float dt0 = dc0 * (1.f - b0v * b0v);
      const float dt2 = dl31 * (1.f - b2 * b2);
      const float dt3 = dl31 * b3 * (1.f - b3);
      dzm[0][r] = dt0 * a1 * a0 * (1.f - a0);
      dzm[1][r] = (p[1] > 0.f) ? dt0 * a0 : 0.f;
      dzm[2][r] = db1 * a2 * (1.f - a2);
      const float dp3 = (p[3] > 0.f) ? db1 : 0.f;
      dzm[4][r] = dt2 * a5 * (1.f - a4 * a4);
      dzm[5][r] = dt2 * a4 * a5 * (1.f - a5);
      dzm[6][r] = dt3 * (1.f - a6 * a6);
      dzm[7][r] = dt3 * a7 * (1.f - a7);
      dzm[3][r] = dp3 * zx3v[r];
      dzx3[r] = dp3 * zm3[r];
      dcp[r] = dc0;
    }
    bf16* dz = a.dz_out + (size_t)b * a.dz_out_ld + u0;
#pragma unroll
    for (int g = 0; g < 8; ++g) st4bf(dz + (size_t)g * H, dzm[g][0], dzm[g][1], dzm[g][2], dzm[g][3]);
    bf16* dzx = a.dzx_out + (size_t)b * a.dz_out_ld + u0;
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      if (g == 3) st4bf(dzx + 3 * H, dzx3[0], dzx3[1], dzx3[2], dzx3[3]);
      else st4bf(dzx + (size_t)g * H, dzm[g][0], dzm[g][1], dzm[g][2], dzm[g][3]);
    }
    st4f(a.dc + bh, dcp[0], dcp[1], dcp[2], dcp[3]);
  }
}

// Batch tiles per workgroup: each workgroup reads its 16-unit weight slice once per NBT x 16
// batch rows.  Larger NBT cuts weight traffic (which dominates at large H) but shrinks the grid.
// Measured on 1x MI355X (4-layer LSTM-2048, T=512, B=64): NBT 1/2/4 -> 129/108/141 ms per
// training step; the 3-layer GRU-1024 per-step path lost 20 % at NBT=4 (128 workgroups).  So
// NBT=2 when that still leaves >= 256 workgroups (one per CU), else 1; DCR_DEBUG=step_nbt=1/2/4
// overrides.
static int step_nbt(int G, int B, int H) {
  const int f = debug_int("step_nbt", 0);
  const int forced = (f == 1 || f == 2 || f == 4) ? f : 0;
  const int nbt_tiles = (B + 15) / 16;
  for (int c : {4, 2}) {
    if (G * c > 16 || nbt_tiles < c) continue;
    if (forced) {
      if (c <= forced) return c;
      continue;
    }
    if (c == 2 && (H / 16) * ((nbt_tiles + c - 1) / c) >= 256) return c;
  }
  return 1;
}

static inline int step_blocks(int B, int H, int nbt) {
  return ((B + 16 * nbt - 1) / (16 * nbt)) * (H / 16);
}

// epilogue-only steps (no GEMM): every wave of a workgroup takes a batch tile
static int ew_nbt(int G, int B) { return (G * 4 <= 16 && B >= 64) ? 4 : (G * 2 <= 16 && B >= 32) ? 2 : 1; }

template <int CELL>
static void fwd_launch(const FwdStepArgs& a, hipStream_t s) {
  const int nbt = a.WT ? step_nbt(CellG<CELL>::G, a.B, a.H) : ew_nbt(CellG<CELL>::G, a.B);
  const int nb = step_blocks(a.B, a.H, nbt);
  if constexpr (CellG<CELL>::G * 4 <= 16) {
    if (nbt == 4) { fwd_step_kernel<CELL, 4><<<nb, 256, 0, s>>>(a); return; }
  }
  if constexpr (CellG<CELL>::G * 2 <= 16) {
    if (nbt == 2) { fwd_step_kernel<CELL, 2><<<nb, 256, 0, s>>>(a); return; }
  }
  fwd_step_kernel<CELL, 1><<<nb, 256, 0, s>>>(a);
}

template <int CELL>
static void bwd_launch(const BwdStepArgs& a, hipStream_t s) {
  const int nbt = a.dz_next ? step_nbt(1, a.B, a.H) : ew_nbt(1, a.B);
  const int nb = step_blocks(a.B, a.H, nbt);
  if (nbt == 4) bwd_step_kernel<CELL, 4><<<nb, 256, 0, s>>>(a);
  else if (nbt == 2) bwd_step_kernel<CELL, 2><<<nb, 256, 0, s>>>(a);
  else bwd_step_kernel<CELL, 1><<<nb, 256, 0, s>>>(a);
}

void launch_fwd_step(int cell, const FwdStepArgs& a, hipStream_t s) {
  switch (cell) {
    case CELL_LSTM: fwd_launch<CELL_LSTM>(a, s); break;
    case CELL_GRU_A: fwd_launch<CELL_GRU_A>(a, s); break;
    case CELL_GRU_B: fwd_launch<CELL_GRU_B>(a, s); break;
    case CELL_RNN: fwd_launch<CELL_RNN>(a, s); break;
    case CELL_NAS: fwd_launch<CELL_NAS>(a, s); break;
  }
}

void launch_bwd_step(int cell, const BwdStepArgs& a, hipStream_t s) {
  switch (cell) {
    case CELL_LSTM: bwd_launch<CELL_LSTM>(a, s); break;
    case CELL_GRU_A: bwd_launch<CELL_GRU_A>(a, s); break;
    case CELL_GRU_B: bwd_launch<CELL_GRU_B>(a, s); break;
    case CELL_RNN: bwd_launch<CELL_RNN>(a, s); break;
    case CELL_NAS: bwd_launch<CELL_NAS>(a, s); break;
  }
}

}  // namespace dcr
