// Persistent, weights-resident LSTM recurrence (forward and BPTT) for gfx950.
//
// Reference: TF's statically unrolled LSTMCell chain (model.py:61-73) and its tf.gradients
// backward: per time step and layer one cuBLAS GEMM + ~11 pointwise kernels (K4/K5/K12 of
// SURVEY.md §2.3).  The per-step kernels in rnn_step.hip already fuse GEMM + cell, but they
// re-stream W_h from L2 every step and pay a launch boundary per step; this file removes both.
//
// Decomposition.  One launch runs all T steps of one layer.  Workgroup (ubk, bg) owns UB*16
// hidden units x 16 batch rows for the whole sequence.  Its 4 waves split the GEMM's K range in
// four and keep their slice of the recurrent weights RESIDENT IN VGPRs as ready-made MFMA A
// fragments (mfma_f32_16x16x32_bf16, swapped operands: A = weight rows, B = batch rows), so a
// step streams only activations:
//   fwd: z[b][g*H+u] = sum_k h_{t-1}[b][k] * W_h[k][g*H+u]      (K = H,  A = W_hᵀ rows)
//   bwd: dh[b][u]    = sum_k dZ_{t+1}[b][k] * W_h[u][k]          (K = 4H, A = W_h rows)
// The four K-partials meet in LDS; one wave per 16-unit block runs the fused cell epilogue with
// the cell state c (fwd) / the carry dc (bwd) held in registers across all T steps.
//
// Cross-workgroup hand-off (h_t in fwd, dZ_t in bwd) follows the placement-independent form of
// cdna_hip_programming.md §6 Guideline 16 / MI355X_MICROARCH.md "Valid forms" row 1, with no
// acquire/release fences: every handed-off byte is stored `sc1` (write-through) by the single
// storing wave, which drains with `s_waitcnt vmcnt(0)` before ONE lane does an agent-scope
// atomic add on the (batch group, step) counter; ONE lane of each consumer polls that counter
// with `sc1` loads (+ s_sleep), the workgroup barrier releases the other waves, and EVERY load
// of handed-off bytes is a `buffer_load ... sc1`.  Counters are zeroed by a memset node before
// every launch; every spin is bounded and a timeout sets an error word and drains the grid.
// Residency: the host only launches when the whole grid fits (<= 2 workgroups per CU here) and
// otherwise falls back to the per-step kernels.
#include "common.h"
#include "kernels.h"
#include "persist_common.h"
#include "debug_env.h"

namespace dcr {

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
// DIAG builds record s_memtime stamps of workgroup 0 per step (never used for timing claims,
// only for the share of each phase; cdna_hip_programming.md §7 "In-kernel stamps")
#define STAMP(i)                                                                    \
  if constexpr (DIAG) {                                                             \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                        \
      a.diag[(size_t)t * 8 + (i)] = __builtin_amdgcn_s_memtime();                   \
  }
// XF: the layer's input projection x_t·W_x (+bias) is computed in-kernel from register-resident
// W_xᵀ fragments while the workgroup waits for h_{t-1} (x_t comes from the layer below, already
// complete) -- no separate GEMM, no [T,B,4H] fp32 Zx round trip through HBM.
template <int KS, int UB, bool DIAG = false, bool XF = false>
__global__ void __launch_bounds__(256, 1) lstm_fwd_persist_kernel(PersistArgs a) {
  // partials double-buffered by step parity: without a workgroup barrier before the MFMAs a
  // wave may start step t+1 while the epilogue wave still reads step t's partials
  __shared__ __attribute__((aligned(16))) float part[2][4][UB][4][64][4];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int Bp = (B + 15) / 16 * 16;  // ring rows: a ragged batch pads to whole 16-row tiles
  const int nwg_u = H / (16 * UB);
  int ubk, bg;
  map_block(blockIdx.x, nwg_u, Bp / 16, ubk, bg);
  const int ub0 = ubk * 16 * UB, b0 = bg * 16;
  const int kq = 8 * (lane >> 4);
  const int kbase = w * (KS * 32);
  unsigned* cnt = a.cnt + (size_t)bg * (T + 1) * 4;
  bool dead = false;

  // resident A fragments: rows g*H + ub + (lane&15) of W_hᵀ, this wave's K quarter
  bf16x8 wf[UB][4][KS];
#pragma unroll
  for (int ui = 0; ui < UB; ++ui)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int s = 0; s < KS; ++s)
        wf[ui][g][s] = ld8(a.W + (size_t)(g * H + ub0 + ui * 16 + (lane & 15)) * H + kbase +
                           s * 32 + kq);

  bf16x8 xw[XF ? UB : 1][4][XF ? KS : 1];
  if constexpr (XF) {
#pragma unroll
    for (int ui = 0; ui < UB; ++ui)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int s = 0; s < KS; ++s)
          xw[ui][g][s] = ld8(a.Wx + (size_t)(g * H + ub0 + ui * 16 + (lane & 15)) * H + kbase +
                             s * 32 + kq);
  }

  const int b = b0 + (lane & 15);
  const bool live = b < B;  // padded rows: zero inputs, ring stores only
  const unsigned hoff = (unsigned)(((size_t)b * H + kbase + kq) * sizeof(bf16));

  // epilogue ownership: wave ui (< UB) owns unit block ui; lane: batch b, units u0..u0+3
  const bool epi = w < UB;
  const int u0 = ub0 + (epi ? w : 0) * 16 + 4 * (lane >> 4);
  const size_t bh = (size_t)b * H + u0;
  float c[4] = {0.f, 0.f, 0.f, 0.f};
  if (epi && live) ld4f(a.cbuf + bh, c);
  float bias[4][4];
  if constexpr (XF) {
    if (epi) {
#pragma unroll
      for (int g = 0; g < 4; ++g) ld4f(a.bias + g * H + u0, bias[g]);
    }
  }

  for (int t = 0; t < T; ++t) {
    STAMP(0)
    // x-projection pre-activations of step t (independent of the recurrence: issue early)
    float zx[4][4] = {};
    f32x4 acc[UB][4];
#pragma unroll
    for (int ui = 0; ui < UB; ++ui)
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[ui][g] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (XF) {
      // input projection of step t: independent of the recurrence, runs before the wait
      const bf16* xp = a.xin + ((size_t)t * B + (live ? b : 0)) * H + kbase + kq;
      bf16x8 xf[KS];
#pragma unroll
      for (int s = 0; s < KS; ++s) xf[s] = live ? ld8(xp + s * 32) : zero8();
#pragma unroll
      for (int ui = 0; ui < UB; ++ui)
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[ui][g] = mfma16(xw[ui][g][s], xf[s], acc[ui][g]);
      if (epi) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int r = 0; r < 4; ++r) zx[g][r] = bias[g][r];
      }
    } else if (epi && live) {
      const float* zrow = a.ids ? a.zx + (size_t)a.ids[(size_t)t * B + b] * a.zx_ld
                                : a.zx + ((size_t)t * B + b) * a.zx_ld;
#pragma unroll
      for (int g = 0; g < 4; ++g) ld4f(zrow + (size_t)g * H + u0, zx[g]);
    }
    if (t > 0) {
      // ONE poller per workgroup (pollers cost chip bandwidth); the barrier releases the waves
      if (threadIdx.x == kLstmPollerThread && !dead)
        dead = !poll_counter(cnt + (size_t)t * 4, (unsigned)(H / 16), a.spin_limit, a.err, 1u);
      STAMP(1)
      __syncthreads();
    }
    STAMP(2)
    // h_{t-1} fragments (handed off by other workgroups: sc1 loads only)
    const bool fring = t > 0;  // slot 0 (initial state) is row-major
    const __amdgpu_buffer_rsrc_t hsrc =
        fring ? make_rsrc(a.hring + (size_t)(t & 1) * Bp * H, sizeof(bf16) * (size_t)Bp * H)
              : make_rsrc(a.hbuf + (size_t)t * B * H, sizeof(bf16) * (size_t)B * H);
    bf16x8 hf[KS];
#pragma unroll
    for (int s = 0; s < KS; ++s)
      hf[s] = ld8_sc1(hsrc, fring ? frag_load_off(bg, w * KS + s, H, lane) : hoff + s * 64);
    __builtin_amdgcn_sched_barrier(0);  // keep all KS hand-off loads in flight together
#pragma unroll
    for (int ui = 0; ui < UB; ++ui) {
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[ui][g] = mfma16(wf[ui][g][s], hf[s], acc[ui][g]);
      float* dst = &part[t & 1][w][ui][0][lane][0];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(dst + g * 256) =
            make_float4(acc[ui][g][0], acc[ui][g][1], acc[ui][g][2], acc[ui][g][3]);
    }
    STAMP(3)
    __syncthreads();
    STAMP(4)
    if (epi) {
      float z[4][4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float4 s0 = *reinterpret_cast<const float4*>(&part[t & 1][0][w][g][lane][0]);
        float4 s1 = *reinterpret_cast<const float4*>(&part[t & 1][1][w][g][lane][0]);
        float4 s2 = *reinterpret_cast<const float4*>(&part[t & 1][2][w][g][lane][0]);
        float4 s3 = *reinterpret_cast<const float4*>(&part[t & 1][3][w][g][lane][0]);
        z[g][0] = s0.x + s1.x + s2.x + s3.x + zx[g][0];
        z[g][1] = s0.y + s1.y + s2.y + s3.y + zx[g][1];
        z[g][2] = s0.z + s1.z + s2.z + s3.z + zx[g][2];
        z[g][3] = s0.w + s1.w + s2.w + s3.w + zx[g][3];
      }
      float gi[4], gj[4], gf[4], go[4], h[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        gi[r] = sigmoidf_(z[0][r]);
        gj[r] = tanhf_(z[1][r]);
        gf[r] = sigmoidf_(z[2][r] + a.forget_bias);
        go[r] = sigmoidf_(z[3][r]);
        c[r] = gf[r] * c[r] + gi[r] * gj[r];
        h[r] = go[r] * tanhf_(c[r]);
      }
      const size_t o = (size_t)(t + 1) * B * H + bh;
      STAMP(5)
      // handed off in fragment order (write-through); row-major copy below
      st4bf_sc1(a.hring + (size_t)((t + 1) & 1) * Bp * H + frag_index(b, u0, H), h[0], h[1], h[2],
                h[3]);
      if (t + 1 < T) {
        // each epilogue wave publishes its own 16-unit slab: drain ONLY the hand-off store
        // (the activation-cache stores below are issued after the arrival, so the wait does
        // not cover them), then one lane arrives on the counter of its K-quarter
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        STAMP(6)
        if (lane == 0)
          __hip_atomic_fetch_add(cnt + (size_t)(t + 1) * 4, 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      }
      if (!live) continue;  // (after the hand-off: padded rows exist only in the ring)
      st4bf(a.hbuf + o, h[0], h[1], h[2], h[3]);
      *reinterpret_cast<float4*>(a.cbuf + o) = make_float4(c[0], c[1], c[2], c[3]);
      if (a.gates) {
        bf16* gp = a.gates + ((size_t)t * B + b) * 4 * H + u0;
        st4bf(gp, gi[0], gi[1], gi[2], gi[3]);
        st4bf(gp + H, gj[0], gj[1], gj[2], gj[3]);
        st4bf(gp + 2 * H, gf[0], gf[1], gf[2], gf[3]);
        st4bf(gp + 3 * H, go[0], go[1], go[2], go[3]);
      }
      if (t == T - 1 && a.hlast32)
        *reinterpret_cast<float4*>(a.hlast32 + bh) = make_float4(h[0], h[1], h[2], h[3]);
      if (t == T - 1 && a.clast32)
        *reinterpret_cast<float4*>(a.clast32 + bh) = make_float4(c[0], c[1], c[2], c[3]);
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward (BPTT)
// ------------------------------------------------------------------------------------------
// EXCL: all KS payload loads of a step are forced in flight together (sched_barrier); the extra
// 4*KS live VGPRs push KS=16/UB=2 past 256 registers, i.e. one workgroup per CU, so this variant
// is only launched when nothing can run beside it (see lstm_persist_occupancy and the backend's
// exclusive mode).  Measured at H=512, B=256: 4.32 vs 5.0 us per BPTT step.
template <int KS, int UB, bool DIAG = false, bool EXCL = false>
__global__ void __launch_bounds__(256, 1) lstm_bwd_persist_kernel(PersistArgs a) {
  __shared__ __attribute__((aligned(16))) float part[2][4][UB][64][4];  // parity double buffer
  // optional fused dEW accumulator (layer-0 gather mode): [V][UB*64] fp32, dynamic
  extern __shared__ __attribute__((aligned(16))) float dew_acc[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int Bp = (B + 15) / 16 * 16;  // ring rows (padded batch)
  const int nwg_u = H / (16 * UB);
  int ubk, bg;
  map_block(blockIdx.x, nwg_u, Bp / 16, ubk, bg);
  const int ub0 = ubk * 16 * UB, b0 = bg * 16;
  const int kq = 8 * (lane >> 4);
  unsigned* cnt = a.cnt + (size_t)bg * (T + 1) * 4;
  const int G4H = 4 * H;
  bool dead = false;

  // K = 4H split by hidden-unit quarter: wave w reduces over columns g*H + [w*H/4, (w+1)*H/4)
  // of every gate g, i.e. exactly the dZ produced by the H/64 unit blocks of quarter w.
  constexpr int KSG = KS / 4;  // k-steps per gate segment
  auto kcol = [&](int s) { return (s / KSG) * H + w * (H / 4) + (s % KSG) * 32; };
  bf16x8 wf[UB][KS];
#pragma unroll
  for (int ui = 0; ui < UB; ++ui)
#pragma unroll
    for (int s = 0; s < KS; ++s)
      wf[ui][s] = ld8(a.W + (size_t)(ub0 + ui * 16 + (lane & 15)) * G4H + kcol(s) + kq);

  const int b = b0 + (lane & 15);
  const bool live = b < B;  // padded rows: zero operands and gradients, ring stores only

  const bool epi = w < UB;
  const int u0 = ub0 + (epi ? w : 0) * 16 + 4 * (lane >> 4);
  const size_t bh = (size_t)b * H + u0;
  float dc[4] = {0.f, 0.f, 0.f, 0.f};
  // fused bias-gradient accumulation: sum over this lane's batch row and all steps
  float dbacc[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r) dbacc[g][r] = 0.f;
  const bool fuse_dew = a.dew_part != nullptr;
  const int DW = UB * 64;  // dEW columns owned by this workgroup: UB blocks x 4 gates x 16 units
  // LDS row stride DW + 1: with DW (a multiple of 64 floats) every batch lane's row id*DW fell
  // on the same bank; the odd stride spreads ids over banks
  const int DWP = DW + 1;
  if (fuse_dew) {
    for (int i = threadIdx.x; i < a.V * DWP; i += 256) dew_acc[i] = 0.f;
    __syncthreads();
  }

  for (int t = T - 1; t >= 0; --t) {
    STAMP(0)
    // recurrence-independent epilogue operands, issued before the wait
    float gi[4] = {}, gj[4] = {}, gf[4] = {}, go[4] = {}, cc[4] = {}, cp[4] = {}, dtop[4] = {};
    int tok = 0;  // fused dEW row (issued with the other recurrence-independent operands)
    if (epi && live) {
      if (fuse_dew) tok = a.ids[(size_t)t * B + b];
      const bf16* gp = a.gates + ((size_t)t * B + b) * G4H + u0;
      ld4bf(gp, gi); ld4bf(gp + H, gj); ld4bf(gp + 2 * H, gf); ld4bf(gp + 3 * H, go);
      ld4f(a.cbuf + (size_t)(t + 1) * B * H + bh, cc);
      ld4f(a.cbuf + (size_t)t * B * H + bh, cp);
      ld4f(a.dtop + (size_t)t * B * H + bh, dtop);
    }
    // per-wave partial sums of the recurrent product over this wave's K quarter
    f32x4 pacc[UB];
#pragma unroll
    for (int ui = 0; ui < UB; ++ui) pacc[ui] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (t < T - 1) {
      if (threadIdx.x == kLstmPollerThread && !dead)
        dead = !poll_counter(cnt + (size_t)(t + 1) * 4, (unsigned)(H / 16), a.spin_limit, a.err, 2u);
      STAMP(1)
      __syncthreads();
      STAMP(2)
      // fragment-tiled ring: one contiguous 1 KB load per k-step
      bf16x8 df[KS];
      const __amdgpu_buffer_rsrc_t zsrc =
          make_rsrc(a.zring + (size_t)((t + 1) & 1) * Bp * G4H, sizeof(bf16) * (size_t)Bp * G4H);
#pragma unroll
      for (int s = 0; s < KS; ++s) df[s] = ld8_sc1(zsrc, frag_load_off(bg, kcol(s) >> 5, G4H, lane));
      if constexpr (EXCL) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ui = 0; ui < UB; ++ui)
#pragma unroll
        for (int s = 0; s < KS; ++s) pacc[ui] = mfma16(wf[ui][s], df[s], pacc[ui]);
#pragma unroll
      for (int ui = 0; ui < UB; ++ui)
        *reinterpret_cast<float4*>(&part[t & 1][w][ui][lane][0]) =
            make_float4(pacc[ui][0], pacc[ui][1], pacc[ui][2], pacc[ui][3]);
      STAMP(3)
      __syncthreads();
      STAMP(4)
    }
    if (epi) {
      float dh[4];
      if (t < T - 1) {
        const float4 s0 = *reinterpret_cast<const float4*>(&part[t & 1][0][w][lane][0]);
        const float4 s1 = *reinterpret_cast<const float4*>(&part[t & 1][1][w][lane][0]);
        const float4 s2 = *reinterpret_cast<const float4*>(&part[t & 1][2][w][lane][0]);
        const float4 s3 = *reinterpret_cast<const float4*>(&part[t & 1][3][w][lane][0]);
        dh[0] = s0.x + s1.x + s2.x + s3.x + dtop[0];
        dh[1] = s0.y + s1.y + s2.y + s3.y + dtop[1];
        dh[2] = s0.z + s1.z + s2.z + s3.z + dtop[2];
        dh[3] = s0.w + s1.w + s2.w + s3.w + dtop[3];
      } else {
        dh[0] = dtop[0]; dh[1] = dtop[1]; dh[2] = dtop[2]; dh[3] = dtop[3];
      }
      float di[4], dj[4], df_[4], dO[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float th = tanhf_(cc[r]);
        const float dcv = dc[r] + dh[r] * go[r] * (1.f - th * th);
        dO[r] = dh[r] * th * go[r] * (1.f - go[r]);
        di[r] = dcv * gj[r] * gi[r] * (1.f - gi[r]);
        dj[r] = dcv * gi[r] * (1.f - gj[r] * gj[r]);
        df_[r] = dcv * cp[r] * gf[r] * (1.f - gf[r]);
        dc[r] = dcv * gf[r];
      }
      STAMP(5)
      bf16* dz = a.dz + ((size_t)t * B + b) * G4H + u0;
      // handed-off copy in fragment order; row-major dz after the arrival
      bf16* const zr = a.zring + (size_t)(t & 1) * Bp * G4H;
      st4bf_sc1(zr + frag_index(b, u0, G4H), di[0], di[1], di[2], di[3]);
      st4bf_sc1(zr + frag_index(b, H + u0, G4H), dj[0], dj[1], dj[2], dj[3]);
      st4bf_sc1(zr + frag_index(b, 2 * H + u0, G4H), df_[0], df_[1], df_[2], df_[3]);
      st4bf_sc1(zr + frag_index(b, 3 * H + u0, G4H), dO[0], dO[1], dO[2], dO[3]);
      if (t > 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        STAMP(6)
        if (lane == 0)
          __hip_atomic_fetch_add(cnt + (size_t)t * 4, 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
      }
      if (!live) continue;  // (padded rows: zero gradients, nothing row-major)
      st4bf(dz, di[0], di[1], di[2], di[3]);
      st4bf(dz + H, dj[0], dj[1], dj[2], dj[3]);
      st4bf(dz + 2 * H, df_[0], df_[1], df_[2], df_[3]);
      st4bf(dz + 3 * H, dO[0], dO[1], dO[2], dO[3]);
      // off the critical path (after the arrival): accumulate the bf16-rounded dz exactly as
      // the dW GEMMs will see it
      float q[4][4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        q[0][r] = (float)f2bf(di[r]); q[1][r] = (float)f2bf(dj[r]);
        q[2][r] = (float)f2bf(df_[r]); q[3][r] = (float)f2bf(dO[r]);
      }
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) dbacc[g][r] += q[g][r];
      if (fuse_dew) {
        const int id = tok;
        float* row = dew_acc + (size_t)id * DWP + w * 64 + 4 * (lane >> 4);
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
          for (int r = 0; r < 4; ++r) atomicAdd(row + g * 16 + r, q[g][r]);
      }
    }
  }
  // bias-gradient partial of this batch group: reduce the 16 batch lanes (lane bits 0..3)
  if (epi && a.db_part) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = dbacc[g][r];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        dbacc[g][r] = v;
      }
    if ((lane & 15) == 0) {
      float* dst = a.db_part + (size_t)bg * G4H + u0;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(dst + g * H) =
            make_float4(dbacc[g][0], dbacc[g][1], dbacc[g][2], dbacc[g][3]);
    }
  }
  if (fuse_dew) {
    __syncthreads();
    // dew_part[bg][v][g*H + ub0 + ui*16 + j]
    for (int i = threadIdx.x; i < a.V * DW; i += 256) {
      const int v = i / DW, col = i % DW;
      const int ui = col / 64, g = (col % 64) / 16, j = col % 16;
      a.dew_part[((size_t)bg * a.V + v) * G4H + g * H + ub0 + ui * 16 + j] = dew_acc[v * DWP + col];
    }
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
// Kernel selection returns the exact instantiation so that launch and residency query agree.
enum : int { PF_FUSED = 1, PF_DIAG = 2, PF_EXCL = 4 };

template <int KS, int UB>
static const void* fwd_fn(int flags) {
  // (the fused-input form runs only at H <= 512, lstm_persist_xfuse_supported: KS <= 4; at
  // KS = 6 / 8 its resident W_x and W_h had spilled to scratch, so it is not instantiated)
  if (flags & PF_FUSED) {
    if constexpr (KS <= 4) return (const void*)lstm_fwd_persist_kernel<KS, UB, false, true>;
    return nullptr;
  }
  if (flags & PF_DIAG) return (const void*)lstm_fwd_persist_kernel<KS, UB, true, false>;
  return (const void*)lstm_fwd_persist_kernel<KS, UB, false, false>;
}
template <int KS, int UB>
static const void* bwd_fn(int flags) {
  const bool d = flags & PF_DIAG, e = flags & PF_EXCL;
  if (d && e) return (const void*)lstm_bwd_persist_kernel<KS, UB, true, true>;
  if (d) return (const void*)lstm_bwd_persist_kernel<KS, UB, true, false>;
  if (e) return (const void*)lstm_bwd_persist_kernel<KS, UB, false, true>;
  return (const void*)lstm_bwd_persist_kernel<KS, UB, false, false>;
}

static int ub_for(int H, int B, int cus) {
  // 32-unit workgroups (measured 3.84 vs 4.02 ms/step at B=256, H=512 against 16-unit ones:
  // half the pollers, half the backward hand-off traffic); 16-unit ones only when H/16 is odd
  (void)B; (void)cus;
  return ((H / 16) % 2 == 0) ? 2 : 1;
}

static const void* pick(int bwd, int H, int B, int flags, int cus) {
  // H > 1024: 16-unit x NT-tile workgroups (lstm_persist_nt.hip; no fused input, no fused
  // dEW, no diag stamps: the plain instantiation for every flag)
  if (H > 1024)
    return (flags & PF_FUSED) ? nullptr : lstm_persist_nt_fn(bwd, H, B, cus, flags & PF_DIAG);
  const int ub = ub_for(H, B, cus);
  if (!bwd) {
    const int ks = H / 128;
#define FWD(K, U) \
  if (ks == K && ub == U) return fwd_fn<K, U>(flags);
    FWD(1, 1) FWD(2, 1) FWD(3, 1) FWD(4, 1) FWD(6, 1) FWD(8, 1)
    FWD(1, 2) FWD(2, 2) FWD(3, 2) FWD(4, 2) FWD(6, 2) FWD(8, 2)
#undef FWD
  } else {
    const int ks = H / 32;
#define BWD(K, U) \
  if (ks == K && ub == U) return bwd_fn<K, U>(flags);
    BWD(4, 1) BWD(8, 1) BWD(12, 1) BWD(16, 1) BWD(24, 1) BWD(32, 1)
    BWD(4, 2) BWD(8, 2) BWD(12, 2) BWD(16, 2) BWD(24, 2) BWD(32, 2)
#undef BWD
  }
  return nullptr;
}

static size_t dyn_lds(int bwd, int H, int B, int V, int cus) {
  return (bwd && V > 0 && H <= 1024) ? sizeof(float) * (size_t)V * (ub_for(H, B, cus) * 64 + 1) : 0;
}

int lstm_persist_supported(int H, int B, int cus) {
  // shape support only; whether a grid can be co-resident is lstm_persist_occupancy's job
  if (H > 1024) return lstm_persist_nt_tiles(H, B, cus) > 0 ? 1 : 0;
  if (H % 128 != 0 || B < 1 || H < 128) return 0;
  return (H / 16) % ub_for(H, B, cus) == 0 ? 1 : 0;
}

int lstm_persist_grid(int H, int B, int cus) {
  if (H > 1024) return lstm_persist_nt_grid(H, B, cus);
  return (H / (16 * ub_for(H, B, cus))) * ((B + 15) / 16);
}

int lstm_persist_occupancy(int bwd, int H, int B, int V, int flags, int cus) {
  if (!lstm_persist_supported(H, B, cus)) return 0;
  const void* fn = pick(bwd, H, B, flags, cus);
  if (!fn) return 0;
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 256, dyn_lds(bwd, H, B, V, cus)) !=
      hipSuccess)
    return 0;
  return n;
}

int lstm_persist_xfuse_supported(int H, int B, int cus) {
  // the fused-input variant holds W_x and W_h in registers: the whole grid must still be
  // co-resident with the GPU to itself
  return H <= 512 && lstm_persist_grid(H, B, cus) <=
                         lstm_persist_occupancy(0, H, B, 0, PF_FUSED, cus) * cus;
}

// Every workgroup of a persistent grid spins on its neighbours, so the whole grid must be
// resident at once: refuse (rather than hang or time out) a grid the CUs cannot hold.
static int launch_persist(int bwd, const PersistArgs& a, int flags, int cus, hipStream_t s) {
  const int grid = lstm_persist_grid(a.H, a.B, cus);
  const void* fn = pick(bwd, a.H, a.B, flags, cus);
  if (!fn || (a.H > 1024 && a.dew_part)) return -1;
  const size_t lds = dyn_lds(bwd, a.H, a.B, a.dew_part ? a.V : 0, cus);
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 256, lds) != hipSuccess ||
      grid > occ * cus)
    return -2;
  if (!a.cnt_zeroed)
    (void)hipMemsetAsync(a.cnt, 0, sizeof(unsigned) * (size_t)((a.B + 15) / 16) * (a.T + 1) * 4, s);
  PersistArgs b = a;
  // H > 1024: the poller lane's wave (DCR_DEBUG=nt_poll=w; default wave 0, an epilogue wave)
  b.poller = a.H > 1024 ? 64 * (debug_int("nt_poll", 0) & 3) : 0;
  void* args[] = {&b};
  return hipLaunchKernel(fn, dim3(grid), dim3(256), args, lds, s) == hipSuccess ? 0 : -3;
}

int launch_lstm_fwd_persist(const PersistArgs& a, int cus, hipStream_t s) {
  if (!a.hring) return -1;
  const int flags = (a.Wx ? PF_FUSED : 0) | (a.diag ? PF_DIAG : 0);
  return launch_persist(0, a, flags, cus, s);
}

int launch_lstm_bwd_persist(const PersistArgs& a, int cus, hipStream_t s) {
  if (!a.zring) return -1;
  const int flags = (a.diag ? PF_DIAG : 0) | (a.excl ? PF_EXCL : 0);
  return launch_persist(1, a, flags, cus, s);
}

}  // namespace dcr
