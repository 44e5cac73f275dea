// Persistent, weights-resident GRU recurrence (forward and BPTT) for gfx950 -- the "GRU 3-gate
// fused-GEMM path" of BASELINE.json's 3-layer GRU-1024 config.
//
// Reference semantics: TF 1.8 GRUCell as wired by model.py:15-25 (cell_fn = GRUCell):
//   [r, u] = sigmoid([x, h_{t-1}]·W_g + b_g)                 (gates/gates kernel+bias)
//   c~     = tanh([x, r ⊙ h_{t-1}]·W_c + b_c)                (candidate/candidate kernel+bias)
//   h_t    = u ⊙ h_{t-1} + (1 - u) ⊙ c~
// The reset gate multiplies h BEFORE the candidate matmul, so every step has two dependent
// all-units exchanges: r⊙h_{t-1} after phase A and h_t after phase B.  The per-step kernels
// (rnn_step.hip, CELL_GRU_A/B) paid two launches per step and re-read W_h from L2 each time;
// here one launch runs the whole sequence of one layer, with the recurrent weight slices
// resident in VGPRs as MFMA A fragments and the two exchanges done in-kernel with the same
// placement-independent hand-off as the LSTM (persist_common.h, Guideline 16 row 1).
//
// Work split (swapped-operand mfma_f32_16x16x32_bf16, as lstm_persist.hip): workgroup (ubk, bg)
// owns UB*16 hidden units x 16 batch rows; its 4 waves split K in quarters and keep
//   fwd: W_gᵀ rows (r and u gates of its units, K = H) and W_cᵀ rows (K = H)
//   bwd: W_c rows (d(r⊙h) = dZc·W_cᵀ, K = H) and W_g rows (dh = dZg·W_gᵀ, K = 2H)
// NT > 1 batch tiles per workgroup (batch group = NT*16 rows) reuse the resident weights for
// NT x the MFMA work per hand-off: the recurrence is hand-off-latency bound (MFMA mostly idle),
// so a larger batch runs at nearly the same tick time instead of falling off the persistent path
// (B = 256 at H = 1024 needs NT = 2 to stay within one 256-workgroup co-resident grid).
// Wave w < UB*NT runs the cell epilogue of unit block w % UB, batch tile w / UB, with h_{t-1} /
// the dh carry in registers.
// Counters: two sets per launch (phase A and phase B), one per (batch group, step, K quarter).
// Any batch: a ragged batch is padded to whole 16·NT-row groups (rows >= B read zero through the
// buffer range checks, write only the fragment-tiled hand-off rings -- sized for the padded
// batch -- and never the row-major buffers), so the reference default B = 50 (train.py:46)
// stays on the persistent kernels.
#include "common.h"
#include "kernels.h"
#include "debug_env.h"
#include "persist_common.h"
#include <stdlib.h>

namespace dcr {

// rows of the padded batch: whole groups of NT 16-row tiles
__host__ __device__ __forceinline__ int gru_rows(int B, int nt) {
  return (B + 16 * nt - 1) / (16 * nt) * (16 * nt);
}

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
template <int KS, int UB, int NT>
__global__ void __launch_bounds__(256, 1) gru_fwd_persist_kernel(GruPersistArgs a) {
  // single-buffered partials: every write of partA (partB) is separated from the previous
  // epilogue read by the phase-B (next phase-A) barrier, which the epilogue wave joins last
  __shared__ __attribute__((aligned(16))) float partA[4][NT][UB][64][8];
  __shared__ __attribute__((aligned(16))) float partB[4][NT][UB][64][4];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int Bp = gru_rows(B, NT);  // ring rows (padded batch)
  const int nwg_u = H / (16 * UB);
  int ubk, bg;
  if (!map_block_grid(blockIdx.x, gridDim.x, nwg_u, Bp / (16 * NT), ubk, bg)) return;  // padding
  const int ub0 = ubk * 16 * UB, b0 = bg * 16 * NT;
  const int kq = 8 * (lane >> 4);
  const int kbase = w * (KS * 32);
  const size_t cset = (size_t)(Bp / (16 * NT)) * (T + 1) * 4;
  unsigned* cntH = a.cnt + (size_t)bg * (T + 1) * 4;         // slot t: h_t published
  unsigned* cntR = a.cnt + cset + (size_t)bg * (T + 1) * 4;  // slot t: r⊙h_{t-1} published
  const unsigned target = (unsigned)(H / (64 * UB));  // workgroups per K-quarter shard
  __shared__ unsigned wg_cnt[2];  // LDS last-arriver counters (phase A / phase B)
  __shared__ int loc_s;
  if (threadIdx.x < 2) wg_cnt[threadIdx.x] = 0;
  // XCD-resident hand-offs (persist_common.h): exchange word in slot 0 of the h set (no counter
  // there); local flags (value = published slot + 1 for r⊙h, slot for h) from dword 4 of each set
  unsigned long long* const xw = reinterpret_cast<unsigned long long*>(cntH + 2);
  const bool tryloc = a.xcdloc && T >= 16 && nwg_u <= 64;
  if (tryloc && threadIdx.x == 0) xcd_publish(xw);
  unsigned* const flH = cntH + 4;
  unsigned* const flR = cntR + 4;
  bool dead = false;

  bf16x8 wg[UB][2][KS], wc[UB][KS];
#pragma unroll
  for (int ui = 0; ui < UB; ++ui)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int row = ub0 + ui * 16 + (lane & 15);
#pragma unroll
      for (int g = 0; g < 2; ++g)
        wg[ui][g][s] = ld8(a.WgT + (size_t)(g * H + row) * H + kbase + s * 32 + kq);
      wc[ui][s] = ld8(a.WcT + (size_t)row * H + kbase + s * 32 + kq);
    }
  if (threadIdx.x == 0) {
    loc_s = tryloc ? xcd_decide(xw, (unsigned)nwg_u, a.spin_limit, a.err, 14u) : 0;
    if (loc_s && ubk == 0) cntH[1] = 1u;  // (diagnostics: the column ran XCD-local)
  }
  __syncthreads();
  const bool loc = __builtin_amdgcn_readfirstlane(loc_s) != 0;

  // MFMA operands: batch tile n's row-major offset (rows b0 + 16n + lane%16) / ring tile
  const unsigned hoff = (unsigned)(((size_t)(b0 + (lane & 15)) * H + kbase + kq) * sizeof(bf16));
  const unsigned tile_off = (unsigned)(16 * H * sizeof(bf16));  // + n * tile_off
  // epilogue role: unit block w % UB of batch tile w / UB
  const bool epi = w < UB * NT;
  const int eu = epi ? w % UB : 0, en = epi ? w / UB : 0;
  const int b = b0 + 16 * en + (lane & 15);
  const bool live = b < B;  // padded rows: zero inputs, ring stores only
  const int u0 = ub0 + eu * 16 + 4 * (lane >> 4);
  const size_t bh = (size_t)b * H + u0;
  const int G3 = 3 * H;
  float hp[4] = {0.f, 0.f, 0.f, 0.f};
  if (epi && live) ld4f(a.h32 + bh, hp);  // h_0, fp32
  // input bias added here when the dense zx was written without it (one [T·B, 3H] fp32 pass
  // less behind the input GEMM)
  float bx[3][4] = {};
  if (epi && a.bias_x) {
#pragma unroll
    for (int g = 0; g < 3; ++g) ld4f(a.bias_x + (size_t)g * H + u0, bx[g]);
  }

  for (int t = 0; t < T; ++t) {
    float zx[3][4] = {};
    if (epi && live) {
      const float* zrow = a.ids ? a.zx + (size_t)a.ids[(size_t)t * B + b] * a.zx_ld
                                : a.zx + ((size_t)t * B + b) * a.zx_ld;
#pragma unroll
      for (int g = 0; g < 3; ++g) ld4f(zrow + (size_t)g * H + u0, zx[g]);
    }
    // ---- phase A: [r, u] from h_{t-1}
    if (t > 0) {
      if (loc) {
        if (w == kPollerThread / 64 && !dead)
          dead = !poll_flags1(flH, nwg_u, (unsigned)t, a.spin_limit, a.err, 5u);
      } else if (threadIdx.x == kPollerThread && !dead) {
        dead = !poll_shards4(cntH + (size_t)t * 4, target, a.spin_limit, a.err, 5u);
      }
      __syncthreads();
    }
    {
      const bool fr = a.ring0 && t > 0;  // slot 0 (initial state) is row-major
      const __amdgpu_buffer_rsrc_t src =
          fr ? make_rsrc(a.ring0 + (size_t)(t & 1) * Bp * H, sizeof(bf16) * (size_t)Bp * H)
             : make_rsrc(a.hbuf + (size_t)t * B * H, sizeof(bf16) * (size_t)B * H);
      bf16x8 hf[NT][KS];
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int s = 0; s < KS; ++s)
          hf[n][s] = ld8_sc1(src, fr ? frag_load_off(bg * NT + n, w * KS + s, H, lane)
                                     : hoff + n * tile_off + s * 64);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int ui = 0; ui < UB; ++ui) {
          f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
          for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int g = 0; g < 2; ++g) acc[g] = mfma16(wg[ui][g][s], hf[n][s], acc[g]);
          float4* dst = reinterpret_cast<float4*>(&partA[w][n][ui][lane][0]);
          dst[0] = make_float4(acc[0][0], acc[0][1], acc[0][2], acc[0][3]);
          dst[1] = make_float4(acc[1][0], acc[1][1], acc[1][2], acc[1][3]);
        }
    }
    __syncthreads();
    float uu[4];
    if (epi) {
      float rr[4];
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const float4 s0 = reinterpret_cast<const float4*>(&partA[0][en][eu][lane][0])[g];
        const float4 s1 = reinterpret_cast<const float4*>(&partA[1][en][eu][lane][0])[g];
        const float4 s2 = reinterpret_cast<const float4*>(&partA[2][en][eu][lane][0])[g];
        const float4 s3 = reinterpret_cast<const float4*>(&partA[3][en][eu][lane][0])[g];
        float* o = g == 0 ? rr : uu;
        o[0] = sigmoidf_(s0.x + s1.x + s2.x + s3.x + (zx[g][0] + bx[g][0]));
        o[1] = sigmoidf_(s0.y + s1.y + s2.y + s3.y + (zx[g][1] + bx[g][1]));
        o[2] = sigmoidf_(s0.z + s1.z + s2.z + s3.z + (zx[g][2] + bx[g][2]));
        o[3] = sigmoidf_(s0.w + s1.w + s2.w + s3.w + (zx[g][3] + bx[g][3]));
      }
      const float rh0 = rr[0] * hp[0], rh1 = rr[1] * hp[1], rh2 = rr[2] * hp[2], rh3 = rr[3] * hp[3];
      if (a.ring1)
        st4bf_ho(loc, a.ring1 + (size_t)(t & 1) * Bp * H + frag_index(b, u0, H), rh0, rh1, rh2, rh3);
      else
        st4bf_ho(loc, a.rh + (size_t)t * B * H + bh, rh0, rh1, rh2, rh3);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) {
        if (loc)
          wg_arrive_flag(&wg_cnt[0], UB * NT, flR + ubk, (unsigned)t + 1u);
        else
          wg_arrive(&wg_cnt[0], UB * NT, cntR + (size_t)t * 4 + (u0 / (H / 4)));
      }
      if (live) {
        if (a.ring1) st4bf(a.rh + (size_t)t * B * H + bh, rh0, rh1, rh2, rh3);
        bf16* gp = a.gates + ((size_t)t * B + b) * G3 + u0;
        st4bf(gp, rr[0], rr[1], rr[2], rr[3]);
        st4bf(gp + H, uu[0], uu[1], uu[2], uu[3]);
      }
    }
    // ---- phase B: c~ from r⊙h_{t-1}
    if (loc) {
      if (w == kPollerThread / 64 && !dead)
        dead = !poll_flags1(flR, nwg_u, (unsigned)t + 1u, a.spin_limit, a.err, 6u);
    } else if (threadIdx.x == kPollerThread && !dead) {
      dead = !poll_shards4(cntR + (size_t)t * 4, target, a.spin_limit, a.err, 6u);
    }
    __syncthreads();
    {
      const __amdgpu_buffer_rsrc_t src =
          a.ring1 ? make_rsrc(a.ring1 + (size_t)(t & 1) * Bp * H, sizeof(bf16) * (size_t)Bp * H)
                  : make_rsrc(a.rh + (size_t)t * B * H, sizeof(bf16) * (size_t)B * H);
      bf16x8 rf[NT][KS];
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int s = 0; s < KS; ++s)
          rf[n][s] = ld8_sc1(src, a.ring1 ? frag_load_off(bg * NT + n, w * KS + s, H, lane)
                                          : hoff + n * tile_off + s * 64);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int ui = 0; ui < UB; ++ui) {
          f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KS; ++s) acc = mfma16(wc[ui][s], rf[n][s], acc);
          *reinterpret_cast<float4*>(&partB[w][n][ui][lane][0]) =
              make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
    }
    __syncthreads();
    if (epi) {
      const float4 s0 = *reinterpret_cast<const float4*>(&partB[0][en][eu][lane][0]);
      const float4 s1 = *reinterpret_cast<const float4*>(&partB[1][en][eu][lane][0]);
      const float4 s2 = *reinterpret_cast<const float4*>(&partB[2][en][eu][lane][0]);
      const float4 s3 = *reinterpret_cast<const float4*>(&partB[3][en][eu][lane][0]);
      float cc[4], h[4];
      cc[0] = tanhf_(s0.x + s1.x + s2.x + s3.x + (zx[2][0] + bx[2][0]));
      cc[1] = tanhf_(s0.y + s1.y + s2.y + s3.y + (zx[2][1] + bx[2][1]));
      cc[2] = tanhf_(s0.z + s1.z + s2.z + s3.z + (zx[2][2] + bx[2][2]));
      cc[3] = tanhf_(s0.w + s1.w + s2.w + s3.w + (zx[2][3] + bx[2][3]));
#pragma unroll
      for (int r = 0; r < 4; ++r) h[r] = uu[r] * hp[r] + (1.f - uu[r]) * cc[r];
      const size_t o = (size_t)(t + 1) * B * H + bh;
      if (a.ring0)
        st4bf_ho(loc, a.ring0 + (size_t)((t + 1) & 1) * Bp * H + frag_index(b, u0, H), h[0], h[1],
                 h[2], h[3]);
      else
        st4bf_ho(loc, a.hbuf + o, h[0], h[1], h[2], h[3]);
      if (t + 1 < T) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
          if (loc)
            wg_arrive_flag(&wg_cnt[1], UB * NT, flH + ubk, (unsigned)t + 1u);
          else
            wg_arrive(&wg_cnt[1], UB * NT, cntH + (size_t)(t + 1) * 4 + (u0 / (H / 4)));
        }
      }
      if (live) {
        if (a.ring0) st4bf(a.hbuf + o, h[0], h[1], h[2], h[3]);
        *reinterpret_cast<float4*>(a.h32 + o) = make_float4(h[0], h[1], h[2], h[3]);
        st4bf(a.gates + ((size_t)t * B + b) * G3 + 2 * H + u0, cc[0], cc[1], cc[2], cc[3]);
        if (t == T - 1 && a.hlast32)
          *reinterpret_cast<float4*>(a.hlast32 + bh) = make_float4(h[0], h[1], h[2], h[3]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) hp[r] = h[r];
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward (BPTT); same recurrences as rnn_step.hip's CELL_GRU_A / CELL_GRU_B steps:
//   phase A (step t):   d(r⊙h) = dZc_t · W_cᵀ;  dZr_t, dZu_t;  P = dh'_t·u + d(r⊙h)·r
//   phase B (t -> t-1): dh'_{t-1} = dtop_{t-1} + P + dZg_t · W_gᵀ;  dZc_{t-1}
// dh' and P never leave the epilogue lane's registers.
// ------------------------------------------------------------------------------------------
template <int KA, int UB, int NT>
__global__ void __launch_bounds__(256, 1) gru_bwd_persist_kernel(GruPersistArgs a) {
  constexpr int KB = 2 * KA;  // phase B reduces over K = 2H
  __shared__ __attribute__((aligned(16))) float partA[4][NT][UB][64][4];
  __shared__ __attribute__((aligned(16))) float partB[4][NT][UB][64][4];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int Bp = gru_rows(B, NT);  // ring rows (padded batch)
  const int nwg_u = H / (16 * UB);
  int ubk, bg;
  if (!map_block_grid(blockIdx.x, gridDim.x, nwg_u, Bp / (16 * NT), ubk, bg)) return;  // padding
  const int ub0 = ubk * 16 * UB, b0 = bg * 16 * NT;
  const int kq = 8 * (lane >> 4);
  const int kA = w * (KA * 32), kB = w * (KB * 32);
  const size_t cset = (size_t)(Bp / (16 * NT)) * (T + 1) * 4;
  unsigned* cntC = a.cnt + (size_t)bg * (T + 1) * 4;         // slot t: dZc_t published
  unsigned* cntG = a.cnt + cset + (size_t)bg * (T + 1) * 4;  // slot t: dZg_t published
  const unsigned target = (unsigned)(H / (64 * UB));  // workgroups per K-quarter shard
  __shared__ unsigned wg_cnt[2];  // LDS last-arriver counters (phase A / phase B)
  __shared__ int loc_s;
  if (threadIdx.x < 2) wg_cnt[threadIdx.x] = 0;
  // XCD-resident hand-offs: exchange word in slot 0 of the dZg set (no counter there); local flag
  // value = T - (published slot), monotonic over the reverse sweep
  unsigned long long* const xw = reinterpret_cast<unsigned long long*>(cntG + 2);
  const bool tryloc = a.xcdloc && T >= 16 && nwg_u <= 64;
  if (tryloc && threadIdx.x == 0) xcd_publish(xw);
  unsigned* const flC = cntC + 4;
  unsigned* const flG = cntG + 4;
  const int G3 = 3 * H;
  bool dead = false;

  bf16x8 wc[UB][KA], wg[UB][KB];
#pragma unroll
  for (int ui = 0; ui < UB; ++ui) {
    const int row = ub0 + ui * 16 + (lane & 15);
#pragma unroll
    for (int s = 0; s < KA; ++s) wc[ui][s] = ld8(a.Wc + (size_t)row * H + kA + s * 32 + kq);
#pragma unroll
    for (int s = 0; s < KB; ++s) wg[ui][s] = ld8(a.Wg + (size_t)row * 2 * H + kB + s * 32 + kq);
  }
  if (threadIdx.x == 0) {
    loc_s = tryloc ? xcd_decide(xw, (unsigned)nwg_u, a.spin_limit, a.err, 15u) : 0;
    if (loc_s && ubk == 0) cntG[1] = 1u;  // (diagnostics: the column ran XCD-local)
  }
  __syncthreads();
  const bool loc = __builtin_amdgcn_readfirstlane(loc_s) != 0;

  // epilogue role: unit block w % UB of batch tile w / UB
  const bool epi = w < UB * NT;
  const int eu = epi ? w % UB : 0, en = epi ? w / UB : 0;
  const int b = b0 + 16 * en + (lane & 15);
  const bool live = b < B;  // padded rows: zero inputs, ring stores only
  const int u0 = ub0 + eu * 16 + 4 * (lane >> 4);
  const size_t bh = (size_t)b * H + u0;
  // MFMA operands (row-major dZ path): batch tile n at + n * tile_off
  const int bm = b0 + (lane & 15);
  const unsigned offA = (unsigned)(((size_t)bm * G3 + 2 * H + kA + kq) * sizeof(bf16));
  const unsigned offB = (unsigned)(((size_t)bm * G3 + kB + kq) * sizeof(bf16));
  const unsigned tile_off = (unsigned)(16 * G3 * sizeof(bf16));
  float dhp[4] = {0.f, 0.f, 0.f, 0.f};
  // bias-gradient sums of this lane's row over all steps, of the bf16-rounded dZ values exactly
  // as the weight GEMMs see them (padded rows add zero); reduced over the tile's rows at the end
  float dbr[4] = {0.f, 0.f, 0.f, 0.f}, dbu[4] = {0.f, 0.f, 0.f, 0.f}, dbc[4] = {0.f, 0.f, 0.f, 0.f};

  // dZc_{T-1} from the top gradient alone
  if (epi) {
    float uu[4] = {0.f, 0.f, 0.f, 0.f}, cc[4] = {0.f, 0.f, 0.f, 0.f};
    if (live) {
      ld4f(a.dtop + (size_t)(T - 1) * B * H + bh, dhp);
      const bf16* gp = a.gates + ((size_t)(T - 1) * B + b) * G3 + u0;
      ld4bf(gp + H, uu);
      ld4bf(gp + 2 * H, cc);
    }
    float z0[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      z0[r] = dhp[r] * (1.f - uu[r]) * (1.f - cc[r] * cc[r]);
      dbc[r] += (float)f2bf(z0[r]);
    }
    bf16* const zrow = a.dz + ((size_t)(T - 1) * B + b) * G3 + 2 * H + u0;
    if (a.ring0)
      st4bf_ho(loc, a.ring0 + (size_t)((T - 1) & 1) * Bp * H + frag_index(b, u0, H), z0[0], z0[1],
               z0[2], z0[3]);
    else
      st4bf_ho(loc, zrow, z0[0], z0[1], z0[2], z0[3]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) {
      if (loc)
        wg_arrive_flag(&wg_cnt[1], UB * NT, flC + ubk, 1u);  // slot T-1
      else
        wg_arrive(&wg_cnt[1], UB * NT, cntC + (size_t)(T - 1) * 4 + (u0 / (H / 4)));
    }
    if (a.ring0 && live) st4bf(zrow, z0[0], z0[1], z0[2], z0[3]);
  }

  for (int t = T - 1; t >= 0; --t) {
    // recurrence-independent epilogue operands, issued before the waits
    float rr[4] = {}, uu[4] = {}, cc[4] = {}, hp[4] = {}, dt[4] = {}, up[4] = {}, cp[4] = {};
    if (epi && live) {
      const bf16* gp = a.gates + ((size_t)t * B + b) * G3 + u0;
      ld4bf(gp, rr); ld4bf(gp + H, uu); ld4bf(gp + 2 * H, cc);
      ld4f(a.h32 + (size_t)t * B * H + bh, hp);
      if (t > 0) {
        ld4f(a.dtop + (size_t)(t - 1) * B * H + bh, dt);
        const bf16* gq = a.gates + ((size_t)(t - 1) * B + b) * G3 + u0;
        ld4bf(gq + H, up); ld4bf(gq + 2 * H, cp);
      }
    }
    const __amdgpu_buffer_rsrc_t zsrc =
        make_rsrc(a.dz + (size_t)t * B * G3, sizeof(bf16) * (size_t)B * G3);
    // ---- phase A: d(r⊙h_{t-1}) = dZc_t · W_cᵀ
    if (loc) {
      if (w == kPollerThread / 64 && !dead)
        dead = !poll_flags1(flC, nwg_u, (unsigned)(T - t), a.spin_limit, a.err, 7u);
    } else if (threadIdx.x == kPollerThread && !dead) {
      dead = !poll_shards4(cntC + (size_t)t * 4, target, a.spin_limit, a.err, 7u);
    }
    __syncthreads();
    {
      bf16x8 zf[NT][KA];
      if (a.ring0) {
        const __amdgpu_buffer_rsrc_t rc =
            make_rsrc(a.ring0 + (size_t)(t & 1) * Bp * H, sizeof(bf16) * (size_t)Bp * H);
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int s = 0; s < KA; ++s)
            zf[n][s] = ld8_sc1(rc, frag_load_off(bg * NT + n, w * KA + s, H, lane));
      } else {
#pragma unroll
        for (int n = 0; n < NT; ++n)
#pragma unroll
          for (int s = 0; s < KA; ++s) zf[n][s] = ld8_sc1(zsrc, offA + n * tile_off + s * 64);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int ui = 0; ui < UB; ++ui) {
          f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KA; ++s) acc = mfma16(wc[ui][s], zf[n][s], acc);
          *reinterpret_cast<float4*>(&partA[w][n][ui][lane][0]) =
              make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
    }
    __syncthreads();
    float P[4];
    if (epi) {
      const float4 s0 = *reinterpret_cast<const float4*>(&partA[0][en][eu][lane][0]);
      const float4 s1 = *reinterpret_cast<const float4*>(&partA[1][en][eu][lane][0]);
      const float4 s2 = *reinterpret_cast<const float4*>(&partA[2][en][eu][lane][0]);
      const float4 s3 = *reinterpret_cast<const float4*>(&partA[3][en][eu][lane][0]);
      const float drh[4] = {s0.x + s1.x + s2.x + s3.x, s0.y + s1.y + s2.y + s3.y,
                            s0.z + s1.z + s2.z + s3.z, s0.w + s1.w + s2.w + s3.w};
      float dzr[4], dzu[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float du = dhp[r] * (hp[r] - cc[r]);
        dzu[r] = du * uu[r] * (1.f - uu[r]);
        dzr[r] = drh[r] * hp[r] * rr[r] * (1.f - rr[r]);
        P[r] = dhp[r] * uu[r] + drh[r] * rr[r];
      }
      bf16* dz = a.dz + ((size_t)t * B + b) * G3 + u0;
      if (a.ring1) {
        bf16* gr = a.ring1 + (size_t)(t & 1) * Bp * 2 * H;
        st4bf_ho(loc, gr + frag_index(b, u0, 2 * H), dzr[0], dzr[1], dzr[2], dzr[3]);
        st4bf_ho(loc, gr + frag_index(b, H + u0, 2 * H), dzu[0], dzu[1], dzu[2], dzu[3]);
      } else {
        st4bf_ho(loc, dz, dzr[0], dzr[1], dzr[2], dzr[3]);
        st4bf_ho(loc, dz + H, dzu[0], dzu[1], dzu[2], dzu[3]);
      }
      if (t > 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) {
          if (loc)
            wg_arrive_flag(&wg_cnt[0], UB * NT, flG + ubk, (unsigned)(T - t));
          else
            wg_arrive(&wg_cnt[0], UB * NT, cntG + (size_t)t * 4 + (u0 / (H / 4)));
        }
      }
      if (a.ring1 && live) {
        st4bf(dz, dzr[0], dzr[1], dzr[2], dzr[3]);
        st4bf(dz + H, dzu[0], dzu[1], dzu[2], dzu[3]);
      }
      // (after the arrival: off the hand-off's critical path -- in front of the ring stores
      // this accumulation cost ~0.45 us per step and layer)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dbr[r] += (float)f2bf(dzr[r]);
        dbu[r] += (float)f2bf(dzu[r]);
      }
    }
    if (t == 0) break;  // dh'_{-1} (the initial state's gradient) is not needed
    // ---- phase B: dh'_{t-1} = dtop_{t-1} + P + dZg_t · W_gᵀ
    if (loc) {
      if (w == kPollerThread / 64 && !dead)
        dead = !poll_flags1(flG, nwg_u, (unsigned)(T - t), a.spin_limit, a.err, 8u);
    } else if (threadIdx.x == kPollerThread && !dead) {
      dead = !poll_shards4(cntG + (size_t)t * 4, target, a.spin_limit, a.err, 8u);
    }
    __syncthreads();
    {
      // one batch tile at a time: KB = 2 KA payload fragments per tile is the register limit
      const __amdgpu_buffer_rsrc_t rg =
          a.ring1 ? make_rsrc(a.ring1 + (size_t)(t & 1) * Bp * 2 * H, sizeof(bf16) * (size_t)Bp * 2 * H)
                  : zsrc;
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        bf16x8 zf[KB];
#pragma unroll
        for (int s = 0; s < KB; ++s)
          zf[s] = ld8_sc1(rg, a.ring1 ? frag_load_off(bg * NT + n, w * KB + s, 2 * H, lane)
                                      : offB + n * tile_off + s * 64);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int ui = 0; ui < UB; ++ui) {
          f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KB; ++s) acc = mfma16(wg[ui][s], zf[s], acc);
          *reinterpret_cast<float4*>(&partB[w][n][ui][lane][0]) =
              make_float4(acc[0], acc[1], acc[2], acc[3]);
        }
      }
    }
    __syncthreads();
    if (epi) {
      const float4 s0 = *reinterpret_cast<const float4*>(&partB[0][en][eu][lane][0]);
      const float4 s1 = *reinterpret_cast<const float4*>(&partB[1][en][eu][lane][0]);
      const float4 s2 = *reinterpret_cast<const float4*>(&partB[2][en][eu][lane][0]);
      const float4 s3 = *reinterpret_cast<const float4*>(&partB[3][en][eu][lane][0]);
      dhp[0] = dt[0] + P[0] + s0.x + s1.x + s2.x + s3.x;
      dhp[1] = dt[1] + P[1] + s0.y + s1.y + s2.y + s3.y;
      dhp[2] = dt[2] + P[2] + s0.z + s1.z + s2.z + s3.z;
      dhp[3] = dt[3] + P[3] + s0.w + s1.w + s2.w + s3.w;
      float dzc[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) dzc[r] = dhp[r] * (1.f - up[r]) * (1.f - cp[r] * cp[r]);
      bf16* const crow = a.dz + ((size_t)(t - 1) * B + b) * G3 + 2 * H + u0;
      if (a.ring0)
        st4bf_ho(loc, a.ring0 + (size_t)((t - 1) & 1) * Bp * H + frag_index(b, u0, H), dzc[0],
                 dzc[1], dzc[2], dzc[3]);
      else
        st4bf_ho(loc, crow, dzc[0], dzc[1], dzc[2], dzc[3]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) {
        if (loc)
          wg_arrive_flag(&wg_cnt[1], UB * NT, flC + ubk, (unsigned)(T - t + 1));  // slot t-1
        else
          wg_arrive(&wg_cnt[1], UB * NT, cntC + (size_t)(t - 1) * 4 + (u0 / (H / 4)));
      }
      if (a.ring0 && live) st4bf(crow, dzc[0], dzc[1], dzc[2], dzc[3]);
#pragma unroll
      for (int r = 0; r < 4; ++r) dbc[r] += (float)f2bf(dzc[r]);  // (after the arrival)
    }
  }
  // bias-gradient partial of this lane group's 4 units over the tile's 16 rows (lane bits 0-3)
  if (epi && a.db_part) {
    float v[12];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = dbr[r]; v[4 + r] = dbu[r]; v[8 + r] = dbc[r];
    }
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      v[i] += __shfl_xor(v[i], 1, 64);
      v[i] += __shfl_xor(v[i], 2, 64);
      v[i] += __shfl_xor(v[i], 4, 64);
      v[i] += __shfl_xor(v[i], 8, 64);
    }
    const int tile0 = b0 + 16 * en;
    if ((lane & 15) == 0 && tile0 < B) {
      float* dst = a.db_part + (size_t)(tile0 / 16) * G3 + u0;
#pragma unroll
      for (int g = 0; g < 3; ++g)
        *reinterpret_cast<float4*>(dst + g * H) = make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]);
    }
  }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
template <int K, int U, int N>
static const void* gru_fn(int bwd) {
  return bwd ? (const void*)gru_bwd_persist_kernel<K, U, N>
             : (const void*)gru_fwd_persist_kernel<K, U, N>;
}

static const void* gru_pick(int bwd, int H, int ub, int nt) {
  const int ks = H / 128;
#define GP(K, U, N) \
  if (ks == K && ub == U && nt == N) return gru_fn<K, U, N>(bwd);
  GP(1, 1, 1) GP(2, 1, 1) GP(3, 1, 1) GP(4, 1, 1) GP(6, 1, 1) GP(8, 1, 1)
  GP(1, 2, 1) GP(2, 2, 1) GP(3, 2, 1) GP(4, 2, 1) GP(6, 2, 1) GP(8, 2, 1)
  // NT > 1 (batch tiles sharing the resident weights): the power-of-two widths
  GP(2, 2, 2) GP(4, 2, 2) GP(8, 2, 2)
  GP(2, 1, 4) GP(4, 1, 4) GP(8, 1, 4)
#undef GP
  return nullptr;
}

static int gru_grid(int H, int B, int ub, int nt) {
  return (H / (16 * ub)) * (gru_rows(B, nt) / (16 * nt));
}

// Launch plan: the first (NT, UB) -- fewest batch tiles per workgroup, then the larger unit block
// (32 before 16 units) -- whose forward AND backward grids are co-resident with the GPU to
// themselves.  Returns UB | NT << 4; 0 = not supported (per-step kernels instead).
// DCR_DEBUG=gru_ub=1 forces 16-unit blocks, gru_nt=N forces N batch tiles per workgroup.
int gru_persist_ub(int H, int B, int cus) {
  if (H % 128 != 0 || H < 128 || H > 1024 || B < 1 || cus <= 0) return 0;
  const int first = debug_int("gru_ub", 2) == 1 ? 1 : 2;
  const int force_nt = debug_int("gru_nt", 0);
  for (int nt = 1; nt <= 4; nt *= 2) {
    // (a ragged batch pads to whole groups of nt tiles: prefer the smallest nt that fits)
    if (force_nt > 0 && nt != force_nt) continue;
    for (int ub = first; ub >= 1; --ub) {
      if (ub * nt > 4) continue;  // one epilogue role per wave
      bool ok = true;
      for (int bwd = 0; bwd < 2 && ok; ++bwd) {
        const void* fn = gru_pick(bwd, H, ub, nt);
        int occ = 0;
        ok = fn && hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 256, 0) == hipSuccess &&
             gru_grid(H, B, ub, nt) <= occ * cus;
      }
      if (ok) return ub | nt << 4;
    }
  }
  return 0;
}

// a ragged batch's padded rows exist only in the fragment-tiled rings: the row-major hand-off
// path (no rings) needs whole 16-row tiles
static bool B_ragged_needs_rings(const GruPersistArgs& a) {
  return a.B % 16 != 0 && (!a.ring0 || !a.ring1);
}
// padded rows of the batch under the launch plan (ring sizing)
int gru_persist_rows(int H, int B, int cus) {
  const int plan = gru_persist_ub(H, B, cus);
  return plan ? gru_rows(B, plan >> 4) : 0;
}

int launch_gru_persist(int bwd, const GruPersistArgs& a, int cus, hipStream_t s) {
  const int plan = gru_persist_ub(a.H, a.B, cus);
  if (!plan) return -2;
  const int ub = plan & 15, nt = plan >> 4;
  const void* fn = gru_pick(bwd, a.H, ub, nt);
  if (!fn) return -1;
  if (B_ragged_needs_rings(a)) return -2;
  if (!a.cnt_zeroed)
    (void)hipMemsetAsync(a.cnt, 0,
                         sizeof(unsigned) * 2 * (size_t)(gru_rows(a.B, nt) / (16 * nt)) * (a.T + 1) * 4, s);
  void* args[] = {const_cast<GruPersistArgs*>(&a)};
  // the XCD-padded grid (persist_common.h xcd_grid) when it is co-resident
  int grid = gru_grid(a.H, a.B, ub, nt), o = 0;
  const int padded = xcd_grid(a.H / (16 * ub), gru_rows(a.B, nt) / (16 * nt));
  if (padded != grid && hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, 256, 0) == hipSuccess &&
      padded <= o * cus)
    grid = padded;
  return hipLaunchKernel(fn, dim3(grid), dim3(256), args, 0, s) == hipSuccess ? 0 : -3;
}

}  // namespace dcr
