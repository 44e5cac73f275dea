// fp32-operand recurrent cell kernels (LSTM / GRU / BasicRNN), gfx950 fp32 MFMA: the native
// `--dtype fp32` path.
//
// Reference: the fp32 TF graph of model.py:43-72 (tf.float32 zero state and variables; per step
// and layer a MatMul of [x_t, h_{t-1}] with the cell kernel + the pointwise gate math) and its
// tf.gradients BPTT (model.py:91).  The bf16 kernels (rnn_step.hip, the persistent families)
// round every MFMA operand to bf16; these keep every operand, activation cache and gradient in
// fp32, so a native fp32 run separates operand rounding from a kernel error (the oracle
// comparison is then at fp32 reassociation level, ~1e-6).
//
// Design: one launch per time step (the time loop runs in C++ below, hipGraph-capturable), the
// input projection X·W_x + b of all T steps hoisted out of the recurrence (a library fp32 GEMM
// in engine/native/fp32.py).  A step is the recurrent product on v_mfma_f32_16x16x4_f32 --
// exact fp32 products and sums (64 FLOP/clk/SIMD, 1/16 of the bf16 rate) -- with the cell's
// pointwise forward or backward in the epilogue.  Swapped operands as in rnn_step.hip: A =
// weight rows (gate column g·H + u, k contiguous), B = batch rows, so a lane ends up holding
// every gate of 4 consecutive units of one batch row (rows 4(l>>4)+r, column l&15) and the cell
// update is lane-local.  A lane loads 16 B (4 k values) per operand row and feeds them to four
// MFMAs: MFMA c takes k = k0 + 4(l>>4) + c from A and B alike, so the 16 k of a chunk are summed
// exactly once.  Workgroup = 16 units x 64 batch rows, one 16-row batch tile per wave (no
// cross-wave reduction).
#include "common.h"
#include "kernels.h"

namespace dcr {
namespace {

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// acc[t] += sum_k A[arow[t] lda + k] * Bm[brow ldb + k], k in [0, K), K % 16 == 0
template <int NT>
__device__ __forceinline__ void gemm32(f32x4 (&acc)[NT], const float* __restrict__ A,
                                       const int (&arow)[NT], int lda, const float* __restrict__ Bm,
                                       int brow, int ldb, int K, int lane) {
  const int kq = 4 * (lane >> 4);
  const float* bp = Bm + (size_t)brow * ldb + kq;
  const float* ap[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) ap[t] = A + (size_t)arow[t] * lda + kq;
  for (int k0 = 0; k0 < K; k0 += 16) {
    const float4 b = *reinterpret_cast<const float4*>(bp + k0);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const float4 a = *reinterpret_cast<const float4*>(ap[t] + k0);
      acc[t] = mfma4(a.x, b.x, acc[t]);
      acc[t] = mfma4(a.y, b.y, acc[t]);
      acc[t] = mfma4(a.z, b.z, acc[t]);
      acc[t] = mfma4(a.w, b.w, acc[t]);
    }
  }
}

struct F32Step {
  const float* W;     // A operand rows (fwd: W_hᵀ [G·H, H]; bwd: W_h in TF layout [H, K])
  const float* Bop;   // B operand rows [B, ldb] (fwd: h_{t-1} or r·h; bwd: dZ of step t+1); null: none
  int ldb, K;
  const float* zx;    // fwd: this step's input projection + bias, row stride zx_ld
  int zx_ld;
  const float* dtop;  // bwd: [B, H] gradient from above / the loss (null: zero)
  const float* hprev; // [B, H] h_{t-1} (GRU) / h_t (RNN backward)
  const float* cprev; // [B, H] c_{t-1} (LSTM)
  const float* c;     // [B, H] c_t (LSTM backward)
  float* hout;        // [B, H]
  float* cout;        // [B, H]
  float* gates;       // [B, gld] activation cache (fwd writes, bwd reads)
  int gld;
  float* rh;          // GRU: [B, H] r·h_{t-1}
  float* dz;          // bwd: this step's pre-activation gradient row base, row stride dz_ld
  int dz_ld;
  float* dc;          // LSTM: dc carry (in / out); GRU: dh_t (GRU_A reads, GRU_B writes)
  float* P;           // GRU: the partial dh_{t-1} of GRU_A (GRU_B reads; null: zero)
  int B, H;
  float fb;
};

constexpr int kTileB = 64;  // batch rows per workgroup (4 waves x 16)

template <int CELL>
struct G32;
template <> struct G32<CELL_LSTM> { static constexpr int G = 4; };
template <> struct G32<CELL_GRU_A> { static constexpr int G = 2; };
template <> struct G32<CELL_GRU_B> { static constexpr int G = 1; };
template <> struct G32<CELL_RNN> { static constexpr int G = 1; };

template <int CELL>
__global__ void __launch_bounds__(256) f32_fwd_kernel(F32Step a) {
  constexpr int G = G32<CELL>::G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int H = a.H, B = a.B, nub = H / 16;
  const int ub = (blockIdx.x % nub) * 16, b0 = (blockIdx.x / nub) * kTileB + 16 * w;
  if (b0 >= B) return;
  const int b = b0 + (lane & 15);
  f32x4 acc[G];
  int arow[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
    arow[g] = g * H + ub + (lane & 15);
  }
  if (a.Bop) gemm32<G>(acc, a.W, arow, H, a.Bop, b < B ? b : B - 1, a.ldb, a.K, lane);
  if (b >= B) return;
  const int u0 = ub + 4 * (lane >> 4);
  const float* zr = a.zx + (size_t)b * a.zx_ld + u0;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int u = u0 + r;
    const size_t bh = (size_t)b * H + u;
    if constexpr (CELL == CELL_LSTM) {
      const float gi = sigmoidf_(acc[0][r] + zr[r]);
      const float gj = tanhf_(acc[1][r] + zr[H + r]);
      const float gf = sigmoidf_(acc[2][r] + zr[2 * H + r] + a.fb);
      const float go = sigmoidf_(acc[3][r] + zr[3 * H + r]);
      const float cn = gf * a.cprev[bh] + gi * gj;
      a.cout[bh] = cn;
      a.hout[bh] = go * tanhf_(cn);
      float* gp = a.gates + (size_t)b * a.gld + u;
      gp[0] = gi; gp[H] = gj; gp[2 * H] = gf; gp[3 * H] = go;
    } else if constexpr (CELL == CELL_GRU_A) {
      const float rr = sigmoidf_(acc[0][r] + zr[r]);
      const float uu = sigmoidf_(acc[1][r] + zr[H + r]);
      a.rh[bh] = rr * a.hprev[bh];
      float* gp = a.gates + (size_t)b * a.gld + u;
      gp[0] = rr; gp[H] = uu;
    } else if constexpr (CELL == CELL_GRU_B) {  // zx: the candidate block
      float* gp = a.gates + (size_t)b * a.gld + u;
      const float cc = tanhf_(acc[0][r] + zr[r]);
      const float uu = gp[H];
      gp[2 * H] = cc;
      a.hout[bh] = uu * a.hprev[bh] + (1.f - uu) * cc;
    } else {  // BasicRNN
      a.hout[bh] = tanhf_(acc[0][r] + zr[r]);
    }
  }
}

template <int CELL>
__global__ void __launch_bounds__(256) f32_bwd_kernel(F32Step a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int H = a.H, B = a.B, nub = H / 16;
  const int ub = (blockIdx.x % nub) * 16, b0 = (blockIdx.x / nub) * kTileB + 16 * w;
  if (b0 >= B) return;
  const int b = b0 + (lane & 15);
  f32x4 acc[1] = {f32x4{0.f, 0.f, 0.f, 0.f}};
  const int arow[1] = {ub + (lane & 15)};
  if (a.Bop) gemm32<1>(acc, a.W, arow, a.K, a.Bop, b < B ? b : B - 1, a.ldb, a.K, lane);
  if (b >= B) return;
  const int u0 = ub + 4 * (lane >> 4);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int u = u0 + r;
    const size_t bh = (size_t)b * H + u;
    const float dt = a.dtop ? a.dtop[bh] : 0.f;
    float* dz = a.dz + (size_t)b * a.dz_ld + u;
    const float* gp = a.gates ? a.gates + (size_t)b * a.gld + u : nullptr;
    if constexpr (CELL == CELL_LSTM) {
      const float gi = gp[0], gj = gp[H], gf = gp[2 * H], go = gp[3 * H];
      const float dh = acc[0][r] + dt;
      const float th = tanhf_(a.c[bh]);
      const float dcv = a.dc[bh] + dh * go * (1.f - th * th);
      dz[0] = dcv * gj * gi * (1.f - gi);
      dz[H] = dcv * gi * (1.f - gj * gj);
      dz[2 * H] = dcv * a.cprev[bh] * gf * (1.f - gf);
      dz[3 * H] = dh * th * go * (1.f - go);
      a.dc[bh] = dcv * gf;
    } else if constexpr (CELL == CELL_RNN) {
      const float h = a.hprev[bh];  // h_t
      dz[0] = (acc[0][r] + dt) * (1.f - h * h);
    } else if constexpr (CELL == CELL_GRU_A) {
      // acc = d(r·h_{t-1}) = dZc_t · Wc_hᵀ; a.dc = dh_t; writes dZr, dZu of step t and the
      // partial P = dh_{t-1} - (dtop_{t-1} + dZg_t · Wg_hᵀ)
      const float rr = gp[0], uu = gp[H], cc = gp[2 * H];
      const float hp = a.hprev[bh], dh = a.dc[bh], drh = acc[0][r];
      dz[0] = drh * hp * rr * (1.f - rr);
      dz[H] = dh * (hp - cc) * uu * (1.f - uu);
      a.P[bh] = dh * uu + drh * rr;
    } else {  // GRU_B: acc = dZg_t · Wg_hᵀ; gates of step t-1: dh_{t-1}, dZc_{t-1}
      const float uu = gp[H], cc = gp[2 * H];
      const float dh = dt + (a.P ? a.P[bh] : 0.f) + acc[0][r];
      a.dc[bh] = dh;
      dz[0] = dh * (1.f - uu) * (1.f - cc * cc);
    }
  }
}

template <int CELL>
void fwd1(const F32Step& a, hipStream_t s) {
  const unsigned grid = (unsigned)((a.H / 16) * ((a.B + kTileB - 1) / kTileB));
  f32_fwd_kernel<CELL><<<grid, 256, 0, s>>>(a);
}
template <int CELL>
void bwd1(const F32Step& a, hipStream_t s) {
  const unsigned grid = (unsigned)((a.H / 16) * ((a.B + kTileB - 1) / kTileB));
  f32_bwd_kernel<CELL><<<grid, 256, 0, s>>>(a);
}

}  // namespace

bool f32_seq_supported(int cell, int H) {
  return H >= 16 && H % 16 == 0 && (cell == CELL_LSTM || cell == CELL_GRU_A || cell == CELL_RNN);
}

// cell: CELL_LSTM, CELL_GRU_A (= the GRU), CELL_RNN.  Buffers (fp32, time-major):
//   zx [T, B, GW] input projection + bias; hs [T+1, B, H] (hs[0] = h_0); cs [T+1, B, H] (LSTM,
//   cs[0] = c_0); gates [T, B, GW] (LSTM i,j,f,o; GRU r,u,c~); rh [T, B, H] (GRU).
void launch_f32_fwd_seq(const F32Seq& q, hipStream_t s) {
  const int T = q.T, B = q.B, H = q.H, GW = q.GW;
  const size_t BH = (size_t)B * H, BG = (size_t)B * GW;
  for (int t = 0; t < T; ++t) {
    F32Step a{};
    a.B = B; a.H = H; a.fb = q.forget_bias;
    a.W = q.WT; a.Bop = q.hs + t * BH; a.ldb = H; a.K = H;
    a.zx = q.zx + t * BG; a.zx_ld = GW;
    a.hprev = q.hs + t * BH;
    a.hout = q.hs + (t + 1) * BH;
    a.gates = q.gates ? q.gates + t * BG : nullptr; a.gld = GW;
    if (q.cell == CELL_LSTM) {
      a.cprev = q.cs + t * BH; a.cout = q.cs + (t + 1) * BH;
      fwd1<CELL_LSTM>(a, s);
    } else if (q.cell == CELL_GRU_A) {
      a.rh = q.rh + t * BH;
      fwd1<CELL_GRU_A>(a, s);
      F32Step c = a;
      c.W = q.WT2; c.Bop = q.rh + t * BH;
      c.zx = a.zx + 2 * H;
      fwd1<CELL_GRU_B>(c, s);
    } else {
      fwd1<CELL_RNN>(a, s);
    }
  }
}

//   dtop [T, B, H] (null: zero); dz [T, B, GW] out; work0 [B, H] (LSTM dc / GRU dh, zeroed here
//   by the first step's kernels: LSTM needs it zero on entry, the caller clears it);
//   work1 [B, H] (GRU partial).  W: W_h [H, GW] (GRU: Wc_h [H, H]); W2 (GRU): Wg_h [H, 2H].
void launch_f32_bwd_seq(const F32Seq& q, hipStream_t s) {
  const int T = q.T, B = q.B, H = q.H, GW = q.GW;
  const size_t BH = (size_t)B * H, BG = (size_t)B * GW;
  auto base = [&](int t) {
    F32Step a{};
    a.B = B; a.H = H;
    a.dtop = q.dtop ? q.dtop + t * BH : nullptr;
    a.gates = q.gates ? q.gates + t * BG : nullptr; a.gld = GW;
    a.dz = q.dz + t * BG; a.dz_ld = GW;
    a.dc = q.work0;
    return a;
  };
  if (q.cell == CELL_GRU_A) {
    {  // step T-1 has no recurrent term: dh_{T-1} = dtop_{T-1}
      F32Step a = base(T - 1);
      a.dz += 2 * H;
      bwd1<CELL_GRU_B>(a, s);
    }
    for (int t = T - 1; t >= 0; --t) {
      F32Step a = base(t);
      a.dtop = nullptr;
      a.W = q.W; a.K = H; a.Bop = q.dz + t * BG + 2 * H; a.ldb = GW;  // dZc_t
      a.hprev = q.hs + t * BH;
      a.P = q.work1;
      bwd1<CELL_GRU_A>(a, s);
      if (t > 0) {
        F32Step c = base(t - 1);
        c.W = q.W2; c.K = 2 * H; c.Bop = q.dz + t * BG; c.ldb = GW;  // dZg_t
        c.P = q.work1;
        c.dz += 2 * H;
        bwd1<CELL_GRU_B>(c, s);
      }
    }
    return;
  }
  for (int t = T - 1; t >= 0; --t) {
    F32Step a = base(t);
    if (t < T - 1) {
      a.W = q.W; a.K = GW; a.Bop = q.dz + (t + 1) * BG; a.ldb = GW;
    }
    if (q.cell == CELL_LSTM) {
      a.c = q.cs + (t + 1) * BH; a.cprev = q.cs + t * BH;
      bwd1<CELL_LSTM>(a, s);
    } else {
      a.hprev = q.hs + (t + 1) * BH;
      bwd1<CELL_RNN>(a, s);
    }
  }
}

}  // namespace dcr
