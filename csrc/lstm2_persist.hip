// Two-layer wavefront forward for the persistent LSTM (gfx950).
//
// Reference: the layer stack of model.py:27-36 runs layer l+1's step t on layer l's h_t; the
// single-layer persistent kernels (lstm_persist.hip) therefore run 2T hand-off-latency-bound
// steps for two layers, although layer l+1's step t-1 and layer l's step t are independent.
// One launch here runs both layers as a wavefront: at tick tau layer l computes step tau and
// layer l+1 computes step tau-2.  Layer l's recurrent operand h_l[tau-1] (slot tau) is also
// layer l+1's input at step tau-1: its input-projection MFMAs h_l·W_x,l+1 run right after this
// tick's epilogue (while the workgroup waits for the next hand-off) and are added at the next
// tick, so the critical path of a tick carries only the two recurrent products.  T+2 ticks
// replace 2T steps.  Per-step latency, not bandwidth, bounds these kernels
// (profiles/r1_persist_stamps_vs_batch.txt), which is what makes the wider tick pay.
//
// Workgroup (ubk, bg) owns 16 hidden units x 32 batch rows (two 16-row MFMA tiles) of BOTH
// layers; its 4 waves split K in quarters and keep W_h(l)ᵀ, W_h(l+1)ᵀ and W_x(l+1)ᵀ rows of its
// units resident (3 x 16 x KS fragments).  Wave w runs the epilogue of layer w>>1, batch tile
// w&1.  Hand-off protocol as lstm_persist.hip (persist_common.h): sc1 write-through h stores,
// drain, agent-scope counter add per (layer, batch group, slot, K quarter); ONE poller per
// workgroup watches both layers' counters; every load of published h is buffer_load sc1.
#include "common.h"
#include "kernels.h"
#include "persist_common.h"

namespace dcr {

#define STAMP2(i)                                                                   \
  if constexpr (DIAG) {                                                             \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                        \
      a.diag[(size_t)tau * 8 + (i)] = __builtin_amdgcn_s_memtime();                 \
  }

template <int KS, bool DIAG = false>
__global__ void __launch_bounds__(256, 1) lstm2_fwd_persist_kernel(Lstm2Args a) {
  // partials [wave][layer][tile][gate][lane][r] (16-B lane stride: conflict-free b128 LDS
  // access), single-buffered -- every tick after the first starts with the poll barrier, which
  // each epilogue wave joins after its reads
  __shared__ __attribute__((aligned(16))) float part[4][2][2][4][64][4];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int nwg_u = H / 16;
  int ubk, bg;
  map_block(blockIdx.x, nwg_u, B / 32, ubk, bg);
  const int ub0 = ubk * 16, b0 = bg * 32;
  const int kq = 8 * (lane >> 4);
  const int kbase = w * (KS * 32);
  unsigned* cnt0 = a.cnt0 + (size_t)bg * (T + 1) * 4;
  unsigned* cnt1 = a.cnt1 + (size_t)bg * (T + 1) * 4;
  const unsigned target = (unsigned)(H / 8);  // H/16 unit blocks x 2 batch tiles
  bool dead = false;

  bf16x8 w0[4][KS], w1[4][KS], x1[4][KS];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const size_t row = (size_t)(g * H + ub0 + (lane & 15)) * H + kbase + s * 32 + kq;
      w0[g][s] = ld8(a.W0T + row);
      w1[g][s] = ld8(a.W1T + row);
      x1[g][s] = ld8(a.X1T + row);
    }
  unsigned hoff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    hoff[j] = (unsigned)(((size_t)(b0 + 16 * j + (lane & 15)) * H + kbase + kq) * sizeof(bf16));

  // epilogue role: layer L, batch tile J
  const int L = w >> 1, J = w & 1;
  const int b = b0 + 16 * J + (lane & 15);
  const int u0 = ub0 + 4 * (lane >> 4);
  const size_t bh = (size_t)b * H + u0;
  bf16* const hbL = L ? a.hbuf1 : a.hbuf0;
  float* const cbL = L ? a.cbuf1 : a.cbuf0;
  bf16* const gtL = L ? a.gates1 : a.gates0;
  float* const hlL = L ? a.hlast1 : a.hlast0;
  float* const clL = L ? a.clast1 : a.clast0;
  unsigned* const cntL = L ? cnt1 : cnt0;
  float c[4];
  ld4f(cbL + bh, c);
  float bias1[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g) ld4f(a.bias1 + g * H + u0, bias1[g]);

  // layer l+1's input-projection partials (this wave's K quarter, [tile][gate]) for its NEXT
  // tick: layer l+1 runs two ticks behind layer l, so x_t·W_x = h_l[t]·W_x is computed right
  // after the epilogue of the tick that loaded h_l[t] for layer l's own recurrence -- off the
  // critical path (the MFMAs run while the workgroup waits for the next hand-off)
  f32x4 xs[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) xs[j][g] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int tau = 0; tau <= T + 1; ++tau) {
    const bool on0 = tau < T;                  // layer l   computes step tau
    const bool on1 = tau >= 2;                 // layer l+1 computes step tau-2
    const bool ld0 = tau <= T;                 // slot tau of h_l (layer l's h_{tau-1})
    const bool ld1 = on1;                      // slot tau-2 of h_{l+1}
    STAMP2(0)
    // layer-l input projections of step tau (recurrence independent: issued before the wait)
    float zx[4][4];
    if (L == 0 && on0) {
      const float* zrow = a.ids ? a.zx0 + (size_t)a.ids[(size_t)tau * B + b] * a.zx_ld
                                : a.zx0 + ((size_t)tau * B + b) * a.zx_ld;
#pragma unroll
      for (int g = 0; g < 4; ++g) ld4f(zrow + (size_t)g * H + u0, zx[g]);
    }
    // hand-offs: layer l's slot tau (from tick tau-1; slot 0 is the prep-written initial state)
    // and layer l+1's slot tau-2 (from tick tau-1; slot 0 likewise)
    const bool pw0 = ld0 && tau >= 1, pw1 = ld1 && tau >= 3;
    if (pw0 || pw1) {
      if (threadIdx.x == kLstmPollerThread && !dead) {
        dead = (pw0 && pw1) ? !poll_counter2(cnt0 + (size_t)tau * 4, target,
                                           cnt1 + (size_t)(tau - 2) * 4, target, a.spin_limit,
                                           a.err, 9u)
                          : !poll_counter(pw0 ? cnt0 + (size_t)tau * 4 : cnt1 + (size_t)(tau - 2) * 4,
                                          target, a.spin_limit, a.err, 9u);
      }
      STAMP2(1)
      __syncthreads();
    }
    STAMP2(2)
    bf16x8 hf0[2][KS], hf1[2][KS];
    {
      // slot 0 (initial state, written by the prep launch) is row-major; later slots come from
      // the fragment-tiled rings: one contiguous 1 KB load per (tile, k-step)
      if (ld0) {
        const bool ring0 = a.hring0 && tau > 0;
        const __amdgpu_buffer_rsrc_t r0 =
            ring0 ? make_rsrc(a.hring0 + (size_t)(tau & 1) * B * H, sizeof(bf16) * (size_t)B * H)
                  : make_rsrc(a.hbuf0 + (size_t)tau * B * H, sizeof(bf16) * (size_t)B * H);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < KS; ++s)
            hf0[j][s] = ld8_sc1(r0, ring0 ? frag_load_off(2 * bg + j, w * KS + s, H, lane)
                                          : hoff[j] + s * 64);
      }
      if (ld1) {
        const int s1 = tau - 2;
        const bool ring1 = a.hring1 && s1 > 0;
        const __amdgpu_buffer_rsrc_t r1 =
            ring1 ? make_rsrc(a.hring1 + (size_t)(s1 & 1) * B * H, sizeof(bf16) * (size_t)B * H)
                  : make_rsrc(a.hbuf1 + (size_t)s1 * B * H, sizeof(bf16) * (size_t)B * H);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < KS; ++s)
            hf1[j][s] = ld8_sc1(r1, ring1 ? frag_load_off(2 * bg + j, w * KS + s, H, lane)
                                          : hoff[j] + s * 64);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (on0) {
        f32x4 acc[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[g] = mfma16(w0[g][s], hf0[j][s], acc[g]);
        float* dst = &part[w][0][j][0][lane][0];
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(dst + g * 256) = make_float4(acc[g][0], acc[g][1], acc[g][2], acc[g][3]);
      }
      if (on1) {  // stashed x-part + recurrent part
        f32x4 acc[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = xs[j][g];
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[g] = mfma16(w1[g][s], hf1[j][s], acc[g]);
        float* dst = &part[w][1][j][0][lane][0];
#pragma unroll
        for (int g = 0; g < 4; ++g)
          *reinterpret_cast<float4*>(dst + g * 256) = make_float4(acc[g][0], acc[g][1], acc[g][2], acc[g][3]);
      }
    }
    STAMP2(3)
    __syncthreads();
    STAMP2(4)
    // layer l+1's x-part of its step tau-1 (next tick) from h_l[tau-1] = slot tau.  Issued
    // right after this wave's hand-off arrival (nothing in flight then but the counter add):
    // placed after the row-major stores, the compiler's conservative vmcnt waits made these
    // MFMAs wait for the write-through of those stores
    const bool stash = ld0 && tau >= 1;
    bool stashed = false;
    auto do_stash = [&]() {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int g = 0; g < 4; ++g) xs[j][g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int g = 0; g < 4; ++g) xs[j][g] = mfma16(x1[g][s], hf0[j][s], xs[j][g]);
      }
      stashed = true;
    };
    if (L == 0 ? on0 : on1) {
      const int t = L == 0 ? tau : tau - 2;  // this layer's step
      float z[4][4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 s0 = *reinterpret_cast<const float4*>(&part[0][L][J][g][lane][0]);
        const float4 s1 = *reinterpret_cast<const float4*>(&part[1][L][J][g][lane][0]);
        const float4 s2 = *reinterpret_cast<const float4*>(&part[2][L][J][g][lane][0]);
        const float4 s3 = *reinterpret_cast<const float4*>(&part[3][L][J][g][lane][0]);
        const float* add = L == 0 ? zx[g] : bias1[g];
        z[g][0] = s0.x + s1.x + s2.x + s3.x + add[0];
        z[g][1] = s0.y + s1.y + s2.y + s3.y + add[1];
        z[g][2] = s0.z + s1.z + s2.z + s3.z + add[2];
        z[g][3] = s0.w + s1.w + s2.w + s3.w + add[3];
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
      STAMP2(5)
      bf16* const ringL = L ? a.hring1 : a.hring0;
      if (ringL)
        st4bf_sc1(ringL + (size_t)((t + 1) & 1) * B * H + frag_index(b, u0, H), h[0], h[1], h[2], h[3]);
      else
        st4bf_sc1(hbL + o, h[0], h[1], h[2], h[3]);
      // layer l's slot t+1 feeds both layers (up to slot T); layer l+1's slot t+1 only itself
      if (L == 0 || t + 1 < T) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        STAMP2(6)
        if (lane == 0)
          __hip_atomic_fetch_add(cntL + (size_t)(t + 1) * 4, 1u,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (stash) do_stash();
      if (ringL) st4bf(hbL + o, h[0], h[1], h[2], h[3]);  // row-major copy for the GEMMs
      *reinterpret_cast<float4*>(cbL + o) = make_float4(c[0], c[1], c[2], c[3]);
      if (gtL) {
        bf16* gp = gtL + ((size_t)t * B + b) * 4 * H + u0;
        st4bf(gp, gi[0], gi[1], gi[2], gi[3]);
        st4bf(gp + H, gj[0], gj[1], gj[2], gj[3]);
        st4bf(gp + 2 * H, gf[0], gf[1], gf[2], gf[3]);
        st4bf(gp + 3 * H, go[0], go[1], go[2], go[3]);
      }
      if (t == T - 1 && hlL)
        *reinterpret_cast<float4*>(hlL + bh) = make_float4(h[0], h[1], h[2], h[3]);
      if (t == T - 1 && clL)
        *reinterpret_cast<float4*>(clL + bh) = make_float4(c[0], c[1], c[2], c[3]);
    }
    if (stash && !stashed) do_stash();  // waves without an epilogue this tick
  }
}

template <int KS>
static const void* lstm2_fn(bool diag) {
  return diag ? (const void*)lstm2_fwd_persist_kernel<KS, true>
              : (const void*)lstm2_fwd_persist_kernel<KS, false>;
}

static const void* lstm2_pick(int H, bool diag = false) {
  switch (H / 128) {
    case 1: return lstm2_fn<1>(diag);
    case 2: return lstm2_fn<2>(diag);
    case 3: return lstm2_fn<3>(diag);
    case 4: return lstm2_fn<4>(diag);
  }
  return nullptr;
}

static int lstm2_grid(int H, int B) { return (H / 16) * (B / 32); }

int lstm2_persist_supported(int H, int B, int cus) {
  if (H % 128 != 0 || H < 128 || H > 512 || B % 32 != 0 || B < 32 || cus <= 0) return 0;
  const void* fn = lstm2_pick(H);
  int occ = 0;
  if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 256, 0) != hipSuccess)
    return 0;
  return lstm2_grid(H, B) <= occ * cus ? 1 : 0;
}

int launch_lstm2_fwd_persist(const Lstm2Args& a, int cus, hipStream_t s) {
  if (!lstm2_persist_supported(a.H, a.B, cus)) return -2;
  void* args[] = {const_cast<Lstm2Args*>(&a)};
  return hipLaunchKernel(lstm2_pick(a.H, a.diag != nullptr), dim3(lstm2_grid(a.H, a.B)),
                         dim3(256), args, 0, s) ==
                 hipSuccess ? 0 : -3;
}

// ------------------------------------------------------------------------------------------
// two-layer wavefront BPTT
// ------------------------------------------------------------------------------------------
// Reference: tf.gradients through the unrolled two-layer stack (model.py:72, 91).  The
// single-layer persistent BPTT (lstm_persist.hip) runs layer l+1's T steps, a dX GEMM
// (dZ_{l+1}·W_x,l+1ᵀ), then layer l's T steps: 2T hand-off-latency-bound steps.  Layer l's
// step t needs only layer l+1's dZ_t (its dtop) and its own dZ_{t+1}, so here one launch runs
// both as a reverse wavefront: at tick tau layer l+1 computes step T-1-tau and layer l step
// T+1-tau (two ticks behind).  The slot dZ_{l+1}[T-tau] loaded for layer l+1's recurrence is
// also layer l's dtop operand one tick later: its W_x,l+1 product (fragments in LDS) runs after
// this tick's epilogue, off the critical path, so the dX GEMM disappears and T+2 ticks replace
// 2T steps.
//
// Workgroup (ubk, bg) owns 16 hidden units x 32 batch rows (two 16-row MFMA tiles) of BOTH
// layers.  K = 4H is split by hidden-unit quarter exactly as in lstm_bwd_persist_kernel: wave w
// reduces over the columns g*H + [w*H/4, (w+1)*H/4) of every gate g and keeps the W_h,l,
// W_h,l+1 and W_x,l+1 rows of its units for that K quarter resident (3 x KS fragments).
// Wave w runs the cell-backward epilogue of layer w>>1 (0 = l, 1 = l+1), batch tile w&1.
// Hand-off: as the forward above (sc1 fragment-order ring stores, the storing wave's
// vmcnt(0), one agent-scope add per storing wave; ONE poller per workgroup watches both
// layers' counters; every load of handed-off dZ is buffer_load sc1).
template <int KS, bool DIAG = false>
__global__ void __launch_bounds__(256, 1) lstm2_bwd_persist_kernel(Lstm2BwdArgs a) {
  // partials [wave][layer][tile][lane][unit r]: single-buffered -- every tick that writes them
  // starts with the poll barrier, which each epilogue wave joins after its reads
  __shared__ __attribute__((aligned(16))) float part[4][2][2][64][4];
  // bias-gradient accumulators of each epilogue lane, kept in LDS (registers are the limit:
  // 3 x KS weight and 3 x KS payload fragments live across the MFMA phase)
  __shared__ float dbl[4][16][64];
  // layer l's dtop partial (this wave's K quarter, both tiles) for its NEXT tick, computed off
  // the critical path after this tick's epilogue from the dZ_{l+1} fragments this tick loaded
  __shared__ __attribute__((aligned(16))) float xsl[4][2][64][4];
  // W_x,l+1 fragments [wave][k-step][lane] (64 KB): only the off-critical-path stash product
  // reads them, so they live in LDS and leave the registers to W_h,l / W_h,l+1 and the payload
  __shared__ __attribute__((aligned(16))) bf16x8 wx1l[4][KS][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int G4H = 4 * H;
  int ubk, bg;
  map_block(blockIdx.x, H / 16, B / 32, ubk, bg);
  const int ub0 = ubk * 16, b0 = bg * 32;
  const int kq = 8 * (lane >> 4);
  unsigned* cnt0 = a.cnt0 + (size_t)bg * (T + 1) * 4;
  unsigned* cnt1 = a.cnt1 + (size_t)bg * (T + 1) * 4;
  const unsigned target = (unsigned)(H / 8);  // H/16 unit blocks x 2 batch tiles
  bool dead = false;

  constexpr int KSG = KS / 4;  // k-steps per gate segment
  auto kcol = [&](int s) { return (s / KSG) * H + w * (H / 4) + (s % KSG) * 32; };
  bf16x8 wh0[KS], wh1[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const size_t row = (size_t)(ub0 + (lane & 15)) * G4H + kcol(s) + kq;
    wh0[s] = ld8(a.Wh0 + row);
    wh1[s] = ld8(a.Wh1 + row);
    wx1l[w][s][lane] = ld8(a.Wx1 + row);  // read back only by this wave
  }

  // epilogue role: layer L, batch tile J
  const int L = w >> 1, J = w & 1;
  const int b = b0 + 16 * J + (lane & 15);
  const int u0 = ub0 + 4 * (lane >> 4);
  const size_t bh = (size_t)b * H + u0;
  const bf16* const gtL = L ? a.gates1 : a.gates0;
  const float* const cbL = L ? a.cbuf1 : a.cbuf0;
  bf16* const dzL = L ? a.dz1 : a.dz0;
  bf16* const zrL = L ? a.zring1 : a.zring0;
  unsigned* const cntL = L ? cnt1 : cnt0;
  float dc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 16; ++i) dbl[w][i][lane] = 0.f;

  for (int tau = 0; tau <= T + 1; ++tau) {
    const bool on1 = tau < T;                 // layer l+1 computes step T-1-tau
    const bool on0 = tau >= 2;                // layer l computes step T+1-tau (two ticks behind)
    const bool ld1 = tau >= 1 && tau <= T;    // dZ_{l+1}[T-tau] (published at tick tau-1)
    const bool ld0 = tau >= 3;                // dZ_l[T+2-tau]   (published at tick tau-1)
    const int t = L ? T - 1 - tau : T + 1 - tau;  // this role's step
    const bool act = L ? on1 : on0;
    STAMP2(0)
    // recurrence-independent epilogue operands, issued before the wait
    // (gates stay packed bf16 until the epilogue: registers are the limit here)
    bf16x4 g4[4];
    float cc[4], cp[4], dtop[4];
    if (act) {
      const bf16* gp = gtL + ((size_t)t * B + b) * G4H + u0;
#pragma unroll
      for (int g = 0; g < 4; ++g) g4[g] = *reinterpret_cast<const bf16x4*>(gp + g * H);
      ld4f(cbL + (size_t)(t + 1) * B * H + bh, cc);
      ld4f(cbL + (size_t)t * B * H + bh, cp);
      if (L) {
        ld4f(a.dtop1 + (size_t)t * B * H + bh, dtop);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) dtop[r] = 0.f;
      }
    }
    // after_arrive runs right after the wave's hand-off arrival, before its other stores
    auto epilogue = [&](auto&& after_arrive) {
        float dh[4];
        if (tau >= 1) {
          const float4 s0 = *reinterpret_cast<const float4*>(&part[0][L][J][lane][0]);
          const float4 s1 = *reinterpret_cast<const float4*>(&part[1][L][J][lane][0]);
          const float4 s2 = *reinterpret_cast<const float4*>(&part[2][L][J][lane][0]);
          const float4 s3 = *reinterpret_cast<const float4*>(&part[3][L][J][lane][0]);
          dh[0] = s0.x + s1.x + s2.x + s3.x + dtop[0];
          dh[1] = s0.y + s1.y + s2.y + s3.y + dtop[1];
          dh[2] = s0.z + s1.z + s2.z + s3.z + dtop[2];
          dh[3] = s0.w + s1.w + s2.w + s3.w + dtop[3];
        } else {
  #pragma unroll
          for (int r = 0; r < 4; ++r) dh[r] = dtop[r];
        }
        float gi[4], gj[4], gf[4], go[4];
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          gi[r] = (float)g4[0][r]; gj[r] = (float)g4[1][r];
          gf[r] = (float)g4[2][r]; go[r] = (float)g4[3][r];
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
        STAMP2(5)
        // layer l+1's dZ_t feeds both layers at the next tick (t >= 0); layer l's only itself
        if (L || t >= 1) {
          bf16* const zr = zrL + (size_t)(t & 1) * B * G4H;
          st4bf_sc1(zr + frag_index(b, u0, G4H), di[0], di[1], di[2], di[3]);
          st4bf_sc1(zr + frag_index(b, H + u0, G4H), dj[0], dj[1], dj[2], dj[3]);
          st4bf_sc1(zr + frag_index(b, 2 * H + u0, G4H), df_[0], df_[1], df_[2], df_[3]);
          st4bf_sc1(zr + frag_index(b, 3 * H + u0, G4H), dO[0], dO[1], dO[2], dO[3]);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          STAMP2(6)
          if (lane == 0)
            __hip_atomic_fetch_add(cntL + (size_t)t * 4, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        after_arrive();
        // row-major copy for the weight GEMMs, after the arrival (off the critical path)
        bf16* dz = dzL + ((size_t)t * B + b) * G4H + u0;
        st4bf(dz, di[0], di[1], di[2], di[3]);
        st4bf(dz + H, dj[0], dj[1], dj[2], dj[3]);
        st4bf(dz + 2 * H, df_[0], df_[1], df_[2], df_[3]);
        st4bf(dz + 3 * H, dO[0], dO[1], dO[2], dO[3]);
        // bias gradient of the bf16-rounded dz, exactly as the weight GEMMs see it
  #pragma unroll
        for (int r = 0; r < 4; ++r) {
          dbl[w][r][lane] += (float)f2bf(di[r]);
          dbl[w][4 + r][lane] += (float)f2bf(dj[r]);
          dbl[w][8 + r][lane] += (float)f2bf(df_[r]);
          dbl[w][12 + r][lane] += (float)f2bf(dO[r]);
        }
    };
    if (tau >= 1) {
      bf16x8 p1[2][KS];
      const int s1 = T - tau, s0 = T + 2 - tau;  // ring slots of dZ_{l+1} and dZ_l
      if (threadIdx.x == kLstmPollerThread && !dead && (ld1 || ld0)) {
        dead = (ld1 && ld0)
                   ? !poll_counter2(cnt1 + (size_t)s1 * 4, target, cnt0 + (size_t)s0 * 4, target,
                                    a.spin_limit, a.err, 10u)
                   : !poll_counter(ld1 ? cnt1 + (size_t)s1 * 4 : cnt0 + (size_t)s0 * 4, target,
                                   a.spin_limit, a.err, 10u);
      }
      STAMP2(1)
      __syncthreads();
      STAMP2(2)
      const size_t slab = sizeof(bf16) * (size_t)B * G4H;
      const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a.zring1 + (size_t)(s1 & 1) * B * G4H, slab);
      const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.zring0 + (size_t)(s0 & 1) * B * G4H, slab);
      // register budget (one wave per SIMD, <= ~450 VGPR+AGPR without spills): 3 x KS weight
      // fragments + 3 x KS payload fragments in flight (both tiles of dZ_{l+1}, tile 0 of
      // dZ_l); tile 1 of dZ_l is issued once tile 0's fragments are consumed
      bf16x8 p0[KS];
      if (ld1) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < KS; ++s)
            p1[j][s] = ld8_sc1(r1, frag_load_off(2 * bg + j, kcol(s) >> 5, G4H, lane));
      }
      if (ld0) {
#pragma unroll
        for (int s = 0; s < KS; ++s)
          p0[s] = ld8_sc1(r0, frag_load_off(2 * bg, kcol(s) >> 5, G4H, lane));
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (on1) {  // layer l+1: dh partial = dZ_{l+1}[t+1] · W_h,l+1ᵀ
          f32x4 acc1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KS; ++s) acc1 = mfma16(wh1[s], p1[j][s], acc1);
          *reinterpret_cast<float4*>(&part[w][1][j][lane][0]) =
              make_float4(acc1[0], acc1[1], acc1[2], acc1[3]);
        }
        if (on0) {  // layer l: dtop (stashed last tick) + dZ_l[t+1] · W_h,lᵀ
          const float4 x0 = *reinterpret_cast<const float4*>(&xsl[w][j][lane][0]);
          f32x4 acc0 = f32x4{x0.x, x0.y, x0.z, x0.w};
          if (ld0) {
#pragma unroll
            for (int s = 0; s < KS; ++s) acc0 = mfma16(wh0[s], p0[s], acc0);
            if (j == 0) {
              __builtin_amdgcn_sched_barrier(0);
#pragma unroll
              for (int s = 0; s < KS; ++s)
                p0[s] = ld8_sc1(r0, frag_load_off(2 * bg + 1, kcol(s) >> 5, G4H, lane));
            }
          }
          *reinterpret_cast<float4*>(&part[w][0][j][lane][0]) =
              make_float4(acc0[0], acc0[1], acc0[2], acc0[3]);
        }
      }
      STAMP2(3)
      __syncthreads();
      STAMP2(4)
      // layer l's dtop for its next tick, off the critical path (see xsl), issued right after
      // this wave's arrival: behind its row-major stores the compiler's conservative vmcnt waits
      // would make the MFMAs wait for their write-through
      bool stashed = false;
      auto do_stash = [&]() {
        if (ld1) {
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < KS; ++s) x = mfma16(wx1l[w][s][lane], p1[j][s], x);
            *reinterpret_cast<float4*>(&xsl[w][j][lane][0]) = make_float4(x[0], x[1], x[2], x[3]);
          }
        }
        stashed = true;
      };
      if (act) epilogue(do_stash);
      if (!stashed) do_stash();
    } else if (act) {
      epilogue([] {});
    }
  }
  // bias-gradient partial of this role's 16-row tile: reduce the 16 batch lanes
  float* const dbp = L ? a.db_part1 : a.db_part0;
  if (dbp) {
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = dbl[w][g * 4 + r][lane];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        if ((lane & 15) == 0) dbp[(size_t)(2 * bg + J) * G4H + g * H + u0 + r] = v;
      }
  }
}

template <int KS>
static const void* lstm2_bwd_fn(bool diag) {
  return diag ? (const void*)lstm2_bwd_persist_kernel<KS, true>
              : (const void*)lstm2_bwd_persist_kernel<KS, false>;
}

static const void* lstm2_bwd_pick(int H, bool diag = false) {
  switch (H / 32) {  // KS = 4H / 4 waves / 32
    case 4: return lstm2_bwd_fn<4>(diag);
    case 8: return lstm2_bwd_fn<8>(diag);
    case 12: return lstm2_bwd_fn<12>(diag);
    case 16: return lstm2_bwd_fn<16>(diag);
  }
  return nullptr;
}

int lstm2_bwd_persist_supported(int H, int B, int cus) {
  if (H % 128 != 0 || H < 128 || H > 512 || B % 32 != 0 || B < 32 || cus <= 0) return 0;
  const void* fn = lstm2_bwd_pick(H);
  int occ = 0;
  if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 256, 0) != hipSuccess)
    return 0;
  return lstm2_grid(H, B) <= occ * cus ? 1 : 0;
}

int launch_lstm2_bwd_persist(const Lstm2BwdArgs& a, int cus, hipStream_t s) {
  if (!lstm2_bwd_persist_supported(a.H, a.B, cus)) return -2;
  void* args[] = {const_cast<Lstm2BwdArgs*>(&a)};
  return hipLaunchKernel(lstm2_bwd_pick(a.H, a.diag != nullptr), dim3(lstm2_grid(a.H, a.B)),
                         dim3(256), args, 0, s) == hipSuccess ? 0 : -3;
}

}  // namespace dcr
