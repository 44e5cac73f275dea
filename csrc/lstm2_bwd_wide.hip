// Two-layer wavefront LSTM BPTT with 32-unit x 16-row workgroup tiles (gfx950).
//
// Reference: tf.gradients through the unrolled two-layer stack (model.py:72, 91); the schedule
// is lstm2_persist.hip's reverse wavefront (layer l+1 at step T-1-tau, layer l two ticks
// behind, layer l's dtop = dZ_{l+1}·W_x,l+1ᵀ computed in-kernel).  What changes is the tile.
//
// Why.  Every BPTT tick a workgroup must read the whole 4H-wide dZ rows of its batch rows for
// both layers (dh = dZ·W_hᵀ reduces over all 4H gate columns).  With 16 units x 32 rows per
// workgroup (lstm2_persist.hip) that is 256 KB per workgroup and tick -- 8 MB per XCD per tick
// out of a 4 MB L2 at ~4.3 TB/s: the payload phase was L2-bandwidth bound (42 % of a 5.7 us
// tick, profiles/r2_pair_groups_stamps.txt).  Here a workgroup owns 32 units x 16 rows: the
// same MFMA work per workgroup and tick, HALF the payload bytes (128 KB), half the producer
// arrivals per hand-off counter, and twice the resident weights -- W_h,l and W_h,l+1 for 32
// units (256 VGPRs per lane) in registers, W_x,l+1 for 32 units (128 KB) in LDS.
//
// Geometry.  Workgroup (ubk, col): hidden units [32 ubk, 32 ubk + 32) of both layers, batch
// rows [16 col, 16 col + 16) (rows >= B are padding: zero inputs, zero gradients, written only
// to the hand-off ring).  Grid (H/32) x ceil(B/16), one workgroup per CU.  Wave w reduces over
// the K quarter {g·H + [w·H/4, (w+1)·H/4)} of every gate g (KS = H/32 k-steps of 32) and runs
// the cell-backward epilogue of layer w>>1, unit half w&1 (units 32 ubk + 16 (w&1) + [0, 16)).
//
// Hand-off protocol: persist_common.h / lstm2_persist.hip (sc1 fragment-order ring stores,
// vmcnt(0), one agent-scope counter add per storing wave per (column, slot); one poller per
// workgroup; every load of handed-off bytes is a buffer_load sc1).  Ring rows are 16-row MFMA
// tiles, so the ring layout is the one lstm2_persist.hip uses.
//
// Bias gradients: each epilogue lane's 16 dZ values (4 gates x 4 units) are reduced over the
// 16 rows of its DPP row by a 4-stage butterfly reduce-scatter (row_mirror, row_half_mirror,
// quad_perm xor 2, xor 1) after the hand-off arrival: lane r of a row ends with the row sum of
// value r, accumulated in ONE register over the launch (LDS holds only W_x and the partials).
#include "common.h"
#include "kernels.h"
#include "persist_common.h"
#include "debug_env.h"

namespace dcr {

// Diagnostics.  a.diag [T+2, 8]: s_memtime phase stamps of workgroup 0.  With a.diag_all the
// buffer is [grid, T+2, 8] and every workgroup records s_memrealtime (100 MHz, one clock for the
// whole chip) at the same points, except that slot 5 is layer l+1's hand-off arrival (wave 2)
// and slot 6 layer l's (wave 0): the cross-workgroup skew of every tick (scripts/pair_bench.py
// --skew).
// (only in the DIAG instantiations: a conditional store between the payload loads and the MFMAs
// degrades the compiler's waitcnt counts to vmcnt(0), see PF = 5)
#define STAMPW(i)                                                                    \
  if (DIAG && a.diag && threadIdx.x == 0 && (i) != 5 && (i) != 6) {                  \
    if (a.diag_all)                                                                  \
      a.diag[((size_t)blockIdx.x * (T + 2) + tau) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    else if (blockIdx.x == 0)                                                        \
      a.diag[(size_t)tau * 8 + (i)] = __builtin_amdgcn_s_memtime();                  \
  }
#define STAMP_ARRIVE()                                                               \
  if (DIAG && a.diag && lane == 0 && (w == 0 || w == 2)) {                           \
    if (a.diag_all)                                                                  \
      a.diag[((size_t)blockIdx.x * (T + 2) + tau) * 8 + (w ? 5 : 6)] =               \
          __builtin_amdgcn_s_memrealtime();                                          \
    else if (blockIdx.x == 0 && w == 0)                                              \
      a.diag[(size_t)tau * 8 + 6] = __builtin_amdgcn_s_memtime();                    \
  }

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, true));
}

// One butterfly stage over N values: lanes paired by the DPP involution CTRL exchange the half
// they do not keep (`hi`: keep the upper half) and add; returns N/2 values.
template <int CTRL, int N>
__device__ __forceinline__ void bfly(float (&v)[16], bool hi) {
#pragma unroll
  for (int k = 0; k < N / 2; ++k) {
    const float send = hi ? v[k] : v[k + N / 2];
    const float keep = hi ? v[k + N / 2] : v[k];
    v[k] = keep + dppf<CTRL>(send);
  }
}

// Row-sum reduce-scatter of 16 values over the 16 lanes of a DPP row: returns, in lane r of the
// row, the sum over the row's lanes of v[r].
__device__ __forceinline__ float row_reduce_scatter16(float (&v)[16], int lane) {
  const int r = lane & 15;
  bfly<0x140, 16>(v, (r & 8) != 0);  // row_mirror: r <-> 15 - r
  bfly<0x141, 8>(v, (r & 4) != 0);   // row_half_mirror: r <-> r ^ 7 (within 8)
  bfly<0x4E, 4>(v, (r & 2) != 0);    // quad_perm [2,3,0,1]: r <-> r ^ 2
  bfly<0xB1, 2>(v, (r & 1) != 0);    // quad_perm [1,0,3,2]: r <-> r ^ 1
  return v[0];
}

// PF: where the epilogue operands (gates, c, dtop, dropout bits; HBM reads, ~1.3 us under
// load) are loaded.  vmcnt retires in issue order, so whatever is loaded before the hand-off
// poll delays the poller's first counter check by its latency.
//   0: at the tick start, before the poll (the poll then waits for them: +1.35 us hand-off)
//   1: right behind the tick's payload loads (the MFMA / epilogue phase waits for them instead);
//      the default with the XCD-resident hand-off, whose poll returns ~0.8 us after the last
//      arrival (BPTT 4.80 vs 5.23 us per tick for 2, scripts/pair_bench.py, same box)
//   2: one tick ahead, right after the previous tick's hand-off arrival: their latency runs
//      concurrently with the hand-off's own (~1.7 us from arrival to the consumers' poll with
//      the write-through hand-off: there it was the best, 1.711 vs 1.726 ms/step for 0)
//   3: 2 for waves 1-3, 1 for wave 0, whose lane 0 polls: the poll then waits for no HBM load
//   4: 2 for waves 1-3; wave 0 (the poller) issues no HBM load at all: wave 1 DMAs wave 0's
//      operands (buffer_load ... lds, 16 dwords per lane) into a per-parity LDS buffer one tick
//      ahead, and wave 0 reads them after the tick's second barrier (wave 1's waits on its own
//      younger payload loads have covered the DMA by then).  No dropout variant.
//   5: 1's operand loads, plus the row-major dZ copy of the PREVIOUS tick stored behind the
//      payload loads (kept packed in registers across the tick boundary) and layer l's dtop
//      stash in front of the arrival (its MFMAs overlapping the ring stores' drain), so that no
//      store sits in front of the next poll.  Every vector-memory operation from the payload
//      loads to the MFMAs is unconditional (empty descriptors / out-of-range offsets instead of
//      branches): with conditional ones the compiler's waitcnt analysis assumes the path
//      without them and the MFMA phase's waits degrade to vmcnt(0), covering the stores (the
//      first form of this order measured 1.630 vs 1.619 ms/step against 2 for that reason).
//      Still slower than 1 (1.55 vs 1.52 ms/step, same box): the drain before the arrival now
//      waits for the HBM operand loads and the deferred stores (3.4 k cycles incl. the stash).
//   6 (default): 1, with layer l's dtop stash moved from after the arrival into the MFMA phase, between
//      layer l+1's chain and layer l's: its 32 LDS fragment reads and MFMAs per wave run while
//      layer l's payload -- loaded second, the CU's L2 read port streaming 128 KB per workgroup
//      and tick -- is still arriving.  After the arrival it delayed the next tick's poll (the
//      stamps: ~1.35 us from the arrival to the next tick start, the poll then ~0.4 us, i.e. the
//      hand-off had long landed).
template <int KS, bool DROP, int PFA, bool DIAG>
__global__ void __launch_bounds__(256, 1) lstm2_bwd_wide_kernel(Lstm2BwdArgs a) {
  static_assert(KS % 4 == 0, "K quarter = whole 32-wide k-steps per gate");
  constexpr int PF = PFA == 6 ? 1 : PFA;  // operand load order
  constexpr bool ES = PFA == 6;           // early stash
  // partials [wave][layer][unit half][lane][4]
  __shared__ __attribute__((aligned(16))) float part[4][2][2][64][4];
  // W_x,l+1 fragments [wave][unit half][k-step][lane] (128 KB at H = 512), read back only by
  // the wave that wrote them (the off-critical-path dtop stash)
  __shared__ __attribute__((aligned(16))) bf16x8 wx1l[4][2][KS][64];
  __shared__ unsigned arrl[2];              // per-layer arrivals of the tick (wgarr)
  // PF = 4: wave 0's epilogue operands by tick parity: g4 (8 dwords), c_{t+1} (4), c_t (4)
  __shared__ __attribute__((aligned(16))) unsigned opb[PF == 4 ? 2 : 1][PF == 4 ? 16 : 1][64];
  // wave 0 (the hand-off poller) hands its row-major dZ copy to wave 2 (same rows and units,
  // layer l+1), which stores it one tick later: vmcnt retires in issue order, so the poller's
  // own stores made its flag loads wait for their acknowledgement; by tick parity, [gate][lane]
  constexpr bool OFFL = PF == 1 || PF == 2;
  __shared__ __attribute__((aligned(16))) u32x2 offl[OFFL ? 2 : 1][4][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int G4H = 4 * H;
  const int ncol = a.nbg;  // 16-row columns (the host passes ceil(B / 16))
  int ubk, col;
  if (!map_block_grid(blockIdx.x, gridDim.x, H / 32, ncol, ubk, col)) return;  // padding
  const int ub0 = ubk * 32;
  const int kq = 8 * (lane >> 4);
  unsigned* cnt0 = a.cnt0 + (size_t)col * (T + 1) * 4;
  unsigned* cnt1 = a.cnt1 + (size_t)col * (T + 1) * 4;
  // XCD-resident hand-offs (persist_common.h): publish now, decide after the weight loads
  unsigned long long* const xw = reinterpret_cast<unsigned long long*>(cnt0 + 2);
  const bool tryloc = a.xcdloc && a.wgarr && T >= 8 && H / 32 <= 32;
  if (tryloc && threadIdx.x == 0) xcd_publish(xw);
  unsigned* const fl0 = cnt0 + 4;  // (local form) per-workgroup flags of layer l / l+1
  unsigned* const fl1 = cnt1 + 4;
  // arrivals per (column, slot) and layer: H/32 unit blocks x (one per workgroup | 2 waves)
  const unsigned target = (unsigned)(a.wgarr ? H / 32 : H / 16);
  if (threadIdx.x < 2) arrl[threadIdx.x] = 0u;  // (ordered before any add by tick 0's barrier)
  const size_t slabn = (size_t)ncol * 16 * G4H;  // one ring slot, elements
  bool dead = false;

  constexpr int KSG = KS / 4;  // k-steps per gate segment
  auto kcol = [&](int s) { return (s / KSG) * H + w * (H / 4) + (s % KSG) * 32; };
  bf16x8 wh0[2][KS], wh1[2][KS];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const size_t row = (size_t)(ub0 + 16 * u + (lane & 15)) * G4H + kcol(s) + kq;
      wh0[u][s] = ld8(a.Wh0 + row);
      wh1[u][s] = ld8(a.Wh1 + row);
      wx1l[w][u][s][lane] = ld8(a.Wx1 + row);
    }
  __shared__ int loc_s;
  if (threadIdx.x == 0) {
    loc_s = tryloc ? xcd_decide(xw, (unsigned)(H / 32), a.spin_limit, a.err, 13u) : 0;
    if (loc_s && ubk == 0) cnt0[1] = 1u;  // (diagnostics: the column ran XCD-local)
  }
  __syncthreads();
  const bool loc = __builtin_amdgcn_readfirstlane(loc_s) != 0;

  // epilogue role: layer L, unit half U
  const int L = w >> 1, U = w & 1;
  const int u0 = ub0 + 16 * U + 4 * (lane >> 4);
  const int b = col * 16 + (lane & 15);
  const bool live = b < B;
  const bf16* const gtL = L ? a.gates1 : a.gates0;
  const float* const cbL = L ? a.cbuf1 : a.cbuf0;
  bf16* const dzL = L ? a.dz1 : a.dz0;
  bf16* const zrL = L ? a.zring1 : a.zring0;
  unsigned* const cntL = L ? cnt1 : cnt0;
  const size_t bh = (size_t)b * H + u0;
  float dc[4] = {0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;  // this lane's bias-gradient sum (value lane & 15 of its row, see header)
  // PF = 5: the previous tick's row-major dZ values (bf16, as st4bf rounds them) and their step
  bf16x4 dzp[4];
  int tpend = -1;
  constexpr unsigned kOut = 0x7FFFFFF0u;  // an out-of-range buffer offset: dropped / reads 0
  const __amdgpu_buffer_rsrc_t rdz = make_rsrc(dzL, sizeof(bf16) * (size_t)T * B * G4H);
  auto flush_dz = [&]() {  // (unconditional: see PF = 5)
    const unsigned o = (tpend >= 0 && live)
                           ? (unsigned)((((size_t)tpend * B + b) * G4H + u0) * sizeof(bf16)) : kOut;
#pragma unroll
    for (int gt = 0; gt < 4; ++gt)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, dzp[gt]), rdz,
                                            o + gt * H * (unsigned)sizeof(bf16), 0, 0);
    tpend = -1;
  };
  // layer l's dtop partial of its NEXT tick (this wave's K quarter, both unit halves), computed
  // off the critical path from the tick's dZ_{l+1} fragments
  f32x4 xs[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const __amdgpu_buffer_rsrc_t rz1 = make_rsrc(a.zring1, sizeof(bf16) * 2 * slabn);
  const __amdgpu_buffer_rsrc_t rz0 = make_rsrc(a.zring0, sizeof(bf16) * 2 * slabn);

  // recurrence-independent epilogue operands of a tick (padded rows: zero) and the dropout
  // bits of layer l's dtop (layer l+1's input mask at step T+1-tau: this row's 32 units)
  bf16x4 g4[4];
  float cc[4], cp[4], dtop[4];
  unsigned mrow = 0;
  // buffer loads: a 32-bit per-lane offset fixed for the launch plus a wave-uniform per-tick
  // offset in an SGPR (64-bit per-lane addresses had spilled, the reload a vmcnt(0) drain)
  const __amdgpu_buffer_rsrc_t rg = make_rsrc(gtL, sizeof(bf16) * (size_t)T * B * G4H);
  const __amdgpu_buffer_rsrc_t rc = make_rsrc(cbL, sizeof(float) * (size_t)(T + 1) * B * H);
  const __amdgpu_buffer_rsrc_t rd = make_rsrc(a.dtop1, sizeof(float) * (size_t)T * B * H);
  const __amdgpu_buffer_rsrc_t rm = make_rsrc(a.xmask, DROP ? (size_t)T * B * (H / 8) : 0);
  const unsigned vg = opaque_vgpr((unsigned)(((size_t)b * G4H + u0) * sizeof(bf16)));
  const unsigned vc = opaque_vgpr((unsigned)(bh * sizeof(float)));
  const unsigned vm = (unsigned)(b * (H / 8) + (ub0 >> 3));
  const __amdgpu_buffer_rsrc_t rdL = make_rsrc(a.dtop1, L ? sizeof(float) * (size_t)T * B * H : 0);
  auto prefetch_u = [&](int tk) {  // PF = 5: unconditional, out-of-range lanes read zero
    const int tt = L ? T - 1 - tk : T + 1 - tk;
    const bool ac = L ? tk < T : tk >= 2;
    // (offsets through an opaque move: LLVM turns a select against an out-of-range offset into
    // a branch around the load, and the waitcnt pass then drains everything at the next write
    // of the destination registers)
    const unsigned vgo = opaque_vgpr((ac && live) ? vg : kOut);
    const unsigned vco = opaque_vgpr((ac && live) ? vc : kOut);
    const unsigned sg = ac ? (unsigned)((size_t)tt * B * G4H * sizeof(bf16)) : 0u;
    const unsigned sc = ac ? (unsigned)((size_t)tt * B * H * sizeof(float)) : 0u;
#pragma unroll
    for (int gt = 0; gt < 4; ++gt)
      g4[gt] = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(
                                              rg, vgo, sg + gt * H * (unsigned)sizeof(bf16), 0));
    const f32x4 c1 = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(rc, vco, sc + B * H * (unsigned)sizeof(float), 0));
    const f32x4 c0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rc, vco, sc, 0));
    const f32x4 d = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rdL, vco, sc, 0));
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      cc[r] = c1[r];
      cp[r] = c0[r];
      dtop[r] = d[r];
    }
    if (DROP) {
      const bool md = tk >= 2 && tk <= T + 1 && live;
      mrow = __builtin_amdgcn_raw_buffer_load_b32(
          rm, opaque_vgpr(md ? vm : kOut), md ? (unsigned)((size_t)(T + 1 - tk) * B * (H / 8)) : 0u,
          0);
    }
  };
  auto prefetch = [&](int tk) {
    if constexpr (PF == 5 || ES) {
      prefetch_u(tk);
      return;
    }
    const int tt = L ? T - 1 - tk : T + 1 - tk;
    const bool ac = L ? tk < T : tk >= 2;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int gt = 0; gt < 4; ++gt) g4[gt][r] = (bf16)0.f;
      cc[r] = cp[r] = dtop[r] = 0.f;
    }
    if (ac && live) {
      const unsigned sg = (unsigned)((size_t)tt * B * G4H * sizeof(bf16));
#pragma unroll
      for (int gt = 0; gt < 4; ++gt)
        g4[gt] = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(
                                                rg, vg, sg + gt * H * (unsigned)sizeof(bf16), 0));
      const unsigned sc = (unsigned)((size_t)tt * B * H * sizeof(float));
      // (whole-vector bit casts: clang's __builtin_bit_cast of an ext-vector ELEMENT reads
      // element 0 whatever the index, and the load is narrowed to one dword)
      const f32x4 c1 = __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rc, vc, sc + B * H * (unsigned)sizeof(float), 0));
      const f32x4 c0 = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rc, vc, sc, 0));
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        cc[r] = c1[r];
        cp[r] = c0[r];
      }
      if (L) {
        const f32x4 d = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, vc, sc, 0));
#pragma unroll
        for (int r = 0; r < 4; ++r) dtop[r] = d[r];
      }
    }
    if (DROP && tk >= 2 && tk <= T + 1 && live)
      mrow = __builtin_amdgcn_raw_buffer_load_b32(rm, vm, (unsigned)((size_t)(T + 1 - tk) * B * (H / 8)), 0);
  };

  for (int tau = 0; tau <= T + 1; ++tau) {
    const bool on1 = tau < T;                 // layer l+1 computes step T-1-tau
    const bool on0 = tau >= 2;                // layer l computes step T+1-tau (two ticks behind)
    const bool ld1 = tau >= 1 && tau <= T;    // dZ_{l+1}[T-tau] (published at tick tau-1)
    const bool ld0 = tau >= 3;                // dZ_l[T+2-tau]   (published at tick tau-1)
    const int t = L ? T - 1 - tau : T + 1 - tau;  // this role's step
    const bool act = L ? on1 : on0;
    STAMPW(0)
    if (PF == 0 || ((PF == 1 || PF == 5) && tau == 0) ||
        ((PF >= 2 && PF <= 4) && tau == 0 && !(PF == 4 && w == 0)))
      prefetch(tau);
    const int s1 = T - tau, s0 = T + 2 - tau;  // ring slots of dZ_{l+1} and dZ_l
    if (tau >= 1 && loc) {  // flags of both layers' producing tick (tau - 1) + 1
      if (w == 0 && !dead && (ld1 || ld0))
        dead = !poll_flags2(fl0, ld0, fl1, ld1, H / 32, (unsigned)tau, a.spin_limit, a.err, 10u);
    } else if (tau >= 1) {
      if (threadIdx.x == kLstmPollerThread && !dead && (ld1 || ld0)) {
        dead = (ld1 && ld0)
                   ? !poll_counter2(cnt1 + (size_t)s1 * 4, target, cnt0 + (size_t)s0 * 4, target,
                                    a.spin_limit, a.err, 10u)
                   : !poll_counter(ld1 ? cnt1 + (size_t)s1 * 4 : cnt0 + (size_t)s0 * 4, target,
                                   a.spin_limit, a.err, 10u);
      }
    }
    STAMPW(1)
    // (also: every wave's previous-tick epilogue has read the partials)
    __syncthreads();
    STAMPW(2)
    bf16x8 p1[KS], p0[KS];
    if (tau >= 1) {
      const unsigned o1 = (unsigned)((s1 & 1) * slabn * sizeof(bf16));
      const unsigned o0 = (unsigned)((s0 & 1) * slabn * sizeof(bf16));
      if constexpr (PF == 5 || ES) {  // unconditional: a skipped layer reads an empty descriptor
        const __amdgpu_buffer_rsrc_t r1e = ld1 ? rz1 : make_rsrc(a.zring1, 0);
        const __amdgpu_buffer_rsrc_t r0e = ld0 ? rz0 : make_rsrc(a.zring0, 0);
#pragma unroll
        for (int s = 0; s < KS; ++s)
          p1[s] = ld8_sc1(r1e, frag_load_off(col, kcol(s) >> 5, G4H, lane) + o1);
#pragma unroll
        for (int s = 0; s < KS; ++s)
          p0[s] = ld8_sc1(r0e, frag_load_off(col, kcol(s) >> 5, G4H, lane) + o0);
      } else {
        if (ld1) {
#pragma unroll
          for (int s = 0; s < KS; ++s)
            p1[s] = ld8_sc1(rz1, frag_load_off(col, kcol(s) >> 5, G4H, lane) + o1);
        }
        if (ld0) {
#pragma unroll
          for (int s = 0; s < KS; ++s)
            p0[s] = ld8_sc1(rz0, frag_load_off(col, kcol(s) >> 5, G4H, lane) + o0);
        }
      }
      if (PF == 1 || PF == 5 || (PF == 3 && w == 0)) prefetch(tau);
      if constexpr (PF == 5) flush_dz();  // last tick's dZ rows, behind this tick's loads
      __builtin_amdgcn_sched_barrier(0);
      f32x4 xsn[2];  // (ES) layer l's dtop partial for its next tick
      if constexpr (ES) {
        // layer l+1's dh partial and layer l's next dtop partial in one pass over p1 (both
        // unconditional: p1 reads zero from an empty descriptor when no slot is loaded); the
        // W_x,l+1 fragment reads from LDS interleave with the W_h,l+1 chain
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        f32x4 xn[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        // W_x fragments read two k-steps ahead (a read waited at its use serialised 32 LDS round
        // trips per tick)
        constexpr int kAh = 2;
        bf16x8 wq[kAh + 1][2];
#pragma unroll
        for (int s = 0; s < kAh; ++s) {
          wq[s][0] = wx1l[w][0][s][lane];
          wq[s][1] = wx1l[w][1][s][lane];
        }
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          if (s + kAh < KS) {
            wq[(s + kAh) % (kAh + 1)][0] = wx1l[w][0][s + kAh][lane];
            wq[(s + kAh) % (kAh + 1)][1] = wx1l[w][1][s + kAh][lane];
          }
          acc[0] = mfma16(wh1[0][s], p1[s], acc[0]);
          acc[1] = mfma16(wh1[1][s], p1[s], acc[1]);
          xn[0] = mfma16(wq[s % (kAh + 1)][0], p1[s], xn[0]);
          xn[1] = mfma16(wq[s % (kAh + 1)][1], p1[s], xn[1]);
        }
        if (on1) {
#pragma unroll
          for (int u = 0; u < 2; ++u)
            *reinterpret_cast<float4*>(&part[w][1][u][lane][0]) =
                make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
        }
        xsn[0] = xn[0];
        xsn[1] = xn[1];
      }
      if (!ES && on1) {  // layer l+1: dh partial = dZ_{l+1}[t+1] · W_h,l+1ᵀ, both unit halves
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          acc[0] = mfma16(wh1[0][s], p1[s], acc[0]);
          acc[1] = mfma16(wh1[1][s], p1[s], acc[1]);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
          *reinterpret_cast<float4*>(&part[w][1][u][lane][0]) =
              make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
      }
      if (on0) {  // layer l: dtop (stashed last tick) + dZ_l[t+1] · W_h,lᵀ
        f32x4 acc[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float4 x0 = make_float4(xs[u][0], xs[u][1], xs[u][2], xs[u][3]);
          if constexpr (DROP) {
            // layer l+1's input dropout on layer l's dtop: this lane's 4 units' bits
            const unsigned m = mrow >> (16 * u + 4 * (lane >> 4));
            x0.x = m & 1u ? x0.x * a.xscale : 0.f;
            x0.y = m & 2u ? x0.y * a.xscale : 0.f;
            x0.z = m & 4u ? x0.z * a.xscale : 0.f;
            x0.w = m & 8u ? x0.w * a.xscale : 0.f;
          }
          acc[u] = f32x4{x0.x, x0.y, x0.z, x0.w};
        }
        if (ld0) {
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            acc[0] = mfma16(wh0[0][s], p0[s], acc[0]);
            acc[1] = mfma16(wh0[1][s], p0[s], acc[1]);
          }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
          *reinterpret_cast<float4*>(&part[w][0][u][lane][0]) =
              make_float4(acc[u][0], acc[u][1], acc[u][2], acc[u][3]);
      }
      if constexpr (ES) {
        if (ld1) {
          xs[0] = xsn[0];
          xs[1] = xsn[1];
        }
      }
    } else {
      // tick 0: layer l+1's first step has no recurrent input
      *reinterpret_cast<float4*>(&part[w][1][0][lane][0]) = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(&part[w][1][1][lane][0]) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    STAMPW(3)
    __syncthreads();
    STAMPW(4)
    // layer l's dtop partial for its next tick from this tick's dZ_{l+1} fragments
    bool stashed = false;
    auto do_stash = [&]() {
      if (ld1) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            x = mfma16(wx1l[w][u][s][lane], p1[s], x);
            // (PF = 2: bound the LDS fragments the scheduler hoists ahead of the MFMAs; the
            // prefetched operands are live here too)
            if (PF >= 2 && (s & 3) == 3) __builtin_amdgcn_sched_barrier(0);
          }
          xs[u] = x;
        }
      }
      stashed = true;
    };
    if constexpr (PF == 4) if (w == 0 && act) {  // this wave's operands, DMA'd by wave 1
      const unsigned(&ob)[16][64] = opb[tau & 1];
#pragma unroll
      for (int gt = 0; gt < 4; ++gt)
        g4[gt] = __builtin_bit_cast(bf16x4, u32x2{ob[2 * gt][lane], ob[2 * gt + 1][lane]});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        cc[r] = live ? __builtin_bit_cast(float, ob[8 + r][lane]) : 0.f;
        cp[r] = live ? __builtin_bit_cast(float, ob[12 + r][lane]) : 0.f;
        dtop[r] = 0.f;  // (layer l: its dtop is inside the partials; prefetch() never ran here)
      }
      if (!live) {
#pragma unroll
        for (int gt = 0; gt < 4; ++gt)
#pragma unroll
          for (int r = 0; r < 4; ++r) g4[gt][r] = (bf16)0.f;
      }
    }
    if (act) {
      float dh[4];
      {
        const float4 q0 = *reinterpret_cast<const float4*>(&part[0][L][U][lane][0]);
        const float4 q1 = *reinterpret_cast<const float4*>(&part[1][L][U][lane][0]);
        const float4 q2 = *reinterpret_cast<const float4*>(&part[2][L][U][lane][0]);
        const float4 q3 = *reinterpret_cast<const float4*>(&part[3][L][U][lane][0]);
        dh[0] = q0.x + q1.x + q2.x + q3.x + dtop[0];
        dh[1] = q0.y + q1.y + q2.y + q3.y + dtop[1];
        dh[2] = q0.z + q1.z + q2.z + q3.z + dtop[2];
        dh[3] = q0.w + q1.w + q2.w + q3.w + dtop[3];
      }
      float di[4], dj[4], df_[4], dO[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float gi = (float)g4[0][r], gj = (float)g4[1][r];
        const float gf = (float)g4[2][r], go = (float)g4[3][r];
        const float th = tanhf_(cc[r]);
        const float dcv = dc[r] + dh[r] * go * (1.f - th * th);
        dO[r] = dh[r] * th * go * (1.f - go);
        di[r] = dcv * gj * gi * (1.f - gi);
        dj[r] = dcv * gi * (1.f - gj * gj);
        df_[r] = dcv * cp[r] * gf * (1.f - gf);
        dc[r] = dcv * gf;
      }
      if (DIAG && a.diag && !a.diag_all && blockIdx.x == 0 && threadIdx.x == 0)
        a.diag[(size_t)tau * 8 + 5] = __builtin_amdgcn_s_memtime();
      // layer l+1's dZ_t feeds both layers at the next tick (t >= 0); layer l's only itself
      if (L || t >= 1) {
        bf16* const zr = zrL + (size_t)(t & 1) * slabn;
        st4bf_ho(loc, zr + frag_index(b, u0, G4H), di[0], di[1], di[2], di[3]);
        st4bf_ho(loc, zr + frag_index(b, H + u0, G4H), dj[0], dj[1], dj[2], dj[3]);
        st4bf_ho(loc, zr + frag_index(b, 2 * H + u0, G4H), df_[0], df_[1], df_[2], df_[3]);
        st4bf_ho(loc, zr + frag_index(b, 3 * H + u0, G4H), dO[0], dO[1], dO[2], dO[3]);
        if constexpr (PF == 5) do_stash();  // its MFMAs overlap the ring stores' drain
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        STAMP_ARRIVE()
        if (lane == 0) {
          if (loc)
            wg_arrive_flag(&arrl[L], 2u, (L ? fl1 : fl0) + ubk, (unsigned)tau + 1u);
          else if (a.wgarr)
            wg_arrive(&arrl[L], 2u, cntL + (size_t)t * 4);
          else
            __hip_atomic_fetch_add(cntL + (size_t)t * 4, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      // off the critical path from here: the next tick's epilogue operands, layer l's next
      // dtop, the row-major dZ copy for the weight GEMMs, the bias gradient
      float dcur[16];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dcur[r] = di[r]; dcur[4 + r] = dj[r]; dcur[8 + r] = df_[r]; dcur[12 + r] = dO[r];
      }
      if constexpr (PF == 5) {  // stored behind the next tick's payload loads (flush_dz)
#pragma unroll
        for (int gt = 0; gt < 4; ++gt)
#pragma unroll
          for (int r = 0; r < 4; ++r) dzp[gt][r] = f2bf(dcur[4 * gt + r]);
        tpend = t;
      } else if (OFFL && w == 0) {  // stored by wave 2 one tick later
#pragma unroll
        for (int gt = 0; gt < 4; ++gt) {
          bf16x4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = f2bf(dcur[4 * gt + r]);
          offl[tau & 1][gt][lane] = __builtin_bit_cast(u32x2, v);
        }
      } else if (live) {
        bf16* dz = dzL + ((size_t)t * B + b) * G4H + u0;
        st4bf(dz, dcur[0], dcur[1], dcur[2], dcur[3]);
        st4bf(dz + H, dcur[4], dcur[5], dcur[6], dcur[7]);
        st4bf(dz + 2 * H, dcur[8], dcur[9], dcur[10], dcur[11]);
        st4bf(dz + 3 * H, dcur[12], dcur[13], dcur[14], dcur[15]);
      }
      // bias gradient of the bf16-rounded dz, exactly as the weight GEMMs see it (padded rows
      // add zero)
#pragma unroll
      for (int i = 0; i < 16; ++i) dcur[i] = (float)f2bf(dcur[i]);
      dbacc += row_reduce_scatter16(dcur, lane);
    }
    if ((PF == 2 || ((PF == 3 || PF == 4) && w != 0)) && tau < T + 1) prefetch(tau + 1);
    if constexpr (PF == 4) if (w == 1 && tau + 1 >= 2 && tau + 1 <= T + 1) {
      // wave 0's (layer l, unit half 0) operands of the next tick into opb[(tau + 1) & 1]
      const int tt = T - tau;  // = T + 1 - (tau + 1)
      const unsigned q = 4 * (lane >> 4);
      const unsigned og = (unsigned)(((size_t)b * G4H + ub0 + q) * sizeof(bf16));
      const unsigned oc = (unsigned)(((size_t)b * H + ub0 + q) * sizeof(float));
      const unsigned sg = (unsigned)((size_t)tt * B * G4H * sizeof(bf16));
      const unsigned sc = (unsigned)((size_t)tt * B * H * sizeof(float));
      unsigned(&ob)[16][64] = opb[(tau + 1) & 1];
#pragma unroll
      for (int gt = 0; gt < 4; ++gt)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rg, (__attribute__((address_space(3))) void*)&ob[2 * gt + h][0], 4, og + 4 * h,
              sg + gt * H * (unsigned)sizeof(bf16), 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rc, (__attribute__((address_space(3))) void*)&ob[8 + r][0], 4, oc + 4 * r,
            sc + B * H * (unsigned)sizeof(float), 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rc, (__attribute__((address_space(3))) void*)&ob[12 + r][0], 4, oc + 4 * r, sc, 0, 0);
      }
    }
    if (!ES && !stashed) do_stash();  // every wave (with an epilogue this tick or not)
    // wave 0's dZ copy of tick tau-1 (layer l, step T+2-tau), written before this tick's first
    // barrier (wave 0 is active from tick 2)
    auto store_offl = [&](int tk) {
      const int t0 = T + 1 - tk;
      bf16* dz = a.dz0 + ((size_t)t0 * B + b) * G4H + u0;
#pragma unroll
      for (int gt = 0; gt < 4; ++gt) *reinterpret_cast<u32x2*>(dz + gt * H) = offl[tk & 1][gt][lane];
    };
    if (OFFL && w == 2 && tau >= 3 && live) store_offl(tau - 1);
    STAMPW(7)
  }
  if constexpr (PF == 5) flush_dz();
  if constexpr (OFFL) {  // wave 0's last copy (tick T + 1, step 0)
    __syncthreads();
    if (w == 2 && live) {
      bf16* dz = a.dz0 + (size_t)b * G4H + u0;
#pragma unroll
      for (int gt = 0; gt < 4; ++gt)
        *reinterpret_cast<u32x2*>(dz + gt * H) = offl[(T + 1) & 1][gt][lane];
    }
  }
  // bias-gradient partial of this role's 16-row column: lane r of row q holds value r
  float* const dbp = L ? a.db_part1 : a.db_part0;
  if (dbp) {
    const int r = lane & 15;
    dbp[(size_t)col * G4H + (r >> 2) * H + u0 + (r & 3)] = dbacc;
    // rows of the partial buffer past the last column (the host sizes it for 32-row groups)
    if (col == ncol - 1)
      for (int c2 = ncol; c2 < a.db_rows; ++c2) dbp[(size_t)c2 * G4H + (r >> 2) * H + u0 + (r & 3)] = 0.f;
  }
}

template <bool DROP, int PF, bool DIAG = false>
static const void* lstm2_bwd_wide_pick_t(int H) {
  switch (H / 32) {  // KS = 4H / 4 waves / 32
    case 4: return (const void*)lstm2_bwd_wide_kernel<4, DROP, PF, DIAG>;
    case 8: return (const void*)lstm2_bwd_wide_kernel<8, DROP, PF, DIAG>;
    case 12: return (const void*)lstm2_bwd_wide_kernel<12, DROP, PF, DIAG>;
    case 16: return (const void*)lstm2_bwd_wide_kernel<16, DROP, PF, DIAG>;
  }
  return nullptr;
}
constexpr int kWidePfDefault = 6;  // headline 1.534 vs 1.558 ms, dropout 1.893 vs 1.963 (same box)
// diag: the stamped instantiation (the default operand order, no dropout)
template <bool DROP>
static const void* lstm2_bwd_wide_pick(int H, bool diag = false) {
  const int pf = debug_int("wide_pf", kWidePfDefault);
  if (diag && !DROP && pf == kWidePfDefault) return lstm2_bwd_wide_pick_t<false, kWidePfDefault, true>(H);
  switch (pf) {
    case 0: return lstm2_bwd_wide_pick_t<DROP, 0>(H);
    case 2: return lstm2_bwd_wide_pick_t<DROP, 2>(H);
    case 3: return lstm2_bwd_wide_pick_t<DROP, 3>(H);
    case 4: return DROP ? lstm2_bwd_wide_pick_t<DROP, 2>(H) : lstm2_bwd_wide_pick_t<DROP, 4>(H);
    case 5: return lstm2_bwd_wide_pick_t<DROP, 5>(H);
    case 6: return lstm2_bwd_wide_pick_t<DROP, 6>(H);
  }
  return lstm2_bwd_wide_pick_t<DROP, 1>(H);
}

// The 32-unit x 16-row BPTT applies at (H, B): H a multiple of 128 up to 512, and the grid of
// (H/32) x ceil(B/16) workgroups co-resident (one per CU).  DCR_DEBUG=wide=0 disables it.
bool lstm2_bwd_wide_ok(int H, int B, int cus) {
  if (debug_int("wide", 1) == 0) return false;
  if (H % 128 != 0 || H < 128 || H > 512 || B < 1 || cus <= 0) return false;
  const int grid = (H / 32) * ((B + 15) / 16);
  for (int drop = 0; drop < 2; ++drop) {
    const void* fn = drop ? lstm2_bwd_wide_pick<true>(H) : lstm2_bwd_wide_pick<false>(H);
    int o = 0;
    if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, 256, 0) != hipSuccess || o < 1)
      return false;
    if (grid > o * cus) return false;
  }
  return true;
}

int launch_lstm2_bwd_wide(const Lstm2BwdArgs& a, int cus, hipStream_t s) {
  if (!lstm2_bwd_wide_ok(a.H, a.B, cus) || a.nbg != (a.B + 15) / 16) return -2;
  void* args[] = {const_cast<Lstm2BwdArgs*>(&a)};
  const void* fn = a.xmask ? lstm2_bwd_wide_pick<true>(a.H)
                          : lstm2_bwd_wide_pick<false>(a.H, a.diag != nullptr);
  // the XCD-padded grid (persist_common.h xcd_grid) when it is co-resident
  int grid = (a.H / 32) * a.nbg, o = 0;
  const int padded = xcd_grid(a.H / 32, a.nbg);
  if (padded != grid && hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, 256, 0) == hipSuccess &&
      padded <= o * cus)
    grid = padded;
  return hipLaunchKernel(fn, dim3(grid), dim3(256), args, 0, s) == hipSuccess ? 0 : -3;
}

}  // namespace dcr
