// Two-layer wavefront persistent LSTM (gfx950): forward and BPTT of layers (l, l+1) in one launch
// each, for any batch size.
//
// Reference: the layer stack of model.py:27-36 runs layer l+1's step t on layer l's h_t, and
// tf.gradients runs the reverse chain (model.py:72, 91).  Run as single-layer persistent kernels
// that is 2T hand-off-latency-bound steps per direction, although layer l+1's step t-1 and layer
// l's step t are independent.  One launch here runs both layers as a wavefront.
//
// Geometry.  Workgroup (ubk, col) owns hidden units [16 ubk, 16 ubk + 16) of BOTH layers for the
// 32 G batch rows of column `col` (G "groups" of two 16-row MFMA tiles).  Its 4 waves split K in
// quarters and keep their slices of W_h(l)ᵀ, W_h(l+1)ᵀ and W_x(l+1)ᵀ (forward) or W_h(l),
// W_h(l+1) (+ W_x(l+1) in LDS, BPTT) resident for the whole launch.  The grid is (H/16) x
// ceil(B / 32G) workgroups, one per CU; G (1..4, compile-time) is the smallest value that fits
// the chip.  Batch rows >= B (padding up to whole columns) run with zero inputs and zero
// gradients, write only the hand-off rings (sized for the padded batch) and are never stored
// row-major.
//
// One hand-off per tick and column.  The per-tick latencies are a counter poll (~0.8 us even when
// the data is long there: the load goes to the memory side), the payload loads and the drain of
// the write-through ring stores (~1 us): profiles/r2_pair_groups.md.  A workgroup therefore polls
// ONCE per tick for its whole column, runs its G groups' payload loads, MFMAs and cell epilogues
// one after the other (the LDS partials are reused per group), and drains + signals ONCE at the
// end of the tick; consumers of the column wait for one counter per layer.
//
// Hand-off protocol (persist_common.h, MI355X_MICROARCH.md "Valid forms", third row): sc1
// fragment-order ring stores, the storing wave's vmcnt(0), one agent-scope counter add per
// storing wave per (column, slot); ONE poller per workgroup watches both layers' counters; every
// load of handed-off bytes is a buffer_load sc1.
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "persist_common.h"

namespace dcr {

// s_memtime stamps of workgroup 0 (diagnostics, scripts/pair_bench.py --stamps): diag[tick][g][i]
#define STAMPG(g, i)                                                                \
  if (a.diag && blockIdx.x == 0 && threadIdx.x == 0)                                \
    a.diag[((size_t)tau * G + (g)) * 8 + (i)] = __builtin_amdgcn_s_memtime();
// The forward's stamps exist only in its DIAG instantiation: a conditional store between the
// payload loads and the MFMAs makes the compiler's waitcnt analysis assume the path without it,
// so every later wait degrades to vmcnt(0) (see the G = 1 notes in the kernel)
#define STAMPF(g, i) \
  if constexpr (DIAG) { STAMPG(g, i) }

constexpr int kPairMaxG = 4;

// Dropout (dropout.hip bit masks): zero the elements of a bf16 MFMA fragment whose mask bit is
// clear (8 consecutive k, bit e of `m` = element e); the 1/keep scale is applied to the product.
// The same in 5 full-rate VALU ops per dword: the bit pair x of the dword is spread to bits 0
// and 16 (x | x << 15, & 0x10001) and multiplied by 0xFFFF into the dword's keep mask (a 24-bit
// multiply: the spread value is < 2^17).
__device__ __forceinline__ bf16x8 mask_frag_fast(const bf16x8& v, unsigned m) {
  u32x4 u = __builtin_bit_cast(u32x4, v);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const unsigned x = (m >> (2 * i)) & 3u;
    u[i] &= __umul24((x | (x << 15)) & 0x10001u, 0xFFFFu);
  }
  return __builtin_bit_cast(bf16x8, u);
}

__device__ __forceinline__ bf16x8 mask_frag(const bf16x8& v, unsigned m) {
  u32x4 u = __builtin_bit_cast(u32x4, v);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    u[i] &= ((m >> (2 * i)) & 1u ? 0x0000FFFFu : 0u) | ((m >> (2 * i + 1)) & 1u ? 0xFFFF0000u : 0u);
  return __builtin_bit_cast(bf16x8, u);
}

// ------------------------------------------------------------------------------------------
// forward.  G = 1: at tick tau (0..T+1) layer l computes step tau and layer l+1 step tau-2.
// Layer l's slot tau (h_l[tau-1], its recurrent operand) is also layer l+1's input of step
// tau-1: that product h_l·W_x,l+1 runs right after the epilogue (while its stores drain) into
// registers and is added at the next tick, so the MFMA phase carries only the two recurrent
// products.  G > 1: layer l+1 runs one tick behind (step tau-1, T+1 ticks) and takes the input
// product in the group's MFMA phase: the ticks are work-bound there (the G phases run back to
// back, one drain per tick), and the stash would cost 32 registers per group.
// ------------------------------------------------------------------------------------------
// XIN (G = 1): layer l's input projection x_t·W_x,l runs in-kernel from bf16 input rows a.x0
// ([T·B, H], time-major; e.g. the dropout-masked embedding rows) instead of a library GEMM's
// fp32 [T·B, 4H] zx0: W_x,lᵀ fragments sit in LDS, the rows' fragments are loaded and the
// product accumulated BEFORE the tick's poll (it does not depend on the hand-off), and the
// recurrent product is added on top after it.
template <int KS, int G, bool DROP, bool XIN, bool DIAG>
__global__ void __launch_bounds__(256, 1) lstm2_fwd_persist_kernel(Lstm2Args a) {
  static_assert(!XIN || G == 1, "in-kernel input projection: one batch group per workgroup");
  // partials [wave][layer][tile][gate][lane][r] (16-B lane stride: conflict-free b128 access),
  // reused by every group: a barrier separates one group's epilogue reads from the next
  // group's stores
  __shared__ __attribute__((aligned(16))) float part[4][2][2][4][64][4];
  // dropout: the tick's input-mask bytes of the workgroup's rows, [row][H/8] (H <= 512),
  // double-buffered by tick (the G = 1 stash reads them after the tick's last barrier)
  constexpr int kMaskDw = 2 * G;  // DMA dwords per lane: 32 G rows x H/32 dwords / 256 lanes
  __shared__ __attribute__((aligned(16))) unsigned mlds[2][DROP ? G * 512 : 1];
  // XIN: W_x,lᵀ fragments [wave][gate][k-step][lane] (64 KB at H = 512), read back only by the
  // wave that wrote them
  __shared__ __attribute__((aligned(16))) bf16x8 wx0l[XIN ? 4 : 1][4][XIN ? KS : 1][64];
  // G = 1 gather mode (the headline): the workgroup's slice of the zx0 table -- 16 units x 4
  // gates of every vocabulary row, rows padded to 68 floats so 16 lanes reading 16 different
  // rows hit distinct banks -- and the gather ids of its 32 rows for every tick live in LDS, so
  // a tick issues no per-row loads (vmcnt retires in order: the one-tick-ahead row loads had
  // made every later wait of the tick cover them; 4.10 -> 3.72 us per tick without them)
  constexpr bool ZTAB = G == 1 && !XIN;
  constexpr int kTabMaxV = 128, kTabLd = 68, kTabMaxT = 256;
  __shared__ __attribute__((aligned(16))) float ztab[ZTAB ? kTabMaxV * kTabLd : 4];
  __shared__ int idsl[ZTAB ? kTabMaxT * 32 : 1];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int nwg_u = H / 16;
  int ubk, col;
  if (!map_block_grid(blockIdx.x, gridDim.x, nwg_u, a.nbg / G, ubk, col)) return;  // padding
  const int ub0 = ubk * 16;
  const int kq = 8 * (lane >> 4);
  const int kbase = w * (KS * 32);
  unsigned* const cnt0 = a.cnt0 + (size_t)col * (T + 1) * 4;
  unsigned* const cnt1 = a.cnt1 + (size_t)col * (T + 1) * 4;
  // XCD-resident hand-offs (persist_common.h): publish this workgroup's XCD now, decide after
  // the weight loads (the exchange's round trip overlaps them)
  unsigned long long* const xw = reinterpret_cast<unsigned long long*>(cnt0 + 2);
  const bool tryloc = a.xcdloc && a.wgarr && T >= 8 && nwg_u <= 32;
  if (tryloc && threadIdx.x == 0) xcd_publish(xw);
  unsigned* const fl0 = cnt0 + 4;  // (local form) per-workgroup flags of layer l / l+1
  unsigned* const fl1 = cnt1 + 4;
  // arrivals per (column, slot) and layer: H/16 unit blocks x (one per workgroup | 2 waves)
  const unsigned target = (unsigned)(a.wgarr ? H / 16 : H / 8);
  __shared__ unsigned arrl[2];  // per-layer arrivals of the tick (wgarr)
  __shared__ int loc_s;
  if (threadIdx.x < 2) arrl[threadIdx.x] = 0u;  // (ordered before any add by tick 0's barrier)
  const size_t ringsz = (size_t)a.nbg * 32 * H;  // one ring slot (padded batch)
  bool dead = false;
  // row-major slot-0 fragment offsets (rows >= B read as zero: buffer range check)
  const unsigned rm_lane = (unsigned)(((lane & 15) * H + kq) * sizeof(bf16));
  auto rm_off = [&](int bg, int j, int s) {
    return (unsigned)((((size_t)bg * 32 + 16 * j) * H + kbase + s * 32) * sizeof(bf16));
  };
  // the same for the h buffers (row stride hld: H, or 2H in the pair-interleaved layout)
  const int hld = a.hld;
  const unsigned rmh_lane = (unsigned)(((lane & 15) * hld + kq) * sizeof(bf16));
  auto rmh_off = [&](int bg, int j, int s) {
    return (unsigned)((((size_t)bg * 32 + 16 * j) * hld + kbase + s * 32) * sizeof(bf16));
  };

  bf16x8 w0[4][KS], w1[4][KS], x1[4][KS];
#pragma unroll
  for (int gt = 0; gt < 4; ++gt)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const size_t row = (size_t)(gt * H + ub0 + (lane & 15)) * H + kbase + s * 32 + kq;
      w0[gt][s] = ld8(a.W0T + row);
      w1[gt][s] = ld8(a.W1T + row);
      x1[gt][s] = ld8(a.X1T + row);
      if constexpr (XIN) wx0l[w][gt][s][lane] = ld8(a.X0T + row);
    }
  // the gather table slice and ids (ZTAB; read after the barrier below)
  const bool ztl = ZTAB && a.ids && a.zx_rows > 0 && a.zx_rows <= kTabMaxV && T <= kTabMaxT;
  if (ztl) {
    for (int i = threadIdx.x; i < a.zx_rows * 64; i += 256) {
      const int v = i >> 6, cc = i & 63;  // column cc = gate (cc >> 4), unit ub0 + (cc & 15)
      ztab[v * kTabLd + cc] = a.zx0[(size_t)v * a.zx_ld + (cc >> 4) * H + ub0 + (cc & 15)];
    }
    for (int i = threadIdx.x; i < T * 32; i += 256) {
      const int tk = i >> 5, r = col * 32 + (i & 31);
      idsl[i] = r < B ? a.ids[(size_t)tk * B + r] : 0;
    }
  }
  if (threadIdx.x == 0) {
    loc_s = tryloc ? xcd_decide(xw, (unsigned)nwg_u, a.spin_limit, a.err, 11u) : 0;
    if (loc_s && ubk == 0) cnt0[1] = 1u;  // (diagnostics: the column ran XCD-local)
  }
  __syncthreads();
  const bool loc = __builtin_amdgcn_readfirstlane(loc_s) != 0;

  // epilogue role: layer L, batch tile J of every group
  const int L = w >> 1, J = w & 1;
  const int u0 = ub0 + 4 * (lane >> 4);
  bf16* const hbL = L ? a.hbuf1 : a.hbuf0;
  float* const cbL = L ? a.cbuf1 : a.cbuf0;
  bf16* const gtL = L ? a.gates1 : a.gates0;
  float* const hlL = L ? a.hlast1 : a.hlast0;
  float* const clL = L ? a.clast1 : a.clast0;
  bf16* const ringL = L ? a.hring1 : a.hring0;
  // the role's bias: layer l+1's, or layer l's when its dense zx0 was written without it
  // (saves a [T·B, 4H] fp32 pass over zx0 behind the input GEMM)
  float biasL[4][4] = {};
  const float* bsrc = L ? a.bias1 : a.bias0;
  if (bsrc) {
#pragma unroll
    for (int gt = 0; gt < 4; ++gt) ld4f(bsrc + gt * H + u0, biasL[gt]);
  }
  constexpr int LAG = G == 1 ? 2 : 1;  // ticks layer l+1 runs behind layer l
  constexpr int NXS = 1;  // (unused for G > 1)
  float c[G][4];
  // (G = 1) layer l+1's input-projection partials (this wave's K quarter, [tile][gate]) for
  // its next tick
  f32x4 xs[NXS][2][4];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int b = (col * G + g) * 32 + 16 * J + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) c[g][r] = 0.f;
    if (b < B) ld4f(cbL + (size_t)b * H + u0, c[g]);  // slot 0 of cbuf (padded rows: zero)
  }
#pragma unroll
  for (int i = 0; i < NXS; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int gt = 0; gt < 4; ++gt) xs[i][j][gt] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto zx_row = [&](int tk, int g) -> const float* {
    const int b = (col * G + g) * 32 + 16 * J + (lane & 15);
    if (XIN || !(L == 0 && tk < T && b < B)) return nullptr;
    return a.ids ? a.zx0 + (size_t)a.ids[(size_t)tk * B + b] * a.zx_ld
                 : a.zx0 + ((size_t)tk * B + b) * a.zx_ld;
  };
  auto zx_load = [&](const float* zr, float (&dst)[4][4]) {
    if (zr) {
#pragma unroll
      for (int gt = 0; gt < 4; ++gt) ld4f(zr + (size_t)gt * H + u0, dst[gt]);
    }
  };
  float zxn[4][4] = {};
  // G = 1: the layer-l input projection rows are loaded one tick ahead (at the previous tick's
  // group start, behind its payload loads) and the gather ids two ticks ahead.  vmcnt retires in
  // issue order, so rows loaded at the tick start (an id load, then the dependent table row: two
  // round trips) had made the poller's first counter check wait for them every tick.
  constexpr bool ZXA = G == 1 && !XIN;
  const int bz = col * G * 32 + 16 * J + (lane & 15);  // (G = 1) this lane's row
  const bool zl = ZXA && L == 0 && bz < B && !ztl;
  int idn = 0;  // gather id of the next tick's row
  auto zx_row1 = [&](int tk, int id) -> const float* {
    return a.ids ? a.zx0 + (size_t)id * a.zx_ld : a.zx0 + ((size_t)tk * B + bz) * a.zx_ld;
  };
  if (zl) {
    const int id0 = a.ids ? a.ids[bz] : 0;
    zx_load(zx_row1(0, id0), zxn);
    if (a.ids && T > 1) idn = a.ids[(size_t)B + bz];
  }
  // G = 1: the tick keeps the compiler's waitcnt analysis exact between its payload loads and
  // its MFMAs -- straight-line, unconditional vector-memory operations only (out-of-range
  // buffer offsets / empty buffer descriptors instead of branches) -- so that the MFMA phase
  // waits for the payload alone.  That makes it free to store the previous tick's row-major
  // h / c / gates copies right behind the payload loads (their acknowledgement then overlaps
  // the MFMA and epilogue phases), instead of after the arrival, where vmcnt's in-order
  // retirement had made the poller's flag loads wait for them (4.10 -> 3.33 us per tick
  // without any row-major store, scripts/pair_bench.py).
  constexpr bool DEFER = G == 1;
  // XIN: layer l's input rows of a tick, loaded one tick ahead into registers by unconditional
  // buffer loads behind the payload (rows >= B and ticks >= T read zero); loading them at the
  // tick start had put their HBM latency in front of the poll's flag loads (vmcnt in order)
  bf16x8 xpf[XIN ? 2 : 1][XIN ? KS : 1];
  const __amdgpu_buffer_rsrc_t r_x = make_rsrc(a.x0, XIN ? sizeof(bf16) * (size_t)T * B * H : 0);
  auto x_prefetch = [&](int tk) {
    if constexpr (XIN) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bool ok = tk < T && col * 32 + 16 * j + (lane & 15) < B;
#pragma unroll
        for (int s = 0; s < KS; ++s)
          // (the offset through an opaque move: LLVM otherwise turns the select into a branch
          // around the load, and the waitcnt pass then waits for everything at its use)
          xpf[j][s] = ld8_sc1(r_x, opaque_vgpr(ok ? (unsigned)((size_t)tk * B * H * sizeof(bf16)) +
                                                        rm_lane + rm_off(col, j, s)
                                                  : 0x7FFFFFF0u));
      }
    }
  };
  x_prefetch(0);
  // (G = 1) dropout: the mask bytes of tick tk (layer l's h of step tk-1) into mlds[tk & 1],
  // DMA'd one tick ahead behind the payload loads by unconditional buffer loads (rows >= B
  // and ticks without an input mask read zero).  Issued before the poll (G > 1), the DMA sat
  // in front of the flag loads in vmcnt order, and the barrier after the poll -- which the
  // compiler makes wait for every LDS-DMA (vmcnt(0)) -- exposed its whole latency every tick.
  auto mask_dma = [&](int tk) {
    if constexpr (DROP && G == 1) {
      const int r0 = col * 32;
      const bool okt = tk >= 1 && tk <= T;
      const __amdgpu_buffer_rsrc_t rm = make_rsrc(a.xmask, sizeof(uint8_t) * (size_t)T * B * (H / 8));
#pragma unroll
      for (int k = 0; k < kMaskDw; ++k) {
        const int i0 = 256 * k + 64 * w;  // this wave's 64 dwords of the 32 rows x H/32
        const int di = i0 + lane;
        const bool ok = okt && i0 < H && r0 + di / (H / 32) < B;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rm, (__attribute__((address_space(3))) void*)&mlds[tk & 1][i0], 4,
            opaque_vgpr(ok ? (unsigned)(((size_t)(tk - 1) * B + r0) * (H / 8) + 4 * (size_t)di)
                           : 0x7FFFFFF0u),
            0, 0, 0);
      }
    }
  };
  bf16x4 rm_h = {}, rm_g[4] = {};
  float rm_c[4] = {};
  int rm_t = -1;
  const __amdgpu_buffer_rsrc_t r_h = make_rsrc(hbL, sizeof(bf16) * (size_t)(T + 1) * B * hld);
  const __amdgpu_buffer_rsrc_t r_c = make_rsrc(cbL, sizeof(float) * (size_t)(T + 1) * B * H);
  const __amdgpu_buffer_rsrc_t r_g = make_rsrc(gtL, gtL ? sizeof(bf16) * (size_t)T * B * 4 * H : 0);
  const __amdgpu_buffer_rsrc_t r_xd =
      make_rsrc(a.xdst, a.xdst ? sizeof(bf16) * (size_t)T * B * a.xdld : 0);
  const __amdgpu_buffer_rsrc_t r_od = make_rsrc(a.odst, a.odst ? sizeof(bf16) * (size_t)T * B * H : 0);
  const __amdgpu_buffer_rsrc_t r_om =
      make_rsrc(a.omask, (DROP && a.odst) ? sizeof(uint8_t) * (size_t)T * B * (H / 8) : 0);
  unsigned rm_m = 0;  // (dropout) the output-mask byte of this lane's deferred layer l+1 row
  const int brow = col * G * 32 + 16 * J + (lane & 15);  // (G = 1) this lane's row
  auto flush_rm = [&]() {
    constexpr unsigned kOut = 0x7FFFFFF0u;  // out of range: dropped
    const bool ok = rm_t >= 0 && brow < B;
    const unsigned oh = ok ? (unsigned)((((size_t)(rm_t + 1) * B + brow) * hld + u0) * sizeof(bf16)) : kOut;
    const unsigned oc = ok ? (unsigned)(((size_t)(rm_t + 1) * B * H + (size_t)brow * H + u0) * sizeof(float)) : kOut;
    const unsigned og = ok ? (unsigned)((((size_t)rm_t * B + brow) * 4 * H + u0) * sizeof(bf16)) : kOut;
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, rm_h), r_h, oh, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(
        __builtin_bit_cast(u32x4, f32x4{rm_c[0], rm_c[1], rm_c[2], rm_c[3]}), r_c, oc, 0, 0);
#pragma unroll
    for (int gt = 0; gt < 4; ++gt)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, rm_g[gt]), r_g,
                                            og + gt * H * (unsigned)sizeof(bf16), 0, 0);
    if constexpr (DROP && G == 1) {
      // layer l+1's masked input row h_l(t) ⊙ mask / keep for its weight gradient (the separate
      // mask pass over [T·B, H] otherwise): the mask bytes of step t are the ones the tick-t
      // DMA staged in mlds[(t + 1) & 1] for the stash (overwritten two ticks later)
      if (L == 0 && a.xdst) {
        const uint8_t* mb = reinterpret_cast<const uint8_t*>(mlds[(rm_t + 1) & 1]);
        const unsigned m = mb[(16 * J + (lane & 15)) * (H / 8) + (u0 >> 3)] >> (u0 & 7);
        bf16x4 xd;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          xd[r] = f2bf((m >> r & 1u) ? bf2f(rm_h[r]) * a.xscale : 0.f);
        const unsigned ox = ok ? (unsigned)((((size_t)rm_t * B + brow) * a.xdld + u0) * sizeof(bf16)) : kOut;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, xd), r_xd, ox, 0, 0);
      }
      // the top layer's output dropout rows (the head's input) from the byte loaded a tick ago
      if (L == 1 && a.odst) {
        const unsigned m = rm_m >> (u0 & 7);
        bf16x4 od;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          od[r] = f2bf((m >> r & 1u) ? bf2f(rm_h[r]) * a.oscale : 0.f);
        const unsigned oo = ok ? (unsigned)((((size_t)rm_t * B + brow) * H + u0) * sizeof(bf16)) : kOut;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, od), r_od, oo, 0, 0);
      }
    }
    rm_t = -1;
  };

  // one tick; SDY (steady): LAG + 1 <= tau <= T - 3, where every edge condition below is a
  // compile-time constant (both layers active, every slot a ring slot, no final step)
  auto tick = [&](int tau, auto sdy_c) __attribute__((always_inline)) {
    constexpr bool SDY = decltype(sdy_c)::value;
    const bool on0 = SDY || tau < T;           // layer l   computes step tau
    const bool on1 = SDY || tau >= LAG;        // layer l+1 computes step tau-LAG
    const bool ld0 = SDY || tau <= T;          // slot tau of h_l (layer l's h_{tau-1})
    const bool ld1 = on1;                      // slot tau-LAG of h_{l+1}
    const int t = L == 0 ? tau : tau - LAG;    // this role's step
    const bool act = L == 0 ? on0 : on1;
    // this role's slot t+1 is read by a later tick: layer l's up to slot T, layer l+1's up to
    // slot T-1 (by itself)
    const bool signal = act && (SDY || L == 0 || t + 1 < T);
    STAMPF(0, 0)
    // layer-l input projections of step tau (independent of the hand-off): group 0's rows are
    // loaded before the poll, group g+1's right behind group g's payload (a gathered row needs
    // its id first; loaded for all groups here, the wait overlaps the poll).  (Loading group 0's
    // rows at the end of the previous tick measured slower: 603 -> 691 us per launch.)
    const float* zrows[G];
    if constexpr (!ZXA) {
#pragma unroll
      for (int g = 0; g < G; ++g) zrows[g] = zx_row(tau, g);
      zx_load(zrows[0], zxn);
    }
    // XIN: layer l's input product of step tau (this wave's K quarter, both tiles, all gates),
    // the recurrent product is accumulated on top after the poll
    // (the rows were loaded one tick ahead, behind the previous tick's payload; zero past T)
    f32x4 xin[XIN ? 2 : 1][4];
    if constexpr (XIN) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int gt = 0; gt < 4; ++gt) xin[j][gt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int gt = 0; gt < 4; ++gt) xin[j][gt] = mfma16(wx0l[w][gt][s][lane], xpf[j][s], xin[j][gt]);
    }
    // dropout of layer l+1's input (layer l's h of step tau-1): the mask bytes of the
    // workgroup's 32G rows for this tick, DMA'd into LDS before the poll (no registers; the
    // poll barrier waits for them).  A global byte load at each use had put its latency on the
    // tick's critical path.
    const bool xdrop = DROP && ld0 && (SDY || tau >= 1);
    if (G > 1 && xdrop) {
      const int r0 = col * G * 32;
      const __amdgpu_buffer_rsrc_t rm =
          make_rsrc(a.xmask + ((size_t)(tau - 1) * B + r0) * (H / 8),
                    B > r0 ? (size_t)(B - r0) * (H / 8) : 0);  // rows >= B read as zero
#pragma unroll
      for (int k = 0; k < kMaskDw; ++k) {
        const int i0 = 256 * k + 64 * w;  // this wave's 64 dwords (G H is a multiple of 64)
        if (i0 < G * H)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rm, (__attribute__((address_space(3))) void*)&mlds[tau & 1][i0], 4,
              4 * (i0 + lane), 0, 0, 0);
      }
    }
    // hand-offs of the previous tick: layer l's slot tau, layer l+1's slot tau-LAG (slot 0 of
    // either is the prep-written initial state)
    const bool pw0 = ld0 && (SDY || tau >= 1), pw1 = ld1 && (SDY || tau >= LAG + 1);
    if (loc) {  // flags of both layers' producing ticks (tau - 1) + 1
      if ((pw0 || pw1) && w == 0 && !dead)
        dead = !poll_flags2(fl0, pw0, fl1, pw1, nwg_u, (unsigned)tau, a.spin_limit, a.err, 9u);
    } else if ((pw0 || pw1) && threadIdx.x == kLstmPollerThread && !dead) {
      dead = (pw0 && pw1) ? !poll_counter2(cnt0 + (size_t)tau * 4, target,
                                           cnt1 + (size_t)(tau - LAG) * 4, target, a.spin_limit,
                                           a.err, 9u)
                          : !poll_counter(pw0 ? cnt0 + (size_t)tau * 4
                                              : cnt1 + (size_t)(tau - LAG) * 4,
                                          target, a.spin_limit, a.err, 9u);
    }
    STAMPF(0, 1)
    // (also orders this tick's first partial stores after the previous tick's epilogue reads)
    __syncthreads();
    STAMPF(0, 2)
    // payload fragments of group g: slot 0 is row-major [B, H] (rows >= B read as zero: buffer
    // bounds); later slots come from the fragment-tiled rings: one contiguous 1 KB load per
    // (tile, k-step).  Double-buffered by group: group g+1's loads are issued before group g's
    // MFMAs (the column's hand-off covers all its groups), so their latency overlaps group g's
    // MFMA and epilogue phases instead of opening group g+1's.
    // (only while the second buffer fits: at KS = 4 it spilled from G = 2 on -- G = 2 without it,
    // spill-free: 3.10 vs 3.24 ms per step at B = 512, same box)
    constexpr bool PREF = G > 1 && KS * G <= 8 && KS < 4;
    bf16x8 pf0[PREF ? 2 : 1][2][KS], pf1[PREF ? 2 : 1][2][KS];
    auto load_group = [&](int g, bf16x8 (&hf0)[2][KS], bf16x8 (&hf1)[2][KS]) {
      const int bg = col * G + g;
      if constexpr (G == 1) {  // unconditional: a skipped layer reads an empty descriptor
        const bool ring0 = SDY || tau > 0;
        const __amdgpu_buffer_rsrc_t r0 =
            !ld0 ? make_rsrc(a.hring0, 0)
                 : ring0 ? make_rsrc(a.hring0 + (size_t)(tau & 1) * ringsz, sizeof(bf16) * ringsz)
                         : make_rsrc(a.hbuf0, sizeof(bf16) * (size_t)B * hld);
        const int s1 = tau - LAG;
        const bool ring1 = SDY || s1 > 0;
        const __amdgpu_buffer_rsrc_t r1 =
            !ld1 ? make_rsrc(a.hring1, 0)
                 : ring1 ? make_rsrc(a.hring1 + (size_t)(s1 & 1) * ringsz, sizeof(bf16) * ringsz)
                         : make_rsrc(a.hbuf1, sizeof(bf16) * (size_t)B * hld);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const unsigned of = frag_load_off(2 * bg + j, w * KS + s, H, lane);
            const unsigned orow = rmh_lane + rmh_off(bg, j, s);
            hf0[j][s] = ld8_sc1(r0, ring0 ? of : orow);
            hf1[j][s] = ld8_sc1(r1, ring1 ? of : orow);
          }
        return;
      }
      if (ld0) {
        const bool ring0 = SDY || tau > 0;
        const __amdgpu_buffer_rsrc_t r0 =
            ring0 ? make_rsrc(a.hring0 + (size_t)(tau & 1) * ringsz, sizeof(bf16) * ringsz)
                  : make_rsrc(a.hbuf0, sizeof(bf16) * (size_t)B * hld);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < KS; ++s)
            hf0[j][s] = ring0 ? ld8_sc1(r0, frag_load_off(2 * bg + j, w * KS + s, H, lane))
                              : ld8_sc1(r0, rmh_lane + rmh_off(bg, j, s));
      }
      if (ld1) {
        const int s1 = tau - LAG;
        const bool ring1 = SDY || s1 > 0;
        const __amdgpu_buffer_rsrc_t r1 =
            ring1 ? make_rsrc(a.hring1 + (size_t)(s1 & 1) * ringsz, sizeof(bf16) * ringsz)
                  : make_rsrc(a.hbuf1, sizeof(bf16) * (size_t)B * hld);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < KS; ++s)
            hf1[j][s] = ring1 ? ld8_sc1(r1, frag_load_off(2 * bg + j, w * KS + s, H, lane))
                              : ld8_sc1(r1, rmh_lane + rmh_off(bg, j, s));
      }
    };
    load_group(0, pf0[0], pf1[0]);
    if constexpr (DEFER) flush_rm();  // the previous tick's row-major copies
    if constexpr (DROP && G == 1) mask_dma(tau + 1);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      STAMPF(g, 7)  // group phase start
      const int bg = col * G + g;
      const int b = bg * 32 + 16 * J + (lane & 15);
      const bool live = b < B;
      const size_t bh = (size_t)b * H + u0;
      float zx[4][4];
#pragma unroll
      for (int gt = 0; gt < 4; ++gt)
#pragma unroll
        for (int r = 0; r < 4; ++r) zx[gt][r] = zxn[gt][r];
      if (ZTAB && ztl && L == 0 && on0) {  // this row's table entry (padded rows: id 0, unused)
        const float* zt = &ztab[idsl[tau * 32 + 16 * J + (lane & 15)] * kTabLd + 4 * (lane >> 4)];
#pragma unroll
        for (int gt = 0; gt < 4; ++gt) {
          const float4 v = *reinterpret_cast<const float4*>(zt + 16 * gt);
          zx[gt][0] = v.x; zx[gt][1] = v.y; zx[gt][2] = v.z; zx[gt][3] = v.w;
        }
      }
      bf16x8 (&hf0)[2][KS] = pf0[PREF ? (g & 1) : 0];
      bf16x8 (&hf1)[2][KS] = pf1[PREF ? (g & 1) : 0];
      if constexpr (PREF) {
        if (g + 1 < G) load_group(g + 1, pf0[(g + 1) & 1], pf1[(g + 1) & 1]);
      } else {
        if (g > 0) load_group(g, pf0[0], pf1[0]);
      }
      if constexpr (XIN) x_prefetch(tau + 1);
      if constexpr (ZXA) {
        // the next tick's row (and the id of the one after), behind this tick's payload loads
        if (zl && (SDY || tau + 1 < T)) {
          zx_load(zx_row1(tau + 1, idn), zxn);
          if (a.ids && (SDY || tau + 2 < T)) idn = a.ids[(size_t)(tau + 2) * B + bz];
        }
      } else {
        if (g + 1 < G) zx_load(zrows[g + 1], zxn);
      }
      // mask byte of this lane's x-part fragment (row 16 j + lane%16 of the group, k = kbase +
      // 32 s + kq .. +7), from the LDS stage (read at its use: no register is held for it
      // across the payload phase)
      auto mbyte = [&](int j, int s2) -> unsigned {
        const uint8_t* m = reinterpret_cast<const uint8_t*>(mlds[tau & 1]);
        return m[(g * 32 + 16 * j + (lane & 15)) * (H / 8) + ((kbase + s2 * 32 + kq) >> 3)];
      };
      if (g > 0) __syncthreads();  // the previous group's epilogue has read the partials
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if (on0) {
          f32x4 acc[4];
#pragma unroll
          for (int gt = 0; gt < 4; ++gt) {
            if constexpr (XIN) {
              acc[gt] = xin[j][gt];
            } else {
              acc[gt] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
          }
#pragma unroll
          for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int gt = 0; gt < 4; ++gt) acc[gt] = mfma16(w0[gt][s], hf0[j][s], acc[gt]);
          float* dst = &part[w][0][j][0][lane][0];
#pragma unroll
          for (int gt = 0; gt < 4; ++gt)
            *reinterpret_cast<float4*>(dst + gt * 256) =
                make_float4(acc[gt][0], acc[gt][1], acc[gt][2], acc[gt][3]);
        }
        if (on1) {  // input part (stashed last tick for G = 1) + recurrent part
          f32x4 acc[4];
#pragma unroll
          for (int gt = 0; gt < 4; ++gt) {
            if constexpr (G == 1) {
              acc[gt] = xs[0][j][gt];
            } else {
              acc[gt] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
          }
          if constexpr (G > 1) {
            if (xdrop) {  // masked input part, scaled by 1/keep, then the recurrent part
#pragma unroll
              for (int s = 0; s < KS; ++s) {
                const bf16x8 hm = mask_frag(hf0[j][s], mbyte(j, s));
#pragma unroll
                for (int gt = 0; gt < 4; ++gt) acc[gt] = mfma16(x1[gt][s], hm, acc[gt]);
              }
#pragma unroll
              for (int gt = 0; gt < 4; ++gt) acc[gt] *= a.xscale;
#pragma unroll
              for (int s = 0; s < KS; ++s)
#pragma unroll
                for (int gt = 0; gt < 4; ++gt) acc[gt] = mfma16(w1[gt][s], hf1[j][s], acc[gt]);
            } else {
#pragma unroll
              for (int s = 0; s < KS; ++s)
#pragma unroll
                for (int gt = 0; gt < 4; ++gt) {
                  acc[gt] = mfma16(x1[gt][s], hf0[j][s], acc[gt]);
                  acc[gt] = mfma16(w1[gt][s], hf1[j][s], acc[gt]);
                }
            }
          } else {
#pragma unroll
            for (int s = 0; s < KS; ++s)
#pragma unroll
              for (int gt = 0; gt < 4; ++gt) acc[gt] = mfma16(w1[gt][s], hf1[j][s], acc[gt]);
          }
          float* dst = &part[w][1][j][0][lane][0];
#pragma unroll
          for (int gt = 0; gt < 4; ++gt)
            *reinterpret_cast<float4*>(dst + gt * 256) =
                make_float4(acc[gt][0], acc[gt][1], acc[gt][2], acc[gt][3]);
        }
      }
      STAMPF(g, 3)
      __syncthreads();
      STAMPF(g, 4)
      // (G = 1) layer l+1's x-part of its step tau-1 (next tick) from slot tau of layer l
      auto do_stash = [&]() {
        if constexpr (G == 1) {
          if (ld0 && (SDY || tau >= 1)) {
            // dropout: the mask dwords of this lane's fragments, all read before any use (one
            // LDS wait; a byte read at each use had serialised 8 LDS round trips); the byte of
            // fragment (j, s) is byte lane/16 of dword s of its row's K range
            unsigned mw[2][KS];
            if (xdrop) {
              const unsigned* mr = &mlds[tau & 1][(kbase >> 5)];
#pragma unroll
              for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int s = 0; s < KS; ++s) mw[j][s] = mr[(16 * j + (lane & 15)) * (H / 32) + s];
              __builtin_amdgcn_sched_barrier(0);  // (keeps the reads together, ahead of the uses)
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
#pragma unroll
              for (int gt = 0; gt < 4; ++gt) xs[0][j][gt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
              for (int s = 0; s < KS; ++s) {
                const bf16x8 hm =
                    xdrop ? mask_frag_fast(hf0[j][s], (mw[j][s] >> (8 * (lane >> 4))) & 0xFFu)
                          : hf0[j][s];
#pragma unroll
                for (int gt = 0; gt < 4; ++gt) xs[0][j][gt] = mfma16(x1[gt][s], hm, xs[0][j][gt]);
              }
              if (xdrop) {
#pragma unroll
                for (int gt = 0; gt < 4; ++gt) xs[0][j][gt] *= a.xscale;
              }
            }
          }
        }
      };
      if (act) {
        float z[4][4];
#pragma unroll
        for (int gt = 0; gt < 4; ++gt) {
          const float4 s0 = *reinterpret_cast<const float4*>(&part[0][L][J][gt][lane][0]);
          const float4 s1 = *reinterpret_cast<const float4*>(&part[1][L][J][gt][lane][0]);
          const float4 s2 = *reinterpret_cast<const float4*>(&part[2][L][J][gt][lane][0]);
          const float4 s3 = *reinterpret_cast<const float4*>(&part[3][L][J][gt][lane][0]);
          float add[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) add[r] = L == 0 ? zx[gt][r] + biasL[gt][r] : biasL[gt][r];
          z[gt][0] = s0.x + s1.x + s2.x + s3.x + add[0];
          z[gt][1] = s0.y + s1.y + s2.y + s3.y + add[1];
          z[gt][2] = s0.z + s1.z + s2.z + s3.z + add[2];
          z[gt][3] = s0.w + s1.w + s2.w + s3.w + add[3];
        }
        float gi[4], gj[4], gf[4], go[4], h[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          gi[r] = sigmoidf_(z[0][r]);
          gj[r] = tanhf_(z[1][r]);
          gf[r] = sigmoidf_(z[2][r] + a.forget_bias);
          go[r] = sigmoidf_(z[3][r]);
          c[g][r] = gf[r] * c[g][r] + gi[r] * gj[r];
          h[r] = go[r] * tanhf_(c[g][r]);
        }
        STAMPF(g, 5)
        st4bf_ho(loc, ringL + (size_t)((t + 1) & 1) * ringsz + frag_index(b, u0, H), h[0], h[1],
                 h[2], h[3]);
        // the stash MFMAs run while the ring stores drain (with dropout too, now that its mask
        // reads are batched and the masking is 5 VALU ops per dword: 1.856 vs 1.860 ms with the
        // stash behind the arrival, same box)
        do_stash();
        if (g == G - 1 && signal) {
          // one arrival per wave and tick, for all its groups' ring stores
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          STAMPF(g, 6)
          if (lane == 0) {
            unsigned* const c = (L ? cnt1 : cnt0) + (size_t)(t + 1) * 4;
            if (loc)
              wg_arrive_flag(&arrl[L], 2u, (L ? fl1 : fl0) + ubk, (unsigned)tau + 1u);
            else if (a.wgarr)
              wg_arrive(&arrl[L], 2u, c);
            else
              __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        }
        if (DEFER) {  // row-major copies: stored behind the next tick's payload loads
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            rm_h[r] = f2bf(h[r]);
            rm_c[r] = c[g][r];
            rm_g[0][r] = f2bf(gi[r]); rm_g[1][r] = f2bf(gj[r]);
            rm_g[2][r] = f2bf(gf[r]); rm_g[3][r] = f2bf(go[r]);
          }
          rm_t = t;
          if constexpr (DROP) {
            if (L == 1 && a.odst)  // consumed by the next tick's flush (rows >= B read zero)
              rm_m = __builtin_amdgcn_raw_buffer_load_b8(
                  r_om, live ? (unsigned)(((size_t)t * B + b) * (H / 8) + (u0 >> 3)) : 0x7FFFFFF0u, 0, 0);
          }
          if (live && (!SDY && t == T - 1) && hlL)
            *reinterpret_cast<float4*>(hlL + bh) = make_float4(h[0], h[1], h[2], h[3]);
          if (live && (!SDY && t == T - 1) && clL)
            *reinterpret_cast<float4*>(clL + bh) = make_float4(c[g][0], c[g][1], c[g][2], c[g][3]);
        } else if (live) {  // row-major copies for the GEMMs / head (not handed off)
          const size_t o = (size_t)(t + 1) * B * H + bh;
          st4bf(hbL + ((size_t)(t + 1) * B + b) * hld + u0, h[0], h[1], h[2], h[3]);
          *reinterpret_cast<float4*>(cbL + o) = make_float4(c[g][0], c[g][1], c[g][2], c[g][3]);
          if (gtL) {
            bf16* gp = gtL + ((size_t)t * B + b) * 4 * H + u0;
            st4bf(gp, gi[0], gi[1], gi[2], gi[3]);
            st4bf(gp + H, gj[0], gj[1], gj[2], gj[3]);
            st4bf(gp + 2 * H, gf[0], gf[1], gf[2], gf[3]);
            st4bf(gp + 3 * H, go[0], go[1], go[2], go[3]);
          }
          if ((!SDY && t == T - 1) && hlL)
            *reinterpret_cast<float4*>(hlL + bh) = make_float4(h[0], h[1], h[2], h[3]);
          if ((!SDY && t == T - 1) && clL)
            *reinterpret_cast<float4*>(clL + bh) = make_float4(c[g][0], c[g][1], c[g][2], c[g][3]);
        }
      } else {
        do_stash();  // waves without an epilogue this tick
      }
    }
    };
  {
    using sdy_t = std::integral_constant<bool, true>;
    using edge_t = std::integral_constant<bool, false>;
    const int sdy_lo = LAG + 1, sdy_hi = a.steady ? T - 3 : -1;  // (steady range)
    int tau = 0;
    for (; tau <= T + LAG - 1 && tau < sdy_lo; ++tau) tick(tau, edge_t{});
    for (; tau <= sdy_hi; ++tau) tick(tau, sdy_t{});
    for (; tau <= T + LAG - 1; ++tau) tick(tau, edge_t{});
  }
  if constexpr (DEFER) flush_rm();
}

// ------------------------------------------------------------------------------------------
// two-layer wavefront BPTT
// ------------------------------------------------------------------------------------------
// Reference: tf.gradients through the unrolled two-layer stack (model.py:72, 91).  Layer l's
// step t needs only layer l+1's dZ_t (its dtop) and its own dZ_{t+1}, so one launch runs both as
// a reverse wavefront: at tick tau layer l+1 computes step T-1-tau and layer l step T+1-tau (two
// ticks behind).  The slot dZ_{l+1}[T-tau] loaded for layer l+1's recurrence is also layer l's
// dtop operand one tick later: its W_x,l+1 product (fragments in LDS) runs after the group's
// epilogue, off the critical path, so the dX GEMM disappears.  T+2 ticks replace 2T steps.
//
// K = 4H is split by hidden-unit quarter: wave w reduces over the columns g*H + [w*H/4,
// (w+1)*H/4) of every gate g and keeps the W_h,l / W_h,l+1 rows of its units for that K quarter
// in registers (W_x,l+1 in LDS).  Wave w runs the cell-backward epilogue of layer w>>1 (0 = l,
// 1 = l+1), batch tile w&1, of every group.
template <int KS, int G, bool DROP>
__global__ void __launch_bounds__(256, 1) lstm2_bwd_persist_kernel(Lstm2BwdArgs a) {
  // partials [wave][layer][tile][lane][unit r]: single-buffered -- every group phase that
  // writes them starts with a barrier, which each epilogue wave joins after its reads
  __shared__ __attribute__((aligned(16))) float part[4][2][2][64][4];
  // bias-gradient accumulators of each epilogue lane (all its groups' rows), kept in LDS
  // (registers are the limit: 2 x KS weight and 3 x KS payload fragments live across the MFMA
  // phase)
  __shared__ float dbl[4][16][64];
  // layer l's dtop partial (this wave's K quarter, both tiles) of each group for its NEXT tick,
  // computed off the critical path after the group's epilogue from its dZ_{l+1} fragments
  __shared__ __attribute__((aligned(16))) float xsl[G][4][2][64][4];
  // dc carry of each epilogue lane, per group
  __shared__ __attribute__((aligned(16))) float dcs[G][4][64][4];
  // W_x,l+1 fragments [wave][k-step][lane] (64 KB at H = 512): only the off-critical-path stash
  // product reads them, so they live in LDS and leave the registers to W_h,l / W_h,l+1 and the
  // payload
  __shared__ __attribute__((aligned(16))) bf16x8 wx1l[4][KS][64];
  __shared__ unsigned short mb16[DROP ? G * 32 : 1];  // dropout bits of the tick (see mdrop)
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int G4H = 4 * H;
  int ubk, col;
  if (!map_block_grid(blockIdx.x, gridDim.x, H / 16, a.nbg / G, ubk, col)) return;  // padding
  const int ub0 = ubk * 16;
  const int kq = 8 * (lane >> 4);
  unsigned* cnt0 = a.cnt0 + (size_t)col * (T + 1) * 4;
  unsigned* cnt1 = a.cnt1 + (size_t)col * (T + 1) * 4;
  unsigned long long* const xw = reinterpret_cast<unsigned long long*>(cnt0 + 2);
  const bool tryloc = a.xcdloc && a.wgarr && T >= 8 && H / 16 <= 32;
  if (tryloc && threadIdx.x == 0) xcd_publish(xw);
  unsigned* const fl0 = cnt0 + 4;  // (local form) per-workgroup flags of layer l / l+1
  unsigned* const fl1 = cnt1 + 4;
  // arrivals per (column, slot) and layer: H/16 unit blocks x (one per workgroup | 2 waves)
  const unsigned target = (unsigned)(a.wgarr ? H / 16 : H / 8);
  __shared__ unsigned arrl[2];  // per-layer arrivals of the tick (wgarr)
  __shared__ int loc_s;
  if (threadIdx.x < 2) arrl[threadIdx.x] = 0u;  // (ordered before any add by tick 0's barrier)
  const size_t slabn = (size_t)a.nbg * 32 * G4H;  // one ring slot (padded batch), elements
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
  if (threadIdx.x == 0) {
    loc_s = tryloc ? xcd_decide(xw, (unsigned)(H / 16), a.spin_limit, a.err, 12u) : 0;
    if (loc_s && ubk == 0) cnt0[1] = 1u;  // (diagnostics: the column ran XCD-local)
  }
  __syncthreads();
  const bool loc = __builtin_amdgcn_readfirstlane(loc_s) != 0;

  // epilogue role: layer L, batch tile J of every group
  const int L = w >> 1, J = w & 1;
  const int u0 = ub0 + 4 * (lane >> 4);
  const bf16* const gtL = L ? a.gates1 : a.gates0;
  const float* const cbL = L ? a.cbuf1 : a.cbuf0;
  bf16* const dzL = L ? a.dz1 : a.dz0;
  bf16* const zrL = L ? a.zring1 : a.zring0;
  unsigned* const cntL = L ? cnt1 : cnt0;
#pragma unroll
  for (int i = 0; i < 16; ++i) dbl[w][i][lane] = 0.f;
#pragma unroll
  for (int g = 0; g < G; ++g)
    *reinterpret_cast<float4*>(&dcs[g][w][lane][0]) = make_float4(0.f, 0.f, 0.f, 0.f);

  for (int tau = 0; tau <= T + 1; ++tau) {
    const bool on1 = tau < T;                 // layer l+1 computes step T-1-tau
    const bool on0 = tau >= 2;                // layer l computes step T+1-tau (two ticks behind)
    const bool ld1 = tau >= 1 && tau <= T;    // dZ_{l+1}[T-tau] (published at tick tau-1)
    const bool ld0 = tau >= 3;                // dZ_l[T+2-tau]   (published at tick tau-1)
    const int t = L ? T - 1 - tau : T + 1 - tau;  // this role's step
    const bool act = L ? on1 : on0;
    // dropout of layer l's dtop (layer l+1's input mask, step T+1-tau): the 16 units' bits of
    // the workgroup's 32G rows, loaded here and staged in LDS after the poll (read in the MFMA
    // phases, each followed by a barrier: one buffer)
    const bool mdrop = DROP && on0;
    unsigned short mreg = 0;
    if (mdrop && threadIdx.x < G * 32) {
      const int r = col * G * 32 + threadIdx.x;
      if (r < B)
        mreg = *reinterpret_cast<const unsigned short*>(
            a.xmask + ((size_t)(T + 1 - tau) * B + r) * (H / 8) + (ub0 >> 3));
    }
    // (a rolled loop: unrolled, the scheduler hoists the next group's operand loads into this
    // group's MFMA phase and the KS = 16 kernel spills)
#pragma unroll 1
    for (int g = 0; g < G; ++g) {
      const int b = (col * G + g) * 32 + 16 * J + (lane & 15);
      const bool live = b < B;
      const size_t bh = (size_t)b * H + u0;
      STAMPG(g, 0)
      // recurrence-independent epilogue operands, issued before the wait (padded rows: zero)
      // (gates stay packed bf16 until the epilogue: registers are the limit here)
      bf16x4 g4[4];
      float cc[4] = {0.f, 0.f, 0.f, 0.f}, cp[4] = {0.f, 0.f, 0.f, 0.f};
      float dtop[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int gt = 0; gt < 4; ++gt)
#pragma unroll
        for (int r = 0; r < 4; ++r) g4[gt][r] = (bf16)0.f;
      if (act && live) {
        const bf16* gp = gtL + ((size_t)t * B + b) * G4H + u0;
#pragma unroll
        for (int gt = 0; gt < 4; ++gt) g4[gt] = *reinterpret_cast<const bf16x4*>(gp + gt * H);
        ld4f(cbL + (size_t)(t + 1) * B * H + bh, cc);
        ld4f(cbL + (size_t)t * B * H + bh, cp);
        if (L) ld4f(a.dtop1 + (size_t)t * B * H + bh, dtop);
      }
      // after_arrive runs right after the wave's ring stores (and, for the last group, its
      // hand-off arrival), before its other stores
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
        float dc[4];
        ld4f(&dcs[g][w][lane][0], dc);
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
        *reinterpret_cast<float4*>(&dcs[g][w][lane][0]) = make_float4(dc[0], dc[1], dc[2], dc[3]);
        STAMPG(g, 5)
        // layer l+1's dZ_t feeds both layers at the next tick (t >= 0); layer l's only itself
        if (L || t >= 1) {
          bf16* const zr = zrL + (size_t)(t & 1) * slabn;
          st4bf_ho(loc, zr + frag_index(b, u0, G4H), di[0], di[1], di[2], di[3]);
          st4bf_ho(loc, zr + frag_index(b, H + u0, G4H), dj[0], dj[1], dj[2], dj[3]);
          st4bf_ho(loc, zr + frag_index(b, 2 * H + u0, G4H), df_[0], df_[1], df_[2], df_[3]);
          st4bf_ho(loc, zr + frag_index(b, 3 * H + u0, G4H), dO[0], dO[1], dO[2], dO[3]);
          if (g == G - 1) {  // one arrival per wave and tick, for all its groups' ring stores
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            STAMPG(g, 6)
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
        }
        after_arrive();
        // row-major copy for the weight GEMMs, after the arrival (off the critical path)
        if (live) {
          bf16* dz = dzL + ((size_t)t * B + b) * G4H + u0;
          st4bf(dz, di[0], di[1], di[2], di[3]);
          st4bf(dz + H, dj[0], dj[1], dj[2], dj[3]);
          st4bf(dz + 2 * H, df_[0], df_[1], df_[2], df_[3]);
          st4bf(dz + 3 * H, dO[0], dO[1], dO[2], dO[3]);
        }
        // bias gradient of the bf16-rounded dz, exactly as the weight GEMMs see it (padded rows
        // add zero)
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
        if (g == 0) {  // the column's hand-off of the previous tick, for all groups
          if (loc) {  // flags of both layers' producing tick (tau - 1) + 1
            if (w == 0 && !dead && (ld1 || ld0))
              dead = !poll_flags2(fl0, ld0, fl1, ld1, H / 16, (unsigned)tau, a.spin_limit, a.err,
                                  10u);
          } else if (threadIdx.x == kLstmPollerThread && !dead && (ld1 || ld0)) {
            dead = (ld1 && ld0)
                       ? !poll_counter2(cnt1 + (size_t)s1 * 4, target, cnt0 + (size_t)s0 * 4,
                                        target, a.spin_limit, a.err, 10u)
                       : !poll_counter(ld1 ? cnt1 + (size_t)s1 * 4 : cnt0 + (size_t)s0 * 4,
                                       target, a.spin_limit, a.err, 10u);
          }
          if (mdrop && threadIdx.x < G * 32) mb16[threadIdx.x] = mreg;
          STAMPG(g, 1)
        }
        // (for g > 0: the previous group's epilogue has read the partials)
        __syncthreads();
        STAMPG(g, 2)
        const size_t slab = sizeof(bf16) * slabn;
        const __amdgpu_buffer_rsrc_t r1 = make_rsrc(a.zring1 + (size_t)(s1 & 1) * slabn, slab);
        const __amdgpu_buffer_rsrc_t r0 = make_rsrc(a.zring0 + (size_t)(s0 & 1) * slabn, slab);
        const int tile0 = 2 * (col * G + g);
        // register budget (one wave per SIMD, <= ~450 VGPR+AGPR without spills): 2 x KS weight
        // fragments + 3 x KS payload fragments in flight (both tiles of dZ_{l+1}, tile 0 of
        // dZ_l); tile 1 of dZ_l is issued once tile 0's fragments are consumed
        bf16x8 p0[KS];
        if (ld1) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int s = 0; s < KS; ++s)
              p1[j][s] = ld8_sc1(r1, frag_load_off(tile0 + j, kcol(s) >> 5, G4H, lane));
        }
        if (ld0) {
#pragma unroll
          for (int s = 0; s < KS; ++s)
            p0[s] = ld8_sc1(r0, frag_load_off(tile0, kcol(s) >> 5, G4H, lane));
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
            float4 x0 = *reinterpret_cast<const float4*>(&xsl[g][w][j][lane][0]);
            if constexpr (DROP) {
              // dropout of layer l+1's input on layer l's dtop (step T+1-tau): this lane's 4
              // units' bits from the LDS stage
              const unsigned m = (unsigned)mb16[g * 32 + 16 * j + (lane & 15)] >> (u0 - ub0);
              x0.x = m & 1u ? x0.x * a.xscale : 0.f;
              x0.y = m & 2u ? x0.y * a.xscale : 0.f;
              x0.z = m & 4u ? x0.z * a.xscale : 0.f;
              x0.w = m & 8u ? x0.w * a.xscale : 0.f;
            }
            f32x4 acc0 = f32x4{x0.x, x0.y, x0.z, x0.w};
            if (ld0) {
#pragma unroll
              for (int s = 0; s < KS; ++s) acc0 = mfma16(wh0[s], p0[s], acc0);
              if (j == 0) {
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int s = 0; s < KS; ++s)
                  p0[s] = ld8_sc1(r0, frag_load_off(tile0 + 1, kcol(s) >> 5, G4H, lane));
              }
            }
            *reinterpret_cast<float4*>(&part[w][0][j][lane][0]) =
                make_float4(acc0[0], acc0[1], acc0[2], acc0[3]);
          }
        }
        STAMPG(g, 3)
        __syncthreads();
        STAMPG(g, 4)
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
              *reinterpret_cast<float4*>(&xsl[g][w][j][lane][0]) = make_float4(x[0], x[1], x[2], x[3]);
            }
          }
          stashed = true;
        };
        if (act) epilogue(do_stash);
        if (!stashed) do_stash();
      } else if (act) {
        epilogue([] {});
      }
      STAMPG(g, 7)  // group phase end
    }
  }
  // bias-gradient partial of this role's 16-row tile column: reduce the 16 batch lanes
  float* const dbp = L ? a.db_part1 : a.db_part0;
  if (dbp) {
#pragma unroll
    for (int gt = 0; gt < 4; ++gt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = dbl[w][gt * 4 + r][lane];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        if ((lane & 15) == 0) dbp[(size_t)(2 * col + J) * G4H + gt * H + u0 + r] = v;
      }
  }
}

// DROP: the dropout instantiation (layer l+1's input masks in-kernel); without dropout that
// code is compiled out (same-box A/B: the runtime-conditional form cost 2.5 % per step)
template <int KS, bool DROP>
static const void* lstm2_fwd_g(int G, bool xin, bool diag) {
  if (xin)
    return G != 1 ? nullptr
           : diag ? (const void*)lstm2_fwd_persist_kernel<KS, 1, DROP, true, true>
                  : (const void*)lstm2_fwd_persist_kernel<KS, 1, DROP, true, false>;
  switch (G) {
    case 1:
      // (the stamped instantiation exists for the stamp-diagnosed shape only)
      if (diag) return (const void*)lstm2_fwd_persist_kernel<KS, 1, DROP, false, true>;
      return (const void*)lstm2_fwd_persist_kernel<KS, 1, DROP, false, false>;
    case 2: return (const void*)lstm2_fwd_persist_kernel<KS, 2, DROP, false, false>;
    case 3: return (const void*)lstm2_fwd_persist_kernel<KS, 3, DROP, false, false>;
    case 4: return (const void*)lstm2_fwd_persist_kernel<KS, 4, DROP, false, false>;
  }
  return nullptr;
}

template <bool DROP>
static const void* lstm2_pick_t(int H, int G, bool xin, bool diag) {
  switch (H / 128) {
    case 1: return lstm2_fwd_g<1, DROP>(G, xin, diag);
    case 2: return lstm2_fwd_g<2, DROP>(G, xin, diag);
    case 3: return lstm2_fwd_g<3, DROP>(G, xin, diag);
    case 4: return lstm2_fwd_g<4, DROP>(G, xin, diag);
  }
  return nullptr;
}
static const void* lstm2_pick(int H, int G, bool drop, bool xin = false, bool diag = false) {
  return drop ? lstm2_pick_t<true>(H, G, xin, diag) : lstm2_pick_t<false>(H, G, xin, diag);
}

// the in-kernel input projection variant exists and is co-resident (G = 1 only); the answer
// per (H, cus) is cached (the launcher asks on every step)
bool lstm2_xin_ok(int H, int cus) {
  static int cache_key = -1, cache_val = 0;
  const int key = H * 4096 + cus;
  if (key == cache_key) return cache_val != 0;
  cache_key = key;
  cache_val = 0;
  for (int drop = 0; drop < 2; ++drop) {
    const void* fn = lstm2_pick(H, 1, drop, true);
    int o = 0;
    if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, 256, 0) != hipSuccess || o < 1)
      return false;
  }
  cache_val = cus > 0;
  return cache_val != 0;
}

template <int KS, bool DROP>
static const void* lstm2_bwd_g(int G) {
  switch (G) {
    case 1: return (const void*)lstm2_bwd_persist_kernel<KS, 1, DROP>;
    case 2: return (const void*)lstm2_bwd_persist_kernel<KS, 2, DROP>;
    case 3: return (const void*)lstm2_bwd_persist_kernel<KS, 3, DROP>;
    case 4: return (const void*)lstm2_bwd_persist_kernel<KS, 4, DROP>;
  }
  return nullptr;
}

template <bool DROP>
static const void* lstm2_bwd_pick_t(int H, int G) {
  switch (H / 32) {  // KS = 4H / 4 waves / 32
    case 4: return lstm2_bwd_g<4, DROP>(G);
    case 8: return lstm2_bwd_g<8, DROP>(G);
    case 12: return lstm2_bwd_g<12, DROP>(G);
    case 16: return lstm2_bwd_g<16, DROP>(G);
  }
  return nullptr;
}
static const void* lstm2_bwd_pick(int H, int G, bool drop) {
  return drop ? lstm2_bwd_pick_t<true>(H, G) : lstm2_bwd_pick_t<false>(H, G);
}

static bool lstm2_fits(int H, int G, int cols, int cus) {
  // every instantiation a launch at (H, G) may use must be co-resident
  const void* fns[4] = {lstm2_pick(H, G, false), lstm2_bwd_pick(H, G, false),
                        lstm2_pick(H, G, true), lstm2_bwd_pick(H, G, true)};
  for (const void* fn : fns) {
    int o = 0;
    if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, 256, 0) != hipSuccess || o < 1)
      return false;
    if ((H / 16) * cols > o * cus) return false;
  }
  return true;
}

// Smallest G (batch groups per workgroup) whose grid of (H/16) x ceil(nbg/G) workgroups is
// co-resident for both kernels; 0 if none.  `force` (> 0) pins G.
int lstm2_plan_g(int H, int B, int cus, int force) {
  if (H % 128 != 0 || H < 128 || H > 512 || B < 1 || cus <= 0) return 0;
  const int nbg = (B + 31) / 32;
  for (int G = force > 0 ? force : 1; G <= kPairMaxG; ++G) {
    if (lstm2_fits(H, G, (nbg + G - 1) / G, cus)) return G;
    if (force > 0) return 0;
  }
  return 0;
}

// the XCD-padded grid (persist_common.h xcd_grid) when it is co-resident, else the plain one
static int lstm2_grid(const void* fn, const int H, const int nbg, const int G, const int cus) {
  const int plain = (H / 16) * (nbg / G), padded = xcd_grid(H / 16, nbg / G);
  int o = 0;
  if (padded != plain && hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, 256, 0) == hipSuccess &&
      padded <= o * cus)
    return padded;
  return plain;
}

static bool lstm2_args_ok(int H, int B, int nbg, int G, int cus) {
  if (G < 1 || G > kPairMaxG || nbg % G != 0 || nbg * 32 < B) return false;
  return lstm2_plan_g(H, B, cus, G) == G;
}

int launch_lstm2_fwd_persist(const Lstm2Args& a, int cus, hipStream_t s) {
  if (!lstm2_args_ok(a.H, a.B, a.nbg, a.G, cus) || !a.hring0 || !a.hring1) return -2;
  void* args[] = {const_cast<Lstm2Args*>(&a)};
  if (a.x0 && (a.G != 1 || !lstm2_xin_ok(a.H, cus))) return -2;
  const void* fn = lstm2_pick(a.H, a.G, a.xmask != nullptr, a.x0 != nullptr, a.diag != nullptr);
  return hipLaunchKernel(fn, dim3(lstm2_grid(fn, a.H, a.nbg, a.G, cus)), dim3(256), args, 0, s) ==
                 hipSuccess ? 0 : -3;
}

int launch_lstm2_bwd_persist(const Lstm2BwdArgs& a, int cus, hipStream_t s) {
  if (!lstm2_args_ok(a.H, a.B, a.nbg, a.G, cus)) return -2;
  void* args[] = {const_cast<Lstm2BwdArgs*>(&a)};
  const void* fn = lstm2_bwd_pick(a.H, a.G, a.xmask != nullptr);
  return hipLaunchKernel(fn, dim3(lstm2_grid(fn, a.H, a.nbg, a.G, cus)), dim3(256), args, 0, s) ==
                 hipSuccess ? 0 : -3;
}

}  // namespace dcr
