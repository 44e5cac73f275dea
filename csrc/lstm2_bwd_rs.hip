// Two-layer wavefront LSTM BPTT with a reduce-scatter hand-off (gfx950).
//
// Reference: tf.gradients through the unrolled two-layer stack (model.py:72, 91) -- the same
// schedule and tile as lstm2_bwd_wide.hip (workgroup = 32 hidden units x 16 batch rows of both
// layers, layer l+1 and layer l advancing together); what changes is WHAT crosses workgroups.
//
// lstm2_bwd_wide.hip hands off the dZ rows themselves (all-gather): every tick a workgroup reads
// the 4H-wide dZ rows of its 16 batch rows for both layers -- 128 KB, the same bytes as the 15
// other unit blocks of its column, all at once (the tick's payload + MFMA phase: 58 % of a 4.6 us
// tick, scripts/pair_bench.py --stamps) -- and multiplies them by its resident W_h slice for its
// own 32 units.  Here the reduction is split the other way (reduce-scatter): a workgroup
// multiplies only the dZ columns it computed itself (its 32 units x 4 gates) by the resident W
// slices of EVERY unit, dh_partial[16 rows, H] = dZ_own[16, 128] · W[H, own 128]ᵀ, and sends each
// unit block its [16 x 32] fp32 slice; a workgroup then sums the 16 slices addressed to it (64 KB
// for both layers, each byte read by one workgroup).  The dZ never leaves the workgroup except as
// the row-major copy for the weight GEMMs.
//
// Products per tick (waves split the H output units, each keeps its quarter's weights):
//   P1 = dZ_{l+1}[s]·W_h,l+1ᵀ            -> layer l+1, step s-1   (W_h,l+1 in VGPRs)
//   C0 = dZ_{l+1}[s]·W_x,l+1ᵀ + dZ_l[s+1]·W_h,lᵀ -> layer l, step s (W_h,l in VGPRs, W_x,l+1 in LDS)
// Layer l's dtop (the first term) and its recurrent term go out as ONE partial, so layer l runs
// one tick behind layer l+1 (LAG = 1; the all-gather kernel needs 2): T + 1 ticks.
//
// Tick tau (layer l+1 at step T-1-tau while tau < T, layer l at step T-tau from tau = 1):
//   poll (tick tau-1's arrivals of the column) -> every epilogue wave loads its 16 partial slices
//   (sc1) and its epilogue operands -> cell backward -> own dZ (bf16) into LDS -> barrier -> the
//   two products (96 MFMAs per wave) -> partial stores -> drain -> one arrival per workgroup ->
//   (off the critical path) row-major dZ copy by waves 2 and 3 from LDS, bias reduce.
// Hand-off forms as lstm2_bwd_wide.hip (persist_common.h): XCD-local columns store plain and
// signal per-workgroup L2 flags; otherwise sc1 stores and one agent counter per (column, tick).
// No dropout form (layer l+1's input mask applies to the SUM of the dtop slices): the launcher
// keeps the all-gather kernel for dropout steps.
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "persist_common.h"
#include "debug_env.h"

namespace dcr {

namespace {
constexpr int kRsLd = 136;  // LDS dZ row stride in bf16 (128 + 8: conflict-free b128 reads)

template <int CTRL, int N>
__device__ __forceinline__ void rs_bfly(float (&v)[16], bool hi) {
#pragma unroll
  for (int k = 0; k < N / 2; ++k) {
    const float send = hi ? v[k] : v[k + N / 2];
    const float keep = hi ? v[k + N / 2] : v[k];
    v[k] = keep + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                                0, __builtin_bit_cast(int, send), CTRL, 0xF, 0xF, true));
  }
}
// LDS reads the compiler does not track (head_wide.hip's pattern): retired by rs_lgkm_wait,
// which also pins the results' first use behind the wait
__device__ __forceinline__ unsigned rs_lds(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void rs_rd128(u32x4& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(addr));
}
template <int N>
__device__ __forceinline__ void rs_lgkm_wait(u32x4 (&d)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(d[0]), "+v"(d[1]), "+v"(d[2]), "+v"(d[3]) : "n"(N));
}
}  // namespace

// DIAG: workgroup 0's s_memtime phase stamps [T+2][8], or with a.diag_all every workgroup's
// s_memrealtime stamps [grid][T+2][8] (one 100 MHz clock for the chip: the cross-workgroup skew)
#define RS_STAMP(i)                                                                      \
  if (DIAG && a.diag && threadIdx.x == 0) {                                              \
    if (a.diag_all)                                                                      \
      a.diag[((size_t)blockIdx.x * (T + 2) + tau) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
    else if (blockIdx.x == 0)                                                            \
      a.diag[(size_t)tau * 8 + (i)] = __builtin_amdgcn_s_memtime();                      \
  }

// NT = H / 64 output-unit tiles of 16 per wave (a wave owns H/4 output units)
template <int NT, bool DIAG>
__global__ void __launch_bounds__(256, 1) lstm2_bwd_rs_kernel(Lstm2BwdArgs a) {
  constexpr int H = NT * 64;
  constexpr int NU = H / 32;      // unit blocks = workgroups per column = partial senders
  constexpr int G4H = 4 * H;
  constexpr int CH = 16 * 32;     // floats per [16 rows x 32 units] partial slice
  // W_x,l+1 fragments [wave][tile][gate][lane] (128 KB at H = 512)
  __shared__ __attribute__((aligned(16))) bf16x8 wxl[4][NT][4][64];
  // own dZ of the tick, bf16 [layer][row][4 gates x 32 units (+ pad)]
  __shared__ __attribute__((aligned(16))) bf16 dzx[2][16][kRsLd];
  // the tick's epilogue operands (one tick ahead, see opnd_dma): gates [layer][gate][row][32]
  // bf16, c [layer][c_t | c_{t-1}][row][32] fp32, layer l+1's dtop [row][32] fp32
  __shared__ __attribute__((aligned(16))) bf16 opg[2][4][16][32];
  __shared__ __attribute__((aligned(16))) float opc[2][2][16][32];
  __shared__ __attribute__((aligned(16))) float opd[16][32];
  __shared__ unsigned arr_s;
  __shared__ int loc_s;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int B = a.B, T = a.T;
  const int ncol = a.nbg;
  int ubk, col;
  if (!map_block_grid(blockIdx.x, gridDim.x, NU, ncol, ubk, col)) return;  // padding
  const int ub0 = ubk * 32;
  unsigned* const cnt = a.cnt0 + (size_t)col * (T + 1) * 4;
  unsigned long long* const xw = reinterpret_cast<unsigned long long*>(cnt + 2);
  const bool tryloc = a.xcdloc && T >= 8 && NU <= 32;
  if (tryloc && threadIdx.x == 0) xcd_publish(xw);
  unsigned* const fl = cnt + 4;  // (local form) per-workgroup flags
  if (threadIdx.x == 0) arr_s = 0u;

  // resident weights: rows = this wave's output units w H/4 + 16 j + (lane & 15), columns = the
  // workgroup's own gate columns g H + ub0 + 8 (lane >> 4) + [0, 8)
  bf16x8 wh1[NT][4], wh0[NT][4];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const size_t off = (size_t)(w * (H / 4) + 16 * j + (lane & 15)) * G4H + g * H + ub0 +
                         8 * (lane >> 4);
      wh1[j][g] = ld8(a.Wh1 + off);
      wh0[j][g] = ld8(a.Wh0 + off);
      wxl[w][j][g][lane] = ld8(a.Wx1 + off);
    }
  if (threadIdx.x == 0) {
    loc_s = tryloc ? xcd_decide(xw, (unsigned)NU, a.spin_limit, a.err, 14u) : 0;
    if (loc_s && ubk == 0) cnt[1] = 1u;  // (diagnostics: the column ran XCD-local)
  }
  __syncthreads();
  const bool loc = __builtin_amdgcn_readfirstlane(loc_s) != 0;
  bool dead = false;

  // partial ring [layer][slot][col][dest][src][16][32] fp32
  const size_t slot_f = (size_t)ncol * NU * NU * CH;
  const __amdgpu_buffer_rsrc_t rp = make_rsrc(a.pring, sizeof(float) * 4 * slot_f);
  auto chunk_off = [=](int Lr, int slot, int dest, int src) -> unsigned {  // bytes
    return (unsigned)(((((size_t)(Lr * 2 + slot) * ncol + col) * NU + dest) * NU + src) * CH *
                      sizeof(float));
  };

  // epilogue role: layer L (1: l+1, 0: l), unit half U
  const int L = w >> 1, U = w & 1;
  const int u0 = ub0 + 16 * U + 4 * (lane >> 4);
  float dc[4] = {0.f, 0.f, 0.f, 0.f};
  float dbacc = 0.f;
  constexpr unsigned kOut = 0x7FFFFFF0u;  // out-of-range buffer offset: reads zero
  // A [16 rows x 32 units] slice is two 1 KB halves (units [0, 16), [16, 32)), each laid out in
  // the MFMA output order [unit quad q][row][4 units]: a sender's tile store and a receiver's
  // load of its unit half are then ONE contiguous 1 KB per wave instruction (lane l at 16 l;
  // row-strided 64-B segments had made every instruction 16 half-line L2 requests)
  const unsigned vr = (unsigned)(U * 1024 + 16 * lane);
  const unsigned vs = (unsigned)(16 * lane);
  // Epilogue operands of the NEXT tick, DMA'd into LDS by waves 1-3 after their arrival (the
  // poller, wave 0, keeps no load in flight across its poll: vmcnt retires in order): per layer
  // the 4 gate rows (bf16), c_t and c_{t-1}; layer l+1's dtop.  1 KB pieces, lane l -> 16 B.
  const int pr = lane >> 2, pp = lane & 3;          // gate pieces: row pr, 16-B part pp
  const int cr = lane >> 3, cpp = lane & 7;         // fp32 pieces: row 8 h + cr, part cpp
  // piece: 0..7 gates (layer, gate), 8..15 c (layer, which, half), 16..17 dtop (half); called
  // with compile-time pieces (a wave-dependent piece index had put the destinations in scratch)
  auto dma_piece = [=](const int piece, int tk) __attribute__((always_inline)) {
    {
      if (piece < 8) {
        const int Lp = piece >> 2, g = piece & 3;
        const bool on = Lp ? tk < T : tk >= 1;
        const int tt = Lp ? T - 1 - tk : T - tk;
        const int br = col * 16 + pr;
        // (the descriptor built from a selected base: a select between two descriptors went
        // through scratch)
        const __amdgpu_buffer_rsrc_t r =
            make_rsrc(Lp ? a.gates1 : a.gates0, sizeof(bf16) * (size_t)T * B * G4H);
        const unsigned off = (on && br < B)
                                 ? (unsigned)((((size_t)tt * B + br) * G4H + g * H + ub0 + 8 * pp) * sizeof(bf16))
                                 : kOut;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)&opg[Lp][g][0][0], 16, opaque_vgpr(off), 0, 0, 0);
      } else {
        const int q = piece - 8;  // c: (layer, which, half); dtop: half
        const int Lp = q < 8 ? q >> 2 : 1, which = q < 8 ? (q >> 1) & 1 : 2, h = q & 1;
        const bool on = Lp ? tk < T : tk >= 1;
        const int tt = Lp ? T - 1 - tk : T - tk;
        const int br = col * 16 + 8 * h + cr;
        // which 0: c_t = cbuf[t + 1], 1: c_{t-1} = cbuf[t], 2: dtop1[t]
        const __amdgpu_buffer_rsrc_t r = make_rsrc(
            which == 2 ? a.dtop1 : (Lp ? a.cbuf1 : a.cbuf0),
            sizeof(float) * (size_t)(which == 2 ? T : T + 1) * B * H);
        const size_t slot_t = which == 0 ? (size_t)tt + 1 : (size_t)tt;
        const unsigned off = (on && br < B)
                                 ? (unsigned)(((slot_t * B + br) * H + ub0 + 4 * cpp) * sizeof(float))
                                 : kOut;
        float* dst = which == 2 ? &opd[8 * h][0] : &opc[Lp][which][8 * h][0];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)dst, 16, opaque_vgpr(off), 0, 0, 0);
      }
    }
  };
  auto opnd_dma = [=](int tk) __attribute__((always_inline)) {
    if (tk > T) return;
    if (w == 1) {
#pragma unroll
      for (int i = 0; i < 6; ++i) dma_piece(i, tk);
    } else if (w == 2) {
#pragma unroll
      for (int i = 6; i < 12; ++i) dma_piece(i, tk);
    } else if (w == 3) {
#pragma unroll
      for (int i = 12; i < 18; ++i) dma_piece(i, tk);
    }
  };
  opnd_dma(0);

  for (int tau = 0; tau <= T; ++tau) {
    const bool on1 = tau < T;   // layer l+1 computes step T-1-tau
    const bool on0 = tau >= 1;  // layer l   computes step T-tau
    const bool act = L ? on1 : on0;
    RS_STAMP(0)
    if (tau >= 1 && !dead) {  // tick tau-1's partials of every unit block of the column
      if (loc) {
        if (w == 0) dead = !poll_flags1(fl, NU, (unsigned)tau, a.spin_limit, a.err, 10u);
      } else if (threadIdx.x == kLstmPollerThread) {
        dead = !poll_counter(cnt + (size_t)(tau - 1) * 4, (unsigned)NU, a.spin_limit, a.err, 10u);
      }
    }
    RS_STAMP(1)
    // waves 1-3: this tick's operand DMA (issued after their previous arrival) has landed
    if (w != 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // (also: every wave's MFMA reads of dzx are done)
    // ---- receive (16 slices of this unit half) + the epilogue operands from LDS
    f32x4 ps = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x4 g4[4];
    float cc[4], cp[4], dtop[4];
    {
      const bool rcv = act && tau >= 1;
      const int slot = (tau - 1) & 1;
      f32x4 pv[NU];
#pragma unroll
      for (int s = 0; s < NU; ++s)
        pv[s] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                              rp, opaque_vgpr(rcv ? vr : kOut),
                                              rcv ? chunk_off(L, slot, ubk, s) : 0u, kAuxSc1));
      const int row = lane & 15, uq = 16 * U + 4 * (lane >> 4);
#pragma unroll
      for (int gt = 0; gt < 4; ++gt) g4[gt] = *reinterpret_cast<const bf16x4*>(&opg[L][gt][row][uq]);
      const float4 c1 = *reinterpret_cast<const float4*>(&opc[L][0][row][uq]);
      const float4 c0 = *reinterpret_cast<const float4*>(&opc[L][1][row][uq]);
      const float4 d = *reinterpret_cast<const float4*>(&opd[row][uq]);
      cc[0] = c1.x; cc[1] = c1.y; cc[2] = c1.z; cc[3] = c1.w;
      cp[0] = c0.x; cp[1] = c0.y; cp[2] = c0.z; cp[3] = c0.w;
      dtop[0] = L ? d.x : 0.f; dtop[1] = L ? d.y : 0.f; dtop[2] = L ? d.z : 0.f; dtop[3] = L ? d.w : 0.f;
#pragma unroll
      for (int s = 0; s < NU; ++s) ps += pv[s];
    }
    RS_STAMP(2)
    // ---- cell backward (zero rows where this role is idle: the products then add nothing)
    float dcur[16];
    {
      float di[4], dj[4], df_[4], dO[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float dh = ps[r] + dtop[r];
        const float gi = (float)g4[0][r], gj = (float)g4[1][r];
        const float gf = (float)g4[2][r], go = (float)g4[3][r];
        const float th = tanhf_(cc[r]);
        const float dcv = dc[r] + dh * go * (1.f - th * th);
        dO[r] = dh * th * go * (1.f - go);
        di[r] = dcv * gj * gi * (1.f - gi);
        dj[r] = dcv * gi * (1.f - gj * gj);
        df_[r] = dcv * cp[r] * gf * (1.f - gf);
        dc[r] = act ? dcv * gf : dc[r];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        dcur[r] = act ? di[r] : 0.f;
        dcur[4 + r] = act ? dj[r] : 0.f;
        dcur[8 + r] = act ? df_[r] : 0.f;
        dcur[12 + r] = act ? dO[r] : 0.f;
      }
#pragma unroll
      for (int gt = 0; gt < 4; ++gt) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = f2bf(dcur[4 * gt + r]);
        *reinterpret_cast<bf16x4*>(&dzx[L][lane & 15][gt * 32 + 16 * U + 4 * (lane >> 4)]) = v;
      }
    }
    RS_STAMP(3)
    __syncthreads();
    RS_STAMP(4)
    // ---- products for tick tau + 1 and their partial stores
    if (tau < T && !dead) {
      const bool need1 = tau + 1 < T;  // layer l+1 still active next tick
      bf16x8 z1[4], z0[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        z1[g] = *reinterpret_cast<const bf16x8*>(&dzx[1][lane & 15][g * 32 + 8 * (lane >> 4)]);
        z0[g] = *reinterpret_cast<const bf16x8*>(&dzx[0][lane & 15][g * 32 + 8 * (lane >> 4)]);
      }
      const int slot = tau & 1;
      // Explicitly pipelined (inline-asm LDS reads, counted waits): tile j+1's four W_x,l+1
      // fragments are read from LDS while tile j's register-operand MFMAs run (P1, then C0's
      // W_h,l term), and C0's W_x term comes last.  Plain reads waited at their use had put one
      // LDS round trip in front of every W_x MFMA (~4.6 k cycles for the 96 MFMAs).
      auto products = [&](auto sc1_c) __attribute__((always_inline)) {
        constexpr bool SC1 = decltype(sc1_c)::value;
        u32x4 xa[2][4];
        const unsigned xbase = rs_lds(&wxl[w][0][0][lane]);  // + (4 j + g) KB: tile j, gate g
#pragma unroll
        for (int g = 0; g < 4; ++g) rs_rd128(xa[0][g], xbase + g * 1024);
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          if (j + 1 < NT) {
#pragma unroll
            for (int g = 0; g < 4; ++g) rs_rd128(xa[(j + 1) & 1][g], xbase + ((j + 1) * 4 + g) * 1024);
          }
          const int ug = w * (H / 4) + 16 * j;  // first output unit of the tile
          const int dest = ug >> 5;
          const unsigned toff = vs + (unsigned)(((ug & 31) >> 4) * 1024);  // its unit half
          f32x4 c1 = f32x4{0.f, 0.f, 0.f, 0.f}, c0 = f32x4{0.f, 0.f, 0.f, 0.f};
          if (need1) {
#pragma unroll
            for (int g = 0; g < 4; ++g) c1 = mfma16(wh1[j][g], z1[g], c1);
          }
#pragma unroll
          for (int g = 0; g < 4; ++g) c0 = mfma16(wh0[j][g], z0[g], c0);
          if (j + 1 < NT)
            rs_lgkm_wait<4>(xa[j & 1]);
          else
            rs_lgkm_wait<0>(xa[j & 1]);
#pragma unroll
          for (int g = 0; g < 4; ++g) c0 = mfma16(__builtin_bit_cast(bf16x8, xa[j & 1][g]), z1[g], c0);
          const unsigned o0 = toff + chunk_off(0, slot, dest, ubk);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, c0), rp, o0, 0,
                                                 SC1 ? kAuxSc1 : 0);
          if (need1) {
            const unsigned o1 = toff + chunk_off(1, slot, dest, ubk);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, c1), rp, o1, 0,
                                                   SC1 ? kAuxSc1 : 0);
          }
        }
      };
      if (loc)
        products(std::integral_constant<bool, false>{});
      else
        products(std::integral_constant<bool, true>{});
      RS_STAMP(5)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      RS_STAMP(6)
      if (lane == 0) {
        if (loc)
          wg_arrive_flag(&arr_s, 4u, fl + ubk, (unsigned)tau + 1u);
        else
          wg_arrive(&arr_s, 4u, cnt + (size_t)tau * 4);
      }
    }
    RS_STAMP(7)
    // the next tick's epilogue operands (after the epilogue's reads: behind the dzx barrier)
    opnd_dma(tau + 1);
    // ---- off the critical path: row-major dZ copies for the weight GEMMs (waves 2 / 3 from
    // LDS, so the poller wave 0 has no store in flight at its next poll) and the bias gradient
    if (w >= 2) {
      const int Lc = w == 2 ? 1 : 0;
      const bool on = Lc ? on1 : on0;
      const int tc = Lc ? T - 1 - tau : T - tau;
      const int r = lane >> 2, q = lane & 3;  // row r, gate q: 32 units = 4 x 16 B
      const int br = col * 16 + r;
      if (on && br < B) {
        bf16* dz = (Lc ? a.dz1 : a.dz0) + ((size_t)tc * B + br) * G4H + q * H + ub0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
          *reinterpret_cast<u32x4*>(dz + 8 * k) =
              *reinterpret_cast<const u32x4*>(&dzx[Lc][r][q * 32 + 8 * k]);
      }
    }
    if (act) {
#pragma unroll
      for (int i = 0; i < 16; ++i) dcur[i] = (float)f2bf(dcur[i]);
      // (the row reduce-scatter of lstm2_bwd_wide.hip: lane r of a DPP row ends with the row
      // sum of value r)
      const int rr = lane & 15;
      rs_bfly<0x140, 16>(dcur, (rr & 8) != 0);  // row_mirror
      rs_bfly<0x141, 8>(dcur, (rr & 4) != 0);   // row_half_mirror
      rs_bfly<0x4E, 4>(dcur, (rr & 2) != 0);    // quad_perm [2,3,0,1]
      rs_bfly<0xB1, 2>(dcur, (rr & 1) != 0);    // quad_perm [1,0,3,2]
      dbacc += dcur[0];
    }
  }
  float* const dbp = L ? a.db_part1 : a.db_part0;
  if (dbp) {
    const int r = lane & 15;
    dbp[(size_t)col * G4H + (r >> 2) * H + u0 + (r & 3)] = dbacc;
    if (col == ncol - 1)
      for (int c2 = ncol; c2 < a.db_rows; ++c2) dbp[(size_t)c2 * G4H + (r >> 2) * H + u0 + (r & 3)] = 0.f;
  }
}

namespace {
template <bool DIAG>
const void* rs_pick(int H) {
  switch (H) {
    case 128: return (const void*)lstm2_bwd_rs_kernel<2, DIAG>;
    case 256: return (const void*)lstm2_bwd_rs_kernel<4, DIAG>;
    case 512: return (const void*)lstm2_bwd_rs_kernel<8, DIAG>;
  }
  return nullptr;
}
}  // namespace

// fp32 floats of the partial ring for (H, B): [2 layers][2 slots][ncol][NU][NU][16 x 32]
size_t lstm2_bwd_rs_ring_floats(int H, int B) {
  const size_t nu = (size_t)H / 32, ncol = (size_t)(B + 15) / 16;
  return 4 * ncol * nu * nu * 512;
}

bool lstm2_bwd_rs_ok(int H, int B, int cus) {
  const void* fn = rs_pick<false>(H);
  if (!fn || B < 1 || cus <= 0) return false;
  const int grid = (H / 32) * ((B + 15) / 16);
  int o = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, 256, 0) != hipSuccess || o < 1)
    return false;
  return grid <= o * cus;
}

int launch_lstm2_bwd_rs(const Lstm2BwdArgs& a, int cus, hipStream_t s) {
  if (!a.pring || a.xmask || !lstm2_bwd_rs_ok(a.H, a.B, cus) || a.nbg != (a.B + 15) / 16 ||
      a.T < 1)
    return -2;
  void* args[] = {const_cast<Lstm2BwdArgs*>(&a)};
  const void* fn = a.diag ? rs_pick<true>(a.H) : rs_pick<false>(a.H);
  int grid = (a.H / 32) * a.nbg, o = 0;
  const int padded = xcd_grid(a.H / 32, a.nbg);
  if (padded != grid && hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, fn, 256, 0) == hipSuccess &&
      padded <= o * cus)
    grid = padded;
  return hipLaunchKernel(fn, dim3(grid), dim3(256), args, 0, s) == hipSuccess ? 0 : -3;
}

}  // namespace dcr
