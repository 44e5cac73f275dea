// Persistent weights-resident LSTM recurrence for LARGE hidden sizes (H = 2048) at small batch
// (gfx950).  BASELINE config 4 (4-layer LSTM-2048, seq 512) at B = 64.
//
// Reference: TF's statically unrolled LSTMCell chain (model.py:61-73) and its tf.gradients
// backward (model.py:91) -- the same recurrence as lstm_persist.hip, which covers H <= 1024.
//
// Why a separate kernel.  At H = 2048 one 16-unit block of W_h is 4 gates x 16 units x 2048 K
// (fwd) / 16 units x 8192 K (bwd) = 256 KB of bf16: split over the 4 waves' K quarters that is
// 256 VGPRs per lane, the whole arch-VGPR file, so a workgroup is alone on its CU and the
// (H/16) x (B/16) grid of lstm_persist.hip (512 workgroups at B = 64) cannot be co-resident.
// Here a workgroup owns 16 units x NT 16-row batch tiles: the resident weight slice is reused
// for NT tiles per step, and the grid is (H/16) x ceil(B / 16NT) = 256 workgroups at B = 64
// (NT = 2).  The per-step library path it replaces re-streams all 32 MB of W_h from the MALL
// every step (13.7 us fwd / 20.6 us bwd at B = 64, profiles/r3_big_step.md); here a step moves
// only the handed-off activations (h: 256 KB, dZ: 1 MB per step, L2-resident).
//
// Per step (fwd): wave w loads the fragment-tiled h_{t-1} k-steps of its K quarter for every
// tile (ONE contiguous 1 KB sc1 load per k-step), multiplies them against its resident W_hᵀ
// fragments (mfma_f32_16x16x32_bf16, swapped operands: A = weight rows, B = batch rows), the
// four K partials meet in LDS, and wave n < NT runs the cell epilogue of tile n (c in registers
// across all T steps).  BPTT: K = 4H, wave w reduces over the gate columns g*H + [w H/4,
// (w+1) H/4) of every gate (its loads are streamed in 16-k-step chunks to bound registers).
//
// Hand-off (persist_common.h "Valid forms" first row): each epilogue wave stores its tile sc1
// in fragment order, drains (vmcnt(0)) and adds to an LDS counter; the workgroup's last such
// wave does ONE agent-scope add on shard (unit block & 3) of the (batch group, step) counter;
// ONE poller lane per workgroup polls the four shards with one 16-B sc1 load (+ s_sleep); a
// workgroup barrier releases the waves; every load of handed-off bytes is buffer_load sc1.
// 128 unit blocks per batch group would otherwise be 128 atomics on one address per step.
// Every spin is bounded; a timeout sets the error word and the grid still drains.
#include "common.h"
#include "kernels.h"
#include "persist_common.h"
#include "debug_env.h"

namespace dcr {

// DIAG builds record s_memtime stamps of workgroup 0 per step (phase shares only, never timing
// claims; cdna_hip_programming.md §7 "In-kernel stamps"); scripts/persist_stamps.py --H 2048
#define STAMP(i)                                                                    \
  if constexpr (DIAG) {                                                             \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                        \
      a.diag[(size_t)t * 8 + (i)] = __builtin_amdgcn_s_memtime();                   \
  }

// one LDS fragment read (16 B per lane) at a byte offset, invisible to the compiler's waitcnt
// pass (the DMA forward below counts its own lgkmcnt)
template <int OFF>
__device__ __forceinline__ void ds_rd128(bf16x8& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF) : "memory");
}
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& d) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(d) : "i"(N) : "memory");
}

template <int KS, int NT, bool DIAG = false, bool DMA = false>
__global__ void __launch_bounds__(256, 1) lstm_fwd_persist_nt_kernel(PersistArgs a) {
  // single-buffered partials [wave][tile][gate][lane] (float4): every step starts with a
  // workgroup barrier that the epilogue waves reach only after reading the previous step's
  // partials.  DMA (NT = 4): the h tiles arrive by LDS-DMA, two per step through each of xa /
  // xb ([wave][k-step][lane], each wave its own K quarter: 16 KB), and the partials go into
  // slices already read (128 KB in all)
  static_assert(!DMA || (NT == 4 && KS == 16), "LDS-DMA forward: NT = 4, H = 2048");
  constexpr int kXtF4 = 4 * KS * 64;
  __shared__ __attribute__((aligned(16))) float part[DMA ? 1 : 4][NT][4][64][4];
  __shared__ __attribute__((aligned(16))) float4 xa[DMA ? kXtF4 : 1];
  __shared__ __attribute__((aligned(16))) float4 xb[DMA ? kXtF4 : 1];
  __shared__ unsigned arr;
  // partial slot (wave wv, tile n, gate g): 64 float4.  DMA: tile 2 -> xa, 3 -> xb, 0 / 1 ->
  // xb +8 / +12 KB (the last tile read out of each)
  auto pslot = [&](int wv, int n, int g) -> float4* {
    if constexpr (DMA)
      return (n == 2 ? xa : xb) + wv * KS * 64 + (n < 2 ? (n + 2) * 4 * 64 : 0) + g * 64;
    else
      return reinterpret_cast<float4*>(&part[wv][n][g][0][0]);
  };
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int Bp = (B + 15) / 16 * 16;
  const int ntile = Bp / 16, nbg = (ntile + NT - 1) / NT;
  const int nwg_u = H / 16;
  int ubk, bg;
  map_block(blockIdx.x, nwg_u, nbg, ubk, bg);
  const int ub0 = ubk * 16, tile0 = bg * NT;
  const int ntl = ntile - tile0 < NT ? ntile - tile0 : NT;  // tiles of this batch group
  const int kq = 8 * (lane >> 4);
  const int kbase = w * (KS * 32);
  unsigned* cnt = a.cnt + (size_t)bg * (T + 1) * 4;
  const unsigned target = (unsigned)(nwg_u / 4);
  bool dead = false;
  if (threadIdx.x == 0) arr = 0u;

  // resident A fragments: rows g*H + ub0 + (lane&15) of W_hᵀ, this wave's K quarter
  bf16x8 wf[4][KS];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int s = 0; s < KS; ++s)
      wf[g][s] = ld8(a.W + (size_t)(g * H + ub0 + (lane & 15)) * H + kbase + s * 32 + kq);

  // epilogue: wave w < ntl owns tile tile0 + w (lane: batch row b, units u0..u0+3)
  const bool epi = w < ntl;
  const int b = (tile0 + (epi ? w : 0)) * 16 + (lane & 15);
  const bool live = epi && b < B;
  const int u0 = ub0 + 4 * (lane >> 4);
  const size_t bh = (size_t)b * H + u0;
  float c[4] = {0.f, 0.f, 0.f, 0.f};
  if (live) ld4f(a.cbuf + bh, c);
  // input bias added here when the dense zx was written without it (the library GEMM with a
  // bias ran as a separate 1 GB fp32 broadcast pass, 155 us per layer at B = 64)
  float bx[4][4] = {};
  if (epi && a.bias) {
#pragma unroll
    for (int g = 0; g < 4; ++g) ld4f(a.bias + (size_t)g * H + u0, bx[g]);
  }
  __syncthreads();  // arr
  if constexpr (DMA) {
    // h_0 published into ring slot 0 in fragment order (padded rows as zeros) and signalled on
    // counter 0: every step's tiles are then the same fragment-ring loads
    if (epi) {
      float h0[4] = {0.f, 0.f, 0.f, 0.f};
      if (live) ld4bf(a.hbuf + bh, h0);
      st4bf_sc1(a.hring + frag_index(b, u0, H), h0[0], h0[1], h0[2], h0[3]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) wg_arrive(&arr, (unsigned)ntl, cnt + (ubk & 3));
    }
  }

  for (int t = 0; t < T; ++t) {
    STAMP(0);
    float zx[4][4] = {};
    if (live) {
      const float* zrow = a.ids ? a.zx + (size_t)a.ids[(size_t)t * B + b] * a.zx_ld
                                : a.zx + ((size_t)t * B + b) * a.zx_ld;
#pragma unroll
      for (int g = 0; g < 4; ++g) ld4f(zrow + (size_t)g * H + u0, zx[g]);
    }
    if (DMA || t > 0) {
      if ((int)threadIdx.x == a.poller && !dead)
        dead = !poll_shards4(cnt + (size_t)t * 4, target, a.spin_limit, a.err, 1u);
    }
    STAMP(1);
    __syncthreads();
    STAMP(2);
    const bool fring = DMA || t > 0;  // slot 0 (initial state) is row-major (DMA: published)
    const __amdgpu_buffer_rsrc_t hsrc =
        fring ? make_rsrc(a.hring + (size_t)(t & 1) * Bp * H, sizeof(bf16) * (size_t)Bp * H)
              : make_rsrc(a.hbuf, sizeof(bf16) * (size_t)B * H);
    // the tiles' h fragments stream through two register buffers: tile n+1's loads are issued
    // before tile n's MFMAs (NT = 4 would not fit every tile's fragments next to the 256 weight
    // VGPRs; at NT <= 2 this is the all-tiles-first order).  Unconditional: a tile past the
    // batch reads an empty descriptor (its MFMAs feed a partial slot no epilogue reads)
    bf16x8 hb[2][KS];
    const __amdgpu_buffer_rsrc_t hnone = make_rsrc(a.hring, 0);
    auto load_tile = [&](int n, bf16x8 (&d)[KS]) {
      const int tile = tile0 + n;
      const __amdgpu_buffer_rsrc_t src = n < ntl ? hsrc : hnone;
      const unsigned roff =
          (unsigned)(((size_t)(tile * 16 + (lane & 15)) * H + kbase + kq) * sizeof(bf16));
#pragma unroll
      for (int s = 0; s < KS; ++s)
        d[s] = fring ? ld8_sc1(src, (unsigned)lane * 16u, frag_tile_off(tile, w * KS + s, H))
                     : ld8_sc1(src, roff + s * 64);
    };
    auto put = [&](int n, const f32x4 (&acc)[4]) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if constexpr (DMA) {
          // (inline asm: the waitcnt pass would hold a plain LDS store behind every LDS-DMA in
          // flight; this slice was read by this wave already)
          const unsigned addr =
              (unsigned)(size_t)(__attribute__((address_space(3))) void*)(pslot(w, n, g) + lane);
          asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(acc[g]) : "memory");
        } else {
          pslot(w, n, g)[lane] = make_float4(acc[g][0], acc[g][1], acc[g][2], acc[g][3]);
        }
      }
    };
    if constexpr (DMA) {
      // tiles 0-1 by LDS-DMA (sc1, like every hand-off load) at once, tile 2 into xa as soon as
      // tile 0 has been multiplied out of it, tile 3 into xb after tile 1: two round trips per
      // step instead of the register double buffer's chain of four
      auto dma_tile = [&](int n, float4* dst) {
        const __amdgpu_buffer_rsrc_t src = n < ntl ? hsrc : hnone;
        dst += w * KS * 64;
#pragma unroll
        for (int s = 0; s < KS; ++s)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              src, (__attribute__((address_space(3))) void*)(dst + s * 64), 16,
              (unsigned)lane * 16u, frag_tile_off(tile0 + n, w * KS + s, H), 0, kAuxSc1);
      };
      // a tile's fragments out of LDS three k-steps ahead of their MFMAs (one LDS round trip is
      // longer than a k-step's four MFMAs), the waits counted here
      auto lds_tile = [&](const float4* src, f32x4 (&acc)[4]) {
        const unsigned base =
            (unsigned)(size_t)(__attribute__((address_space(3))) const void*)(src + w * KS * 64 +
                                                                               lane);
        bf16x8 q[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
        ds_rd128<0 * 1024>(q[0], base);
        ds_rd128<1 * 1024>(q[1], base);
        ds_rd128<2 * 1024>(q[2], base);
#define DCR_NT_KSTEP(S)                                                              \
  if constexpr ((S) + 3 < KS) ds_rd128<((S) + 3) * 1024>(q[((S) + 3) & 3], base);   \
  if constexpr ((S) + 3 < KS) lgkm_wait<3>(q[(S) & 3]);                              \
  else if constexpr ((S) + 2 < KS) lgkm_wait<2>(q[(S) & 3]);                         \
  else if constexpr ((S) + 1 < KS) lgkm_wait<1>(q[(S) & 3]);                         \
  else lgkm_wait<0>(q[(S) & 3]);                                                     \
  _Pragma("unroll") for (int g = 0; g < 4; ++g) acc[g] = mfma16(wf[g][S], q[(S) & 3], acc[g]);
        DCR_NT_KSTEP(0) DCR_NT_KSTEP(1) DCR_NT_KSTEP(2) DCR_NT_KSTEP(3)
        DCR_NT_KSTEP(4) DCR_NT_KSTEP(5) DCR_NT_KSTEP(6) DCR_NT_KSTEP(7)
        DCR_NT_KSTEP(8) DCR_NT_KSTEP(9) DCR_NT_KSTEP(10) DCR_NT_KSTEP(11)
        DCR_NT_KSTEP(12) DCR_NT_KSTEP(13) DCR_NT_KSTEP(14) DCR_NT_KSTEP(15)
#undef DCR_NT_KSTEP
      };
      f32x4 a0[4], a1[4], acc[4];
      dma_tile(0, xa);
      dma_tile(1, xb);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 landed
      lds_tile(xa, a0);
      dma_tile(2, xa);  // (tile 0's reads have returned: the MFMAs above consumed them)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 1 landed
      lds_tile(xb, a1);
      dma_tile(3, xb);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 2 landed
      lds_tile(xa, acc);
      put(2, acc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile 3 landed
      lds_tile(xb, acc);
      put(3, acc);
      put(0, a0);
      put(1, a1);
      // the partial stores above are inline asm, invisible to the compiler's waitcnt pass, and
      // the barrier below does not wait for LDS operations by itself: drain them here so that
      // other waves' pslot() reads after the barrier see every partial
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      load_tile(0, hb[0]);
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        if (n + 1 < NT) load_tile(n + 1, hb[(n + 1) & 1]);
        const bf16x8 (&hf)[KS] = hb[n & 1];
        f32x4 acc[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[g] = mfma16(wf[g][s], hf[s], acc[g]);
        put(n, acc);
      }
    }
    STAMP(3);
    __syncthreads();
    STAMP(4);
    if (epi) {
      float z[4][4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 s0 = pslot(0, w, g)[lane];
        const float4 s1 = pslot(1, w, g)[lane];
        const float4 s2 = pslot(2, w, g)[lane];
        const float4 s3 = pslot(3, w, g)[lane];
        z[g][0] = s0.x + s1.x + s2.x + s3.x + (zx[g][0] + bx[g][0]);
        z[g][1] = s0.y + s1.y + s2.y + s3.y + (zx[g][1] + bx[g][1]);
        z[g][2] = s0.z + s1.z + s2.z + s3.z + (zx[g][2] + bx[g][2]);
        z[g][3] = s0.w + s1.w + s2.w + s3.w + (zx[g][3] + bx[g][3]);
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
      // (padded rows are handed off too: zero inputs, finite values, never read back)
      STAMP(5);
      st4bf_sc1(a.hring + (size_t)((t + 1) & 1) * Bp * H + frag_index(b, u0, H), h[0], h[1], h[2],
                h[3]);
      if (t + 1 < T) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) wg_arrive(&arr, (unsigned)ntl, cnt + (size_t)(t + 1) * 4 + (ubk & 3));
        STAMP(6);
      }
      if (live) {
        const size_t o = (size_t)(t + 1) * B * H + bh;
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
}

// KS = 4H / 128 k-steps per wave (K = 4H split by unit quarter inside every gate, as in
// lstm_persist.hip); the payload of one tile is streamed in chunks of KSG = KS / 4 k-steps (one
// gate segment), two chunks in flight next to the 256 weight VGPRs.
template <int KS, int NT, bool DIAG = false>
__global__ void __launch_bounds__(256, 1) lstm_bwd_persist_nt_kernel(PersistArgs a) {
  __shared__ __attribute__((aligned(16))) float part[4][NT][64][4];
  __shared__ unsigned arr;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int Bp = (B + 15) / 16 * 16;
  const int ntile = Bp / 16, nbg = (ntile + NT - 1) / NT;
  const int nwg_u = H / 16;
  int ubk, bg;
  map_block(blockIdx.x, nwg_u, nbg, ubk, bg);
  const int ub0 = ubk * 16, tile0 = bg * NT;
  const int ntl = ntile - tile0 < NT ? ntile - tile0 : NT;
  const int kq = 8 * (lane >> 4);
  const int G4H = 4 * H;
  unsigned* cnt = a.cnt + (size_t)bg * (T + 1) * 4;
  const unsigned target = (unsigned)(nwg_u / 4);
  bool dead = false;
  if (threadIdx.x == 0) arr = 0u;

  constexpr int KSG = KS / 4;  // k-steps per gate segment
  bf16x8 wf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s)
    wf[s] = ld8(a.W + (size_t)(ub0 + (lane & 15)) * G4H + (s / KSG) * H + w * (H / 4) +
                (s % KSG) * 32 + kq);

  const bool epi = w < ntl;
  const int b = (tile0 + (epi ? w : 0)) * 16 + (lane & 15);
  const bool live = epi && b < B;
  const int u0 = ub0 + 4 * (lane >> 4);
  const size_t bh = (size_t)b * H + u0;
  float dc[4] = {0.f, 0.f, 0.f, 0.f};
  float dbacc[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r) dbacc[g][r] = 0.f;
  __syncthreads();  // arr

  for (int t = T - 1; t >= 0; --t) {
    STAMP(0);
    float gi[4] = {}, gj[4] = {}, gf[4] = {}, go[4] = {}, cc[4] = {}, cp[4] = {}, dtop[4] = {};
    if (live) {
      const bf16* gp = a.gates + ((size_t)t * B + b) * G4H + u0;
      ld4bf(gp, gi); ld4bf(gp + H, gj); ld4bf(gp + 2 * H, gf); ld4bf(gp + 3 * H, go);
      ld4f(a.cbuf + (size_t)(t + 1) * B * H + bh, cc);
      ld4f(a.cbuf + (size_t)t * B * H + bh, cp);
      ld4f(a.dtop + (size_t)t * B * H + bh, dtop);
    }
    if (t < T - 1) {
      if ((int)threadIdx.x == a.poller && !dead)
        dead = !poll_shards4(cnt + (size_t)(t + 1) * 4, target, a.spin_limit, a.err, 2u);
      STAMP(1);
      __syncthreads();
      STAMP(2);
      const __amdgpu_buffer_rsrc_t zsrc =
          make_rsrc(a.zring + (size_t)((t + 1) & 1) * Bp * G4H, sizeof(bf16) * (size_t)Bp * G4H);
      // chunk c = (tile n = c / 4, gate g = c % 4); two chunk buffers: the loads of chunk c+1
      // are issued before the MFMAs of chunk c (two chunks = 128 VGPRs in flight)
      const int nch = 4 * ntl;
      bf16x8 db[2][KSG];
      auto load_chunk = [&](int c, bf16x8 (&d)[KSG]) {
        const int tile = tile0 + c / 4, g = c % 4;
#pragma unroll
        for (int s = 0; s < KSG; ++s)
          d[s] = ld8_sc1(zsrc, (unsigned)lane * 16u,
                         frag_tile_off(tile, (g * H + w * (H / 4)) / 32 + s, G4H));
      };
      load_chunk(0, db[0]);
      // a tile loop that is not unrolled around the four gate chunks of a tile (c = 4 n + g:
      // the chunk buffer parity is g's); fully unrolled over NT = 4 tiles the register
      // allocator had spilled 1.5 KB per lane
#pragma unroll 1
      for (int n = 0; n < ntl; ++n) {
        f32x4 pacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = 4 * n + g;
          if (c + 1 < nch) load_chunk(c + 1, db[(g + 1) & 1]);
#pragma unroll
          for (int s = 0; s < KSG; ++s) pacc = mfma16(wf[g * KSG + s], db[g & 1][s], pacc);
        }
        *reinterpret_cast<float4*>(&part[w][n][lane][0]) =
            make_float4(pacc[0], pacc[1], pacc[2], pacc[3]);
      }
      STAMP(3);
      __syncthreads();
      STAMP(4);
    }
    if (epi) {
      float dh[4];
      if (t < T - 1) {
        const float4 s0 = *reinterpret_cast<const float4*>(&part[0][w][lane][0]);
        const float4 s1 = *reinterpret_cast<const float4*>(&part[1][w][lane][0]);
        const float4 s2 = *reinterpret_cast<const float4*>(&part[2][w][lane][0]);
        const float4 s3 = *reinterpret_cast<const float4*>(&part[3][w][lane][0]);
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
      bf16* const zr = a.zring + (size_t)(t & 1) * Bp * G4H;
      STAMP(5);
      st4bf_sc1(zr + frag_index(b, u0, G4H), di[0], di[1], di[2], di[3]);
      st4bf_sc1(zr + frag_index(b, H + u0, G4H), dj[0], dj[1], dj[2], dj[3]);
      st4bf_sc1(zr + frag_index(b, 2 * H + u0, G4H), df_[0], df_[1], df_[2], df_[3]);
      st4bf_sc1(zr + frag_index(b, 3 * H + u0, G4H), dO[0], dO[1], dO[2], dO[3]);
      if (t > 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) wg_arrive(&arr, (unsigned)ntl, cnt + (size_t)t * 4 + (ubk & 3));
        STAMP(6);
      }
      if (live) {
        bf16* dz = a.dz + ((size_t)t * B + b) * G4H + u0;
        st4bf(dz, di[0], di[1], di[2], di[3]);
        st4bf(dz + H, dj[0], dj[1], dj[2], dj[3]);
        st4bf(dz + 2 * H, df_[0], df_[1], df_[2], df_[3]);
        st4bf(dz + 3 * H, dO[0], dO[1], dO[2], dO[3]);
        // the bias gradient sums the bf16-rounded dz exactly as the dW GEMMs see it
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          dbacc[0][r] += (float)f2bf(di[r]);
          dbacc[1][r] += (float)f2bf(dj[r]);
          dbacc[2][r] += (float)f2bf(df_[r]);
          dbacc[3][r] += (float)f2bf(dO[r]);
        }
      }
    }
  }
  // bias-gradient partial of each 16-row tile: reduce its 16 batch lanes (lane bits 0..3)
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
      float* dst = a.db_part + (size_t)(tile0 + w) * G4H + u0;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(dst + g * H) =
            make_float4(dbacc[g][0], dbacc[g][1], dbacc[g][2], dbacc[g][3]);
    }
  }
}

// ------------------------------------------------------------------------------------------
// host side (called from lstm_persist.hip's selection for H > 1024)
// ------------------------------------------------------------------------------------------
// Batch tiles per workgroup: the smallest NT in {1, 2, 4} whose (H/16) x ceil(B/16NT) grid fits
// one workgroup per CU; 0 if none does (the large-batch steps stay on the library form, where
// the per-step GEMMs are efficient) or the shape has no instantiation.
int lstm_persist_nt_tiles(int H, int B, int cus) {
  if (H != 2048 || B < 1 || cus <= 0) return 0;
  const int ntile = (B + 15) / 16;
  for (int nt = 1; nt <= 4; nt *= 2)
    if ((H / 16) * ((ntile + nt - 1) / nt) <= cus) return nt;
  return 0;
}

int lstm_persist_nt_grid(int H, int B, int cus) {
  const int nt = lstm_persist_nt_tiles(H, B, cus);
  return nt ? (H / 16) * (((B + 15) / 16 + nt - 1) / nt) : 0;
}

const void* lstm_persist_nt_fn(int bwd, int H, int B, int cus, int diag) {
  switch (lstm_persist_nt_tiles(H, B, cus) * (diag ? -1 : 1)) {
    case 1: return bwd ? (const void*)lstm_bwd_persist_nt_kernel<64, 1>
                       : (const void*)lstm_fwd_persist_nt_kernel<16, 1>;
    case 2: return bwd ? (const void*)lstm_bwd_persist_nt_kernel<64, 2>
                       : (const void*)lstm_fwd_persist_nt_kernel<16, 2>;
    // NT = 4 forward: h tiles by LDS-DMA (DCR_DEBUG=nt_dma=0: register double buffer)
    case 4: return bwd ? (const void*)lstm_bwd_persist_nt_kernel<64, 4>
                   : debug_int("nt_dma", 1) ? (const void*)lstm_fwd_persist_nt_kernel<16, 4, false, true>
                                            : (const void*)lstm_fwd_persist_nt_kernel<16, 4>;
    case -1: return bwd ? (const void*)lstm_bwd_persist_nt_kernel<64, 1, true>
                        : (const void*)lstm_fwd_persist_nt_kernel<16, 1, true>;
    case -2: return bwd ? (const void*)lstm_bwd_persist_nt_kernel<64, 2, true>
                        : (const void*)lstm_fwd_persist_nt_kernel<16, 2, true>;
    case -4: return bwd ? (const void*)lstm_bwd_persist_nt_kernel<64, 4, true>
                    : debug_int("nt_dma", 1) ? (const void*)lstm_fwd_persist_nt_kernel<16, 4, true, true>
                                             : (const void*)lstm_fwd_persist_nt_kernel<16, 4, true>;
  }
  return nullptr;
}

}  // namespace dcr
