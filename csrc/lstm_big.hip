// Persistent LSTM forward for large hidden sizes (1024 < H <= 2048) on gfx950.
//
// Reference: the TF LSTMCell chain (model.py:61-73; K4/K5 of SURVEY.md §2.3).  For H = 2048 one
// layer's W_hᵀ is 32 MB of bf16: the 16-unit workgroups of lstm_persist.hip would need 256 KB of
// it per CU, so those shapes ran the per-step kernels, which re-stream every workgroup's weight
// slice from L2/MALL/HBM at every step (bandwidth bound).  Here the weights are
// sharded by 8-unit blocks: a workgroup keeps 8 units x 4 gates = 32 rows of W_hᵀ (128 KB at
// H = 2048, 128 VGPRs per lane over 4 waves) resident for the whole sequence and handles NBT
// batch tiles of 16 rows, so the grid is (H/8) x (B / 16·NBT) <= one workgroup per CU.
//
// MFMA layout (mfma_f32_16x16x32_bf16, swapped operands): A-tile a (a = 0, 1) = W_hᵀ rows
// g·H + ub0 + 4a + u' ordered (u' = row>>2, g = row&3), B = the batch rows of h_{t-1}.  The C/D
// row 4·(lane>>4) + reg is then (unit u' = lane>>4, gate g = reg): each lane holds all four gate
// pre-activations of one unit for one batch row and the cell update is lane-local.  The 4 waves
// split K in quarters (partials meet in LDS); wave w runs the epilogue of batch tile w.
//
// Hand-off (persist_common.h, the validated form): every step's h goes to a 2-slot ring in
// MFMA-fragment order.  A wave's 8 units x 16 rows are one contiguous 256-B run there, so the
// wave stages them through LDS and 32 lanes write the two 128-B lines whole with ONE 8-B sc1
// store instruction; the wave drains (vmcnt(0)) and adds to an LDS count, and the workgroup's
// last storing wave adds 1 to its shard of the (batch group, step) counter (the first "valid
// forms" row: one signal per workgroup, 4 shards).  One poller per workgroup polls all four
// shards with one 16-B sc1 load (+ s_sleep), a barrier releases the other waves, every payload
// load is buffer_load sc1.  Spins are bounded (error word).
#include "common.h"
#include "kernels.h"
#include "persist_common.h"

namespace dcr {

#define BSTAMP(i)                                                                   \
  if constexpr (DIAG) {                                                             \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                        \
      a.diag[(size_t)tt * 8 + (i)] = __builtin_amdgcn_s_memtime();                  \
  }

template <int KS, int NBT, bool DIAG = false>
__global__ void __launch_bounds__(256, 1) lstm_big_fwd_kernel(PersistArgs a) {
  __shared__ __attribute__((aligned(16))) float part[4][NBT][2][64][4];
  __shared__ __attribute__((aligned(16))) bf16 stage[4][16][8];  // per-wave h tile [row][unit]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int nwg_u = H / 8;
  const int ubk = blockIdx.x % nwg_u, bgp = blockIdx.x / nwg_u;
  const int ub0 = ubk * 8, b0 = bgp * 16 * NBT;
  const int kq = 8 * (lane >> 4);
  const int kbase = w * (KS * 32);
  // arrivals: one per workgroup (its last storing wave signals for all, after an LDS count),
  // spread over 4 counter shards by unit block; all H/8 workgroups of a batch group signal every
  // step, so a single counter would take hundreds of contended atomics per step
  unsigned* cnt = a.cnt + (size_t)bgp * (T + 1) * 4;
  const unsigned target = (unsigned)(nwg_u / 4);  // workgroups per shard
  unsigned* const my_shard_base = cnt + (ubk & 3);
  __shared__ unsigned lds_arrive;
  if (threadIdx.x == 0) lds_arrive = 0;
  __syncthreads();
  bool dead = false;

  // resident A fragments: row r = lane&15 -> (u' = r>>2, g = r&3)
  bf16x8 wf[2][KS];
  {
    const int r = lane & 15;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const size_t row = (size_t)((r & 3) * H + ub0 + 4 * t + (r >> 2));
#pragma unroll
      for (int s = 0; s < KS; ++s) wf[t][s] = ld8(a.W + row * H + kbase + s * 32 + kq);
    }
  }

  // epilogue role: batch tile j = w (waves >= NBT have none); lane: unit ub0 + 4t + (lane>>4)
  // for t = 0, 1, batch row b
  const bool epi = w < NBT;
  const int up = lane >> 4;
  const int b = b0 + 16 * (epi ? w : 0) + (lane & 15);
  float c[2] = {0.f, 0.f};
  if (epi) {
#pragma unroll
    for (int t = 0; t < 2; ++t) c[t] = a.cbuf[(size_t)b * H + ub0 + 4 * t + up];
  }

  // input projections, prefetched one step ahead: for layers >= 1 they stream from the
  // [T, B, 4H] fp32 GEMM output in HBM, and a load issued in the same step sat in front of the
  // payload loads in the (in-order) vmcnt queue
  auto zx_load = [&](float (&z)[2][4], int step) {
    const float* zrow = a.ids ? a.zx + (size_t)a.ids[(size_t)step * B + b] * a.zx_ld
                              : a.zx + ((size_t)step * B + b) * a.zx_ld;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) z[t][g] = zrow[(size_t)g * H + ub0 + 4 * t + up];
  };
  float zxn[2][4];
  if (epi) zx_load(zxn, 0);

  for (int tt = 0; tt < T; ++tt) {
    float zx[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) zx[t][g] = zxn[t][g];
    if (epi && tt + 1 < T) zx_load(zxn, tt + 1);
    BSTAMP(0)
    if (tt >= 1) {
      if (threadIdx.x == kLstmPollerThread && !dead)
        dead = !poll_shards4(cnt + (size_t)tt * 4, target, a.spin_limit, a.err, 11u);
      BSTAMP(1)
      __syncthreads();
    }
    BSTAMP(2)
    // payload h_{t-1}: slot 0 (initial state, prep-written) row-major, later slots from the
    // fragment-order ring; batch tiles double-buffered (loads of tile j+1 under tile j's MFMAs)
    const bool ring = a.hring && tt > 0;
    const __amdgpu_buffer_rsrc_t rs =
        ring ? make_rsrc(a.hring + (size_t)(tt & 1) * B * H, sizeof(bf16) * (size_t)B * H)
             : make_rsrc(a.hbuf, sizeof(bf16) * (size_t)B * H);
    auto hload = [&](bf16x8 (&hf)[KS], int j) {
      const int bt = b0 / 16 + j;
#pragma unroll
      for (int s = 0; s < KS; ++s)
        hf[s] = ld8_sc1(rs, ring ? frag_load_off(bt, w * KS + s, H, lane)
                                 : (unsigned)((((size_t)(16 * bt + (lane & 15)) * H + kbase + kq) +
                                               s * 32) * sizeof(bf16)));
    };
    bf16x8 hA[KS], hB[KS];
    hload(hA, 0);
#pragma unroll
    for (int j = 0; j < NBT; ++j) {
      bf16x8 (&cur)[KS] = (j & 1) ? hB : hA;
      bf16x8 (&nxt)[KS] = (j & 1) ? hA : hB;
      if (j + 1 < NBT) hload(nxt, j + 1);
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[t] = mfma16(wf[t][s], cur[s], acc[t]);
#pragma unroll
      for (int t = 0; t < 2; ++t)
        *reinterpret_cast<float4*>(&part[w][j][t][lane][0]) =
            make_float4(acc[t][0], acc[t][1], acc[t][2], acc[t][3]);
    }
    BSTAMP(3)
    __syncthreads();
    BSTAMP(4)
    if (epi) {
      float h[2], gi[2], gj[2], gf[2], go[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        float z[4];
        const float4 s0 = *reinterpret_cast<const float4*>(&part[0][w][t][lane][0]);
        const float4 s1 = *reinterpret_cast<const float4*>(&part[1][w][t][lane][0]);
        const float4 s2 = *reinterpret_cast<const float4*>(&part[2][w][t][lane][0]);
        const float4 s3 = *reinterpret_cast<const float4*>(&part[3][w][t][lane][0]);
        z[0] = s0.x + s1.x + s2.x + s3.x + zx[t][0];
        z[1] = s0.y + s1.y + s2.y + s3.y + zx[t][1];
        z[2] = s0.z + s1.z + s2.z + s3.z + zx[t][2];
        z[3] = s0.w + s1.w + s2.w + s3.w + zx[t][3];
        gi[t] = sigmoidf_(z[0]);
        gj[t] = tanhf_(z[1]);
        gf[t] = sigmoidf_(z[2] + a.forget_bias);
        go[t] = sigmoidf_(z[3]);
        c[t] = gf[t] * c[t] + gi[t] * gj[t];
        h[t] = go[t] * tanhf_(c[t]);
      }
      BSTAMP(5)
      // stage the wave's 16 rows x 8 units: row-contiguous 16-B runs
      const int bl = lane & 15;
      stage[w][bl][up] = f2bf(h[0]);
      stage[w][bl][4 + up] = f2bf(h[1]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      if (tt + 1 < T) {  // publish first: the hand-off is the critical path
        // 32 lanes x 8 B = the wave's 256-B run (two whole 128-B lines) in ONE sc1 store
        // instruction: lane l writes units 4(l&1)..+3 of batch row l>>1
        if (lane < 32) {
          const int row = lane >> 1, half = lane & 1;
          const uint64_t v = *reinterpret_cast<const uint64_t*>(&stage[w][row][4 * half]);
          bf16* dst = a.hring + (size_t)((tt + 1) & 1) * B * H +
                      frag_index(b0 + 16 * w + row, ub0, H) + 4 * half;
          __hip_atomic_store(reinterpret_cast<uint64_t*>(dst), v, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        BSTAMP(6)
        if (lane == 0) wg_arrive(&lds_arrive, NBT, my_shard_base + (size_t)(tt + 1) * 4);
      }
      // off the critical path: row-major h, c, gates, final state
      if (lane < 16)
        *reinterpret_cast<bf16x8*>(a.hbuf + ((size_t)(tt + 1) * B + b0 + 16 * w + lane) * H + ub0) =
            *reinterpret_cast<const bf16x8*>(&stage[w][lane][0]);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int u = ub0 + 4 * t + up;
        const size_t o = ((size_t)(tt + 1) * B + b) * H + u;
        a.cbuf[o] = c[t];
        if (a.gates) {
          bf16* gp = a.gates + ((size_t)tt * B + b) * 4 * H + u;
          gp[0] = f2bf(gi[t]);
          gp[H] = f2bf(gj[t]);
          gp[2 * H] = f2bf(gf[t]);
          gp[3 * H] = f2bf(go[t]);
        }
        if (tt == T - 1) {
          if (a.hlast32) a.hlast32[(size_t)b * H + u] = h[t];
          if (a.clast32) a.clast32[(size_t)b * H + u] = c[t];
        }
      }
    }
  }
}

template <int KS>
static const void* big_fn(int nbt, bool diag) {
  if (diag) return KS == 16 && nbt == 4 ? (const void*)lstm_big_fwd_kernel<16, 4, true> : nullptr;
  switch (nbt) {
    case 1: return (const void*)lstm_big_fwd_kernel<KS, 1>;
    case 2: return (const void*)lstm_big_fwd_kernel<KS, 2>;
    case 4: return (const void*)lstm_big_fwd_kernel<KS, 4>;
  }
  return nullptr;
}

static const void* big_pick(int H, int nbt, bool diag = false) {
  switch (H / 128) {
    case 9: return big_fn<9>(nbt, diag);
    case 10: return big_fn<10>(nbt, diag);
    case 12: return big_fn<12>(nbt, diag);
    case 14: return big_fn<14>(nbt, diag);
    case 16: return big_fn<16>(nbt, diag);
  }
  return nullptr;
}

// batch tiles per workgroup: the fewest that keep the grid within one workgroup per CU
static int big_nbt(int H, int B, int cus) {
  const int tiles = B / 16;
  for (int nbt : {1, 2, 4})
    if (tiles % nbt == 0 && (H / 8) * (tiles / nbt) <= cus) return nbt;
  return 0;
}

int lstm_big_supported(int H, int B, int cus) {
  if (H % 128 != 0 || H <= 1024 || H > 2048 || B % 16 != 0 || B < 16 || cus <= 0) return 0;
  const int nbt = big_nbt(H, B, cus);
  const void* fn = nbt ? big_pick(H, nbt) : nullptr;
  if (!fn) return 0;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 256, 0) != hipSuccess) return 0;
  return (H / 8) * (B / 16 / nbt) <= occ * cus ? 1 : 0;
}

int launch_lstm_big_fwd(const PersistArgs& a, int cus, hipStream_t s) {
  if (!lstm_big_supported(a.H, a.B, cus) || !a.hring) return -2;
  const int nbt = big_nbt(a.H, a.B, cus);
  const int grid = (a.H / 8) * (a.B / 16 / nbt);
  if (!a.cnt_zeroed)
    (void)hipMemsetAsync(a.cnt, 0, sizeof(unsigned) * (size_t)(a.B / 16 / nbt) * (a.T + 1) * 4, s);
  void* args[] = {const_cast<PersistArgs*>(&a)};
  const void* fn = big_pick(a.H, nbt, a.diag != nullptr);
  if (!fn) return -2;
  return hipLaunchKernel(fn, dim3(grid), dim3(256), args, 0, s) == hipSuccess ? 0 : -3;
}

}  // namespace dcr
