// Token-reduction weight-gradient GEMM for gfx950:  C_s[m, n] = sum_{k in chunk s} A[k, m] B[k, n]
//
// Reference: the weight gradients of the unrolled cell (tf.gradients through model.py:72, summed
// over all T x B tokens).  Both operands lie token-major in memory (A = h_{t-1} or the layer input
// [K tokens, M], B = dZ [K tokens, N]), i.e. K is the OUTER index of both, so neither is an MFMA
// fragment as stored.  Each workgroup streams [32 x 256] k-row panels of A and B into LDS as they
// lie in memory and reads them back transposed with ds_read_b64_tr_b16 (CDNA4's transposing LDS
// read), which hands every lane the consecutive-k bf16 values of one m (or n) -- the A / B
// fragment of v_mfma_f32_16x16x32_bf16.
//
// Tiling.  A workgroup owns a 256 x 256 output tile (8 waves of 128 x 64 = 8 x 4 MFMA tiles, 128
// fp32 accumulators per lane; two waves per SIMD, so one wave's LDS reads and barrier waits
// hide under the other's MFMAs -- 4 waves of 128 x 128 with one fragment set ran at 870 TF/s,
// and a second fragment set did not fit beside 256 accumulators) and one K chunk (split-K slab
// s); the slabs are summed by the step's prep flush (prep.hip SUM), so every output element has
// one fixed summation order.
// Workgroups of one (problem, slab) -- which share their A and B panels -- are placed on one XCD
// (round-robin dispatch), so those panels are fetched into one L2.
//
// Pipeline.  The panels arrive by LDS-DMA (buffer_load ... lds, 16 B per lane, 1 KB = two
// k-rows per instruction) into a ring of kWgStages 32 KB stages, kWgStages - 1 of them in
// flight.  A wave's DMA count per stage is fixed (4), so the wait for a stage is a counted vmcnt;
// the DMA is inline asm, invisible to the compiler's waitcnt pass, which would otherwise wait
// vmcnt(0) for the whole ring before every LDS read.  v3: after the k-step's barrier the wave's
// 32 MFMAs run in four groups of 8 with the stage refill (one DMA pair per group) and the next
// stage's fragment reads between the groups, pinned there by sched_barrier (the A fragments of
// the next stage land in the registers the group before has consumed: one A register set, 32
// VGPRs fewer than two, no spill next to the 128 accumulators): in v2 every wave
// issued its DMAs and all 24 reads right after the barrier, with both waves of a SIMD in
// lockstep, so the matrix pipe idled through that burst (scripts/micro/gemm_lab.hip, headline
// shapes, same box: [1024 x 2048] 127 -> 120 us, [512 x 2048] 70 -> 67 us, both in one launch
// 211 -> 191 us).
//
// Problems of different shapes share one launch (the step's layer-1 [1024 x 2048] and layer-0
// [512 x 2048] gradients, K = 32768): the work items are (problem, slab, tile), one per
// workgroup, each problem with its own split count.
//
// LDS layout.  Row r of a stage holds 256 bf16 (32 chunks of 16 B, no padding); logical chunk c
// sits at physical chunk c ^ f(r), f(r) = 2 (r & 7) + ((r >> 4) & 1).  One transposed read of a
// 16-column tile touches rows {b_q + a} = {0..7, 16..23} (+ 8 for the high half) and two chunks
// per row: under f the 32 (row, chunk) pairs cover each of the 16 bank groups exactly twice -- the
// 2-pass minimum for 512 B -- where the unswizzled rows would all hit the same 8 banks.  The DMA
// writes each lane's 16 B to physical position lane, so a lane fetches the logical chunk that
// belongs there (the global reads stay two whole 512-B rows per instruction).
#include <type_traits>

#include "gemm_common.h"
#include "kernels.h"

namespace dcr {

constexpr int kWgTile = 256;   // output tile edge (M and N)
constexpr int kWgK = 32;       // k rows per stage (one MFMA k step)
constexpr int kWgStages = 4;   // LDS ring stages (kWgStages - 1 in flight)
constexpr int kWgStageB = 2 * kWgK * kWgTile * 2;  // bytes per stage (A + B panels)
constexpr int kWgWaves = 8;                        // 2 per SIMD
constexpr int kWgDmaPerWave = 32 / kWgWaves;       // DMA instructions per wave and stage

__device__ __forceinline__ int wg_swz(int r) { return 2 * (r & 7) + ((r >> 4) & 1); }

// V: measurement variants (scripts/micro/wgrad_lab.hip; the step runs V = 0): bit 0 every k-step
// re-reads the slab's first stage (L2-hot operands), bit 1 no DMA and no stage waits (LDS reads
// of whatever the ring holds), bit 2 (with bit 1) no barriers, bit 3 a 5-stage ring (160 KB),
// bit 4 only the A panel is DMA'd, bit 5 the DMA is issued but never waited for, bit 6 the
// k-step barrier without its lgkmcnt(0), bit 7 no steady-state k-steps (round-5 code: every
// k-step's wait count chosen at run time), bit 8 s_setprio(1) over each MFMA group, bit 9 the
// refill DMA pairs after MFMA groups 1 and 2 (instead of 0 and 1)
template <int V>
__global__ void __launch_bounds__(64 * kWgWaves, kWgWaves / 4) wgrad_kernel(WgradArgs a) {
  constexpr bool HOT = V & 1, NODMA = V & 2, NOBAR = (V & 6) == 6, NOB = V & 16, NOWAIT = V & 34;
  constexpr int ST = (V & 8) ? 5 : kWgStages;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[ST * kWgStageB];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // block -> work item; the items of one (problem, slab) -- which share their A and B panels --
  // are consecutive and dealt to one XCD (round-robin dispatch), so those panels are fetched
  // into one L2
  const int nb = gridDim.x;
  const int lin = (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8;
  if (lin >= a.items) return;  // padding blocks (grid rounded to a multiple of 8)
  int pi = 0;
  while (pi + 1 < a.np && lin >= a.p[pi + 1].item0) ++pi;
  const WgradProblem& P = a.p[pi];
  const int loc = lin - P.item0;
  const int s = loc / P.tiles, tile = loc % P.tiles;
  const int tn = P.N / kWgTile;
  const int m0 = (tile / tn) * kWgTile, n0 = (tile % tn) * kWgTile;
  const int ksteps = a.K / kWgK;
  const int kt0 = (int)((long)ksteps * s / P.S), kt1 = (int)((long)ksteps * (s + 1) / P.S);
  const int nk = kt1 - kt0;

  // DMA: wave w fills k-rows [4 w, 4 w + 4) of both panels, 2 rows per instruction; lane l
  // writes physical chunk (l & 31) of row 4 w + 2 j + (l >> 5)
  const __amdgpu_buffer_rsrc_t ra = gemm_rsrc(P.A);
  const __amdgpu_buffer_rsrc_t rb = gemm_rsrc(P.B);
  unsigned offa[kWgDmaPerWave / 2], offb[kWgDmaPerWave / 2];  // k-step 0 (+ kt * 32 rows)
#pragma unroll
  for (int j = 0; j < kWgDmaPerWave / 2; ++j) {
    const int r = (kWgDmaPerWave) * w + 2 * j + (lane >> 5);
    const int c = (lane & 31) ^ wg_swz(r);  // logical chunk stored at this physical position
    offa[j] = (unsigned)(((size_t)r * P.lda + m0 + 8 * c) * sizeof(bf16));
    offb[j] = (unsigned)(((size_t)r * P.ldb + n0 + 8 * c) * sizeof(bf16));
  }
  const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) void*)lds;
  auto stage_addr = [&](int kt) { return lds0 + ((unsigned)(kt - kt0) % ST) * kWgStageB; };
  // the per-stage strides live in registers: read through P inside the loop, every DMA's
  // "memory" clobber made the compiler reload them (s_load + s_waitcnt lgkmcnt(0) before each
  // DMA pair, which also waits for the wave's in-flight LDS fragment reads; no measurable
  // change on its own, profiles/r5_wgrad_lab.txt wl2 / wl3)
  const unsigned stra = (unsigned)(kWgK * P.lda * sizeof(bf16));
  const unsigned strb = (unsigned)(kWgK * P.ldb * sizeof(bf16));
  auto issue_pair = [&](int kt, int j) {  // this wave's DMA pair j of stage kt
    if constexpr (NODMA) return;
    const unsigned st = stage_addr(kt);
    const unsigned ktd = (unsigned)(HOT ? kt0 : kt);
    const unsigned sa = ktd * stra;
    const unsigned sb = ktd * strb;
    const unsigned r = (unsigned)(kWgDmaPerWave * w + 2 * j);
    gemm_dma(ra, st + r * 512, offa[j], sa);
    if constexpr (!NOB) gemm_dma(rb, st + kWgK * 512 + r * 512, offb[j], sb);
  };

  // fragment read addresses: lane 16q + 4ta + tp reads k-row b_q + ta (lo; + 8 hi), m columns
  // 4 tp .. +3 of its 16-column tile; byte address within a stage panel
  const int q = lane >> 4, ta = (lane & 15) >> 2, tp = lane & 3;
  const int bq = 4 * q + 8 * (q >> 1);
  // wave w: 128 (M) x 64 (N) of the tile = 8 x 4 MFMA tiles
  const int wm = 128 * (w >> 2), wn = 64 * (w & 3);
  // tile i's column chunk is cbase + 2 i with cbase = wm / 8 + tp / 2 in {0, 1, 16, 17}: no bit
  // overlaps 2 i, so its physical chunk is (cbase ^ f(row)) ^ 2 i -- one XOR per read, and only
  // two per-lane constants per half (lo / hi row) instead of 32 addresses
  const int cb_a = (wm >> 3) + (tp >> 1), cb_b = (wn >> 3) + (tp >> 1);
  unsigned rowb[2], xa[2], xb[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = bq + ta + 8 * h;
    rowb[h] = (unsigned)(row * 512 + ((tp & 1) << 3));
    xa[h] = (unsigned)(cb_a ^ wg_swz(row));
    xb[h] = (unsigned)(cb_b ^ wg_swz(row));
  }
  auto rd_a = [&](int kt, u32x4 (&fa)[8], int i0, int i1) {
    const unsigned base = stage_addr(kt);
#pragma unroll
    for (int i = i0; i < i1; ++i) {
      const u32x2 lo = gemm_rd_tr(base + rowb[0] + ((xa[0] ^ (2u * i)) << 4));
      const u32x2 hi = gemm_rd_tr(base + rowb[1] + ((xa[1] ^ (2u * i)) << 4));
      fa[i] = u32x4{lo[0], lo[1], hi[0], hi[1]};
    }
  };
  auto rd_b = [&](int kt, u32x4 (&fb)[4]) {
    const unsigned base = stage_addr(kt) + kWgK * 512;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32x2 lo = gemm_rd_tr(base + rowb[0] + ((xb[0] ^ (2u * j)) << 4));
      const u32x2 hi = gemm_rd_tr(base + rowb[1] + ((xb[1] ^ (2u * j)) << 4));
      fb[j] = u32x4{lo[0], lo[1], hi[0], hi[1]};
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mf = [&](int g, u32x4 (&fa)[8], u32x4 (&fb)[4]) {  // MFMA group g: A tiles 2g, 2g + 1
#pragma unroll
    for (int ii = 2 * g; ii < 2 * g + 2; ++ii)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        acc[ii][jj] = mfma16(__builtin_bit_cast(bf16x8, fa[ii]), __builtin_bit_cast(bf16x8, fb[jj]),
                             acc[ii][jj]);
  };

  // prologue: the first kWgStages stages in flight, stage 0 landed everywhere, its fragments read
  u32x4 fa[8], fb0[4], fb1[4];
  if (nk > 0) {
    const int pro = nk < ST ? nk : ST;
    for (int j = 0; j < pro; ++j) {
      issue_pair(kt0 + j, 0);
      issue_pair(kt0 + j, 1);
    }
    gemm_vm_wait(NOWAIT ? 0 : (pro - 1) * (NOB ? kWgDmaPerWave / 2 : kWgDmaPerWave));
    gemm_barrier();
    rd_b(kt0, fb0);
    rd_a(kt0, fa, 0, 8);
  }
  // k-step i: its fragments are in (fa, fb); between the MFMA groups the next stage's A tiles
  // are read into the registers the previous group has just consumed (ONE A set), its B tiles
  // into the other B set, next to the refill of stage i's slot (two statically indexed B sets:
  // the loop runs two k-steps per trip)
  // STEADY: a k-step with a refill (i + ST < nk), so its conditions and its counted wait are
  // compile-time constants -- no branch cascade of gemm_vm_wait between the barrier-aligned
  // waves' MFMA groups
  auto kstep = [&](int i, u32x4 (&fb)[4], u32x4 (&nb_)[4], auto steady) {
    constexpr bool STEADY = decltype(steady)::value;
    const int kt = kt0 + i;
    const bool more = STEADY || i + 1 < nk;
    const bool refill = STEADY || (more && i + ST < nk);
    if (more) {
      // stage kt+1 landed (the later in-flight stages may stay outstanding), visible to every
      // wave; stage kt's slot was read by every wave before this barrier: it may be refilled
      constexpr int per = NOB ? kWgDmaPerWave / 2 : kWgDmaPerWave;
      if constexpr (NOWAIT) {
      } else if constexpr (STEADY) {
        gemm_vm_wait((ST - 2) * per);
      } else {
        const int later = nk - 2 - i < ST - 2 ? nk - 2 - i : ST - 2;
        gemm_vm_wait(later * per);
      }
      if constexpr (V & 64)
        asm volatile("s_barrier" ::: "memory");
      else if constexpr (!NOBAR)
        gemm_barrier();
    }
    constexpr bool PRIO = V & 256, LATE = V & 512;
    auto mfp = [&](int g) {
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
      mf(g, fa, fb);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    };
    __builtin_amdgcn_sched_barrier(0);
    mfp(0);
    __builtin_amdgcn_sched_barrier(0);
    if (!LATE && refill) issue_pair(kt + ST, 0);
    if (more) {
      rd_b(kt + 1, nb_);
      rd_a(kt + 1, fa, 0, 2);
    }
    __builtin_amdgcn_sched_barrier(0);
    mfp(1);
    __builtin_amdgcn_sched_barrier(0);
    if (!LATE && refill) issue_pair(kt + ST, 1);
    if (LATE && refill) issue_pair(kt + ST, 0);
    if (more) rd_a(kt + 1, fa, 2, 4);
    __builtin_amdgcn_sched_barrier(0);
    mfp(2);
    __builtin_amdgcn_sched_barrier(0);
    if (LATE && refill) issue_pair(kt + ST, 1);
    if (more) rd_a(kt + 1, fa, 4, 6);
    __builtin_amdgcn_sched_barrier(0);
    mfp(3);
    __builtin_amdgcn_sched_barrier(0);
    if (more) rd_a(kt + 1, fa, 6, 8);
  };
  using steady_t = std::integral_constant<bool, true>;
  using tail_t = std::integral_constant<bool, false>;
  int i = 0;
  if constexpr (!(V & 128))
    for (; i + 1 + ST < nk; i += 2) {
      kstep(i, fb0, fb1, steady_t{});
      kstep(i + 1, fb1, fb0, steady_t{});
    }
  for (; i < nk; i += 2) {
    kstep(i, fb0, fb1, tail_t{});
    if (i + 1 < nk) kstep(i + 1, fb1, fb0, tail_t{});
  }

  // D[4q + r][l & 15] of tile (i, j): row m0 + wm + 16 i + 4 q + r, column n0 + wn + 16 j + l%16
  float* c = P.C + (size_t)s * P.slab + (size_t)(m0 + wm + 4 * q) * P.ldc + n0 + wn + (lane & 15);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j) c[(size_t)(16 * i + r) * P.ldc + 16 * j] = acc[i][j][r];
}

bool wgrad_supported(int M, int N, int K) {
  return M > 0 && N > 0 && M % kWgTile == 0 && N % kWgTile == 0 && K % kWgK == 0 && K > 0;
}

// One split count for a launch of problems with `tiles` output tiles in all (M, N multiples of
// 256).  One workgroup per CU (128 KB of LDS ring), so a grid of tiles x S workgroups runs in
// ceil(blocks / cus) rounds of K / S tokens each; every slab adds an M x N fp32 write + read
// (summed by the step tail).  Modelled time: rounds x (K / S) x 0.85 us per 32-token k-step
// + S x tiles x 0.1 us, each slab at least 1024 tokens deep.  (A second partial round costs a
// full round: 3 x 16 tiles x 6 slabs = 288 workgroups ran 367 us vs 230 us at 5 slabs.  The
// round-5 score -- CU utilisation less 1 % per slab -- chose S = 1 for a 2-tile launch, one
// bucket's softmax_w gradient under data parallelism: 2 workgroups, 639 us.)
int wgrad_splits_tiles(int tiles, int K, int cus, double* cost_out) {
  if (cus <= 0) cus = 256;  // (no device: the MI355X's count)
  const int smax = K / 1024 > 1 ? (K / 1024 < kWgradMaxSplit ? K / 1024 : kWgradMaxSplit) : 1;
  int best = 1;
  double best_cost = 1e300;
  for (int S = 1; S <= smax; ++S) {
    const long blocks = (long)tiles * S;
    const long rounds = (blocks + cus - 1) / cus;
    const double cost = (double)rounds * ((double)K / S / kWgK) * 0.85 + 0.1 * S * tiles;
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = S;
    }
  }
  if (cost_out) *cost_out = tiles > 0 ? best_cost : 0.0;
  return best;
}

int wgrad_splits(int np, int M, int N, int K, int cus) {
  return wgrad_splits_tiles(np * (M / kWgTile) * (N / kWgTile), K, cus);
}

void launch_wgrad(WgradArgs& a, hipStream_t s) {
  int items = 0;
  for (int i = 0; i < a.np; ++i) {
    a.p[i].tiles = (a.p[i].M / kWgTile) * (a.p[i].N / kWgTile);
    a.p[i].item0 = items;
    items += a.p[i].tiles * a.p[i].S;
  }
  a.items = items;
  const int grid = (items + 7) / 8 * 8;
  wgrad_kernel<0><<<grid, 64 * kWgWaves, 0, s>>>(a);
}

}  // namespace dcr
