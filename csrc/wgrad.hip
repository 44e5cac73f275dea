// Token-reduction weight-gradient GEMM for gfx950:  C_s[m, n] = sum_{k in chunk s} A[k, m] B[k, n]
//
// Reference: the weight gradients of the unrolled cell (tf.gradients through model.py:72, summed
// over all T x B tokens).  Both operands lie token-major in memory (A = h_{t-1} or the layer input
// [K tokens, M], B = dZ [K tokens, N]), i.e. K is the OUTER index of both, so neither is an MFMA
// fragment as stored.  Each workgroup streams [32 x 256] k-row panels of A and B through LDS as
// they lie in memory (coalesced 512-B rows) and reads them back transposed with
// ds_read_b64_tr_b16 (CDNA4's transposing LDS read), which hands every lane the 8 consecutive-k
// bf16 values of one m (or n) -- exactly the A / B fragment of v_mfma_f32_16x16x32_bf16.
//
// Tiling.  A workgroup owns a 256 x 256 output tile (4 waves of 128 x 128 = 8 x 8 MFMA tiles, 256
// fp32 accumulators per lane) and one K chunk (split-K slab s); the slabs are summed by the
// step's prep flush (prep.hip SUM), so every output element has one fixed summation order.  The
// 256 x 256 tile halves the operand traffic of a 256 x 128 library tile (the three headline
// gradients are operand-stream bound: 2 x 32768 x (512 + 2048) bf16 per GEMM, read by every
// tile of a row / column).  Workgroups of one (problem, slab) -- which share their A and B panels
// -- are placed on one XCD (round-robin dispatch), so those panels are fetched into one L2.
//
// LDS layout.  A stage holds 32 k-rows of 256 bf16 at a row stride of 272 bf16 (136 dwords =
// 8 mod 64 banks).  The 8 k values of lane group q (lanes 16q .. 16q+15) are the k-rows
// {b_q .. b_q+3} (lo read) and {b_q+8 .. b_q+11} (hi read), b_q = 4q + 8 (q >> 1): the 32 lanes
// of each half-wave then hit 64 distinct banks.  A and B use the same k permutation, so the
// products are unchanged.  Two stages (69.6 KB), one barrier per k step; the next stage's global
// loads are issued before the current stage's MFMAs and written to LDS after them.
//
// Measured (scripts/micro/wgrad_bench.py, same box as the library form): the three headline
// gradients in one launch 230 us vs 279 us as split-K library bmm's in isolation, but on par in
// the training step (228 vs ~220 us: there the library GEMMs find dZ partly in L2 / MALL right
// after the BPTT), so the step keeps the library GEMMs by default (DCR_DEBUG=wgrad=1 selects this
// kernel).  Rejected variants: BK = 64 (274 us), a second register stage (spills), a 4-stage
// LDS-DMA pipeline with counted vmcnt and raw barriers (312 vs 299 us library on its box).
#include "common.h"
#include "kernels.h"

namespace dcr {

constexpr int kWgTile = 256;             // output tile edge (M and N)
constexpr int kWgK = 32;                 // k rows per stage (one MFMA k step)
constexpr int kWgLd = kWgTile + 16;      // LDS row stride (bf16): 136 dwords = 8 mod 64

typedef short s16x4_wg __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 wg_frag(const bf16* base) {
  // base = &stage[b_q + a][col0 + 4 p]  for lane 16q + 4a + p
  const s16x4_wg lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_wg*)base);
  const s16x4_wg hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4_wg*)(base + 8 * kWgLd));
  u32x4 u;
  u[0] = (unsigned)(unsigned short)lo[0] | ((unsigned)(unsigned short)lo[1] << 16);
  u[1] = (unsigned)(unsigned short)lo[2] | ((unsigned)(unsigned short)lo[3] << 16);
  u[2] = (unsigned)(unsigned short)hi[0] | ((unsigned)(unsigned short)hi[1] << 16);
  u[3] = (unsigned)(unsigned short)hi[2] | ((unsigned)(unsigned short)hi[3] << 16);
  return __builtin_bit_cast(bf16x8, u);
}

__global__ void __launch_bounds__(256, 1) wgrad_kernel(WgradArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 lds[2][2][kWgK][kWgLd];  // [stage][A/B][k][col]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // block -> (group = (problem, slab), tile in group); a group's tiles on one XCD
  const int nb = gridDim.x;
  const int lin = (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8;
  const int grp = lin / a.tiles, tile = lin % a.tiles;
  if (grp >= a.np * a.S) return;  // padding blocks (grid rounded to a multiple of 8)
  const int p = grp / a.S, s = grp % a.S;
  const WgradProblem& P = a.p[p];
  const int tn = a.N / kWgTile;
  const int m0 = (tile / tn) * kWgTile, n0 = (tile % tn) * kWgTile;
  const int ksteps = a.K / kWgK;
  const int kt0 = (int)((long)ksteps * s / a.S), kt1 = (int)((long)ksteps * (s + 1) / a.S);

  // staging: thread t -> k-row (t >> 5) + 8 j, columns 8 (t & 31) .. +7, for j < 4
  const int srow = threadIdx.x >> 5, scol = 8 * (threadIdx.x & 31);
  const bf16* ga = P.A + (size_t)srow * P.lda + m0 + scol;
  const bf16* gb = P.B + (size_t)srow * P.ldb + n0 + scol;
  bf16x8 st[2][4];  // [A/B][j]
  auto fetch = [&](int kt) {
    const size_t k0 = (size_t)kt * kWgK;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      st[0][j] = ld8(ga + (k0 + 8 * j) * P.lda);
      st[1][j] = ld8(gb + (k0 + 8 * j) * P.ldb);
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      *reinterpret_cast<bf16x8*>(&lds[buf][0][srow + 8 * j][scol]) = st[0][j];
      *reinterpret_cast<bf16x8*>(&lds[buf][1][srow + 8 * j][scol]) = st[1][j];
    }
  };

  // fragment read addresses: lane 16q + 4a + pp reads k-row b_q + a, columns 4 pp .. +3 of
  // its 16-column tile
  const int q = lane >> 4, ta = (lane & 15) >> 2, tp = lane & 3;
  const int bq = 4 * q + 8 * (q >> 1);
  const int wm = 128 * (w >> 1), wn = 128 * (w & 1);
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kt0 < kt1) {
    fetch(kt0);
    stash(0);
  }
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const int buf = (kt - kt0) & 1;
    if (kt + 1 < kt1) fetch(kt + 1);
    const bf16* la = &lds[buf][0][bq + ta][wm + 4 * tp];
    const bf16* lb = &lds[buf][1][bq + ta][wn + 4 * tp];
    bf16x8 fa[8], fb[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = wg_frag(la + 16 * i);
#pragma unroll
    for (int j = 0; j < 8; ++j) fb[j] = wg_frag(lb + 16 * j);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
    if (kt + 1 < kt1) stash(buf ^ 1);  // that stage was last read before the previous barrier
    __syncthreads();
  }

  // D[4q + r][l & 15] of tile (i, j): row m0 + wm + 16 i + 4 q + r, column n0 + wn + 16 j + l%16
  float* c = P.C + (size_t)s * P.slab + (size_t)(m0 + wm + 4 * q) * P.ldc + n0 + wn + (lane & 15);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 8; ++j) c[(size_t)(16 * i + r) * P.ldc + 16 * j] = acc[i][j][r];
}

bool wgrad_supported(int M, int N, int K) {
  return M > 0 && N > 0 && M % kWgTile == 0 && N % kWgTile == 0 && K % kWgK == 0 && K > 0;
}

// Slabs per problem.  One workgroup per CU (256 accumulators per lane), so a grid of np x tiles x S
// workgroups runs in ceil(blocks / cus) rounds; pick the S with the best CU utilisation
// blocks / (rounds x cus), less 1 % per slab (each slab is an extra M x N fp32 write + read in the
// flush), each slab at least 1024 tokens deep.  (A second partial round costs a full round:
// 3 x 16 tiles x 6 slabs = 288 workgroups ran 367 us vs 230 us at 5 slabs.)
int wgrad_splits(int np, int M, int N, int K, int cus) {
  const int tiles = (M / kWgTile) * (N / kWgTile);
  const int smax = K / 1024 > 1 ? (K / 1024 < kWgradMaxSplit ? K / 1024 : kWgradMaxSplit) : 1;
  int best = 1;
  double best_score = -1.0;
  for (int S = 1; S <= smax; ++S) {
    const long blocks = (long)np * tiles * S;
    const long rounds = (blocks + cus - 1) / cus;
    const double score = (double)blocks / ((double)rounds * cus) - 0.01 * S;
    if (score > best_score + 1e-9) {
      best_score = score;
      best = S;
    }
  }
  return best;
}

void launch_wgrad(const WgradArgs& a, hipStream_t s) {
  const int blocks = a.np * a.S * a.tiles;
  const int grid = (blocks + 7) / 8 * 8;
  wgrad_kernel<<<grid, 256, 0, s>>>(a);
}

}  // namespace dcr
