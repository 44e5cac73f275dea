// Fused large-H LSTM time step for gfx950: one MFMA GEMM over the step's recurrent product with
// the cell (forward) or cell-backward (BPTT) epilogue in registers.
//
// Reference: the static unroll of model.py:72 (per time step a MatMul of [x_t, h_{t-1}] with the
// LSTM kernel + BiasAdd + the pointwise gate math, model.py:15-36 / TF's BasicLSTMCell) and its
// tf.gradients BPTT (model.py:91).  For rnn_size > 1024 (BASELINE config 4: 4-layer LSTM-2048) no
// weights-resident persistent kernel fits the register file (W_h is 32 MB bf16 per layer), so a
// step is one launch; the input projection of all T steps ran before as one token GEMM (or, for
// layer 0, is the [V, 4H] table gathered by id).
//
//   forward  : Z^T[4H, B] = W_hᵀ[4H, H] · h_{t-1}[B, H]ᵀ   -> c_t, h_t, gates (bf16)
//   backward : dh^T[H, B] = W_h[H, 4H] · dZ_{t+1}[B, 4H]ᵀ  -> dZ_t (bf16), dc carry
//
// Both operands are K-contiguous rows (W_hᵀ / W_h in their bf16 layouts, h / dZ row-major), so
// mfma_f32_16x16x32_bf16 takes them swapped (A = weight rows, B = batch rows) and a lane ends up
// with 4 consecutive hidden units of one batch row in each accumulator.  In the forward the
// workgroup tile's weight rows are [gate][unit] (4 x BU rows), so the wave that owns 16 units
// holds their i, j, f, o pre-activations in 4 accumulators of the same lane: the cell update is
// lane-local, and every epilogue access is a 16-B (fp32) / 8-B (bf16) vector of 4 units -- no
// fp32 [B, 4H] pre-activation round trip through memory (the library path wrote and re-read it).
//
// Pipeline.  The A (weights) and B (activations) k-tiles of a stage are DMA'd straight into LDS
// (buffer_load ... lds, 16 B per lane, 1 KB per instruction) through three stage buffers; the
// source address is pre-swizzled so the LDS image is lane-linear for the DMA yet the fragment
// reads (ds_read_b128, 16 rows x 16 B per quarter-wave) hit 16 distinct bank groups.  One raw
// barrier per stage (no __syncthreads: its fence would drain the in-flight DMAs); every wait on
// the DMAs is a counted vmcnt, every fragment read inline asm (the compiler cannot tell the
// buffer being read from those being filled and would otherwise wait vmcnt(0)); the next
// k-step's fragments are read while the current one's MFMAs run.  Activation rows >= B read
// zero through the buffer range check, so any batch works.
//
// Decomposition (per launch = one time step of one layer): tiles of BU units x BN batch rows;
// WK > 1 splits a stage's k-steps over waves (reduced through LDS), S > 1 splits K over
// workgroups (the last-arriving slice sums the others' fp32 slabs, cdna_hip_programming.md §5
// "in-launch split-K reduction", then runs the epilogue).  Workgroups of one unit block (same
// weight rows) and a tile's slices are placed on one XCD.
#include "common.h"
#include "kernels.h"
#include "persist_common.h"
#include "debug_env.h"

namespace dcr {

// (outside the anonymous namespace: the kernel template is instantiated on it, and a kernel's
// host stub must have external linkage)
template <int BU_, int BN_, int WM_, int WN_, int WK_, bool BWD_>
struct BsCfg {
  static constexpr int BU = BU_, BN = BN_, WM = WM_, WN = WN_, WK = WK_;
  static constexpr bool BWD = BWD_;
  static constexpr int BM = BWD ? BU : 4 * BU;       // weight rows per tile
  static constexpr int NW = WM * WN * WK;            // waves
  static constexpr int BK = 32 * WK > 64 ? 32 * WK : 64;
  static constexpr int NSUB = BK / 32;               // k-steps per stage
  static constexpr int NSW = NSUB / WK;              // k-steps per stage and wave
  static constexpr int ROWB = BK * 2;                // LDS row bytes
  static constexpr int CPR = BK / 8;                 // 16-B chunks per row
  static constexpr int RPD = 1024 / ROWB;            // rows per 1 KB DMA instruction
  static constexpr int SROWS = BM + BN;
  static constexpr int SBYTES = SROWS * ROWB;
  static constexpr int NSTAGE = 3;
  static constexpr int DPS = SROWS / RPD;            // DMA instructions per stage
  static constexpr int DPW = DPS / NW;               // ... per wave
  static constexpr int UFW = BU / WM / 16;           // 16-unit fragments per wave
  static constexpr int FM = BWD ? UFW : 4 * UFW;     // weight-row fragments per wave
  static constexpr int FN = BN / WN / 16;            // batch fragments per wave
  static constexpr int FNR = FN / WK;                // batch fragments a wave finishes
  static constexpr int LDS = NSTAGE * SBYTES > NW * FM * FN * 1024 ? NSTAGE * SBYTES
                                                                    : NW * FM * FN * 1024;
  static_assert(DPS % NW == 0, "DMA rows must split evenly over waves");
  static_assert(NSUB % WK == 0 && FN % WK == 0 && UFW >= 1 && FN >= 1, "tile shape");
  static_assert(BM % 16 == 0 && RPD * ROWB == 1024, "row geometry");
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
};

namespace {

// wave-uniform wait until at most n of this wave's vector-memory operations are outstanding
__device__ __forceinline__ void bs_vm_wait(int n) {
#define BS_VMW(k) \
  case k:         \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
  switch (n) {
    BS_VMW(1) BS_VMW(2) BS_VMW(3) BS_VMW(4) BS_VMW(5) BS_VMW(6) BS_VMW(7) BS_VMW(8) BS_VMW(9)
    BS_VMW(10) BS_VMW(11) BS_VMW(12) BS_VMW(13) BS_VMW(14) BS_VMW(15) BS_VMW(16) BS_VMW(17)
    BS_VMW(18) BS_VMW(19) BS_VMW(20) BS_VMW(21) BS_VMW(22) BS_VMW(23) BS_VMW(24)
    default:
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#undef BS_VMW
}
__device__ __forceinline__ void bs_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ unsigned bs_lds(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}
// (inline asm only inside __device__ helpers: in a __global__ body the host-side parse rejects
// the "v" constraint and silently drops the kernel's host stub)
__device__ __forceinline__ void bs_vm_wait0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// one 1 KB LDS-DMA: lane l's 16 source bytes land at lds + 16 l
__device__ __forceinline__ void bs_dma(__amdgpu_buffer_rsrc_t r, unsigned char* lds, unsigned voff,
                                       unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           voff, soff, 0, 0);
}

__device__ __forceinline__ float4 bs_ld4f(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void bs_st4f(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
__device__ __forceinline__ void bs_ld4bf(const bf16* p, float (&o)[4]) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  o[0] = (float)v[0]; o[1] = (float)v[1]; o[2] = (float)v[2]; o[3] = (float)v[3];
}
__device__ __forceinline__ void bs_st4bf(bf16* p, float a, float b, float c, float d) {
  bf16x4 v;
  v[0] = f2bf(a); v[1] = f2bf(b); v[2] = f2bf(c); v[3] = f2bf(d);
  *reinterpret_cast<bf16x4*>(p) = v;
}

// XOR swizzle of a row's 16-B chunks: the 16 rows of a fragment read land on 16 distinct bank
// groups (128-B rows: two rows share a 256-B bank row, so rows 2i and 2i+1 differ in the bank
// half and (r >> 1) spreads the chunk; 256-B rows: r itself)
template <int CPR>
__device__ __forceinline__ int bs_swz(int r) {
  return CPR == 8 ? ((r >> 1) & 7) : (r & 15);
}

}  // namespace

template <class C>
__global__ void __launch_bounds__(C::NW * 64, 1) lstm_gemm_step_kernel(BigStepArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[C::LDS];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w % C::WM, wn = (w / C::WM) % C::WN, wk = w / (C::WM * C::WN);
  const int H = a.H, B = a.B, S = a.S;
  const int K = C::BWD ? 4 * H : H;
  const int tiles_b = (B + C::BN - 1) / C::BN;
  const int tiles_u = H / C::BU;

  // XCD-aware bijective remap (blocks b, b+8, ... share an XCD): consecutive `lin` on one XCD
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb / 8, r8 = nb % 8, xcd = bid % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int split = lin % S, tb = (lin / S) % tiles_b, tu = lin / (S * tiles_b);
  if (tu >= tiles_u) return;
  const int u0 = tu * C::BU, n0 = tb * C::BN;
  const int tile = tu * tiles_b + tb;
  const int nkt = K / C::BK;
  const int kt0 = (int)((long)nkt * split / S), kt1 = (int)((long)nkt * (split + 1) / S);
  const int nk = kt1 - kt0;

  const __amdgpu_buffer_rsrc_t ra = make_rsrc(a.A, sizeof(bf16) * (size_t)(C::BWD ? H : 4 * H) * K);
  const __amdgpu_buffer_rsrc_t rx = make_rsrc(a.X, sizeof(bf16) * (size_t)B * K);

  // this wave's DMA instructions: stage rows [j RPD, (j+1) RPD), j = w DPW + i; lane l fills
  // LDS row j RPD + l / CPR, chunk l % CPR, from the source chunk (l % CPR) ^ swz(row)
  unsigned doff[C::DPW];
#pragma unroll
  for (int i = 0; i < C::DPW; ++i) {
    const int j = w * C::DPW + i;
    const int row = j * C::RPD + lane / C::CPR;
    const int lch = (lane % C::CPR) ^ bs_swz<C::CPR>(row);
    size_t grow;
    if (j * C::RPD < C::BM) {
      grow = C::BWD ? (size_t)(u0 + row) : (size_t)(row / C::BU) * H + u0 + row % C::BU;
    } else {
      grow = (size_t)(n0 + row - C::BM);
    }
    doff[i] = (unsigned)((grow * K + (size_t)kt0 * C::BK + 8 * lch) * sizeof(bf16));
  }
  auto dma = [&](int it) {  // stage it (k-tile kt0 + it) into buffer it % 3
    unsigned char* sb = lds + (it % C::NSTAGE) * C::SBYTES;
    const unsigned koff = (unsigned)(it * C::BK * sizeof(bf16));
#pragma unroll
    for (int i = 0; i < C::DPW; ++i) {
      const int j = w * C::DPW + i;
      if (j * C::RPD < C::BM)
        bs_dma(ra, sb + j * 1024, doff[i], koff);
      else
        bs_dma(rx, sb + j * 1024, doff[i], koff);
    }
  };

  // fragment read offsets: lane reads row (lane & 15) of a 16-row fragment, logical chunk
  // 4 s + (lane >> 4) of k-step s
  const int fi = lane & 15, fq = lane >> 4;
  unsigned roff[C::NSW];
#pragma unroll
  for (int j = 0; j < C::NSW; ++j) {
    const int s = wk + j * C::WK;
    roff[j] = (unsigned)(fi * C::ROWB + (((4 * s + fq) ^ bs_swz<C::CPR>(fi)) * 16));
  }
  int arow[C::FM], brow[C::FN];  // fragment base rows in the stage
#pragma unroll
  for (int m = 0; m < C::FM; ++m) {
    if (C::BWD) {
      arow[m] = wm * (C::BU / C::WM) + 16 * m;
    } else {
      const int g = m / C::UFW, uf = m % C::UFW;
      arow[m] = g * C::BU + wm * (C::BU / C::WM) + 16 * uf;
    }
  }
#pragma unroll
  for (int n = 0; n < C::FN; ++n) brow[n] = C::BM + wn * (C::BN / C::WN) + 16 * n;

  f32x4 acc[C::FM][C::FN];
#pragma unroll
  for (int m = 0; m < C::FM; ++m)
#pragma unroll
    for (int n = 0; n < C::FN; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // two fragment register sets, addressed only with compile-time slots (a runtime slot index
  // would make the compiler move registers whose LDS reads are still in flight)
  u32x4 fa0[C::FM], fb0[C::FN], fa1[C::FM], fb1[C::FN];
  // plain LDS loads: the compiler tracks their lgkmcnt itself (with ONE __shared__ array it
  // does not make them wait for the in-flight DMAs)
  auto reads = [&](int it, int j, u32x4 (&fa)[C::FM], u32x4 (&fb)[C::FN]) {
    const unsigned char* base = lds + (it % C::NSTAGE) * C::SBYTES + roff[j];
#pragma unroll
    for (int m = 0; m < C::FM; ++m) fa[m] = *reinterpret_cast<const u32x4*>(base + arow[m] * C::ROWB);
#pragma unroll
    for (int n = 0; n < C::FN; ++n) fb[n] = *reinterpret_cast<const u32x4*>(base + brow[n] * C::ROWB);
  };
  auto mfmas = [&](u32x4 (&fa)[C::FM], u32x4 (&fb)[C::FN]) {
#pragma unroll
    for (int n = 0; n < C::FN; ++n) {
      const bf16x8 b8 = __builtin_bit_cast(bf16x8, fb[n]);
#pragma unroll
      for (int m = 0; m < C::FM; ++m)
        acc[m][n] = mfma16(__builtin_bit_cast(bf16x8, fa[m]), b8, acc[m][n]);
    }
  };
  // one k-step: queue the next k-step's fragment reads into the other set, run this set's
  // MFMAs
  auto sub = [&](int it, int j, u32x4 (&fa)[C::FM], u32x4 (&fb)[C::FN], u32x4 (&na)[C::FM],
                 u32x4 (&nb)[C::FN]) {
    if (j + 1 < C::NSW) {
      reads(it, j + 1, na, nb);
    } else if (it + 1 < nk) {
      // stage it+1 landed (only stage it+2 may still be in flight), every wave is done
      // reading stage it (retired above): refill its buffer with stage it+3
      if (it + 2 < nk)  // (a constant count per branch: no runtime-count switch in the loop)
        bs_vm_wait(C::DPW);
      else
        bs_vm_wait0();
      bs_barrier();
      if (it + 3 < nk) dma(it + 3);
      reads(it + 1, 0, na, nb);
    }
    mfmas(fa, fb);
  };

  if (nk > 0) {
#pragma unroll
    for (int p = 0; p < C::NSTAGE; ++p)
      if (p < nk) dma(p);
    bs_vm_wait(C::DPW * (nk - 1 < C::NSTAGE - 1 ? nk - 1 : C::NSTAGE - 1));
    bs_barrier();
    reads(0, 0, fa0, fb0);
    if constexpr (C::NSW % 2 == 0) {  // k-step q of the wave uses set q & 1 = j & 1
      for (int it = 0; it < nk; ++it) {
#pragma unroll
        for (int j = 0; j < C::NSW; j += 2) {
          sub(it, j, fa0, fb0, fa1, fb1);
          sub(it, j + 1, fa1, fb1, fa0, fb0);
        }
      }
    } else {  // one k-step per stage: set it & 1
      static_assert(C::NSW == 1, "k-steps per stage and wave: 1 or even");
      int it = 0;
      for (; it + 1 < nk; it += 2) {
        sub(it, 0, fa0, fb0, fa1, fb1);
        sub(it + 1, 0, fa1, fb1, fa0, fb0);
      }
      if (it < nk) sub(it, 0, fa0, fb0, fa1, fb1);
    }
  }

  // ---- reduce the wave k-split (WK > 1) through LDS: wave (wm, wn, wk) finishes the batch
  // fragments [wk FNR, (wk+1) FNR) of its (wm, wn) tile
  f32x4 red[C::FM][C::FNR];
  if constexpr (C::WK > 1) {
    __syncthreads();  // every stage read has retired (no DMA in flight)
    f32x4* part = reinterpret_cast<f32x4*>(lds);
#pragma unroll
    for (int m = 0; m < C::FM; ++m)
#pragma unroll
      for (int n = 0; n < C::FN; ++n) part[((w * C::FM + m) * C::FN + n) * 64 + lane] = acc[m][n];
    __syncthreads();
#pragma unroll
    for (int m = 0; m < C::FM; ++m)
#pragma unroll
      for (int r = 0; r < C::FNR; ++r) {
        const int n = wk * C::FNR + r;
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < C::WK; ++k) {
          const int ww = (k * C::WN + wn) * C::WM + wm;
          v += part[((ww * C::FM + m) * C::FN + n) * 64 + lane];
        }
        red[m][r] = v;
      }
  } else {
#pragma unroll
    for (int m = 0; m < C::FM; ++m)
#pragma unroll
      for (int r = 0; r < C::FNR; ++r) red[m][r] = acc[m][r];
  }

  // ---- split-K over workgroups: the last-arriving slice sums the others' slabs
  if (S > 1) {
    constexpr int TILE_F4 = C::NW * C::FM * C::FNR * 64;  // f32x4 per slab
    f32x4* slab = reinterpret_cast<f32x4*>(a.ws) + ((size_t)tile * S) * TILE_F4;
#pragma unroll
    for (int m = 0; m < C::FM; ++m)
#pragma unroll
      for (int r = 0; r < C::FNR; ++r)
        slab[(size_t)split * TILE_F4 + ((w * C::FM + m) * C::FNR + r) * 64 + lane] = red[m][r];
    bs_vm_wait0();
    __syncthreads();
    unsigned* flag = reinterpret_cast<unsigned*>(lds);
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      bs_vm_wait0();
      const unsigned t = __hip_atomic_fetch_add(a.cnt + tile, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      const unsigned last = t == (unsigned)(S - 1);
      if (last) {
        __hip_atomic_store(a.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        bs_vm_wait0();
      }
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    for (int s2 = 0; s2 < S; ++s2) {
      if (s2 == split) continue;
#pragma unroll
      for (int m = 0; m < C::FM; ++m)
#pragma unroll
        for (int r = 0; r < C::FNR; ++r)
          red[m][r] += slab[(size_t)s2 * TILE_F4 + ((w * C::FM + m) * C::FNR + r) * 64 + lane];
    }
  }

  // ---- epilogue: lane -> batch row b, 4 consecutive units per fragment
  const LstmEwArgs& e = a.ew;
  const size_t G = 4 * (size_t)H;
#pragma unroll
  for (int r = 0; r < C::FNR; ++r) {
    const int n = wk * C::FNR + r;
    const int b = n0 + wn * (C::BN / C::WN) + 16 * n + fi;
    if (b >= B) continue;
    if constexpr (!C::BWD) {
      const float* zrow = e.ids ? e.zx + (size_t)e.ids[b] * G : e.zx + (size_t)b * G;
#pragma unroll
      for (int uf = 0; uf < C::UFW; ++uf) {
        const int u = u0 + wm * (C::BU / C::WM) + 16 * uf + 4 * fq;
        const size_t bh = (size_t)b * H + u;
        float z[4][4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 v = bs_ld4f(zrow + (size_t)g * H + u);
          const f32x4 c4 = red[g * C::UFW + uf][r];
          z[g][0] = c4[0] + v.x; z[g][1] = c4[1] + v.y; z[g][2] = c4[2] + v.z; z[g][3] = c4[3] + v.w;
          if (e.bias) {
            const float4 bv = bs_ld4f(e.bias + (size_t)g * H + u);
            z[g][0] += bv.x; z[g][1] += bv.y; z[g][2] += bv.z; z[g][3] += bv.w;
          }
        }
        const float4 cpv = bs_ld4f(e.cprev + bh);
        const float cp[4] = {cpv.x, cpv.y, cpv.z, cpv.w};
        float gi[4], gj[4], gf[4], go[4], cn[4], hc[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          gi[k] = sigmoidf_(z[0][k]);
          gj[k] = tanhf_(z[1][k]);
          gf[k] = sigmoidf_(z[2][k] + e.forget_bias);
          go[k] = sigmoidf_(z[3][k]);
          cn[k] = gf[k] * cp[k] + gi[k] * gj[k];
          hc[k] = go[k] * tanhf_(cn[k]);
        }
        bs_st4f(e.cout + bh, cn[0], cn[1], cn[2], cn[3]);
        bs_st4bf(e.hout + bh, hc[0], hc[1], hc[2], hc[3]);
        if (e.hout32) bs_st4f(e.hout32 + bh, hc[0], hc[1], hc[2], hc[3]);
        bf16* gp = e.gates + (size_t)b * G + u;
        bs_st4bf(gp, gi[0], gi[1], gi[2], gi[3]);
        bs_st4bf(gp + H, gj[0], gj[1], gj[2], gj[3]);
        bs_st4bf(gp + 2 * H, gf[0], gf[1], gf[2], gf[3]);
        bs_st4bf(gp + 3 * H, go[0], go[1], go[2], go[3]);
      }
    } else {
#pragma unroll
      for (int mf = 0; mf < C::FM; ++mf) {
        const int u = u0 + wm * (C::BU / C::WM) + 16 * mf + 4 * fq;
        const size_t bh = (size_t)b * H + u;
        const float4 dt = bs_ld4f(e.dtop + bh);
        const f32x4 c4 = red[mf][r];
        const float dh[4] = {c4[0] + dt.x, c4[1] + dt.y, c4[2] + dt.z, c4[3] + dt.w};
        float gi[4], gj[4], gf[4], go[4];
        const bf16* gp = e.gates_in + (size_t)b * G + u;
        bs_ld4bf(gp, gi); bs_ld4bf(gp + H, gj); bs_ld4bf(gp + 2 * H, gf); bs_ld4bf(gp + 3 * H, go);
        const float4 cv = bs_ld4f(e.c + bh), cpv = bs_ld4f(e.cprev + bh), dcv4 = bs_ld4f(e.dc + bh);
        const float cc[4] = {cv.x, cv.y, cv.z, cv.w}, cp[4] = {cpv.x, cpv.y, cpv.z, cpv.w};
        const float dcin[4] = {dcv4.x, dcv4.y, dcv4.z, dcv4.w};
        float di[4], dj[4], df[4], dO[4], dcp[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {  // same math as lstm_ew.hip / rnn_step.hip
          const float th = tanhf_(cc[k]);
          const float dcv = dcin[k] + dh[k] * go[k] * (1.f - th * th);
          dO[k] = dh[k] * th * go[k] * (1.f - go[k]);
          di[k] = dcv * gj[k] * gi[k] * (1.f - gi[k]);
          dj[k] = dcv * gi[k] * (1.f - gj[k] * gj[k]);
          df[k] = dcv * cp[k] * gf[k] * (1.f - gf[k]);
          dcp[k] = dcv * gf[k];
        }
        bf16* dz = e.dz_out + (size_t)b * G + u;
        bs_st4bf(dz, di[0], di[1], di[2], di[3]);
        bs_st4bf(dz + H, dj[0], dj[1], dj[2], dj[3]);
        bs_st4bf(dz + 2 * H, df[0], df[1], df[2], df[3]);
        bs_st4bf(dz + 3 * H, dO[0], dO[1], dO[2], dO[3]);
        bs_st4f(e.dc + bh, dcp[0], dcp[1], dcp[2], dcp[3]);
      }
    }
  }
}

// Configurations (id: shape).  L = large batch (one K slice per tile where the tile count fills
// the chip), S = small batch (16- / 64-unit tiles, a stage's k-steps split over the 4 waves);
// *8 = 8 waves (two per SIMD).  DCR_DEBUG=bigstep_cfg=<id> forces one (same direction).
using Cfg0 = BsCfg<64, 128, 4, 1, 1, false>;   // FwdL : 256 weight rows x 128 batch, 4 waves
using Cfg1 = BsCfg<16, 64, 1, 1, 4, false>;    // FwdS : 64 x 64, BK = 128
using Cfg2 = BsCfg<128, 128, 2, 2, 1, true>;   // BwdL : 128 x 128
using Cfg3 = BsCfg<64, 64, 1, 1, 4, true>;     // BwdS : 64 x 64, BK = 128
using Cfg4 = BsCfg<64, 128, 4, 2, 1, false>;   // FwdL8: 256 x 128, 8 waves of 64 x 64
using Cfg5 = BsCfg<128, 128, 2, 4, 1, true>;   // BwdL8: 128 x 128, 8 waves of 64 x 32
using Cfg6 = BsCfg<32, 128, 2, 4, 1, false>;   // FwdM8: 128 x 128, 8 waves of 64 x 32
using Cfg7 = BsCfg<32, 256, 2, 4, 1, false>;   // FwdW8: 128 x 256, 8 waves of 64 x 64
using Cfg8 = BsCfg<64, 128, 1, 4, 1, true>;    // BwdN : 64 x 128, 4 waves of 64 x 32 (no split)
using Cfg9 = BsCfg<64, 128, 1, 4, 2, true>;    // BwdN8: 64 x 128, 8 waves (2-way wave k split)
using Cfg10 = BsCfg<128, 64, 2, 2, 1, true>;   // BwdM : 128 x 64, 4 waves of 64 x 32
using Cfg11 = BsCfg<64, 256, 1, 4, 1, true>;   // BwdW : 64 x 256, 4 waves of 64 x 64

namespace {
struct BsPlan {
  int cfg, BU, BN, BK, NW, tiles, S;
};

template <class C>
BsPlan bs_fill(int cfg) {
  BsPlan p{};
  p.cfg = cfg;
  p.BU = C::BU;
  p.BN = C::BN;
  p.BK = C::BK;
  p.NW = C::NW;
  return p;
}

BsPlan bs_cfg(int id) {
  switch (id) {
    case 0: return bs_fill<Cfg0>(0);
    case 1: return bs_fill<Cfg1>(1);
    case 2: return bs_fill<Cfg2>(2);
    case 3: return bs_fill<Cfg3>(3);
    case 4: return bs_fill<Cfg4>(4);
    case 5: return bs_fill<Cfg5>(5);
    case 6: return bs_fill<Cfg6>(6);
    case 8: return bs_fill<Cfg8>(8);
    case 9: return bs_fill<Cfg9>(9);
    case 10: return bs_fill<Cfg10>(10);
    case 11: return bs_fill<Cfg11>(11);
    default: return bs_fill<Cfg7>(7);
  }
}
bool bs_cfg_bwd(int id) { return id == 2 || id == 3 || id == 5 || id >= 8; }

BsPlan bs_plan(bool bwd, int B, int H, int cus, int force_S) {
  // forward: the configuration whose grid is closest to one workgroup per CU without a K split
  // (scripts/micro/big_step_bench.py at H = 2048: B = 128 cfg 1 13.7 us, B = 512 cfg 6 26.9 us,
  // B = 1024 cfg 4 45.7 us; split-K slices of large tiles lose to the serial slab reduction)
  int id = bwd ? (B >= 256 ? 2 : 3) : (B <= 160 ? 1 : B <= 640 ? 6 : 7);
  const int forced = debug_int("bigstep_cfg", -1);
  if (forced >= 0 && forced <= 11 && bs_cfg_bwd(forced) == bwd && H % bs_cfg(forced).BU == 0)
    id = forced;
  BsPlan p = bs_cfg(id);
  p.tiles = (H / p.BU) * ((B + p.BN - 1) / p.BN);
  const int nkt = (bwd ? 4 * H : H) / p.BK;
  int S = 1;
  // split K until the grid fills the chip, each slice keeping >= 4 k-tiles
  while (p.tiles * S * 2 <= cus && nkt / (S * 2) >= 4) S *= 2;
  if (force_S > 0) S = force_S;
  p.S = S;
  return p;
}
}  // namespace

bool big_step_supported(int B, int H) {
  return B >= 1 && H >= 128 && H % 128 == 0;
}

// fp32 workspace floats and tickets a launch of this shape needs
void big_step_workspace(bool bwd, int B, int H, int cus, int force_S, int64_t* ws_floats,
                        int64_t* tickets) {
  const BsPlan p = bs_plan(bwd, B, H, cus, force_S);
  const int BM = bwd ? p.BU : 4 * p.BU;
  *ws_floats = p.S > 1 ? (int64_t)p.tiles * p.S * BM * p.BN : 0;
  *tickets = p.tiles;
}

template <class C>
void bs_launch(unsigned grid, const BigStepArgs& a, hipStream_t s) {
  lstm_gemm_step_kernel<C><<<grid, C::NW * 64, 0, s>>>(a);
}

int launch_big_step(bool bwd, const BigStepArgs& a0, int cus, int force_S, hipStream_t s) {
  const BsPlan p = bs_plan(bwd, a0.B, a0.H, cus, force_S);
  BigStepArgs a = a0;
  a.S = p.S;
  const unsigned grid = (unsigned)(p.tiles * p.S);
  switch (p.cfg) {
    case 0: bs_launch<Cfg0>(grid, a, s); break;
    case 1: bs_launch<Cfg1>(grid, a, s); break;
    case 2: bs_launch<Cfg2>(grid, a, s); break;
    case 3: bs_launch<Cfg3>(grid, a, s); break;
    case 4: bs_launch<Cfg4>(grid, a, s); break;
    case 5: bs_launch<Cfg5>(grid, a, s); break;
    case 6: bs_launch<Cfg6>(grid, a, s); break;
    case 8: bs_launch<Cfg8>(grid, a, s); break;
    case 9: bs_launch<Cfg9>(grid, a, s); break;
    case 10: bs_launch<Cfg10>(grid, a, s); break;
    case 11: bs_launch<Cfg11>(grid, a, s); break;
    default: bs_launch<Cfg7>(grid, a, s); break;
  }
  return p.S;
}

}  // namespace dcr
