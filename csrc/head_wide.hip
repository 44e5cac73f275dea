// Fused wide-vocabulary softmax head (BASELINE.json's 8k-token config): logits, softmax
// cross-entropy and bf16 dlogits without ever writing the fp32 logits.
//
// Reference: logits = output·softmax_w + softmax_b (model.py:76), the sequence loss
// (model.py:79-85) and its gradient.  The library route is a logits GEMM writing fp32 [N, V]
// (1.07 GB at N = 32768, V = 8192; 420 us) and a one-read CE kernel over it (350 us).  Here:
//
//   pass 1 (stats): a workgroup owns 256 tokens (8 waves x 32, O rows resident in VGPRs) and ONE
//           half of the vocabulary; softmax_wᵀ streams through LDS in 32-vocab tiles; each
//           lane keeps an online max / sum-exp over its vocab subset (no cross-lane traffic in
//           the loop), merged over the token's 4 lanes at the end -> (max, sum) per token and
//           half, and the target logit by the half that holds it;
//   pass 2 (grad): the same grid merges the two halves' stats into lse, recomputes its half's
//           logits and stores dlog = (exp(l - lse) - onehot) * scale as bf16 (what the dW_s /
//           dtop GEMMs read), plus the bf16 values' column sums over its tokens (d softmax_b
//           partials, one DPP butterfly per tile); the half-0 workgroups write the row losses.
//
// Why this shape: every workgroup streams the softmax_wᵀ rows it covers once per pass, so the
// L2 -> LDS traffic is (token blocks) x (V x H x 2 B) per pass: 256-token blocks halve it against
// 128-token ones (the register file holds at most 32 tokens' O rows per wave at H = 512), and
// the vocabulary split keeps 256 workgroups on the chip.  The XCD-aware block map puts each
// half on 4 XCDs, so an XCD's L2 sees one 4 MB half.  Four LDS buffers keep three tiles of DMA
// in flight per CU; every wait on them is a counted vmcnt (the LDS reads are inline asm: the
// compiler would otherwise wait vmcnt(0) for the whole prefetch before any LDS read).
//
// MFMA: mfma_f32_16x16x32_bf16 with swapped operands (A = softmax_wᵀ rows from LDS, B = the
// wave's O rows), so a lane holds 4 consecutive vocab entries of one token.  softmax_wᵀ rows
// arrive by LDS-DMA (one 1 KB buffer_load ... lds per row at H = 512) into a padded 1056-B row
// stride: conflict-free ds_read_b128 fragment reads.
#include <type_traits>

#include "common.h"
#include "kernels.h"
#include "persist_common.h"
#include "debug_env.h"

namespace dcr {

constexpr int kHwTok = 256;   // tokens per workgroup (8 waves x 32)
constexpr int kHwVt = 32;     // vocab rows per LDS tile
constexpr int kHwBuf = 4;     // LDS tile buffers (3 tiles of DMA in flight)
constexpr int kHwRow = 1056;  // LDS row stride in bytes (H = 512: 1024 + 32, conflict-free)
constexpr int kHwSplit = 2;   // vocabulary halves
constexpr int kHwStg = 80;    // dlogits staging row stride in bytes (64 B of a tile row + pad)

template <int CTRL>
__device__ __forceinline__ float hw_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                               0xF, 0xF, true));
}
template <int CTRL, int NV>
__device__ __forceinline__ void hw_bfly(float (&v)[16], bool hi) {
#pragma unroll
  for (int k = 0; k < NV / 2; ++k) {
    const float send = hi ? v[k] : v[k + NV / 2];
    const float keep = hi ? v[k + NV / 2] : v[k];
    v[k] = keep + hw_dpp<CTRL>(send);
  }
}
// sum over the 16 lanes of a DPP row of v[i]; lane r of the row returns the sum of v[r]
__device__ __forceinline__ float hw_row_reduce_scatter(float (&v)[16], int lane) {
  const int r = lane & 15;
  hw_bfly<0x140, 16>(v, (r & 8) != 0);
  hw_bfly<0x141, 8>(v, (r & 4) != 0);
  hw_bfly<0x4E, 4>(v, (r & 2) != 0);
  hw_bfly<0xB1, 2>(v, (r & 1) != 0);
  return v[0];
}

// raw workgroup barrier: __syncthreads()' fence would add vmcnt(0) while an LDS-DMA (or the
// dlogits stores behind it) is in flight, draining the prefetch
__device__ __forceinline__ void hw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// wait until at most n vector-memory operations of this wave are outstanding (n wave-uniform)
__device__ __forceinline__ void hw_vm_wait(int n) {
#define HW_VMW(k) \
  case k:         \
    asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); \
    break;
  switch (n) {
    HW_VMW(1) HW_VMW(2) HW_VMW(3) HW_VMW(4) HW_VMW(5) HW_VMW(6) HW_VMW(7) HW_VMW(8) HW_VMW(9)
    HW_VMW(10) HW_VMW(11) HW_VMW(12) HW_VMW(13) HW_VMW(14) HW_VMW(15) HW_VMW(16) HW_VMW(17)
    HW_VMW(18) HW_VMW(19) HW_VMW(20) HW_VMW(21) HW_VMW(22) HW_VMW(23) HW_VMW(24) HW_VMW(25)
    HW_VMW(26) HW_VMW(27) HW_VMW(28) HW_VMW(29) HW_VMW(30) HW_VMW(31) HW_VMW(32) HW_VMW(33)
    HW_VMW(34) HW_VMW(35) HW_VMW(36) HW_VMW(37) HW_VMW(38) HW_VMW(39) HW_VMW(40)
    default:
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#undef HW_VMW
}
// LDS reads the compiler does not see: its waitcnt pass cannot tell the tile being read from the
// ones the LDS-DMA is filling (no alias scopes on __shared__ arrays), so a plain read would wait
// vmcnt(0) for the whole in-flight prefetch.  The caller retires them with hw_lgkm_wait, which
// also pins the results' first use after the wait.
__device__ __forceinline__ unsigned hw_lds(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ void hw_rd128(u32x4& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(addr));
}
template <int N>
__device__ __forceinline__ void hw_lgkm_wait(u32x4 (&d)[2]) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(d[0]), "+v"(d[1]) : "n"(N));
}

struct HwMap {
  int tb, half;
};
// XCD-aware: workgroups are dispatched round-robin over the 8 XCDs (blockIdx % 8); XCDs 0-3 take
// vocabulary half 0, XCDs 4-7 half 1
__device__ __forceinline__ HwMap hw_map(int g, int nblk) {
  const int total = nblk * kHwSplit;
  if (total % 8 == 0) {
    const int xcd = g & 7, slot = g >> 3;
    return {slot * 4 + (xcd & 3), xcd >> 2};
  }
  return {g >> 1, g & 1};
}

// PASS 1: stats; PASS 2: lse, row loss, dlogits / logits, d softmax_b partials.  FL >= 0: the
// argument flags at compile time (bit 0 softmax_b, 1 dlogits, 2 logits, 3 colpart; the training
// step's combinations), so the per-tile counted waits are constants; FL = -1 reads them from a.
template <int KS, int PASS, int FL>
__global__ void __launch_bounds__(512, 1) head_wide_kernel(HeadWideArgs a) {
  static_assert(KS * 32 * 2 == 1024, "one 1 KB LDS-DMA instruction per vocab row (H = 512)");
  __shared__ __attribute__((aligned(16))) unsigned char wl[kHwBuf][kHwVt * kHwRow];
  __shared__ __attribute__((aligned(16))) float bl[kHwBuf][64];  // softmax_b of the tile
  // per-wave dlogits staging: the MFMA layout (a lane holds 4 vocab of one token, the 4 lanes
  // of a token 8 B apart) becomes 16-B row chunks with adjacent lanes adjacent in memory
  __shared__ __attribute__((aligned(16))) unsigned char stg[8][32 * kHwStg];
  __shared__ float lred[8];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int N = a.N, V = a.V, H = a.H;
  const int q = lane >> 4, nl = lane & 15;
  const int nblk = (N + kHwTok - 1) / kHwTok;
  const HwMap mp = hw_map(blockIdx.x, nblk);
  const int n0 = mp.tb * kHwTok + w * 32;  // this wave's 32 tokens
  const int Vh = V / kHwSplit;
  const int vbase = mp.half * Vh;
  const int ntile = Vh / kHwVt;  // (V % 64 == 0: head_wide_supported)
  float* stats = a.stats;        // [2][N] (max, sum-exp) pairs, then [N] target logits
  float* tlog = a.stats + 2 * kHwSplit * (size_t)N;

  int y[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int n = n0 + 16 * tt + nl;
    y[tt] = (a.targets && n < N) ? a.targets[n] : -1;
  }
  const bool grad = PASS == 2 && (FL < 0 ? a.dlogits != nullptr : (FL & 2) != 0);
  const bool want_logits = PASS == 2 && (FL < 0 ? a.logits != nullptr : (FL & 4) != 0);
  const bool has_colpart = FL < 0 ? a.colpart != nullptr : (FL & 8) != 0;
  float lse[2] = {0.f, 0.f};
  if constexpr (PASS == 2) {
    // merge the two halves' stats; the half-0 workgroups write the row losses
    float lacc = 0.f;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int n = n0 + 16 * tt + nl;
      if (n < N) {
        const float2 s0 = reinterpret_cast<const float2*>(stats)[n];
        const float2 s1 = reinterpret_cast<const float2*>(stats)[N + n];
        const float M = fmaxf(s0.x, s1.x);
        lse[tt] = M + __logf(s0.y * __expf(s0.x - M) + s1.y * __expf(s1.x - M));
        if (mp.half == 0 && q == 0 && y[tt] >= 0) {
          const float loss = lse[tt] - tlog[n];
          if (a.row_loss) a.row_loss[n] = loss;
          lacc += loss;
        }
      }
    }
    lacc = wave_sum(lacc);
    if (lane == 0) lred[w] = lacc;
    // (the stats loads retire here, before any LDS-DMA is queued behind them)
    asm volatile("" ::"v"(lse[0]), "v"(lse[1]) : "memory");
    if (!grad && !want_logits) {
      __syncthreads();
      if (threadIdx.x == 0 && mp.half == 0 && a.partial) {
        float t = 0.f;
        for (int k = 0; k < 8; ++k) t += lred[k];
        a.partial[mp.tb] = t;
      }
      return;
    }
  }

  // O rows of the wave: B fragments [token tile][k-step] (rows >= N: zero)
  bf16x8 ofr[2][KS];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int n = n0 + 16 * tt + nl;
#pragma unroll
    for (int s = 0; s < KS; ++s)
      ofr[tt][s] = n < N ? ld8(a.O + (size_t)n * a.ldo + s * 32 + 8 * q) : zero8();
  }
  // retire the O and target loads here, before the first DMA: a first use inside the tile loop
  // would make the compiler wait vmcnt(0) there on every iteration
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" ::"v"(__builtin_bit_cast(u32x4, ofr[tt][s])));
  asm volatile("" ::"v"(y[0]), "v"(y[1]) : "memory");

  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.WsT, sizeof(bf16) * (size_t)V * H);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc(a.bias, sizeof(float) * (size_t)V);
  // outputs by range-checked buffer stores: rows >= N fall off the end of the buffer, so every
  // wave issues the same number of stores per tile (the counted vmcnt waits rely on it)
  const __amdgpu_buffer_rsrc_t rdl = make_rsrc(a.dlogits, sizeof(bf16) * (size_t)N * V);
  const __amdgpu_buffer_rsrc_t rlg = make_rsrc(a.logits, sizeof(float) * (size_t)N * V);
  const bool has_bias = FL < 0 ? a.bias != nullptr : (FL & 1) != 0;
  // the bias row: wave 0 (FL < 0) or every wave (FL >= 0: the same 256 B into the same LDS
  // words, so every wave's count is the same constant)
  const bool bias_dma = has_bias && (FL >= 0 || w == 0);
  // vector-memory operations this wave issues per tile: DMA rows (+ the bias row) and pass-2
  // stores (dlogits, logits, the wave's colpart row)
  const int dper = 4 + (bias_dma ? 1 : 0);
  const int sper = (grad ? 2 : 0) + (want_logits ? 4 : 0) + ((grad && has_colpart) ? 1 : 0);

  // softmax_wᵀ rows of tile i into buffer i % 4: wave w DMAs rows [4 w, 4 w + 4); wave 0 also
  // the tile's softmax_b values.  Everything a tile reads arrives through this DMA.
  auto load_tile = [&](int i) {
    const int b = i & (kHwBuf - 1);
    const int v0 = vbase + i * kHwVt;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = 4 * w + j;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rw, (__attribute__((address_space(3))) void*)&wl[b][r * kHwRow], 16,
          (unsigned)(lane * 16), (unsigned)((size_t)(v0 + r) * H * sizeof(bf16)), 0, 0);
    }
    if (bias_dma)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void*)&bl[b][0],
                                               4, (unsigned)(lane * 4),
                                               (unsigned)(v0 * sizeof(float)), 0, 0);
  };
  // logits of tile i: acc[vt][tt] rows = vocab v0 + 16 vt + 4 q + r, column = token
  auto tile_logits = [&](int i, f32x4 (&acc)[2][2]) {
    const int b = i & (kHwBuf - 1);
#pragma unroll
    for (int vt = 0; vt < 2; ++vt)
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) acc[vt][tt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // A fragments of k-step s (one ds_read_b128 per 16-vocab sub-tile), read one k-step ahead
    const unsigned base = hw_lds(&wl[b][nl * kHwRow + 16 * q]);
    u32x4 af[2][2];
#pragma unroll
    for (int vt = 0; vt < 2; ++vt) hw_rd128(af[0][vt], base + vt * 16 * kHwRow);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      if (s + 1 < KS) {
#pragma unroll
        for (int vt = 0; vt < 2; ++vt)
          hw_rd128(af[(s + 1) & 1][vt], base + vt * 16 * kHwRow + (s + 1) * 64);
        hw_lgkm_wait<2>(af[s & 1]);
      } else {
        hw_lgkm_wait<0>(af[s & 1]);
      }
#pragma unroll
      for (int vt = 0; vt < 2; ++vt) {
        const bf16x8 a8 = __builtin_bit_cast(bf16x8, af[s & 1][vt]);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) acc[vt][tt] = mfma16(a8, ofr[tt][s], acc[vt][tt]);
      }
    }
    if (has_bias) {
      u32x4 bv[2];
#pragma unroll
      for (int vt = 0; vt < 2; ++vt) hw_rd128(bv[vt], hw_lds(&bl[b][16 * vt + 4 * q]));
      hw_lgkm_wait<0>(bv);
#pragma unroll
      for (int vt = 0; vt < 2; ++vt) {
        const f32x4 bb = __builtin_bit_cast(f32x4, bv[vt]);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) acc[vt][tt] += bb;
      }
    }
  };
  // top of tile i: this wave's DMA of tile i has landed once only the operations issued after
  // it remain: the DMAs of tiles i+1, i+2 (those that exist) and the stores of tiles
  // max(0, i-3) .. i-1; then every wave's rows have landed after the barrier
  // A steady tile (3 <= i, i + 3 < ntile) has both later DMAs and three tiles of stores behind
  // its own DMA: with the flags compile-time (FL >= 0) its count is a constant -- one s_waitcnt
  // instead of hw_vm_wait's branch tree -- and its refill unconditional
  auto wait_tile = [&](int i, auto steady) {
    if constexpr (decltype(steady)::value) {
      hw_vm_wait(2 * dper + 3 * sper);
      hw_barrier();
      load_tile(i + 3);
    } else {
      const int nd = (i + 1 < ntile ? 1 : 0) + (i + 2 < ntile ? 1 : 0);
      hw_vm_wait(nd * dper + (i < 3 ? i : 3) * sper);
      hw_barrier();
      if (i + 3 < ntile) load_tile(i + 3);  // into the buffer tile i-1 was read from
    }
  };
  auto run_tiles = [&](auto& body) {
    using steady_t = std::integral_constant<bool, true>;
    using edge_t = std::integral_constant<bool, false>;
    int i = 0;
    for (; i < ntile && i < 3; ++i) body(i, edge_t{});
    if constexpr (FL >= 0)
      for (; i + 3 < ntile; ++i) body(i, steady_t{});
    for (; i < ntile; ++i) body(i, edge_t{});
  };

#pragma unroll
  for (int i = 0; i < 3; ++i)
    if (i < ntile) load_tile(i);

  if constexpr (PASS == 1) {
    float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f}, ty[2] = {0.f, 0.f};
    float found[2] = {0.f, 0.f};
    auto body = [&](int i, auto steady) {
      wait_tile(i, steady);
      f32x4 acc[2][2];
      tile_logits(i, acc);
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        float mx = m[tt];
#pragma unroll
        for (int vt = 0; vt < 2; ++vt)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, acc[vt][tt][r]);
        float s = l[tt] * __expf(m[tt] - mx);  // (m = -inf on the first tile: exp(-inf) = 0)
#pragma unroll
        for (int vt = 0; vt < 2; ++vt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s += __expf(acc[vt][tt][r] - mx);
            if (vbase + i * kHwVt + 16 * vt + 4 * q + r == y[tt]) {
              ty[tt] = acc[vt][tt][r];
              found[tt] = 1.f;
            }
          }
        m[tt] = mx;
        l[tt] = s;
      }
    };
    run_tiles(body);
    // merge the 4 lanes of each token (lanes nl, nl + 16, nl + 32, nl + 48)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      float M = fmaxf(m[tt], __shfl_xor(m[tt], 16, 64));
      M = fmaxf(M, __shfl_xor(M, 32, 64));
      float L = l[tt] * __expf(m[tt] - M);
      L += __shfl_xor(L, 16, 64);
      L += __shfl_xor(L, 32, 64);
      float t = ty[tt], f = found[tt];
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      f += __shfl_xor(f, 16, 64);
      f += __shfl_xor(f, 32, 64);
      const int n = n0 + 16 * tt + nl;
      if (q == 0 && n < N) {
        reinterpret_cast<float2*>(stats)[(size_t)mp.half * N + n] = make_float2(M, L);
        if (f > 0.f) tlog[n] = t;
      }
    }
  } else {
    auto body = [&](int i, auto steady) {
      wait_tile(i, steady);
      f32x4 acc[2][2];
      tile_logits(i, acc);
      float cs[16];  // this lane's column sums over its 2 tokens: [4 vt + r], 8..15 zero
#pragma unroll
      for (int k = 0; k < 16; ++k) cs[k] = 0.f;
#pragma unroll
      for (int vt = 0; vt < 2; ++vt) {
        const int v0 = vbase + i * kHwVt + 16 * vt + 4 * q;
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          const int n = n0 + 16 * tt + nl;
          const unsigned off = (unsigned)n * (unsigned)V + (unsigned)v0;  // element offset
          if (want_logits)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[vt][tt]), rlg,
                                                   off * 4u, 0, 0);
          if (grad) {
            bf16x4 o;
            const bool live = n < N;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float p = __expf(acc[vt][tt][r] - lse[tt]);
              const float d = (p - (v0 + r == y[tt] ? 1.f : 0.f)) * a.grad_scale;
              o[r] = f2bf(live ? d : 0.f);
              cs[4 * vt + r] += (float)o[r];
            }
            asm volatile("ds_write_b64 %0, %1" ::"v"(hw_lds(&stg[w][(16 * tt + nl) * kHwStg +
                                                               32 * vt + 8 * q])),
                         "v"(__builtin_bit_cast(u32x2, o))
                         : "memory");
          }
        }
      }
      if (grad) {
        // the wave's 32 x 32 bf16 tile: lanes 4 r .. 4 r + 3 store row r's 64 B (2 rows of 16)
        u32x4 rd[2];
#pragma unroll
        for (int k = 0; k < 2; ++k)
          hw_rd128(rd[k], hw_lds(&stg[w][(16 * k + (lane >> 2)) * kHwStg + 16 * (lane & 3)]));
        hw_lgkm_wait<0>(rd);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const unsigned n = (unsigned)(n0 + 16 * k + (lane >> 2));
          const unsigned off = (n * (unsigned)V + (unsigned)(vbase + i * kHwVt)) * 2u + 16u * (lane & 3);
          __builtin_amdgcn_raw_buffer_store_b128(rd[k], rdl, off, 0, 0);
        }
      }
      if (grad && has_colpart) {
        // over the wave's 16 token lanes: lane nl < 8 of lane group q ends with value nl =
        // 4 vt + r -> vocab 16 vt + 4 q + r of the tile, stored into the wave's own partial row
        // (no cross-wave step: the finalize kernel sums 8 rows per token block)
        const float sv = hw_row_reduce_scatter(cs, lane);
        if (nl < 8)
          a.colpart[(size_t)(mp.tb * 8 + w) * V + vbase + i * kHwVt + 16 * (nl >> 2) + 4 * q +
                    (nl & 3)] = sv;
      }
    };
    run_tiles(body);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0 && mp.half == 0 && a.partial) {
      float t = 0.f;
      for (int k = 0; k < 8; ++k) t += lred[k];
      a.partial[mp.tb] = t;
    }
  }
}

int head_wide_blocks(int N) { return (N + kHwTok - 1) / kHwTok; }
int head_wide_colpart_rows(int N) { return 8 * head_wide_blocks(N); }
size_t head_wide_stats_floats(int N) { return (size_t)(2 * kHwSplit + 1) * (size_t)N; }
// (V a whole number of 64-row tiles: each half is whole 32-row tiles and the softmax_wᵀ DMA
// never leaves the buffer)
int head_wide_supported(int V, int H) { return H == 512 && V >= 64 && V % 64 == 0 ? 1 : 0; }

int launch_head_wide(const HeadWideArgs& a, float* db, float* loss_out, hipStream_t s) {
  if (!head_wide_supported(a.V, a.H) || a.N <= 0 || !a.stats) return -1;
  // 32-bit buffer offsets of the outputs, up to the last block's padded rows (which the range
  // check drops).  Larger token counts run as chunks of whole 256-token blocks that each fit:
  // every per-token / per-block output is offset to the chunk, each chunk keeps its own stats
  // region ((2 kHwSplit + 1) floats per token, so the chunks tile head_wide_stats_floats(N)),
  // and one finalize sums all blocks' partials.
  const int nb = head_wide_blocks(a.N);
  const size_t bpr = a.logits ? 4 * (size_t)a.V : a.dlogits ? 2 * (size_t)a.V : 0;  // bytes / row
  int chunk_blocks = nb;
  if (bpr) {
    const size_t max_rows = ((1ull << 32) - 1) / bpr;
    chunk_blocks = (int)(max_rows / kHwTok);
    if (chunk_blocks < 1) return -2;
  }
  const int force = debug_int("hw_chunk", 0);  // (tests: chunking at small N)
  if (force > 0 && force < chunk_blocks) chunk_blocks = force;
  for (int b0 = 0; b0 < nb; b0 += chunk_blocks) {
    const int cb = nb - b0 < chunk_blocks ? nb - b0 : chunk_blocks;
    const size_t n0 = (size_t)b0 * kHwTok;
    HeadWideArgs c = a;
    c.N = (int)((size_t)a.N - n0 < (size_t)cb * kHwTok ? (size_t)a.N - n0 : (size_t)cb * kHwTok);
    c.O = a.O + n0 * a.ldo;
    if (a.targets) c.targets = a.targets + n0;
    if (a.row_loss) c.row_loss = a.row_loss + n0;
    if (a.dlogits) c.dlogits = a.dlogits + n0 * a.V;
    if (a.logits) c.logits = a.logits + n0 * a.V;
    if (a.colpart) c.colpart = a.colpart + (size_t)b0 * 8 * a.V;
    if (a.partial) c.partial = a.partial + b0;
    c.stats = a.stats + (size_t)(2 * kHwSplit + 1) * n0;
    // the training step's flags (softmax_b, dlogits, colpart, no logits) take the
    // compile-time-flag kernels; other combinations the generic ones
    const bool train = c.bias && c.dlogits && c.colpart && !c.logits && debug_int("hw_fl", 1);
    if (c.targets || c.dlogits) {
      if (train)
        hipLaunchKernelGGL((head_wide_kernel<16, 1, 11>), dim3(cb * kHwSplit), dim3(512), 0, s, c);
      else
        hipLaunchKernelGGL((head_wide_kernel<16, 1, -1>), dim3(cb * kHwSplit), dim3(512), 0, s, c);
    }
    if (train)
      hipLaunchKernelGGL((head_wide_kernel<16, 2, 11>), dim3(cb * kHwSplit), dim3(512), 0, s, c);
    else
      hipLaunchKernelGGL((head_wide_kernel<16, 2, -1>), dim3(cb * kHwSplit), dim3(512), 0, s, c);
  }
  launch_xent_finalize(a.partial, nb, a.N, loss_out, a.dlogits ? a.colpart : nullptr, 8 * nb, a.V,
                       db, s);
  return 0;
}

}  // namespace dcr
