// Fused softmax head, forward + backward in one launch (K9 + K10 + the bias/dtop halves of the
// head backward in SURVEY.md §2.3).
//
// Reference: logits = output·softmax_w + softmax_b (model.py:75-77), the sequence loss
// (model.py:79-85: sparse softmax CE summed and divided by batch*seq) and its gradient flowing
// to softmax_b and back into the top RNN layer.  The library path ran this as five launches
// (logits GEMM on 28 workgroups for a 65-column output, CE, a column sum and a reduce for
// d softmax_b, the dtop GEMM).  Here one wave owns a chunk of TPW x 16 tokens:
//
//   logits  C[v, n] = WsT[v, :] · O[n, :]ᵀ        mfma_f32_16x16x32_bf16, swapped operands:
//           lane (n = lane&15, g = lane>>4) holds v = 16*vt + 4g + r for one token, so a
//           token's V logits live in 4 lanes and max / sum-exp / target pick are 2 shuffles;
//   CE      online over the lane's NVT x 4 logits, lse, row loss, dlogits (bf16, the values the
//           weight-gradient GEMM will see), bias-gradient partials;
//   dtop    C[h, n] = Ws[h, :] · dlog[n, :]ᵀ     dlog staged per wave in LDS (K = v rows of
//           16 B), Ws rows streamed from L2; the output lane holds 4 consecutive h of one
//           token -> float4 stores straight into dtop [N, H].
//
// d softmax_w = Oᵀ·dlog stays a split-K library GEMM (token reduction, engine/native_backend.py).
#include "common.h"
#include "kernels.h"
#include "debug_env.h"

namespace dcr {

constexpr int kHeadWaves = 8;   // (two waves per SIMD: one wave's L2 round trips hide behind the other's work)
constexpr int kHeadThreads = 64 * kHeadWaves;
constexpr int kHeadTPW = 1;  // token tiles (16 tokens each) per wave chunk

template <int NVT>
__global__ void __launch_bounds__(kHeadThreads) head_kernel(HeadArgs a) {
  constexpr int VP = 16 * NVT;             // padded vocab (logit rows)
  constexpr int VK = 32 * ((VP + 31) / 32);  // padded K for the dtop MFMA
  constexpr int SLD = VK + 8;              // LDS row stride (bf16), keeps 16-B alignment
  constexpr int TPW = kHeadTPW;
  __shared__ __attribute__((aligned(16))) bf16 sdl[kHeadWaves][TPW * 16][SLD];
  __shared__ float red[kHeadWaves][VP + 1];
  // softmax_wᵀ [VP, H] staged once per workgroup (shared by its 4 waves), 16-B chunk c of row r
  // at chunk c ^ (r & 15): the 16 rows of a fragment read hit 16 distinct bank groups
  extern __shared__ __attribute__((aligned(16))) bf16 swt[];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nl = lane & 15, g = lane >> 4;
  const int N = a.N, H = a.H, V = a.V;
  const bool train = a.dtop != nullptr || a.dlogits != nullptr;

  // zero the K padding columns [VP, VK) of this wave's dlog tile once (never rewritten)
  for (int i = lane; i < TPW * 16 * (VK - VP); i += 64)
    sdl[w][i / (VK - VP)][VP + i % (VK - VP)] = f2bf(0.f);

  float bias[NVT][4];
#pragma unroll
  for (int vt = 0; vt < NVT; ++vt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int v = 16 * vt + 4 * g + r;
      bias[vt][r] = v < V ? a.bias[v] : 0.f;
    }
  float dbacc[NVT][4];
#pragma unroll
  for (int vt = 0; vt < NVT; ++vt)
#pragma unroll
    for (int r = 0; r < 4; ++r) dbacc[vt][r] = 0.f;
  float lacc = 0.f;

  const int nchunks = (N + TPW * 16 - 1) / (TPW * 16);
  const int hc = H / 8;  // 16-B chunks per softmax_wᵀ row
  if (a.lds_wst) {
    // every thread's loads issued together (8 per batch), then the swizzled LDS stores
    for (int i0 = threadIdx.x; i0 < VP * hc; i0 += 8 * kHeadThreads) {
      bf16x8 v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + j * kHeadThreads;
        v[j] = i < VP * hc ? ld8(a.WsT + (size_t)(i / hc) * H + 8 * (i % hc)) : zero8();
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = i0 + j * kHeadThreads;
        const int r = i / hc, c = i % hc;
        if (i < VP * hc) *reinterpret_cast<bf16x8*>(&swt[(size_t)r * H + 8 * (c ^ (r & 15))]) = v[j];
      }
    }
    __syncthreads();
  }
  for (int chunk = blockIdx.x * kHeadWaves + w; chunk < nchunks; chunk += gridDim.x * kHeadWaves) {
    const int nb = chunk * TPW * 16;
    // ---- logits
    f32x4 acc[TPW][NVT];
#pragma unroll
    for (int tp = 0; tp < TPW; ++tp)
#pragma unroll
      for (int vt = 0; vt < NVT; ++vt) acc[tp][vt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16* orow[TPW];
#pragma unroll
    for (int tp = 0; tp < TPW; ++tp)
      orow[tp] = a.O + (size_t)min(nb + tp * 16 + nl, N - 1) * a.ldo + 8 * g;
    if (a.lds_wst) {
      // A fragments from the LDS image; the chunk's O fragments in groups of 8 k-steps, each
      // group's 16 loads issued together (one L2 round trip per group instead of per k-step)
      for (int k0 = 0; k0 < H; k0 += 256) {
        bf16x8 bo[8][TPW];
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int tp = 0; tp < TPW; ++tp)
            bo[j][tp] = ld8(orow[tp] + min(k0 + 32 * j, H - 32));  // (clamped: unused past H)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (k0 + 32 * j >= H) break;
          const int c = (k0 + 32 * j) / 8 + g;  // logical chunk of this lane's 8 k
#pragma unroll
          for (int vt = 0; vt < NVT; ++vt) {
            const bf16x8 af =
                *reinterpret_cast<const bf16x8*>(&swt[(size_t)(16 * vt + nl) * H + 8 * (c ^ nl)]);
#pragma unroll
            for (int tp = 0; tp < TPW; ++tp) acc[tp][vt] = mfma16(af, bo[j][tp], acc[tp][vt]);
          }
        }
      }
    } else {
      const bf16* wrow = a.WsT + (size_t)nl * H + 8 * g;
#pragma unroll 2
      for (int k = 0; k < H; k += 32) {
        bf16x8 bo[TPW];
#pragma unroll
        for (int tp = 0; tp < TPW; ++tp) bo[tp] = ld8(orow[tp] + k);
#pragma unroll
        for (int vt = 0; vt < NVT; ++vt) {
          const bf16x8 af = ld8(wrow + (size_t)vt * 16 * H + k);
#pragma unroll
          for (int tp = 0; tp < TPW; ++tp) acc[tp][vt] = mfma16(af, bo[tp], acc[tp][vt]);
        }
      }
    }
    // ---- softmax cross-entropy per token
#pragma unroll
    for (int tp = 0; tp < TPW; ++tp) {
      const int n = nb + tp * 16 + nl;
      const bool valid = n < N;
      float x[NVT][4];
      float m = -INFINITY;
#pragma unroll
      for (int vt = 0; vt < NVT; ++vt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int v = 16 * vt + 4 * g + r;
          x[vt][r] = v < V ? acc[tp][vt][r] + bias[vt][r] : -INFINITY;
          m = fmaxf(m, x[vt][r]);
        }
      m = fmaxf(m, __shfl_xor(m, 16, 64));
      m = fmaxf(m, __shfl_xor(m, 32, 64));
      float s = 0.f;
#pragma unroll
      for (int vt = 0; vt < NVT; ++vt)
#pragma unroll
        for (int r = 0; r < 4; ++r) s += __expf(x[vt][r] - m);  // exp(-inf) = 0 on padding
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      const float lse = m + __logf(s);
      int y = -1;
      if (a.targets) {
        y = a.targets[min(n, N - 1)];
        if (!valid) y = 0;
        float xy = 0.f;
#pragma unroll
        for (int vt = 0; vt < NVT; ++vt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (16 * vt + 4 * g + r == y) xy = x[vt][r];
        xy += __shfl_xor(xy, 16, 64);
        xy += __shfl_xor(xy, 32, 64);
        const float loss = lse - xy;
        if (g == 0 && valid) {
          if (a.row_loss) a.row_loss[n] = loss;
          lacc += loss;
        }
      }
      if (a.logits && valid) {
#pragma unroll
        for (int vt = 0; vt < NVT; ++vt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int v = 16 * vt + 4 * g + r;
            if (v < V) a.logits[(size_t)n * V + v] = x[vt][r];
          }
      }
      if (train) {
        const float inv = 1.f / s;
#pragma unroll
        for (int vt = 0; vt < NVT; ++vt) {
          float q[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int v = 16 * vt + 4 * g + r;
            const float d = (__expf(x[vt][r] - m) * inv - (v == y ? 1.f : 0.f)) * a.grad_scale;
            const bf16 db = f2bf(valid && v < V ? d : 0.f);
            q[r] = (float)db;
            dbacc[vt][r] += q[r];
            if (a.dlogits && valid && v < V) a.dlogits[(size_t)n * a.ldl + v] = db;
          }
          bf16x4 pk;
          pk[0] = f2bf(q[0]); pk[1] = f2bf(q[1]); pk[2] = f2bf(q[2]); pk[3] = f2bf(q[3]);
          *reinterpret_cast<bf16x4*>(&sdl[w][tp * 16 + nl][16 * vt + 4 * g]) = pk;
        }
      }
    }
    if (a.dtop == nullptr) continue;
    // ---- dtop = dlog · Wsᵀ (this wave's tile only: a wave-local LDS hand-off)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // Ws fragments for HG h-tiles are issued together (the loop is otherwise L2-latency bound:
    // 3 loads per tile, 32 tiles); the dlog B fragments are re-read from LDS per tile
    constexpr int HG = VK <= 96 ? 8 : (VK <= 160 ? 4 : 2);
    const bf16* wk = a.Wsk + (size_t)nl * VK + 8 * g;
    for (int ht0 = 0; ht0 < H / 16; ht0 += HG) {
      bf16x8 af[HG][VK / 32];
#pragma unroll
      for (int j = 0; j < HG; ++j)
#pragma unroll
        for (int ks = 0; ks < VK / 32; ++ks)
          af[j][ks] = ld8(wk + (size_t)min(ht0 + j, H / 16 - 1) * 16 * VK + ks * 32);  // (clamped)
#pragma unroll
      for (int j = 0; j < HG; ++j) {
        if (ht0 + j >= H / 16) break;
        f32x4 d[TPW];
#pragma unroll
        for (int tp = 0; tp < TPW; ++tp) d[tp] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < VK / 32; ++ks)
#pragma unroll
          for (int tp = 0; tp < TPW; ++tp) {
            const bf16x8 bfr =
                *reinterpret_cast<const bf16x8*>(&sdl[w][tp * 16 + nl][ks * 32 + 8 * g]);
            d[tp] = mfma16(af[j][ks], bfr, d[tp]);
          }
#pragma unroll
        for (int tp = 0; tp < TPW; ++tp) {
          const int n = nb + tp * 16 + nl;
          const int h0 = (ht0 + j) * 16 + 4 * g;
          if (n < N) {
            if (a.omask) {  // output dropout: this lane's 4 units' bits of token n
              const unsigned m = (unsigned)a.omask[(size_t)n * (H / 8) + (h0 >> 3)] >> (h0 & 7);
#pragma unroll
              for (int r = 0; r < 4; ++r) d[tp][r] = (m >> r) & 1u ? d[tp][r] * a.oscale : 0.f;
            }
            *reinterpret_cast<float4*>(a.dtop + (size_t)n * H + h0) =
                make_float4(d[tp][0], d[tp][1], d[tp][2], d[tp][3]);
          }
        }
      }
    }
    // the next chunk rewrites this wave's tile: its reads above must be complete
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }

  // ---- per-workgroup partials: loss, bias gradient (deterministic, reduced by head_finalize)
#pragma unroll
  for (int vt = 0; vt < NVT; ++vt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float v = dbacc[vt][r];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      v += __shfl_xor(v, 8, 64);
      if (nl == 0) red[w][16 * vt + 4 * g + r] = v;
    }
  lacc = wave_sum(lacc);
  if (lane == 0) red[w][VP] = lacc;
  __syncthreads();
  float* part = a.part + (size_t)blockIdx.x * (VP + 1);
  for (int i = threadIdx.x; i <= VP; i += kHeadThreads) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < kHeadWaves; ++k) t += red[k][i];
    part[i] = t;
  }
}

// one wave per output column, lanes stride the partial rows (deterministic order per lane,
// fixed shuffle tree): 256 x 81 partials in a few microseconds instead of a serial walk
__global__ void __launch_bounds__(kHeadThreads) head_finalize_kernel(const float* __restrict__ part,
                                                                    int nparts, int VP, int V,
                                                                    float loss_scale,
                                                                    float* __restrict__ db,
                                                                    float* __restrict__ loss) {
  const int lane = threadIdx.x & 63;
  const int wv = blockIdx.x * (kHeadThreads / 64) + (threadIdx.x >> 6);
  const int nw = gridDim.x * (kHeadThreads / 64);
  for (int i = wv; i <= VP; i += nw) {
    float s = 0.f;
    for (int k = lane; k < nparts; k += 64) s += part[(size_t)k * (VP + 1) + i];
    s = wave_sum(s);
    if (lane == 0) {
      if (i == VP) {
        if (loss) loss[0] = s * loss_scale;
      } else if (db && i < V) {
        db[i] = s;
      }
    }
  }
}

int head_vpad(int V) { return 16 * ((V + 15) / 16); }
int head_kpad(int V) { return 32 * ((head_vpad(V) + 31) / 32); }
int head_supported(int V, int H) { return V >= 1 && V <= 256 && H % 32 == 0 && H >= 32; }

int head_num_partials(int N, int cus) {
  const int nchunks = (N + kHeadTPW * 16 - 1) / (kHeadTPW * 16);
  int g = (nchunks + kHeadWaves - 1) / kHeadWaves;
  const int cap = 2 * (cus > 0 ? cus : 256);
  return g < cap ? (g > 0 ? g : 1) : cap;
}

// dynamic LDS of the staged softmax_wᵀ image: VP x H bf16 while it fits beside the static
// arrays (V <= 80 at H = 512: 80 KB); larger heads stream it from L2 (lds_wst = 0)
constexpr size_t kHeadLdsWst = 96 * 1024;

template <int NVT>
static void head_inst(const HeadArgs& a0, int grid, hipStream_t s) {
  HeadArgs a = a0;
  const size_t bytes = (size_t)16 * NVT * a.H * sizeof(bf16);
  // (the chunk swizzle c ^ (r & 15) needs whole groups of 16 chunks per row: H % 128 == 0)
  a.lds_wst = bytes <= kHeadLdsWst && a.H % 128 == 0 && debug_int("head_lds", 1) != 0 ? 1 : 0;
  if (a.lds_wst) {
    static bool attr_set = false;  // opt in to > 64 KB of dynamic LDS once per instantiation
    if (!attr_set) {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&head_kernel<NVT>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)kHeadLdsWst);
      attr_set = true;
    }
  }
  head_kernel<NVT><<<grid, kHeadThreads, a.lds_wst ? bytes : 0, s>>>(a);
}

int launch_head(const HeadArgs& a, int cus, float* db_out, float* loss_out, hipStream_t s) {
  if (!head_supported(a.V, a.H) || a.N <= 0) return -1;
  const int grid = head_num_partials(a.N, cus);
  const int nvt = head_vpad(a.V) / 16;
  switch (nvt) {
#define HC(K) \
  case K: head_inst<K>(a, grid, s); break;
    HC(1) HC(2) HC(3) HC(4) HC(5) HC(6) HC(7) HC(8)
    HC(9) HC(10) HC(11) HC(12) HC(13) HC(14) HC(15) HC(16)
#undef HC
    default: return -1;
  }
  const int fw = (head_vpad(a.V) + 1 + kHeadWaves - 1) / kHeadWaves;  // one wave per column
  head_finalize_kernel<<<fw, kHeadThreads, 0, s>>>(a.part, grid, head_vpad(a.V), a.V,
                                                  1.0f / (float)a.N, db_out, loss_out);
  return 0;
}

}  // namespace dcr
