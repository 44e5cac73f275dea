// Single-launch autoregressive generation for the LSTM char model (gfx950): every layer's
// recurrence, the softmax head and the categorical draw for ALL characters in one persistent
// launch, weights resident in LDS across the grid.
//
// Reference: Model.sample (model.py:105-140) -- zero state, prime[:-1] fed to warm the state,
// then one Session.run per character for probs = softmax(h·W_s + b_s) (model.py:76-77) and a
// host-side pick: argmax (sampling_type 0), inverse-CDF weighted pick searchsorted(cumsum(p),
// rand * sum(p)) (1), or the weighted pick only after a space, else argmax (2).  SURVEY.md K16.
//
// Geometry.  G = H / 4 workgroups, one per CU, all co-resident.  Workgroup j owns hidden units
// [4 j, 4 j + 4) of every layer: the 16 gate columns {g H + u} of W_h,l (and of W_x,l for l > 0)
// sit in its LDS as bf16 rows of K (16-B row padding: the 16 column rows of one k-chunk fall on
// distinct banks), next to softmax_wᵀ [V, H] when it fits.  Layer 0's input projection is the
// E·W_x0 + b0 gather table row of the current id (fp32, as in the training forward).
//
// Per character, per layer l: z = x·W_x + h_prev·W_h (+ table row / bias) -- a GEMV over the
// workgroup's 16 columns, 16 k-chunks per column reduced in LDS -- then the cell update of the
// 4 owned units (c in registers), and an all-gather of h_l: each owner stores its units as
// 8-byte {value, tag} granules with agent-scope 8-byte atomic stores (MI355X_MICROARCH.md:
// a granule written by one store needs no ordering), every workgroup sweeps the S x H granules
// with 8-byte agent-scope loads until all carry the tag of (character, layer).  Two slots per
// layer (by character parity): a producer can only reach character c + 2 after every
// workgroup has consumed character c's slot.  After the top layer every workgroup computes the
// V logits and the pick itself (identical inputs and summation order: identical picks), so no
// second exchange is needed; workgroup 0 writes the generated ids.  Every spin is bounded
// (the error word is set and the grid drains).
//
// Numerics follow the training kernels: bf16 weights and bf16-rounded h as GEMV inputs, fp32
// accumulation, fp32 cell state; the draw uses the counter hash of sample.hip (uniform01 of
// seed, stream, per-stream counter).
#include "common.h"
#include "kernels.h"
#include "debug_env.h"

namespace dcr {

constexpr int kGenThreads = 256;
constexpr int kGenU = 4;           // units per workgroup per layer
constexpr int kGenCols = 4 * kGenU;  // gate columns per workgroup per layer
constexpr int kGenChunks = kGenThreads / kGenCols;  // k-chunks per column (16)
constexpr int kGenGather = 8;      // granules of the all-gather in flight per thread

__device__ __forceinline__ unsigned long long gen_pack(float v, unsigned tag) {
  return (unsigned long long)__float_as_uint(v) | ((unsigned long long)tag << 32);
}

extern __shared__ __attribute__((aligned(16))) unsigned char gen_lds[];

// diagnostics: the 100-MHz real-time counter at phase points of characters 8..15, first and last
// workgroup (GenArgs::stamps)
__device__ __forceinline__ void gen_stamp(const GenArgs& a, int c, int point) {
  if (a.stamps && threadIdx.x == 0 && c >= 8 && c < 16 && point < 16 &&
      (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1))
    a.stamps[((blockIdx.x ? 1 : 0) * 8 + (c - 8)) * 16 + point] = __builtin_amdgcn_s_memrealtime();
  // (points 0 and 13 also record the shader-clock counter in slots 11 / 12: the clock rate)
  if (a.stamps && threadIdx.x == 0 && c >= 8 && c < 16 && (point == 0 || point == 13) &&
      (blockIdx.x == 0 || blockIdx.x == gridDim.x - 1))
    a.stamps[((blockIdx.x ? 1 : 0) * 8 + (c - 8)) * 16 + (point ? 12 : 11)] = __builtin_amdgcn_s_memtime();
}

__global__ void __launch_bounds__(kGenThreads, 1) generate_kernel(GenArgs a) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int H = a.H, V = a.V, S = a.S, L = a.L;
  const int u0 = blockIdx.x * kGenU;
  const int rowb = 2 * H + 16;  // bytes per LDS weight row (one gate column, K = H) + pad
  // ---- LDS carve-up
  unsigned char* p = gen_lds;
  bf16* Wl = reinterpret_cast<bf16*>(p);                 // [(2L-1) slices][16 cols][H + 8]
  p += (size_t)(2 * L - 1) * kGenCols * rowb;
  float* hcur = reinterpret_cast<float*>(p);             // [L][S][H] latest h of every layer
  p += (size_t)L * S * H * 4;
  float* part = reinterpret_cast<float*>(p);             // [S][chunks][cols]
  p += (size_t)S * kGenChunks * kGenCols * 4;
  float* z = reinterpret_cast<float*>(p);                // [S][cols]
  p += (size_t)S * kGenCols * 4;
  float* lg = reinterpret_cast<float*>(p);               // [S][V] logits / probabilities
  p += (size_t)S * V * 4;
  float* red = reinterpret_cast<float*>(p);              // [kGenThreads] scan / reductions
  p += kGenThreads * 4;
  int* ids = reinterpret_cast<int*>(p);                  // [S] this character's input ids
  p += 16 * 4;
  int* pk = reinterpret_cast<int*>(p);                   // [S] picks
  p += 16 * 4;
  unsigned* flag = reinterpret_cast<unsigned*>(p);
  p += 16;
  float* cst = reinterpret_cast<float*>(p);              // [L][S][U] cell state of the owned units
  p += (size_t)L * S * kGenU * 4;
  float* bsL = reinterpret_cast<float*>(p);              // [V] softmax_b
  p += (size_t)((V + 3) & ~3) * 4;
  float* biasL = reinterpret_cast<float*>(p);            // [L][cols] the owned gate biases
  p += (size_t)kGenMaxLayers * kGenCols * 4;
  bf16* WsL = a.ws_lds ? reinterpret_cast<bf16*>(p) : nullptr;  // [V][H + 8] softmax_wᵀ
  const int wsld = H + 8;  // (16-B row pad: the 16 rows of an MFMA fragment read on distinct banks)

  // ---- resident weights: slice 0 = W_h,0; slice 2l-1 = W_x,l, 2l = W_h,l (l > 0).  LDS row c
  // (gate g = c / 4, unit u0 + c % 4) holds column g H + u0 + c % 4 of the [K, 4H] TF kernel
  for (int sl = 0; sl < 2 * L - 1; ++sl) {
    const int l = (sl + 1) / 2;
    const bf16* W = (sl == 0 || sl % 2 == 0) ? a.Wh[l] : a.Wx[l];
    bf16* dst = reinterpret_cast<bf16*>(reinterpret_cast<unsigned char*>(Wl) + (size_t)sl * kGenCols * rowb);
    for (int i = tid; i < kGenCols * H; i += kGenThreads) {
      const int c = i / H, k = i % H;
      const int col = (c / kGenU) * H + u0 + (c % kGenU);
      *reinterpret_cast<bf16*>(reinterpret_cast<unsigned char*>(dst) + (size_t)c * rowb + 2 * k) =
          W[(size_t)k * 4 * H + col];
    }
  }
  if (WsL)
    for (int i = tid; i < V * H; i += kGenThreads) WsL[(size_t)(i / H) * wsld + i % H] = a.WsT[i];
  for (int i = tid; i < V; i += kGenThreads) bsL[i] = a.bs[i];
  for (int i = tid; i < L * kGenCols; i += kGenThreads) {
    const int l = i / kGenCols, cc = i % kGenCols;
    biasL[i] = a.bias[l][(cc / kGenU) * H + u0 + (cc % kGenU)];
  }
  // initial state: full h of every layer (bf16-rounded like the training forward's h rows);
  // the owned units' c in registers of threads t < S * U
  for (int i = tid; i < L * S * H; i += kGenThreads) hcur[i] = (float)f2bf(a.h0[i]);
  const int cs = tid / kGenU, cu = tid % kGenU;  // (stream, unit) of this thread's cell
  const bool cell = tid < S * kGenU;
  if (cell)
    for (int l = 0; l < L; ++l) cst[(l * S + cs) * kGenU + cu] = a.c0[((size_t)l * S + cs) * H + u0 + cu];
  __syncthreads();

  const int NC = a.P - 1 + a.num;  // characters stepped: prime[:-1] warm-up, then num draws
  const int col = tid % kGenCols, kc = tid / kGenCols;
  const int KC = H / kGenChunks;   // k per chunk
  bool dead = false;
  for (int c = 0; c < NC; ++c) {
    if (tid < S) {  // (two stores, not a select of a global and an LDS pointer: a flat load)
      if (c < a.P) ids[tid] = a.prime[c];
      else ids[tid] = pk[tid];
    }
    gen_stamp(a, c, 0);
    __syncthreads();
    // layer 0's table row of this character's id: loaded now, used after the GEMV
    float trow = 0.f;
    if (tid < S * kGenCols) {
      const int s = tid / kGenCols, cc = tid % kGenCols;
      trow = a.table[(size_t)ids[s] * 4 * H + (cc / kGenU) * H + u0 + (cc % kGenU)];
    }
    for (int l = 0; l < L; ++l) {
      // ---- z[s][col] = sum_k x[s][k] Wx[col][k] + h[s][k] Wh[col][k] over this thread's chunk
      const float* x = l ? hcur + (size_t)(l - 1) * S * H : nullptr;
      const float* hp = hcur + (size_t)l * S * H;
      const unsigned char* wh = reinterpret_cast<const unsigned char*>(Wl) +
                                (size_t)(l ? 2 * l : 0) * kGenCols * rowb + (size_t)col * rowb;
      const unsigned char* wx = reinterpret_cast<const unsigned char*>(Wl) +
                                (size_t)(2 * l - 1) * kGenCols * rowb + (size_t)col * rowb;
      // (operands as 16-B LDS reads, a chunk's reads issued together: KC = H / 16 is a
      // multiple of 8)
      auto dot8 = [](const bf16x8& wv, const float* v) {
        const float4 v0 = *reinterpret_cast<const float4*>(v);
        const float4 v1 = *reinterpret_cast<const float4*>(v + 4);
        return (float)wv[0] * v0.x + (float)wv[1] * v0.y + (float)wv[2] * v0.z +
               (float)wv[3] * v0.w + (float)wv[4] * v1.x + (float)wv[5] * v1.y +
               (float)wv[6] * v1.z + (float)wv[7] * v1.w;
      };
      for (int s = 0; s < S; ++s) {
        float acc = 0.f;
        const float* hv = hp + (size_t)s * H;
        if (l) {
          const float* xs = x + (size_t)s * H;
#pragma unroll 4
          for (int k = kc * KC; k < (kc + 1) * KC; k += 8)
            acc += dot8(*reinterpret_cast<const bf16x8*>(wh + 2 * k), hv + k) +
                   dot8(*reinterpret_cast<const bf16x8*>(wx + 2 * k), xs + k);
        } else {
#pragma unroll 4
          for (int k = kc * KC; k < (kc + 1) * KC; k += 8)
            acc += dot8(*reinterpret_cast<const bf16x8*>(wh + 2 * k), hv + k);
        }
        part[((size_t)s * kGenChunks + kc) * kGenCols + col] = acc;
      }
      gen_stamp(a, c, 1 + 4 * l);
      __syncthreads();
      if (tid < S * kGenCols) {
        const int s = tid / kGenCols, cc = tid % kGenCols;
        float t = 0.f;
        for (int i = 0; i < kGenChunks; ++i) t += part[((size_t)s * kGenChunks + i) * kGenCols + cc];
        t += l == 0 ? trow : biasL[l * kGenCols + cc];
        z[s * kGenCols + cc] = t;
      }
      __syncthreads();
      // ---- cell update of the owned units; publish h as tagged granules
      const unsigned tag = (unsigned)(c * L + l + 1);
      unsigned long long* slot = a.hx + ((size_t)l * 2 + (c & 1)) * S * H;
      if (cell) {
        const float* zz = z + cs * kGenCols;
        const float gi = sigmoidf_(zz[cu]), gj = tanhf_(zz[kGenU + cu]);
        const float gf = sigmoidf_(zz[2 * kGenU + cu] + a.forget_bias), go = sigmoidf_(zz[3 * kGenU + cu]);
        float& cv = cst[(l * S + cs) * kGenU + cu];  // (only this thread touches it)
        cv = gf * cv + gi * gj;
        const float h = go * tanhf_(cv);
        const float hb = (float)f2bf(h);
        __hip_atomic_store(slot + (size_t)cs * H + u0 + cu, gen_pack(hb, tag), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        if (c == NC - 1) {
          a.h_out[((size_t)l * S + cs) * H + u0 + cu] = h;
          a.c_out[((size_t)l * S + cs) * H + u0 + cu] = cv;
        }
      }
      gen_stamp(a, c, 2 + 4 * l);
      // ---- all-gather h_l: every granule of a thread's batch is loaded at once, then only
      // the ones not yet carrying the tag are polled again (one round trip per batch, not
      // one per granule)
      float* hl = hcur + (size_t)l * S * H;
      const int n = S * H;
      for (int base = tid; base < n; base += kGenThreads * kGenGather) {
        unsigned long long g[kGenGather];
#pragma unroll
        for (int j = 0; j < kGenGather; ++j) {
          const int i = base + kGenThreads * j;
          g[j] = i < n ? __hip_atomic_load(slot + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                       : ((unsigned long long)tag << 32);
        }
        unsigned spins = 0;
        for (;;) {
          bool all = true;
#pragma unroll
          for (int j = 0; j < kGenGather; ++j) all = all && (unsigned)(g[j] >> 32) == tag;
          if (all || dead) break;
          __builtin_amdgcn_s_sleep(1);
#pragma unroll
          for (int j = 0; j < kGenGather; ++j) {
            const int i = base + kGenThreads * j;
            if ((unsigned)(g[j] >> 32) != tag)
              g[j] = __hip_atomic_load(slot + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          if (++spins > a.spin_limit) {
            dead = true;
            atomicOr(a.err, 0x40u);
          }
        }
#pragma unroll
        for (int j = 0; j < kGenGather; ++j) {
          const int i = base + kGenThreads * j;
          if (i < n) hl[i] = __uint_as_float((unsigned)g[j]);
        }
      }
      gen_stamp(a, c, 3 + 4 * l);
      __syncthreads();
      gen_stamp(a, c, 4 + 4 * l);
    }
    // ---- head: logits of every stream on MFMA, all streams at once: D[v][s] = sum_k
    // Ws[v][k] h[s][k] as 16-row vocabulary blocks (one per wave in turn) x the <= 16 streams
    // as the 16 columns; lane l supplies A row (l & 15), B column (l & 15) = stream, k-chunk
    // l >> 4 of each 32-deep k-step (h is bf16-exact: the rounded values of the all-gather)
    {
      const float* ht = hcur + (size_t)(L - 1) * S * H;
      const int m = lane & 15, q = lane >> 4;
      const bool sv = m < S;
      for (int rb = w; rb * 16 < V && a.dbg != 1; rb += kGenThreads / 64) {
        const int row = min(16 * rb + m, V - 1);
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        // every operand load unconditional (a guarded LDS read is a branch with its own
        // lgkmcnt(0): one serialised round trip per element), 4 k-steps per batch
        const float* hrow = ht + (size_t)(sv ? m : 0) * H;
        const float zs = sv ? 1.f : 0.f;
        // (two accumulator chains over alternate k-steps: their operand reads overlap; H is a
        // multiple of 128, so the k-steps pair up)
        f32x4 acc2 = f32x4{0.f, 0.f, 0.f, 0.f};
        auto step2 = [&](int k0) {
          bf16x8 av0, av1;
          if (WsL) {
            av0 = *reinterpret_cast<const bf16x8*>(WsL + (size_t)row * wsld + k0);
            av1 = *reinterpret_cast<const bf16x8*>(WsL + (size_t)row * wsld + k0 + 32);
          } else {
            av0 = ld8(a.WsT + (size_t)row * H + k0);
            av1 = ld8(a.WsT + (size_t)row * H + k0 + 32);
          }
          const float4 h0 = *reinterpret_cast<const float4*>(hrow + k0);
          const float4 h1 = *reinterpret_cast<const float4*>(hrow + k0 + 4);
          const float4 h2 = *reinterpret_cast<const float4*>(hrow + k0 + 32);
          const float4 h3 = *reinterpret_cast<const float4*>(hrow + k0 + 36);
          bf16x8 b0, b1;
          b0[0] = (bf16)(h0.x * zs); b0[1] = (bf16)(h0.y * zs); b0[2] = (bf16)(h0.z * zs);
          b0[3] = (bf16)(h0.w * zs); b0[4] = (bf16)(h1.x * zs); b0[5] = (bf16)(h1.y * zs);
          b0[6] = (bf16)(h1.z * zs); b0[7] = (bf16)(h1.w * zs);
          b1[0] = (bf16)(h2.x * zs); b1[1] = (bf16)(h2.y * zs); b1[2] = (bf16)(h2.z * zs);
          b1[3] = (bf16)(h2.w * zs); b1[4] = (bf16)(h3.x * zs); b1[5] = (bf16)(h3.y * zs);
          b1[6] = (bf16)(h3.z * zs); b1[7] = (bf16)(h3.w * zs);
          acc = mfma16(av0, b0, acc);
          acc2 = mfma16(av1, b1, acc2);
        };
        if (WsL) {
#pragma unroll 2
          for (int k0 = 8 * q; k0 < H; k0 += 64) step2(k0);
        } else {
#pragma unroll 2
          for (int k0 = 8 * q; k0 < H; k0 += 64) step2(k0);
        }
        acc += acc2;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int v = 16 * rb + 4 * q + r;
          if (v < V && sv) lg[(size_t)m * V + v] = acc[r] + bsL[v];
        }
      }
    }
    gen_stamp(a, c, 13);
    __syncthreads();
    const bool draw = c >= a.P - 1;
    if (draw && a.logits_out && blockIdx.x == 0)
      for (int i = tid; i < S * V; i += kGenThreads)
        a.logits_out[(size_t)(c - (a.P - 1)) * S * V + i] = lg[i];
    // ---- the pick of every stream (sample.hip's rules), identical in every workgroup: one
    // wave per stream, wave-level reductions and scan only (no block barrier inside)
    for (int s = w; s < S; s += kGenThreads / 64) {
      const float* ls = lg + (size_t)s * V;
      // lane l owns the contiguous chunk [l C, l C + C) of the vocabulary
      const int C = (V + 63) / 64;
      const int lo = lane * C, hi = min(lo + C, V);
      float m = -INFINITY;
      for (int v = lo; v < hi; ++v) m = fmaxf(m, ls[v]);
      m = wave_max(m);
      int first = V;
      for (int v = hi - 1; v >= lo; --v)
        if (ls[v] == m) first = v;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) first = min(first, __shfl_xor(first, o, 64));
      int pick = first;
      const bool weighted = a.mode == 1 || (a.mode == 2 && ids[s] == a.space_id);
      if (draw && weighted) {
        float csum = 0.f;
        for (int v = lo; v < hi; ++v) csum += __expf(ls[v] - m);
        // inclusive prefix sum over the lanes' chunk sums
        float incl = csum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const float t = __shfl_up(incl, o, 64);
          if (lane >= o) incl += t;
        }
        const float total = __shfl(incl, 63, 64);
        const float u = uniform01(a.seed, (uint64_t)s, (uint64_t)(a.ctr0[s] + (unsigned)(c - (a.P - 1))));
        const float r = u * total;
        const float before = incl - csum;
        // the first lane whose inclusive sum reaches r scans its chunk
        const unsigned long long hit_lanes = __ballot(lo < hi && r <= incl);
        const int owner = hit_lanes ? __ffsll((long long)hit_lanes) - 1 : -1;
        int hit = V - 1;
        if (lane == owner) {
          float cc = before;
          hit = hi - 1;
          for (int v = lo; v < hi; ++v) {
            cc += __expf(ls[v] - m);
            if (cc >= r) { hit = v; break; }
          }
        }
        pick = owner >= 0 ? __shfl(hit, owner, 64) : V - 1;
      }
      if (lane == 0) {
        pk[s] = pick;
        if (draw && blockIdx.x == 0) a.out[(size_t)s * a.num + (c - (a.P - 1))] = pick;
      }
    }
    gen_stamp(a, c, 14);
    __syncthreads();
  }
}

size_t gen_lds_bytes(int L, int H, int V, int S, bool ws_lds) {
  size_t b = (size_t)(2 * L - 1) * kGenCols * (2 * H + 16) + (size_t)L * S * H * 4 +
             (size_t)S * kGenChunks * kGenCols * 4 + (size_t)S * kGenCols * 4 + (size_t)S * V * 4 +
             kGenThreads * 4 + 16 * 4 + 16 * 4 + 16 + (size_t)L * S * kGenU * 4 +
             (size_t)((V + 3) & ~3) * 4 + (size_t)kGenMaxLayers * kGenCols * 4;
  if (ws_lds) b += (size_t)V * (H + 8) * 2;
  return b;
}

int generate_supported(int L, int H, int V, int S, int cus) {
  if (L < 1 || L > kGenMaxLayers || H % (kGenChunks * 8) != 0 || H / kGenU > cus || S < 1 ||
      S > kGenMaxStreams || V < 1)
    return 0;
  return gen_lds_bytes(L, H, V, S, false) <= 160 * 1024 ? 1 : 0;
}

int launch_generate(GenArgs& a, int cus, hipStream_t s) {
  if (!generate_supported(a.L, a.H, a.V, a.S, cus)) return -1;
  a.ws_lds = gen_lds_bytes(a.L, a.H, a.V, a.S, true) <= 160 * 1024 ? 1 : 0;
  a.dbg = debug_int("gen_dbg", 0);
  const size_t lds = gen_lds_bytes(a.L, a.H, a.V, a.S, a.ws_lds != 0);
  if (hipFuncSetAttribute((const void*)generate_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return -2;
  hipLaunchKernelGGL(generate_kernel, dim3(a.H / kGenU), dim3(kGenThreads), lds, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace dcr
