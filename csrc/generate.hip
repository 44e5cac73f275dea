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

namespace dcr {

constexpr int kGenThreads = 256;
constexpr int kGenU = 4;           // units per workgroup per layer
constexpr int kGenCols = 4 * kGenU;  // gate columns per workgroup per layer
constexpr int kGenChunks = kGenThreads / kGenCols;  // k-chunks per column (16)

__device__ __forceinline__ unsigned long long gen_pack(float v, unsigned tag) {
  return (unsigned long long)__float_as_uint(v) | ((unsigned long long)tag << 32);
}

extern __shared__ __attribute__((aligned(16))) unsigned char gen_lds[];

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
  bf16* WsL = a.ws_lds ? reinterpret_cast<bf16*>(p) : nullptr;  // [V][H] softmax_wᵀ

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
    for (int i = tid; i < V * H; i += kGenThreads) WsL[i] = a.WsT[i];
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
    if (tid < S) ids[tid] = c < a.P ? a.prime[c] : pk[tid];
    __syncthreads();
    for (int l = 0; l < L; ++l) {
      // ---- z[s][col] = sum_k x[s][k] Wx[col][k] + h[s][k] Wh[col][k] over this thread's chunk
      const float* x = l ? hcur + (size_t)(l - 1) * S * H : nullptr;
      const float* hp = hcur + (size_t)l * S * H;
      const unsigned char* wh = reinterpret_cast<const unsigned char*>(Wl) +
                                (size_t)(l ? 2 * l : 0) * kGenCols * rowb + (size_t)col * rowb;
      const unsigned char* wx = reinterpret_cast<const unsigned char*>(Wl) +
                                (size_t)(2 * l - 1) * kGenCols * rowb + (size_t)col * rowb;
      for (int s = 0; s < S; ++s) {
        float acc = 0.f;
        for (int k = kc * KC; k < (kc + 1) * KC; k += 8) {
          const bf16x8 wv = *reinterpret_cast<const bf16x8*>(wh + 2 * k);
          const float* hv = hp + (size_t)s * H + k;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc += (float)wv[j] * hv[j];
          if (l) {
            const bf16x8 xv = *reinterpret_cast<const bf16x8*>(wx + 2 * k);
            const float* xs = x + (size_t)s * H + k;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc += (float)xv[j] * xs[j];
          }
        }
        part[((size_t)s * kGenChunks + kc) * kGenCols + col] = acc;
      }
      __syncthreads();
      if (tid < S * kGenCols) {
        const int s = tid / kGenCols, cc = tid % kGenCols;
        float t = 0.f;
        for (int i = 0; i < kGenChunks; ++i) t += part[((size_t)s * kGenChunks + i) * kGenCols + cc];
        const int gcol = (cc / kGenU) * H + u0 + (cc % kGenU);
        t += l == 0 ? a.table[(size_t)ids[s] * 4 * H + gcol] : a.bias[l][gcol];
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
      // ---- all-gather h_l: sweep the S x H granules until every tag matches
      float* hl = hcur + (size_t)l * S * H;
      for (int i = tid; i < S * H; i += kGenThreads) {
        unsigned long long g = __hip_atomic_load(slot + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned n = 0;
        while ((unsigned)(g >> 32) != tag && !dead) {
          __builtin_amdgcn_s_sleep(1);
          g = __hip_atomic_load(slot + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (++n > a.spin_limit) {
            dead = true;
            atomicOr(a.err, 0x40u);
          }
        }
        hl[i] = __uint_as_float((unsigned)g);
      }
      __syncthreads();
    }
    // ---- head: logits of every stream (wave per vocabulary row, lanes split H)
    const float* ht = hcur + (size_t)(L - 1) * S * H;
    for (int s = 0; s < S; ++s)
      for (int v = w; v < V; v += kGenThreads / 64) {
        const bf16* wr = WsL ? WsL + (size_t)v * H : a.WsT + (size_t)v * H;
        float acc = 0.f;
        for (int k = lane * 8; k < H; k += 64 * 8) {
          const bf16x8 y = ld8(wr + k);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc += ht[(size_t)s * H + k + j] * (float)y[j];
        }
        acc = wave_sum(acc);
        if (lane == 0) lg[(size_t)s * V + v] = acc + a.bs[v];
      }
    __syncthreads();
    const bool draw = c >= a.P - 1;
    if (draw && a.logits_out && blockIdx.x == 0)
      for (int i = tid; i < S * V; i += kGenThreads)
        a.logits_out[(size_t)(c - (a.P - 1)) * S * V + i] = lg[i];
    // ---- the pick of every stream (sample.hip's rules), identical in every workgroup
    for (int s = 0; s < S; ++s) {
      float* ls = lg + (size_t)s * V;
      float m = -INFINITY;
      for (int v = tid; v < V; v += kGenThreads) m = fmaxf(m, ls[v]);
      m = wave_max(m);
      if (lane == 0) red[w] = m;
      __syncthreads();
      m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
      __syncthreads();
      if (tid == 0) flag[0] = (unsigned)V;
      __syncthreads();
      for (int v = tid; v < V; v += kGenThreads)
        if (ls[v] == m) atomicMin(flag, (unsigned)v);
      __syncthreads();
      int pick = (int)flag[0];
      const bool weighted = a.mode == 1 || (a.mode == 2 && ids[s] == a.space_id);
      if (draw && weighted) {
        const int C = (V + kGenThreads - 1) / kGenThreads;
        const int lo = tid * C, hi = min(lo + C, V);
        float csum = 0.f;
        for (int v = lo; v < hi; ++v) {
          const float e = __expf(ls[v] - m);
          ls[v] = e;
          csum += e;
        }
        red[tid] = csum;
        __syncthreads();
        for (int off = 1; off < kGenThreads; off <<= 1) {
          const float add = tid >= off ? red[tid - off] : 0.f;
          __syncthreads();
          red[tid] += add;
          __syncthreads();
        }
        const float total = red[kGenThreads - 1];
        const float u = uniform01(a.seed, (uint64_t)s, (uint64_t)(a.ctr0[s] + (unsigned)(c - (a.P - 1))));
        const float r = u * total;
        if (tid == 0) flag[0] = (unsigned)(V - 1);
        __syncthreads();
        const float before = tid ? red[tid - 1] : 0.f;
        if (lo < hi && r <= red[tid] && (tid == 0 || r > before)) {
          float cc = before;
          int hit = hi - 1;
          for (int v = lo; v < hi; ++v) {
            cc += ls[v];
            if (cc >= r) { hit = v; break; }
          }
          flag[0] = (unsigned)hit;
        }
        __syncthreads();
        pick = (int)flag[0];
      }
      __syncthreads();
      if (tid == 0) {
        pk[s] = pick;
        if (draw && blockIdx.x == 0) a.out[(size_t)s * a.num + (c - (a.P - 1))] = pick;
      }
    }
    __syncthreads();
  }
}

size_t gen_lds_bytes(int L, int H, int V, int S, bool ws_lds) {
  size_t b = (size_t)(2 * L - 1) * kGenCols * (2 * H + 16) + (size_t)L * S * H * 4 +
             (size_t)S * kGenChunks * kGenCols * 4 + (size_t)S * kGenCols * 4 + (size_t)S * V * 4 +
             kGenThreads * 4 + 16 * 4 + 16 * 4 + 16 + (size_t)L * S * kGenU * 4;
  if (ws_lds) b += (size_t)V * H * 2;
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
  const size_t lds = gen_lds_bytes(a.L, a.H, a.V, a.S, a.ws_lds != 0);
  if (hipFuncSetAttribute((const void*)generate_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds) != hipSuccess)
    return -2;
  hipLaunchKernelGGL(generate_kernel, dim3(a.H / kGenU), dim3(kGenThreads), lds, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace dcr
