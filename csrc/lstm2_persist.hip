// Two-layer wavefront forward for the persistent LSTM (gfx950).
//
// Reference: the layer stack of model.py:27-36 runs layer l+1's step t on layer l's h_t; the
// single-layer persistent kernels (lstm_persist.hip) therefore run 2T hand-off-latency-bound
// steps for two layers, although layer l+1's step t-1 and layer l's step t are independent.
// One launch here runs both layers as a wavefront: at tick tau layer l computes step tau and
// layer l+1 computes step tau-1.  Both consume the same published slot h_l[tau] (layer l's
// recurrent input and layer l+1's input x), so a tick loads one extra payload (h_{l+1}) and
// T+1 ticks replace 2T steps.  Per-step latency, not bandwidth, bounds these kernels
// (profiles/r1_persist_stamps_vs_batch.txt), which is what makes the wider tick pay.
//
// Workgroup (ubk, bg) owns 16 hidden units x 32 batch rows (two 16-row MFMA tiles) of BOTH
// layers; its 4 waves split K in quarters and keep W_h(l)ᵀ, W_h(l+1)ᵀ and W_x(l+1)ᵀ rows of its
// units resident (3 x 16 x KS fragments).  Wave w runs the epilogue of layer w>>1, batch tile
// w&1.  Hand-off protocol as lstm_persist.hip (persist_common.h): sc1 write-through h stores,
// drain, agent-scope counter add per (layer, batch group, slot, K quarter); ONE poller per
// workgroup watches both layers' counters; every load of published h is buffer_load sc1.
#include "common.h"
#include "kernels.h"
#include "persist_common.h"

namespace dcr {

#define STAMP2(i)                                                                   \
  if constexpr (DIAG) {                                                             \
    if (blockIdx.x == 0 && threadIdx.x == 0)                                        \
      a.diag[(size_t)tau * 8 + (i)] = __builtin_amdgcn_s_memtime();                 \
  }

template <int KS, bool DIAG = false>
__global__ void __launch_bounds__(256, 1) lstm2_fwd_persist_kernel(Lstm2Args a) {
  // partials [wave][layer][tile][lane][gate*4 + r]: single-buffered -- every tick after the
  // first starts with the poll barrier, which each epilogue wave joins after its reads
  __shared__ __attribute__((aligned(16))) float part[4][2][2][64][16];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int H = a.H, B = a.B, T = a.T;
  const int nwg_u = H / 16;
  int ubk, bg;
  map_block(blockIdx.x, nwg_u, B / 32, ubk, bg);
  const int ub0 = ubk * 16, b0 = bg * 32;
  const int kq = 8 * (lane >> 4);
  const int kbase = w * (KS * 32);
  unsigned* cnt0 = a.cnt0 + (size_t)bg * (T + 1) * 4;
  unsigned* cnt1 = a.cnt1 + (size_t)bg * (T + 1) * 4;
  const unsigned target = (unsigned)(H / 8);  // H/16 unit blocks x 2 batch tiles
  bool dead = false;

  bf16x8 w0[4][KS], w1[4][KS], x1[4][KS];
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const size_t row = (size_t)(g * H + ub0 + (lane & 15)) * H + kbase + s * 32 + kq;
      w0[g][s] = ld8(a.W0T + row);
      w1[g][s] = ld8(a.W1T + row);
      x1[g][s] = ld8(a.X1T + row);
    }
  unsigned hoff[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    hoff[j] = (unsigned)(((size_t)(b0 + 16 * j + (lane & 15)) * H + kbase + kq) * sizeof(bf16));

  // epilogue role: layer L, batch tile J
  const int L = w >> 1, J = w & 1;
  const int b = b0 + 16 * J + (lane & 15);
  const int u0 = ub0 + 4 * (lane >> 4);
  const size_t bh = (size_t)b * H + u0;
  bf16* const hbL = L ? a.hbuf1 : a.hbuf0;
  float* const cbL = L ? a.cbuf1 : a.cbuf0;
  bf16* const gtL = L ? a.gates1 : a.gates0;
  float* const hlL = L ? a.hlast1 : a.hlast0;
  float* const clL = L ? a.clast1 : a.clast0;
  unsigned* const cntL = L ? cnt1 : cnt0;
  float c[4];
  ld4f(cbL + bh, c);
  float bias1[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g) ld4f(a.bias1 + g * H + u0, bias1[g]);

  for (int tau = 0; tau <= T; ++tau) {
    const bool on0 = tau < T, on1 = tau >= 1;
    STAMP2(0)
    // layer-l input projections of step tau (recurrence independent: issued before the wait)
    float zx[4][4];
    if (L == 0 && on0) {
      const float* zrow = a.ids ? a.zx0 + (size_t)a.ids[(size_t)tau * B + b] * a.zx_ld
                                : a.zx0 + ((size_t)tau * B + b) * a.zx_ld;
#pragma unroll
      for (int g = 0; g < 4; ++g) ld4f(zrow + (size_t)g * H + u0, zx[g]);
    }
    if (tau >= 1) {
      if (threadIdx.x == kLstmPollerThread && !dead) {
        // layer l+1's slot tau-1 exists from tick 2 on; before that poll layer l's twice
        dead = tau >= 2 ? !poll_counter2(cnt0 + (size_t)tau * 4, target,
                                         cnt1 + (size_t)(tau - 1) * 4, target, a.spin_limit,
                                         a.err, 9u)
                        : !poll_counter(cnt0 + (size_t)tau * 4, target, a.spin_limit, a.err, 9u);
      }
      STAMP2(1)
      __syncthreads();
    }
    STAMP2(2)
    // payloads: h_l[tau] (both layers' input) and h_{l+1}[tau-1]
    bf16x8 hf0[2][KS], hf1[2][KS];
    {
      // slot 0 (initial state, written by the prep launch) is row-major; later slots come from
      // the fragment-tiled rings: one contiguous 1 KB load per (tile, k-step)
      const bool ring0 = a.hring0 && tau > 0, ring1 = a.hring1 && tau > 1;
      const __amdgpu_buffer_rsrc_t r0 =
          ring0 ? make_rsrc(a.hring0 + (size_t)(tau & 1) * B * H, sizeof(bf16) * (size_t)B * H)
                : make_rsrc(a.hbuf0 + (size_t)tau * B * H, sizeof(bf16) * (size_t)B * H);
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int s = 0; s < KS; ++s)
          hf0[j][s] = ld8_sc1(r0, ring0 ? frag_load_off(2 * bg + j, w * KS + s, H, lane)
                                        : hoff[j] + s * 64);
      if (on1) {
        const __amdgpu_buffer_rsrc_t r1 =
            ring1 ? make_rsrc(a.hring1 + (size_t)((tau - 1) & 1) * B * H, sizeof(bf16) * (size_t)B * H)
                  : make_rsrc(a.hbuf1 + (size_t)(tau - 1) * B * H, sizeof(bf16) * (size_t)B * H);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int s = 0; s < KS; ++s)
            hf1[j][s] = ld8_sc1(r1, ring1 ? frag_load_off(2 * bg + j, w * KS + s, H, lane)
                                          : hoff[j] + s * 64);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (on0) {
        f32x4 acc[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[g] = mfma16(w0[g][s], hf0[j][s], acc[g]);
        float4* dst = reinterpret_cast<float4*>(&part[w][0][j][lane][0]);
#pragma unroll
        for (int g = 0; g < 4; ++g) dst[g] = make_float4(acc[g][0], acc[g][1], acc[g][2], acc[g][3]);
      }
      if (on1) {
        f32x4 acc[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            acc[g] = mfma16(x1[g][s], hf0[j][s], acc[g]);
            acc[g] = mfma16(w1[g][s], hf1[j][s], acc[g]);
          }
        float4* dst = reinterpret_cast<float4*>(&part[w][1][j][lane][0]);
#pragma unroll
        for (int g = 0; g < 4; ++g) dst[g] = make_float4(acc[g][0], acc[g][1], acc[g][2], acc[g][3]);
      }
    }
    STAMP2(3)
    __syncthreads();
    STAMP2(4)
    if (L == 0 ? on0 : on1) {
      const int t = L == 0 ? tau : tau - 1;  // this layer's step
      float z[4][4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 s0 = reinterpret_cast<const float4*>(&part[0][L][J][lane][0])[g];
        const float4 s1 = reinterpret_cast<const float4*>(&part[1][L][J][lane][0])[g];
        const float4 s2 = reinterpret_cast<const float4*>(&part[2][L][J][lane][0])[g];
        const float4 s3 = reinterpret_cast<const float4*>(&part[3][L][J][lane][0])[g];
        const float* add = L == 0 ? zx[g] : bias1[g];
        z[g][0] = s0.x + s1.x + s2.x + s3.x + add[0];
        z[g][1] = s0.y + s1.y + s2.y + s3.y + add[1];
        z[g][2] = s0.z + s1.z + s2.z + s3.z + add[2];
        z[g][3] = s0.w + s1.w + s2.w + s3.w + add[3];
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
      const size_t o = (size_t)(t + 1) * B * H + bh;
      STAMP2(5)
      bf16* const ringL = L ? a.hring1 : a.hring0;
      if (ringL)
        st4bf_sc1(ringL + (size_t)((t + 1) & 1) * B * H + frag_index(b, u0, H), h[0], h[1], h[2], h[3]);
      else
        st4bf_sc1(hbL + o, h[0], h[1], h[2], h[3]);
      // layer l's slot t+1 feeds both layers (up to slot T); layer l+1's slot t+1 only itself
      if (L == 0 || t + 1 < T) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        STAMP2(6)
        if (lane == 0)
          __hip_atomic_fetch_add(cntL + (size_t)(t + 1) * 4, 1u,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (ringL) st4bf(hbL + o, h[0], h[1], h[2], h[3]);  // row-major copy for the GEMMs
      *reinterpret_cast<float4*>(cbL + o) = make_float4(c[0], c[1], c[2], c[3]);
      if (gtL) {
        bf16* gp = gtL + ((size_t)t * B + b) * 4 * H + u0;
        st4bf(gp, gi[0], gi[1], gi[2], gi[3]);
        st4bf(gp + H, gj[0], gj[1], gj[2], gj[3]);
        st4bf(gp + 2 * H, gf[0], gf[1], gf[2], gf[3]);
        st4bf(gp + 3 * H, go[0], go[1], go[2], go[3]);
      }
      if (t == T - 1 && hlL)
        *reinterpret_cast<float4*>(hlL + bh) = make_float4(h[0], h[1], h[2], h[3]);
      if (t == T - 1 && clL)
        *reinterpret_cast<float4*>(clL + bh) = make_float4(c[0], c[1], c[2], c[3]);
    }
  }
}

template <int KS>
static const void* lstm2_fn(bool diag) {
  return diag ? (const void*)lstm2_fwd_persist_kernel<KS, true>
              : (const void*)lstm2_fwd_persist_kernel<KS, false>;
}

static const void* lstm2_pick(int H, bool diag = false) {
  switch (H / 128) {
    case 1: return lstm2_fn<1>(diag);
    case 2: return lstm2_fn<2>(diag);
    case 3: return lstm2_fn<3>(diag);
    case 4: return lstm2_fn<4>(diag);
  }
  return nullptr;
}

static int lstm2_grid(int H, int B) { return (H / 16) * (B / 32); }

int lstm2_persist_supported(int H, int B, int cus) {
  if (H % 128 != 0 || H < 128 || H > 512 || B % 32 != 0 || B < 32 || cus <= 0) return 0;
  const void* fn = lstm2_pick(H);
  int occ = 0;
  if (!fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, 256, 0) != hipSuccess)
    return 0;
  return lstm2_grid(H, B) <= occ * cus ? 1 : 0;
}

int launch_lstm2_fwd_persist(const Lstm2Args& a, int cus, hipStream_t s) {
  if (!lstm2_persist_supported(a.H, a.B, cus)) return -2;
  void* args[] = {const_cast<Lstm2Args*>(&a)};
  return hipLaunchKernel(lstm2_pick(a.H, a.diag != nullptr), dim3(lstm2_grid(a.H, a.B)),
                         dim3(256), args, 0, s) ==
                 hipSuccess ? 0 : -3;
}

}  // namespace dcr
