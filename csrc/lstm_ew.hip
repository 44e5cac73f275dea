// Epilogue-only LSTM cell kernels of the large-H library-step path (native_backend._lstm_*_lib):
// the recurrent GEMM of the step ran as a library (or split-K) GEMM; these apply the cell
// forward / backward of model.py's LSTMCell (gate order i, j, f, o; forget bias added at run
// time) exactly as the fused per-step kernels (rnn_step.hip) do, with a thread mapping made for
// streaming: thread -> (batch row b, 4 consecutive units), consecutive threads -> consecutive
// units, so every gate read / write of a wave is one contiguous 1 KB (fp32) / 512 B (bf16)
// segment.  (Launching the MFMA step kernel without its GEMM instead measured 10.4 / 9.3 us per
// step at B = 256, H = 2048: its 16-row x 64-unit lane tiles touch 64-B pieces of 16 rows.)
#include "common.h"
#include "kernels.h"

namespace dcr {

constexpr int kEwThreads = 256;

__device__ __forceinline__ float4 ew_ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void ew_st4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
__device__ __forceinline__ void ew_st4bf(bf16* p, float a, float b, float c, float d) {
  bf16x4 v;
  v[0] = f2bf(a); v[1] = f2bf(b); v[2] = f2bf(c); v[3] = f2bf(d);
  *reinterpret_cast<bf16x4*>(p) = v;
}
__device__ __forceinline__ void ew_ld4bf(const bf16* p, float (&o)[4]) {
  const bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  o[0] = bf2f(v[0]); o[1] = bf2f(v[1]); o[2] = bf2f(v[2]); o[3] = bf2f(v[3]);
}

__global__ void __launch_bounds__(kEwThreads) lstm_ew_fwd_kernel(LstmEwArgs a) {
  const int H = a.H, H4 = H / 4;
  const int64_t n = (int64_t)a.B * H4;
  const int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x;
  if (i >= n) return;
  const int b = (int)(i / H4), u = (int)(i % H4) * 4;
  const size_t G = 4 * (size_t)H;
  const float* zx = a.ids ? a.zx + (size_t)a.ids[b] * G : a.zx + (size_t)b * G;
  float z[4][4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 v = ew_ld4(zx + (size_t)g * H + u);
    z[g][0] = v.x; z[g][1] = v.y; z[g][2] = v.z; z[g][3] = v.w;
  }
  if (a.bias) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 v = ew_ld4(a.bias + (size_t)g * H + u);
      z[g][0] += v.x; z[g][1] += v.y; z[g][2] += v.z; z[g][3] += v.w;
    }
  }
  for (int s = 0; s < a.nsplit; ++s) {
    const float* zr = a.zrec + ((size_t)s * a.B + b) * G + u;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 v = ew_ld4(zr + (size_t)g * H);
      z[g][0] += v.x; z[g][1] += v.y; z[g][2] += v.z; z[g][3] += v.w;
    }
  }
  const size_t bh = (size_t)b * H + u;
  const float4 cpv = ew_ld4(a.cprev + bh);
  const float cp[4] = {cpv.x, cpv.y, cpv.z, cpv.w};
  float gi[4], gj[4], gf[4], go[4], cn[4], hc[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    gi[r] = sigmoidf_(z[0][r]);
    gj[r] = tanhf_(z[1][r]);
    gf[r] = sigmoidf_(z[2][r] + a.forget_bias);
    go[r] = sigmoidf_(z[3][r]);
    cn[r] = gf[r] * cp[r] + gi[r] * gj[r];
    hc[r] = go[r] * tanhf_(cn[r]);
  }
  ew_st4(a.cout + bh, cn[0], cn[1], cn[2], cn[3]);
  ew_st4bf(a.hout + bh, hc[0], hc[1], hc[2], hc[3]);
  if (a.hout32) ew_st4(a.hout32 + bh, hc[0], hc[1], hc[2], hc[3]);
  bf16* gp = a.gates + (size_t)b * G + u;
  ew_st4bf(gp, gi[0], gi[1], gi[2], gi[3]);
  ew_st4bf(gp + H, gj[0], gj[1], gj[2], gj[3]);
  ew_st4bf(gp + 2 * H, gf[0], gf[1], gf[2], gf[3]);
  ew_st4bf(gp + 3 * H, go[0], go[1], go[2], go[3]);
}

__global__ void __launch_bounds__(kEwThreads) lstm_ew_bwd_kernel(LstmEwArgs a) {
  const int H = a.H, H4 = H / 4;
  const int64_t n = (int64_t)a.B * H4;
  const int64_t i = (int64_t)blockIdx.x * kEwThreads + threadIdx.x;
  if (i >= n) return;
  const int b = (int)(i / H4), u = (int)(i % H4) * 4;
  const size_t G = 4 * (size_t)H, bh = (size_t)b * H + u;
  float dh[4];
  {
    const float4 v = ew_ld4(a.dtop + bh);
    dh[0] = v.x; dh[1] = v.y; dh[2] = v.z; dh[3] = v.w;
  }
  for (int s = 0; s < a.nsplit; ++s) {
    const float4 v = ew_ld4(a.dhrec + (size_t)s * a.B * H + bh);
    dh[0] += v.x; dh[1] += v.y; dh[2] += v.z; dh[3] += v.w;
  }
  float gi[4], gj[4], gf[4], go[4];
  const bf16* gp = a.gates_in + (size_t)b * G + u;
  ew_ld4bf(gp, gi); ew_ld4bf(gp + H, gj); ew_ld4bf(gp + 2 * H, gf); ew_ld4bf(gp + 3 * H, go);
  const float4 cv = ew_ld4(a.c + bh), cpv = ew_ld4(a.cprev + bh), dcv4 = ew_ld4(a.dc + bh);
  const float c[4] = {cv.x, cv.y, cv.z, cv.w}, cp[4] = {cpv.x, cpv.y, cpv.z, cpv.w};
  const float dcin[4] = {dcv4.x, dcv4.y, dcv4.z, dcv4.w};
  float di[4], dj[4], df[4], dO[4], dcp[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {  // same math as rnn_step.hip bwd_step_kernel<CELL_LSTM>
    const float th = tanhf_(c[r]);
    const float dcv = dcin[r] + dh[r] * go[r] * (1.f - th * th);
    dO[r] = dh[r] * th * go[r] * (1.f - go[r]);
    di[r] = dcv * gj[r] * gi[r] * (1.f - gi[r]);
    dj[r] = dcv * gi[r] * (1.f - gj[r] * gj[r]);
    df[r] = dcv * cp[r] * gf[r] * (1.f - gf[r]);
    dcp[r] = dcv * gf[r];
  }
  bf16* dz = a.dz_out + (size_t)b * G + u;
  ew_st4bf(dz, di[0], di[1], di[2], di[3]);
  ew_st4bf(dz + H, dj[0], dj[1], dj[2], dj[3]);
  ew_st4bf(dz + 2 * H, df[0], df[1], df[2], df[3]);
  ew_st4bf(dz + 3 * H, dO[0], dO[1], dO[2], dO[3]);
  ew_st4(a.dc + bh, dcp[0], dcp[1], dcp[2], dcp[3]);
}

void launch_lstm_ew(bool bwd, const LstmEwArgs& a, hipStream_t s) {
  const int64_t n = (int64_t)a.B * (a.H / 4);
  const unsigned nb = (unsigned)((n + kEwThreads - 1) / kEwThreads);
  if (bwd)
    lstm_ew_bwd_kernel<<<nb, kEwThreads, 0, s>>>(a);
  else
    lstm_ew_fwd_kernel<<<nb, kEwThreads, 0, s>>>(a);
}

}  // namespace dcr
