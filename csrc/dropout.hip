// Dropout masks as bits (K3 of SURVEY.md §2.3) for the DropoutWrapper(input_keep_prob,
// output_keep_prob) stack and the embedding dropout of the reference (model.py:31-34, 58-59).
//
// One mask per layer input (the embedding dropout x input dropout for layer 0, the output
// dropout of layer l-1 x the input dropout of layer l for l > 0: a product of independent
// Bernoulli draws is one Bernoulli draw of the product keep probability) plus one for the top
// layer's output.  A mask is a [T, B, K/8] byte tensor (time-major rows r = t*B + b, bit i of
// byte (r, j) = element (r, 8j + i)): 1/16 of a bf16 mask's bytes, regenerated per step from a
// counter-based hash of (seed, stream, element) so the backward pass and the tests see exactly
// the forward's draws.  Consumers: the persistent pair kernels (lstm2_persist.hip) read the
// bits of their fragments in-kernel; everything else goes through the apply kernels below.
#include "common.h"
#include "kernels.h"

namespace dcr {

constexpr int kDropThreads = 256;

// thread -> 32 consecutive elements (4 bytes, one dword store).  Each 64-bit hash yields four
// 16-bit uniforms (keep resolution 2^-16): 8 hashes per 32 elements.  One launch fills all the
// step's masks: segment m (nwords each, consecutive in memory) draws from its own stream with
// its own keep threshold, element indices local to the segment (the bits equal a launch per mask).
// With ``e.out``: the words of segment 0 (layer 0's input mask) also write their 32 masked
// embedding elements out[r, 32c .. 32c+31] = E[ids[r], ...] * (bit ? scale : 0) as bf16 -- the
// embed_dropout rows, bit for bit, without a second launch re-reading the bits.
__global__ void __launch_bounds__(kDropThreads) dropout_bits_kernel(unsigned* __restrict__ bits,
                                                                    DropSegs d, uint64_t seed,
                                                                    DropEmbed e) {
  const int64_t total = d.nwords * d.n;
  // (32-bit index math while it fits: a 64-bit division per word had cost more than its hashes)
  const bool small = total < ((int64_t)1 << 31);
  for (int64_t i = blockIdx.x * (int64_t)kDropThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kDropThreads) {
    const int m = small ? (int)((unsigned)i / (unsigned)d.nwords) : (int)(i / d.nwords);
    const int64_t li = i - (int64_t)m * d.nwords;
    const uint64_t key = seed ^ mix64(d.stream[m] * 0x632BE59BD9B4E019ull);
    const unsigned kt = d.kt[m];
    unsigned w = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint64_t r = mix64(key + (uint64_t)li * 8 + q);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        w |= ((unsigned)(r >> (16 * u)) & 0xFFFFu) < kt ? 1u << (4 * q + u) : 0u;
    }
    bits[i] = w;
    if (e.out && m == 0) {
      const int kw = e.K / 32;
      const int64_t r = small ? (int64_t)((unsigned)li / (unsigned)kw) : li / kw;
      const int c0 = 32 * (int)(li - r * kw);
      const float4* src = reinterpret_cast<const float4*>(e.E + (int64_t)e.ids[r] * e.K + c0);
      bf16x8* dst = reinterpret_cast<bf16x8*>(e.out + r * e.K + c0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 a = src[2 * q], b = src[2 * q + 1];
        const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = f2bf((w >> (8 * q + k) & 1u) ? v[k] * e.scale : 0.f);
        dst[q] = o;
      }
    }
  }
}

template <typename T> struct Vec8;
template <> struct Vec8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float (&v)[8]) {
    const bf16x8 x = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (float)x[e];
  }
  static __device__ __forceinline__ void store(bf16* p, const float (&v)[8]) {
    bf16x8 x;
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = f2bf(v[e]);
    *reinterpret_cast<bf16x8*>(p) = x;
  }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float (&v)[8]) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  static __device__ __forceinline__ void store(float* p, const float (&v)[8]) {
    reinterpret_cast<float4*>(p)[0] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
};

// out[r, k] = in[r, k] * (bit ? scale : 0), 8 consecutive k per thread (one mask byte, one
// 16/32-B vector each way).  In/out may alias (in place).  Row strides in elements (multiples
// of 8).
template <typename TI, typename TO>
__global__ void __launch_bounds__(kDropThreads) mask_apply_kernel(
    const TI* in, int64_t ld_in, TO* out, int64_t ld_out, const uint8_t* __restrict__ bits,
    int64_t rows, int K, float scale) {
  const int kb = K / 8;
  const int64_t n = rows * kb;
  for (int64_t i = blockIdx.x * (int64_t)kDropThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kDropThreads) {
    const int64_t r = i / kb;
    const int j = (int)(i - r * kb);
    const unsigned m = bits[i];
    float v[8];
    Vec8<TI>::load(in + r * ld_in + 8 * j, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (m >> e & 1u) ? v[e] * scale : 0.f;
    Vec8<TO>::store(out + r * ld_out + 8 * j, v);
  }
}

// out[r, k] = E[ids[r], k] * (bit ? scale : 0): the masked layer-0 input rows
__global__ void __launch_bounds__(kDropThreads) embed_dropout_kernel(
    const int* __restrict__ ids, const float* __restrict__ E, const uint8_t* __restrict__ bits,
    bf16* __restrict__ out, int64_t rows, int K, float scale) {
  const int kb = K / 8;
  const int64_t n = rows * kb;
  for (int64_t i = blockIdx.x * (int64_t)kDropThreads + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kDropThreads) {
    const int64_t r = i / kb;
    const int j = (int)(i - r * kb);
    const unsigned m = bits ? bits[i] : 0xFFu;
    const float4* src = reinterpret_cast<const float4*>(E + (int64_t)ids[r] * K + 8 * j);
    const float4 a = src[0], b = src[1];
    const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = f2bf((m >> e & 1u) ? v[e] * scale : 0.f);
    *reinterpret_cast<bf16x8*>(out + r * K + 8 * j) = o;
  }
}

static int drop_grid(int64_t n) {
  const int64_t b = (n + kDropThreads - 1) / kDropThreads;
  return (int)(b < 4096 ? (b > 0 ? b : 1) : 4096);
}

unsigned drop_threshold(float keep) {
  const double kt = (double)keep * 65536.0;
  return kt >= 65536.0 ? 65536u : (kt <= 0.0 ? 0u : (unsigned)(kt + 0.5));
}

void launch_dropout_bits(uint8_t* bits, const DropSegs& d, uint64_t seed, hipStream_t s,
                         const DropEmbed& e) {
  dropout_bits_kernel<<<drop_grid(d.nwords * d.n), kDropThreads, 0, s>>>(
      reinterpret_cast<unsigned*>(bits), d, seed, e);
}

void launch_mask_apply(const void* in, bool in_bf16, int64_t ld_in, void* out, bool out_bf16,
                       int64_t ld_out, const uint8_t* bits, int64_t rows, int K, float scale,
                       hipStream_t s) {
  const int g = drop_grid(rows * (K / 8));
  if (in_bf16 && out_bf16)
    mask_apply_kernel<bf16, bf16><<<g, kDropThreads, 0, s>>>(
        (const bf16*)in, ld_in, (bf16*)out, ld_out, bits, rows, K, scale);
  else if (in_bf16)
    mask_apply_kernel<bf16, float><<<g, kDropThreads, 0, s>>>(
        (const bf16*)in, ld_in, (float*)out, ld_out, bits, rows, K, scale);
  else if (out_bf16)
    mask_apply_kernel<float, bf16><<<g, kDropThreads, 0, s>>>(
        (const float*)in, ld_in, (bf16*)out, ld_out, bits, rows, K, scale);
  else
    mask_apply_kernel<float, float><<<g, kDropThreads, 0, s>>>(
        (const float*)in, ld_in, (float*)out, ld_out, bits, rows, K, scale);
}

void launch_embed_dropout(const int* ids, const float* E, const uint8_t* bits, bf16* out,
                          int64_t rows, int K, float scale, hipStream_t s) {
  embed_dropout_kernel<<<drop_grid(rows * (K / 8)), kDropThreads, 0, s>>>(ids, E, bits, out, rows,
                                                                          K, scale);
}

}  // namespace dcr
