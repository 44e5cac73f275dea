// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of distributed_char_rnn_amd.
//
// Everything here is written for 64-lane wavefronts and the gfx950 MFMA register maps
// (see /opt/skills/guides/cdna_hip_programming.md §3):
//   mfma_f32_32x32x16_bf16: lane l (r = l&31, h = l>>5) holds A[r][8h+j], B[8h+j][r] (j = 0..7);
//                          C/D: col = l&31, row = (reg&3) + 8*(reg>>2) + 4*h   (reg = 0..15)
//   mfma_f32_16x16x32_bf16: lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15];
//                          C/D: col = l&15, row = 4*(l>>4) + reg               (reg = 0..3)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dcr {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }  // RNE, v_cvt_pk_bf16_f32

__device__ __forceinline__ f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Activations.  __expf lowers to v_exp_f32 (base-2) with one multiply and the reciprocal to
// v_rcp_f32 (1 ulp): two instructions.  A plain `1.0f / y` is an IEEE division, a ~10-
// instruction v_div_scale / v_rcp / 4 x fma / v_div_fmas / v_div_fixup sequence: with 5
// activations per cell unit it made the LSTM epilogue the longest phase of a persistent
// kernel's tick (profiles/r2_pair_groups.md).  Both forms saturate cleanly: rcp(inf) = 0.
__device__ __forceinline__ float rcpf_(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float sigmoidf_(float x) { return rcpf_(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) {
  // tanh(x) = 1 - 2/(exp(2x)+1): saturates cleanly to +-1 for large |x|.
  return 1.0f - 2.0f * rcpf_(__expf(2.0f * x) + 1.0f);
}
__device__ __forceinline__ float reluf_(float x) { return x > 0.f ? x : 0.f; }

// Wave-level reductions (64 lanes).
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block reduction for a 1-D block of NT threads (NT multiple of 64). `red` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

// 16-byte load of 8 bf16 (caller guarantees 16-B alignment).
__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }
__device__ __forceinline__ bf16x8 zero8() {
  bf16x8 z;
#pragma unroll
  for (int i = 0; i < 8; ++i) z[i] = (bf16)0.0f;
  return z;
}

// Counter-based RNG (splitmix64-style finaliser over (seed, stream, counter)); used for
// dropout masks and on-device categorical sampling.  Deterministic for a given triple.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t stream, uint64_t ctr) {
  const uint64_t r = mix64(seed ^ mix64(stream * 0x632BE59BD9B4E019ull + ctr));
  return (float)(r >> 40) * (1.0f / 16777216.0f);  // [0,1) with 24 bits
}

}  // namespace dcr
