// kml_common.h — shared device/host helpers for the kubeml_amd HIP kernels.
//
// Target: gfx950 (MI355X, CDNA4) only.  Wave64 everywhere; bf16 is handled as raw
// 16-bit payloads (ushort) with explicit round-to-nearest-even conversion so that
// every kernel controls its own vector widths (16 B per lane on the hot loads).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define KML_API extern "C" __attribute__((visibility("default")))

#define KML_WAVE 64

typedef unsigned short bf16_t;  // raw bf16 bits

typedef __attribute__((ext_vector_type(8))) short bf16x8_t;   // MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4_t;    // 16x16 MFMA accumulator
typedef __attribute__((ext_vector_type(16))) float f32x16_t;  // 32x32 MFMA accumulator

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((unsigned)v) << 16);
}


// two floats -> packed bf16 pair with gfx950's v_cvt_pk_bf16_f32 (round-to-nearest-even,
// NaN stays NaN): one VALU instruction instead of two software roundings
typedef __bf16 kml_bf16x2_hw __attribute__((ext_vector_type(2)));
typedef float kml_f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack_bf2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((kml_f32x2_t{a, b}), kml_bf16x2_hw));
}
// round-to-nearest-even; NaN stays NaN
__device__ __forceinline__ bf16_t f2bf(float f) { return (bf16_t)(pack_bf2(f, 0.f) & 0xffffu); }

__device__ __forceinline__ float lo_bf(unsigned w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_bf(unsigned w) { return __uint_as_float(w & 0xffff0000u); }

// erf for the GELU epilogues: Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, far below the
// bf16 output resolution) — one rcp, five FMAs, one v_exp_f32, instead of the device
// library's branchy ~30-instruction erff
__device__ __forceinline__ float kml_erf(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
  float y = fmaf(fmaf(fmaf(fmaf(1.061405429f, t, -1.453152027f), t, 1.421413741f), t, -0.284496736f), t,
                 0.254829592f) * t;
  y = 1.f - y * __builtin_amdgcn_exp2f(-ax * ax * 1.4426950408889634f);
  return copysignf(y, x);
}
__device__ __forceinline__ float kml_gelu(float x) { return 0.5f * x * (1.f + kml_erf(x * 0.70710678118654752f)); }
__device__ __forceinline__ float kml_gelu_grad(float x) {
  return 0.5f * (1.f + kml_erf(x * 0.70710678118654752f)) +
         x * 0.3989422804014327f * __builtin_amdgcn_exp2f(-0.5f * 1.4426950408889634f * x * x);
}

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

// grid sizing for streaming kernels: cap at 256 CUs x 8 blocks, grid-stride the rest
static inline unsigned kml_stream_grid(long long n_items, int block) {
  long long g = (n_items + block - 1) / block;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (unsigned)g;
}

#define KML_LAUNCH_CHECK() return (int)hipGetLastError()
