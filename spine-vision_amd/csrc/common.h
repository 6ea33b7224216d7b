// Shared device/host helpers for the spine-vision MI355X (gfx950) kernel library.
//
// Conventions (see include/sv_kernels.h):
//  * activations are NHWC, i.e. a 2-D [rows = B*H*W][C] matrix with C contiguous;
//  * bf16 travels as uint16_t bit patterns (round-to-nearest-even on store);
//  * every entry point is asynchronous on the caller's hipStream_t and returns an sv_status.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include "../../include/sv_kernels.h"

namespace sv {

// ---- error plumbing (defined in abi.cpp) ---------------------------------------------
int set_error(int code, const char* fmt, ...);
int check_launch(const char* what);

#define SV_REQUIRE(cond, ...)                                                       \
  do {                                                                              \
    if (!(cond)) return ::sv::set_error(SV_ERR_INVALID_ARG, __VA_ARGS__);           \
  } while (0)

// ---- bf16 <-> f32 -------------------------------------------------------------------
__device__ __forceinline__ float bf2f(uint16_t u) { return __uint_as_float((uint32_t)u << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // lowers to v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  return __builtin_bit_cast(uint16_t, b);
}
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// typed element load/store used by dtype-generic kernels (T = float or uint16_t=bf16)
template <typename T> __device__ __forceinline__ float ld(const T* p, size_t i);
template <> __device__ __forceinline__ float ld<float>(const float* p, size_t i) { return p[i]; }
template <> __device__ __forceinline__ float ld<uint16_t>(const uint16_t* p, size_t i) { return bf2f(p[i]); }
template <typename T> __device__ __forceinline__ void st(T* p, size_t i, float v);
template <> __device__ __forceinline__ void st<float>(float* p, size_t i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void st<uint16_t>(uint16_t* p, size_t i, float v) { p[i] = f2bf(v); }

// load/store 4 consecutive elements (caller guarantees alignment of 4 elements)
template <typename T> __device__ __forceinline__ float4 ld4(const T* p, size_t i);
template <> __device__ __forceinline__ float4 ld4<float>(const float* p, size_t i) {
  return *reinterpret_cast<const float4*>(p + i);
}
template <> __device__ __forceinline__ float4 ld4<uint16_t>(const uint16_t* p, size_t i) {
  uint2 u = *reinterpret_cast<const uint2*>(p + i);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                     __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
}
template <typename T> __device__ __forceinline__ void st4(T* p, size_t i, float4 v);
template <> __device__ __forceinline__ void st4<float>(float* p, size_t i, float4 v) {
  *reinterpret_cast<float4*>(p + i) = v;
}
template <> __device__ __forceinline__ void st4<uint16_t>(uint16_t* p, size_t i, float4 v) {
  *reinterpret_cast<uint2*>(p + i) = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
}

// ---- GELU (erf form, = torch.nn.GELU() default) -----------------------------------------
// Phi(x) = 0.5*erfc(-x/sqrt2) with the branch-free Chebyshev-fitted erfc of Numerical Recipes
// (erfcc, |relative error| < 1.2e-7 everywhere): one v_exp, one v_rcp and ten FMAs, no divergent
// ranges -- the GELU epilogues of the fc1/fc2 GEMMs run it on every element.
__device__ __forceinline__ float phi_cdf(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __frcp_rn(1.0f + 0.5f * z);
  float p = 0.17087277f;
  p = fmaf(p, t, -0.82215223f);
  p = fmaf(p, t, 1.48851587f);
  p = fmaf(p, t, -1.13520398f);
  p = fmaf(p, t, 0.27886807f);
  p = fmaf(p, t, -0.18628806f);
  p = fmaf(p, t, 0.09678418f);
  p = fmaf(p, t, 0.37409196f);
  p = fmaf(p, t, 1.00002368f);
  p = fmaf(p, t, -1.26551223f);
  const float r = t * __expf(fmaf(-z, z, p));  // erfc(|x|/sqrt2)
  return x >= 0.f ? fmaf(-0.5f, r, 1.0f) : 0.5f * r;
}
__device__ __forceinline__ float gelu_f(float x) { return x * phi_cdf(x); }
// GELU and its derivative from one Phi evaluation (forward epilogue of fc1)
__device__ __forceinline__ void gelu_and_grad(float x, float& g, float& dg) {
  const float c = phi_cdf(x);
  g = x * c;
  dg = c + x * (0.39894228040143268f * __expf(-0.5f * x * x));
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  // d/dx [x * Phi(x)] = Phi(x) + x * phi(x)
  return phi_cdf(x) + x * (0.39894228040143268f * __expf(-0.5f * x * x));
}

// ---- wave / block reductions (wave64) -------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum; `red` must hold >= blockDim.x/64 floats; all threads get the result
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

}  // namespace sv
