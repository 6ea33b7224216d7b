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

// ---- ISA-checked counted waits (tools/check_vmcnt.py, tests/test_vmcnt_isa.py) ----------------------------------
// A counted s_waitcnt vmcnt(N) retires a DMA only if at least N vector-memory instructions were issued after it, in
// the instruction stream the COMPILER emitted, on every path.  These markers let the checker verify that on the
// device assembly instead of trusting the source order:
//   SV_VMTAG("name")       after the last vector-memory instruction of a group a later counted wait must retire;
//   SV_VMWAIT(N, "name:k") s_waitcnt vmcnt(N) that must retire the k-th most recent instance of each listed group
//                          (k = 1: the latest; several "name:k" separated by spaces);
//   SV_VMCHECK("name:k")   asserts the same at that point without waiting.
// The asm statements clobber memory, so the compiler cannot move vector-memory instructions across them.
#define SV_VMTAG(t) asm volatile("; svtag " t ::: "memory")
#define SV_VMWAIT(n, t) asm volatile("s_waitcnt vmcnt(%0) ; svwait " t ::"n"(n) : "memory")
#define SV_VMCHECK(t) asm volatile("; svcheck " t ::: "memory")

namespace sv {

// ---- error plumbing (defined in abi.cpp) ---------------------------------------------
int set_error(int code, const char* fmt, ...);
int check_launch(const char* what);

// ---- per-device facts (abi.cpp): keyed by the device of the launch's stream, cached per device under a
// mutex -- no launch inherits another device's CU count, and the library is reentrant across devices ----
int stream_device(hipStream_t s);   // the device a stream belongs to (the null stream: the current device)
int device_cus(hipStream_t s);      // compute units of that device
int stream_cus(hipStream_t s);      // compute units a launch on that stream may use (its CU mask, if any)
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device) before its first launch there;
// SV_OK, or the failure reported through set_error (retried on the next launch: only a success is remembered)
int ensure_lds_attr(const void* kernel, int bytes, hipStream_t s);
// the grid of a persistent launch of `total` tiles under `pol` (nullable): one workgroup per tile, or
// wg_per_cu x CUs, then at most pol->grid_cap
int policy_grid(const sv_gemm_policy* pol, int total, int per_cu_default, hipStream_t s);

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
// two floats -> one bf16x2 word in ONE v_cvt_pk_bf16_f32 (RNE); the shift/or form costs three
__device__ __forceinline__ uint32_t pack2bf(float lo, float hi) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  const bf16x2_t v = __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t);
  return __builtin_bit_cast(uint32_t, v);
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
// Phi(x) = 1 - 0.5 erfc(|x|/sqrt2) (x >= 0), 0.5 erfc(|x|/sqrt2) (x < 0) with the Abramowitz-Stegun
// 7.1.26 erfc: t = 1/(1 + 0.3275911 z), erfc(z) = t (a1 + t (a2 + t (a3 + t (a4 + t a5)))) e^{-z^2},
// |error of erf| <= 1.5e-7.  With z = |x|/sqrt2, e^{-z^2} = sqrt(2 pi) * phi(x), phi the Gaussian
// density, so ONE v_exp_f32 gives both pieces:
//     phi(x)  = exp2(x^2 * (-log2(e)/2) + log2(1/sqrt(2 pi)))        (one fma + v_exp)
//     h       = 0.5 erfc(z) = t * P(t) * phi(x),  P = 0.5 sqrt(2 pi) (a1 + ... )  (coefficients folded)
//     Phi(x)  = 0.5 + copysign(0.5 - h, x)                          (v_sub + v_bfi + v_add)
//     GELU(x) = x Phi(x),   GELU'(x) = Phi(x) + x phi(x)            (v_mul, v_fma)
// = 2 transcendental + ~14 VALU per element for GELU and GELU' together; the fc1 epilogue evaluates
// them for every element of the 4C-wide hidden layer.
struct GeluParts {
  float phi, dens;  // Phi(x), phi(x)
};
__device__ __forceinline__ GeluParts gelu_parts(float x) {
  constexpr float K = 1.2533141373155003f;  // 0.5 * sqrt(2 pi)
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  const float dens = __builtin_amdgcn_exp2f(fmaf(x * x, -0.72134752044448170f, -1.3257480647361593f));
  float p = fmaf(1.061405429f * K, t, -1.453152027f * K);
  p = fmaf(p, t, 1.421413741f * K);
  p = fmaf(p, t, -0.284496736f * K);
  p = fmaf(p, t, 0.254829592f * K);
  const float h = (p * t) * dens;  // 0.5 erfc(|x|/sqrt2)
  return {0.5f + copysignf(0.5f - h, x), dens};
}
// two elements at once in packed f32 (v_pk_mul_f32 / v_pk_fma_f32 where the scalar form has one v_mul / v_fma):
// per component the same operations in the same order as gelu_parts, so the same bits
typedef float gelu_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void gelu_parts2(gelu_f2 x, gelu_f2& phi, gelu_f2& dens) {
  constexpr float K = 1.2533141373155003f;
  const gelu_f2 z = __builtin_elementwise_abs(x) * (gelu_f2){0.70710678118654752f, 0.70710678118654752f};
  const gelu_f2 d = __builtin_elementwise_fma((gelu_f2){0.3275911f, 0.3275911f}, z, (gelu_f2){1.0f, 1.0f});
  const gelu_f2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  const gelu_f2 ea = __builtin_elementwise_fma(x * x, (gelu_f2){-0.72134752044448170f, -0.72134752044448170f},
                                               (gelu_f2){-1.3257480647361593f, -1.3257480647361593f});
  dens = (gelu_f2){__builtin_amdgcn_exp2f(ea.x), __builtin_amdgcn_exp2f(ea.y)};
  gelu_f2 p = __builtin_elementwise_fma((gelu_f2){1.061405429f * K, 1.061405429f * K}, t,
                                        (gelu_f2){-1.453152027f * K, -1.453152027f * K});
  p = __builtin_elementwise_fma(p, t, (gelu_f2){1.421413741f * K, 1.421413741f * K});
  p = __builtin_elementwise_fma(p, t, (gelu_f2){-0.284496736f * K, -0.284496736f * K});
  p = __builtin_elementwise_fma(p, t, (gelu_f2){0.254829592f * K, 0.254829592f * K});
  const gelu_f2 h = (p * t) * dens;
  const gelu_f2 r = (gelu_f2){0.5f, 0.5f} - h;
  phi = (gelu_f2){0.5f, 0.5f} + (gelu_f2){copysignf(r.x, x.x), copysignf(r.y, x.y)};
}
__device__ __forceinline__ float phi_cdf(float x) { return gelu_parts(x).phi; }
__device__ __forceinline__ float gelu_f(float x) { return x * gelu_parts(x).phi; }
// GELU and its derivative from one evaluation (forward epilogue of fc1)
__device__ __forceinline__ void gelu_and_grad(float x, float& g, float& dg) {
  const GeluParts q = gelu_parts(x);
  g = x * q.phi;
  dg = fmaf(x, q.dens, q.phi);
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  const GeluParts q = gelu_parts(x);
  return fmaf(x, q.dens, q.phi);
}


// SV_PERMLANE_NOP=n (A/B builds, round 6): n wait states between a v_permlane16/32_swap and the VALU read of its two
// results (an s_nop the compiler cannot schedule around: the results pass through it).  Tests whether a
// permlane-swap-write -> VALU-read hazard is left uncovered by the compiler's hazard recognizer.
#ifndef SV_PERMLANE_NOP
#define SV_PERMLANE_NOP 0
#endif
__device__ __forceinline__ void permlane_guard(uint32_t& a, uint32_t& b) {
#if SV_PERMLANE_NOP
  asm volatile("s_nop %2" : "+v"(a), "+v"(b) : "n"(SV_PERMLANE_NOP - 1));
#else
  (void)a, (void)b;
#endif
}

// xor-butterfly sum over groups of LPR lanes (16, 32 or 64) in __shfl_xor order (partner distance LPR/2 first, then
// halving), the partners taken from the cross-lane unit instead of ds_bpermute round trips: permlane32 / permlane16
// swaps for the exact xor-32 / xor-16 partners, DPP row rotation by 8 (xor 8 inside a 16-lane row), rotations by 4 and
// 2 (they deliver a lane whose value equals the xor partner's: the earlier steps made lanes i, i^8 and then i^4 equal)
// and a quad permutation (xor 1).  Every lane of a group ends with the same sum, bitwise the shuffle butterfly's.
template <int LPR>
__device__ __forceinline__ float xlane_group_sum(float v) {
  static_assert(LPR == 16 || LPR == 32 || LPR == 64, "row-rotation steps need groups of >= 16 lanes");
  const int lane = threadIdx.x & 63;
  if constexpr (LPR >= 64) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    uint32_t r0 = r[0], r1 = r[1];
    permlane_guard(r0, r1);
    v += __uint_as_float(lane < 32 ? r1 : r0);
  }
  if constexpr (LPR >= 32) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    uint32_t r0 = r[0], r1 = r[1];
    permlane_guard(r0, r1);
    v += __uint_as_float((lane & 16) ? r0 : r1);
  }
  v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), 0x128, 0xf, 0xf, false));  // row_ror:8
  v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), 0x124, 0xf, 0xf, false));  // row_ror:4
  v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), 0x122, 0xf, 0xf, false));  // row_ror:2
  v += __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), 0xb1, 0xf, 0xf, false));   // quad [1,0,3,2]
  return v;
}

// the value of lane l ^ OFF, from the cross-lane unit: OFF 1 / 2 = quad permutations, 8 = DPP row rotation by 8 (xor 8
// inside a 16-lane row), 16 / 32 = permlane16 / permlane32 swaps -- each the exact xor partner.  OFF 4 has no single
// DPP form: xlane_xor<4, true> uses the half-row mirror, whose source lane holds the partner's value only where the
// quads are uniform (after xor 1 and xor 2 steps of an ascending butterfly).
template <int OFF, bool QUADS_UNIFORM = false>
__device__ __forceinline__ float xlane_xor(float v) {
  const uint32_t u = __float_as_uint(v);
  if constexpr (OFF == 1) return __uint_as_float(__builtin_amdgcn_update_dpp(0u, u, 0xb1, 0xf, 0xf, false));
  else if constexpr (OFF == 2) return __uint_as_float(__builtin_amdgcn_update_dpp(0u, u, 0x4e, 0xf, 0xf, false));
  else if constexpr (OFF == 4) {
    static_assert(QUADS_UNIFORM, "xor 4 via the half-row mirror needs uniform quads");
    return __uint_as_float(__builtin_amdgcn_update_dpp(0u, u, 0x141, 0xf, 0xf, false));
  } else if constexpr (OFF == 8) return __uint_as_float(__builtin_amdgcn_update_dpp(0u, u, 0x128, 0xf, 0xf, false));
  else if constexpr (OFF == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    uint32_t r0 = r[0], r1 = r[1];
    permlane_guard(r0, r1);
    return __uint_as_float((threadIdx.x & 16) ? r0 : r1);
  } else {
    static_assert(OFF == 32, "xor distance 1, 2, 4, 8, 16 or 32");
    const auto r = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    uint32_t r0 = r[0], r1 = r[1];
    permlane_guard(r0, r1);
    return __uint_as_float((threadIdx.x & 32) ? r0 : r1);
  }
}

// ---- wave / block reductions (wave64) -------------------------------------------------
// the xor butterflies take their partners from the cross-lane unit (above) instead of ds_bpermute; bitwise the same
// sums.  -DSV_XLANE=0 builds the shuffle forms everywhere (A/B builds)
#ifndef SV_XLANE
#define SV_XLANE 1
#endif
__device__ __forceinline__ float wave_sum(float v) {
#if SV_XLANE
  return xlane_group_sum<64>(v);
#else
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
#endif
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
