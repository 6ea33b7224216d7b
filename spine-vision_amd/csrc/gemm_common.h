// Shared pieces of the MFMA GEMM kernels (gemm.hip: register-staged v1 for the f32 parity mode and
// odd shapes; gemm2.hip: LDS-DMA pipelined v2 for bf16): epilogue arguments, the fused epilogue
// math and the LDS-staged wave-tile store.
#pragma once

#include "common.h"

namespace sv {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int EPI_LD = 64 + 4;  // f32 epilogue slab row stride (floats)

struct EpiArgs {
  int M, N;
  int epi;
  void* C; int c_dtype; int64_t ldc;
  void* C2; int c2_dtype;
  const float* bias;
  const float* gamma;
  const void* aux; int aux_dtype; int64_t ld_aux;
};

__device__ __forceinline__ float4 ld4_any(const void* p, int dt, size_t i) {
  return dt == SV_F32 ? ld4(reinterpret_cast<const float*>(p), i) : ld4(reinterpret_cast<const uint16_t*>(p), i);
}
__device__ __forceinline__ void st4_any(void* p, int dt, size_t i, float4 v) {
  if (dt == SV_F32) st4(reinterpret_cast<float*>(p), i, v);
  else st4(reinterpret_cast<uint16_t*>(p), i, v);
}

// apply the epilogue to 4 consecutive columns n..n+3 of row m
__device__ __forceinline__ void epi4(const EpiArgs& e, int m, int n, float4 v, int split) {
  if (e.epi == SV_EPI_SLAB) {
    float* C = reinterpret_cast<float*>(e.C) + (size_t)split * e.M * e.N;
    *reinterpret_cast<float4*>(C + (size_t)m * e.N + n) = v;
    return;
  }
  if (e.bias && e.epi != SV_EPI_GELU_GRAD) {
    const float4 b = *reinterpret_cast<const float4*>(e.bias + n);
    v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
  }
  const size_t ci = (size_t)m * e.ldc + n;
  if (e.epi == SV_EPI_STORE) {
    st4_any(e.C, e.c_dtype, ci, v);
  } else if (e.epi == SV_EPI_BIAS_GELU2) {
    st4_any(e.C, e.c_dtype, ci, v);
    st4_any(e.C2, e.c2_dtype, ci, make_float4(gelu_f(v.x), gelu_f(v.y), gelu_f(v.z), gelu_f(v.w)));
  } else if (e.epi == SV_EPI_BIAS_GAMMA_RES) {
    const float4 g = *reinterpret_cast<const float4*>(e.gamma + n);
    const float4 r = ld4_any(e.aux, e.aux_dtype, (size_t)m * e.ld_aux + n);
    st4_any(e.C, e.c_dtype, ci, make_float4(r.x + g.x * v.x, r.y + g.y * v.y, r.z + g.z * v.z, r.w + g.w * v.w));
  } else {  // SV_EPI_GELU_GRAD
    const float4 h = ld4_any(e.aux, e.aux_dtype, (size_t)m * e.ld_aux + n);
    st4_any(e.C, e.c_dtype, ci,
            make_float4(v.x * gelu_grad_f(h.x), v.y * gelu_grad_f(h.y), v.z * gelu_grad_f(h.z), v.w * gelu_grad_f(h.w)));
  }
}


// Store one wave's 64x64 accumulator (acc[i][j]: 16x16 MFMA fragments, C/D map col = lane&15,
// row = 4*(lane>>4) + r).  Each 16-row slab goes through the wave's private LDS region `slab`
// (16 x EPI_LD floats) and is re-read row-contiguous: lane -> (row = lane>>2, 16 columns), so every
// epilogue load/store is a 16-B vector access.
__device__ __forceinline__ void wave_tile_epilogue(const f32x4 (&acc)[4][4], float* __restrict__ slab, int mb,
                                                   int nb, const EpiArgs& e, int split) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[(4 * (l >> 4) + r) * EPI_LD + j * 16 + (l & 15)] = acc[i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const int row = l >> 2, cb = (l & 3) * 16;
    const int m = mb + i * 16 + row;
    if (m < e.M) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = nb + cb + 4 * g;
        if (n < e.N) {
          const float* sp = slab + row * EPI_LD + cb + 4 * g;
          epi4(e, m, n, make_float4(sp[0], sp[1], sp[2], sp[3]), split);
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
}

// v2 entry (gemm2.hip): returns SV_ERR_UNSUPPORTED when the shape/dtypes are outside its contract
int launch_gemm2(const sv_gemm_desc* d, hipStream_t s);

}  // namespace sv
