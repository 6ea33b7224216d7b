// v1 (register-staged) MFMA tile geometry and fragment readers shared by gemm.hip and conv.hip:
// 128x128 output tile per 256-thread workgroup (4 waves in 2x2, 64x64 per wave), BK = 32, padded
// LDS images; bf16 fragments for v_mfma_f32_16x16x32_bf16, f32 fragments for v_mfma_f32_16x16x4f32.
#pragma once

#include "gemm_common.h"

namespace sv {

constexpr int BM = 128, BN = 128, BKT = 32;
constexpr int kGemmThreads = 256;

// ---------------------------------------------------------------------------------------------
// LDS images.  bf16 compute: k-major [R][BKT+8] (80 B rows), m-major [BKT][R+16] (288 B rows).
//               f32 compute:  k-major [R][BKT+4] (144 B rows), m-major [BKT][R+4] (528 B rows).
template <bool BF16, bool KMAJ>
struct Img {
  static constexpr int LD = BF16 ? (KMAJ ? BKT + 8 : BM + 16) : (KMAJ ? BKT + 4 : BM + 4);
  static constexpr int ROWS = KMAJ ? BM : BKT;
  static constexpr int BYTES = ROWS * LD * (BF16 ? 2 : 4);
};


// bf16 fragment for v_mfma_f32_16x16x32_bf16: lane l holds X[row = base + (l&15)][k = 8(l>>4)+j].
template <bool KMAJ>
__device__ __forceinline__ bf16x8 frag_bf16(const char* __restrict__ img, int base) {
  const int l = threadIdx.x & 63;
  if (KMAJ) {
    constexpr int LD = Img<true, true>::LD;
    return *reinterpret_cast<const bf16x8*>(img + ((size_t)(base + (l & 15)) * LD + 8 * (l >> 4)) * 2);
  } else {
    // [k][row] image: two ds_read_b64_tr_b16, k rows 8g..8g+3 and 8g+4..8g+7 (g = l>>4);
    // lane 4q+p of each 16-lane group addresses row q, columns 4p..4p+3 of the 4x16 block.
    constexpr int LD = Img<true, false>::LD;
    const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
    typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
    const char* a0 = img + ((size_t)(8 * g + q) * LD + base + 4 * p) * 2;
    const char* a1 = a0 + (size_t)4 * LD * 2;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// f32 fragment for v_mfma_f32_16x16x4_f32: lane l holds X[row = base + (l&15)][k = kk + (l>>4)].
template <bool KMAJ>
__device__ __forceinline__ float frag_f32(const char* __restrict__ img, int base, int kk) {
  const int l = threadIdx.x & 63;
  constexpr int LD = Img<false, KMAJ>::LD;
  const float* f = reinterpret_cast<const float*>(img);
  return KMAJ ? f[(size_t)(base + (l & 15)) * LD + kk + (l >> 4)] : f[(size_t)(kk + (l >> 4)) * LD + base + (l & 15)];
}


}  // namespace sv
