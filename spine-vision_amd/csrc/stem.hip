// ConvNeXt stem on MFMA (bf16 mode) and the batch input transform on the GPU.
//
// timm's stem Conv2d(3, C, k=4, s=4) (reached through spine_vision/training/models/backbone.py:166)
// is a GEMM over non-overlapping 4x4 patches: z[p][c] = b[c] + sum_k patch[p][k] * w[c][k] with
// k = ci*16 + kh*4 + kw (= stem.0.weight [C,3,4,4] flattened).  The gather below writes the
// patches as bf16 rows of 64 (k 48..63 zero, one 128-B line per pixel), so the conv is one sv_gemm
// with K = 64 on the v3 MFMA kernel and its weight gradient one split-K wgrad GEMM (N = 48 columns
// of the same patch rows).  The LayerNorm2d after it runs as sv_layernorm_fwd/bwd.
//
// Input kinds (what the drop-in boundary hands the backbone):
//   SV_IMG_F32_NCHW  the reference batch["image"]: [B,3,H,W] f32, already ImageNet-normalised by
//                    the dataset transform (training/datasets/localization.py:196-233);
//   SV_IMG_U8_GRAY   the decoded uint8 grayscale batch [B,H,W]: the transform's ToTensor (/255),
//                    gray->RGB replication (Image.convert("RGB"), localization.py:254) and
//                    Normalize(mean[c], std[c]) are applied in flight, with the same f32 operations
//                    as torchvision ((x / 255 - mean) / std), so both kinds give identical patches.
//
// HBM: the gather reads the image once (f32: 192 B, u8: 16 B per output pixel) and writes one 128-B
// row per output pixel; a thread owns one 16-B chunk (8 k) of one pixel, so a wave writes eight whole
// 128-B rows.  The normalisation constants are HOST arrays of 3 floats (passed by value to the kernel).
#include "common.h"

namespace sv {

constexpr int kStemGatherThreads = 256;

__device__ __forceinline__ float norm_u8(uint32_t u, float mean, float std_) {
  return ((float)u / 255.0f - mean) / std_;
}

template <int KIND>
__global__ void __launch_bounds__(kStemGatherThreads) stem_patchify_kernel(
    const void* __restrict__ img, float m0, float m1, float m2, float s0, float s1, float s2,
    uint16_t* __restrict__ patches, int B, int H, int W) {
  const int Ho = H >> 2, Wo = W >> 2;
  const int64_t total = (int64_t)B * Ho * Wo * 8;
  for (int64_t t = (int64_t)blockIdx.x * kStemGatherThreads + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * kStemGatherThreads) {
    const int chunk = (int)(t & 7);
    const int64_t p = t >> 3;
    uint4 out = make_uint4(0u, 0u, 0u, 0u);
    if (chunk < 6) {
      const int j = (int)(p % Wo), i = (int)((p / Wo) % Ho), b = (int)(p / ((int64_t)Wo * Ho));
      const int ci = chunk >> 1, kh0 = (chunk & 1) * 2;
      float v[8];
      if constexpr (KIND == SV_IMG_F32_NCHW) {
        const float* base = reinterpret_cast<const float*>(img) + (((size_t)b * 3 + ci) * H + 4 * i + kh0) * W + 4 * j;
        const float4 r0 = *reinterpret_cast<const float4*>(base);
        const float4 r1 = *reinterpret_cast<const float4*>(base + W);
        v[0] = r0.x; v[1] = r0.y; v[2] = r0.z; v[3] = r0.w;
        v[4] = r1.x; v[5] = r1.y; v[6] = r1.z; v[7] = r1.w;
      } else {
        const uint8_t* base = reinterpret_cast<const uint8_t*>(img) + ((size_t)b * H + 4 * i + kh0) * W + 4 * j;
        const uint32_t r0 = *reinterpret_cast<const uint32_t*>(base);
        const uint32_t r1 = *reinterpret_cast<const uint32_t*>(base + W);
        const float mean = ci == 0 ? m0 : (ci == 1 ? m1 : m2);
        const float sd = ci == 0 ? s0 : (ci == 1 ? s1 : s2);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          v[q] = norm_u8((r0 >> (8 * q)) & 0xffu, mean, sd);
          v[4 + q] = norm_u8((r1 >> (8 * q)) & 0xffu, mean, sd);
        }
      }
      out = make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
    }
    *reinterpret_cast<uint4*>(patches + (size_t)p * 64 + chunk * 8) = out;
  }
}

__global__ void __launch_bounds__(256) stem_weight_pack_kernel(const float* __restrict__ w,
                                                               uint16_t* __restrict__ wp, int C) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= C * 64) return;
  const int c = i >> 6, k = i & 63;
  wp[i] = k < 48 ? f2bf(w[(size_t)c * 48 + k]) : (uint16_t)0;
}

// reference transform of a decoded grayscale batch: out[b][c][h][w] = (u / 255 - mean[c]) / std[c]
__global__ void __launch_bounds__(256) normalize_u8_gray_kernel(const uint8_t* __restrict__ img, float m0, float m1,
                                                                float m2, float s0, float s1, float s2,
                                                                float* __restrict__ out, int64_t HW, int B) {
  const int64_t n4 = (int64_t)B * HW / 4;  // HW % 4 == 0
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < n4; t += (int64_t)gridDim.x * 256) {
    const int64_t e = t * 4;
    const int64_t b = e / HW, r = e - b * HW;
    const uint32_t u = *reinterpret_cast<const uint32_t*>(img + e);
    float* o = out + (size_t)b * 3 * HW + r;
    const float ms[3] = {m0, m1, m2}, ss[3] = {s0, s1, s2};
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      *reinterpret_cast<float4*>(o + (size_t)c * HW) =
          make_float4(norm_u8(u & 0xffu, ms[c], ss[c]), norm_u8((u >> 8) & 0xffu, ms[c], ss[c]),
                      norm_u8((u >> 16) & 0xffu, ms[c], ss[c]), norm_u8(u >> 24, ms[c], ss[c]));
    }
  }
}

static int grid_for(int64_t work, int threads) {
  const int64_t g = (work + threads - 1) / threads;
  return (int)(g < 65536 ? (g > 0 ? g : 1) : 65536);
}

}  // namespace sv

using namespace sv;

extern "C" {

int sv_stem_patchify(const void* img, int32_t img_kind, const float* norm_mean, const float* norm_std,
                     uint16_t* patches, int32_t B, int32_t H, int32_t W, sv_stream_t stream) {
  SV_REQUIRE(img && patches, "sv_stem_patchify: null pointer");
  SV_REQUIRE(B > 0 && H > 0 && W > 0 && H % 4 == 0 && W % 4 == 0, "sv_stem_patchify: H, W must be multiples of 4");
  SV_REQUIRE(((uintptr_t)patches & 15) == 0, "sv_stem_patchify: patches must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for((int64_t)B * (H / 4) * (W / 4) * 8, kStemGatherThreads);
  if (img_kind == SV_IMG_F32_NCHW) {
    SV_REQUIRE(((uintptr_t)img & 15) == 0, "sv_stem_patchify: f32 image must be 16-byte aligned");
    stem_patchify_kernel<SV_IMG_F32_NCHW><<<grid, kStemGatherThreads, 0, s>>>(img, 0.f, 0.f, 0.f, 1.f, 1.f, 1.f,
                                                                              patches, B, H, W);
  } else if (img_kind == SV_IMG_U8_GRAY) {
    SV_REQUIRE(norm_mean && norm_std, "sv_stem_patchify: u8 input needs the normalisation constants");
    SV_REQUIRE(((uintptr_t)img & 3) == 0, "sv_stem_patchify: u8 image must be 4-byte aligned");
    stem_patchify_kernel<SV_IMG_U8_GRAY><<<grid, kStemGatherThreads, 0, s>>>(
        img, norm_mean[0], norm_mean[1], norm_mean[2], norm_std[0], norm_std[1], norm_std[2], patches, B, H, W);
  } else {
    return set_error(SV_ERR_INVALID_ARG, "sv_stem_patchify: bad image kind %d", img_kind);
  }
  return check_launch("sv_stem_patchify");
}

int sv_stem_weight_pack(const float* w, uint16_t* wpack, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(w && wpack && C > 0, "sv_stem_weight_pack: bad args");
  stem_weight_pack_kernel<<<ceil_div((int64_t)C * 64, 256), 256, 0, (hipStream_t)stream>>>(w, wpack, C);
  return check_launch("sv_stem_weight_pack");
}

int sv_normalize_u8_gray(const uint8_t* img, const float* norm_mean, const float* norm_std, float* out, int32_t B,
                         int32_t H, int32_t W, sv_stream_t stream) {
  SV_REQUIRE(img && norm_mean && norm_std && out, "sv_normalize_u8_gray: null pointer");
  SV_REQUIRE(B > 0 && H > 0 && W > 0 && ((int64_t)H * W) % 4 == 0, "sv_normalize_u8_gray: H*W must be a multiple of 4");
  SV_REQUIRE(((uintptr_t)img & 3) == 0 && ((uintptr_t)out & 15) == 0, "sv_normalize_u8_gray: misaligned buffers");
  const int64_t HW = (int64_t)H * W;
  normalize_u8_gray_kernel<<<grid_for((int64_t)B * HW / 4, 256), 256, 0, (hipStream_t)stream>>>(
      img, norm_mean[0], norm_mean[1], norm_mean[2], norm_std[0], norm_std[1], norm_std[2], out, HW, B);
  return check_launch("sv_normalize_u8_gray");
}

}  // extern "C"
