// Resize of decoded uint8 images on the device (row f1): the reference's first transform,
// torchvision Resize(size) on a PIL image (spine_vision/training/datasets/localization.py:199 and
// classification.py:250) = Image.resize((W, H), BILINEAR) = Pillow's libImaging/Resample.c:
//   * per axis, precompute_coeffs: support = filterscale = max(in/out, 1) (antialiasing when shrinking),
//     taps [xmin, xmin + count) around center = (x + 0.5) * in/out, triangle weights normalised to sum 1,
//     then normalize_coeffs_8bpc: int32 fixed point with PRECISION_BITS = 22 (round half away from 0);
//     these tables are computed on the host in double exactly as Pillow does
//     (training/datasets/resize.py) and passed in;
//   * ImagingResampleHorizontal_8bpc then ImagingResampleVertical_8bpc: ss = 1 << 21 + sum(pixel * k),
//     clip8(ss >> 22) -- the horizontal pass rounds to uint8 before the vertical pass reads it.
// One thread per output pixel (all C channels) recomputes the horizontal results of its vertical taps:
// the same integers in the same order as Pillow's two passes, so the output is bit-identical.
// Ragged batch: desc[b] = {src byte offset, h, w, x-table offset, x taps, y-table offset, y taps, 0}
// (int64); a table at offset o holds bounds[out][2] = {first tap, count} followed by coef[out][taps]
// (int32).  Source [h][w][C], output [B][H][W][C] uint8, C = 1 or 3.
#include "common.h"

namespace sv {
namespace {

constexpr int RS_THREADS = 256;
constexpr int RS_PREC = 22;

__device__ __forceinline__ int clip8(int ss) {
  const int v = ss >> RS_PREC;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

template <int C>
__global__ void __launch_bounds__(RS_THREADS) resize_u8_kernel(const uint8_t* __restrict__ src,
                                                               const int64_t* __restrict__ desc,
                                                               const int32_t* __restrict__ coef,
                                                               uint8_t* __restrict__ dst, int H, int W) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * RS_THREADS + threadIdx.x;
  if (p >= H * W) return;
  const int y = p / W, x = p - y * W;
  const int64_t* d = desc + (size_t)b * 8;
  const uint8_t* img = src + d[0];
  const int w = (int)d[2];
  const int32_t* xt = coef + d[3];
  const int kxs = (int)d[4];
  const int32_t* yt = coef + d[5];
  const int kys = (int)d[6];
  const int xmin = xt[2 * x], xcnt = xt[2 * x + 1];
  const int32_t* kx = xt + 2 * W + (size_t)x * kxs;
  const int ymin = yt[2 * y], ycnt = yt[2 * y + 1];
  const int32_t* ky = yt + 2 * H + (size_t)y * kys;
  int sv[C];
#pragma unroll
  for (int c = 0; c < C; ++c) sv[c] = 1 << (RS_PREC - 1);
  for (int j = 0; j < ycnt; ++j) {
    const uint8_t* row = img + ((size_t)(ymin + j) * w + xmin) * C;
    int sh[C];
#pragma unroll
    for (int c = 0; c < C; ++c) sh[c] = 1 << (RS_PREC - 1);
    for (int i = 0; i < xcnt; ++i) {
      const int k = kx[i];
#pragma unroll
      for (int c = 0; c < C; ++c) sh[c] += (int)row[i * C + c] * k;
    }
    const int k = ky[j];
#pragma unroll
    for (int c = 0; c < C; ++c) sv[c] += clip8(sh[c]) * k;
  }
  uint8_t* o = dst + (((size_t)b * H + y) * W + x) * C;
#pragma unroll
  for (int c = 0; c < C; ++c) o[c] = (uint8_t)clip8(sv[c]);
}

}  // namespace

extern "C" int sv_resize_u8(const uint8_t* src, const int64_t* desc, const int32_t* coef, int32_t B, int32_t H,
                            int32_t W, int32_t C, uint8_t* dst, hipStream_t stream) {
  SV_REQUIRE(src && desc && coef && dst && B > 0 && H > 0 && W > 0, "sv_resize_u8: null pointer or empty shape");
  SV_REQUIRE(C == 1 || C == 3, "sv_resize_u8: C must be 1 or 3");
  SV_REQUIRE((int64_t)H * W < (1 << 30), "sv_resize_u8: output too large");
  const dim3 grid((unsigned)ceil_div(H * W, RS_THREADS), (unsigned)B);
  if (C == 1) resize_u8_kernel<1><<<grid, RS_THREADS, 0, stream>>>(src, desc, coef, dst, H, W);
  else resize_u8_kernel<3><<<grid, RS_THREADS, 0, stream>>>(src, desc, coef, dst, H, W);
  return check_launch("sv_resize_u8");
}

}  // namespace sv
