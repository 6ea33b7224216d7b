// Train-time augmentation of decoded uint8 images on the device (row f1): the reference's torchvision
// chain after Resize (spine_vision/training/datasets/localization.py:202-216 and
// classification.py:276-289):
//     RandomHorizontalFlip(0.5) -> RandomAffine(10 deg, translate 5%, scale 0.95-1.05, NEAREST, fill 0)
//     -> ColorJitter(brightness 0.2, contrast 0.2, random order)
// applied by torchvision to PIL images, i.e. by Pillow's C code.  The random parameters are drawn on
// the host exactly as torchvision draws them (training/datasets/augment.py); these kernels restate the
// PIL arithmetic bit for bit:
//   * affine (Pillow Geometry.c ImagingTransformAffine, NEAREST): when the inverse matrix has no
//     off-diagonal terms, ImagingScaleAffine's incremental DOUBLE walk (xo = a2 + a0/2, xo += a0);
//     otherwise 16.16 fixed point (FIX(v) = floor(v*65536 + 0.5); origin FIX(a2 + a0/2 + a1/2) and
//     steps FIX(a0), FIX(a1), ...: source = xx >> 16) -- or, if a corner leaves the fixed-point
//     range, the incremental double walk of the generic path; samples outside the image are the
//     fill (0);
//   * brightness / contrast (ImageEnhance = Image.blend(degenerate, img, f)): t = d + f*(v - d) in
//     float32 with separately rounded multiply and add (no FMA contraction), truncated, clipped when
//     f > 1; the contrast degenerate is int(mean(L) + 0.5) with L = (R*19595 + G*38470 + B*7471 +
//     0x8000) >> 16 for RGB (Pillow's convert("L")), the plane itself for one channel.
// Layout: [B][H][W][C] uint8, C = 1 (grayscale plane) or 3 (interleaved RGB).
// params: double [B][10] = {flip, a0..a5 (inverse affine, torchvision _get_inverse_affine_matrix),
// brightness, contrast, order (0: brightness first, 1: contrast first)}.
#include "common.h"

namespace sv {
namespace {

constexpr int AUG_THREADS = 256;

__device__ __forceinline__ int coord_pil(double v) { return v < 0.0 ? -1 : (int)v; }
__device__ __forceinline__ int fix16(double v) { return (int)floor(v * 65536.0 + 0.5); }

__device__ __forceinline__ uint8_t blend_u8(int d, int v, float f) {
  // Pillow Blend.c: (int)in1 + alpha * ((int)in2 - (int)in1) in float, truncated (clipped when alpha > 1)
  const float t = __fadd_rn((float)d, __fmul_rn(f, (float)(v - d)));
  if (f >= 0.f && f <= 1.f) return (uint8_t)t;
  if (t <= 0.f) return 0;
  if (t >= 255.f) return 255;
  return (uint8_t)t;
}

__device__ __forceinline__ int luma(const uint8_t* p, int C) {
  if (C == 1) return p[0];
  return (p[0] * 19595 + p[1] * 38470 + p[2] * 7471 + 0x8000) >> 16;
}

// per output row: flip + affine (+ brightness when it comes first), and the row's luma sum
__global__ void __launch_bounds__(AUG_THREADS) augment_affine_kernel(const uint8_t* __restrict__ in,
                                                                     uint8_t* __restrict__ out, int H, int W, int C,
                                                                     const double* __restrict__ params,
                                                                     int* __restrict__ row_sums) {
  const int y = blockIdx.x, b = blockIdx.y;
  const double* prm = params + (size_t)b * 10;
  const bool flip = prm[0] != 0.0;
  const double a0 = prm[1], a1 = prm[2], a2 = prm[3], a3 = prm[4], a4 = prm[5], a5 = prm[6];
  const float bright = (float)prm[7];
  const bool bright_first = prm[9] == 0.0;
  const uint8_t* src = in + (size_t)b * H * W * C;
  uint8_t* dst = out + (size_t)b * H * W * C + (size_t)y * W * C;
  // which Pillow path (decided exactly as ImagingTransformAffine does)
  const bool scale_path = a1 == 0.0 && a3 == 0.0;
  auto in_fixed = [&](double x, double yy) {
    return fabs(a0 * x + a1 * yy + a2) < 32768.0 && fabs(a3 * x + a4 * yy + a5) < 32768.0;
  };
  const bool fixed = !scale_path && in_fixed(0, 0) && in_fixed(W, H) && in_fixed(0, H) && in_fixed(W, 0);
  int sum = 0;
  for (int x = threadIdx.x; x < W; x += AUG_THREADS) {
    int xi, yi;
    if (fixed) {
      // Pillow affine_fixed: the half-pixel offsets are folded in double BEFORE the fixed conversion;
      // integer steps are exact, so the incremental walk equals this direct form
      const int f0 = fix16(a0), f1 = fix16(a1), f3 = fix16(a3), f4 = fix16(a4);
      const int xo = fix16(a2 + a0 * 0.5 + a1 * 0.5), yo = fix16(a5 + a3 * 0.5 + a4 * 0.5);
      xi = (xo + y * f1 + x * f0) >> 16;
      yi = (yo + y * f4 + x * f3) >> 16;
    } else if (scale_path) {
      double xo = a2 + a0 * 0.5, yo = a5 + a4 * 0.5;
      for (int i = 0; i < x; ++i) xo += a0;
      for (int i = 0; i < y; ++i) yo += a4;
      xi = coord_pil(xo);
      yi = coord_pil(yo);
    } else {  // generic double walk (a corner outside the 16.16 range)
      double xo = a2 + a1 * 0.5 + a0 * 0.5, yo = a5 + a4 * 0.5 + a3 * 0.5;
      for (int i = 0; i < y; ++i) {
        xo += a1;
        yo += a4;
      }
      for (int i = 0; i < x; ++i) {
        xo += a0;
        yo += a3;
      }
      xi = coord_pil(xo);
      yi = coord_pil(yo);
    }
    uint8_t px[3] = {0, 0, 0};
    if (xi >= 0 && xi < W && yi >= 0 && yi < H) {
      const int sx = flip ? W - 1 - xi : xi;  // hflip precedes the affine
      const uint8_t* s = src + ((size_t)yi * W + sx) * C;
      for (int c = 0; c < C; ++c) px[c] = s[c];
    }
    if (bright_first)
      for (int c = 0; c < C; ++c) px[c] = blend_u8(0, px[c], bright);
    for (int c = 0; c < C; ++c) dst[(size_t)x * C + c] = px[c];
    sum += luma(px, C);
  }
  // row sum: wave butterfly + LDS (integer: order-independent, exact)
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
  __shared__ int red[AUG_THREADS / 64];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int i = 0; i < AUG_THREADS / 64; ++i) t += red[i];
    row_sums[(size_t)b * H + y] = t;
  }
}

// per image chunk: contrast against int(mean(L) + 0.5) (+ brightness when it comes second), in place
__global__ void __launch_bounds__(AUG_THREADS) augment_color_kernel(uint8_t* __restrict__ img, int H, int W, int C,
                                                                    const double* __restrict__ params,
                                                                    const int* __restrict__ row_sums, int chunk) {
  const int b = blockIdx.y;
  const double* prm = params + (size_t)b * 10;
  const float bright = (float)prm[7], contrast = (float)prm[8];
  const bool bright_first = prm[9] == 0.0;
  __shared__ long long red[AUG_THREADS / 64];
  long long s = 0;
  for (int i = threadIdx.x; i < H; i += AUG_THREADS) s += row_sums[(size_t)b * H + i];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  long long tot = 0;
  for (int i = 0; i < AUG_THREADS / 64; ++i) tot += red[i];
  // ImageStat: sum(i * hist[i]) / count in double, then int(mean + 0.5)
  const int deg = (int)((double)tot / (double)((long long)H * W) + 0.5);
  const size_t npix = (size_t)H * W;
  uint8_t* base = img + (size_t)b * npix * C;
  const size_t p0 = (size_t)blockIdx.x * chunk;
  const size_t p1 = p0 + chunk < npix ? p0 + chunk : npix;
  for (size_t p = p0 + threadIdx.x; p < p1; p += AUG_THREADS) {
    for (int c = 0; c < C; ++c) {
      int v = base[p * C + c];
      v = blend_u8(deg, v, contrast);
      if (!bright_first) v = blend_u8(0, v, bright);
      base[p * C + c] = (uint8_t)v;
    }
  }
}

}  // namespace
}  // namespace sv

extern "C" {

int sv_augment_u8(const uint8_t* in, uint8_t* out, int32_t B, int32_t H, int32_t W, int32_t C, const double* params,
                  int32_t* row_sums, sv_stream_t stream) {
  SV_REQUIRE(in && out && params && row_sums, "sv_augment_u8: null pointer");
  SV_REQUIRE(in != out, "sv_augment_u8: in and out must not alias");
  SV_REQUIRE(B > 0 && H > 0 && W > 0 && (C == 1 || C == 3), "sv_augment_u8: bad shape (C must be 1 or 3)");
  SV_REQUIRE((int64_t)H * W <= (1ll << 23), "sv_augment_u8: image too large for the 32-bit row sums");
  hipStream_t s = (hipStream_t)stream;
  sv::augment_affine_kernel<<<dim3(H, B), sv::AUG_THREADS, 0, s>>>(in, out, H, W, C, params, row_sums);
  int rc = sv::check_launch("sv_augment_u8(affine)");
  if (rc) return rc;
  const int chunk = 4096;
  const int nchunks = (int)(((int64_t)H * W + chunk - 1) / chunk);
  sv::augment_color_kernel<<<dim3(nchunks, B), sv::AUG_THREADS, 0, s>>>(out, H, W, C, params, row_sums, chunk);
  return sv::check_launch("sv_augment_u8(color)");
}

}  // extern "C"
