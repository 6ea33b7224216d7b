// Depthwise 7x7 convolution (pad 3, stride 1) on NHWC activations -- ConvNeXtBlock.conv_dw
// (timm convnext.py; HF equivalent transformers/models/convnext/modeling_convnext.py:130,144).
//
// Layout/tiling (gfx950): a workgroup owns an 8x8 output tile of one image for one 64-channel
// chunk.  The (8+6)x(8+6)x64 f32 input halo tile is staged in LDS as [pixel][64 ch] (16 lanes x
// 16 B per pixel on the global side -> 256 contiguous bytes per pixel, fully coalesced; on the
// LDS side lane == channel, so the per-tap ds_read_b32 of 64 consecutive floats is bank-conflict
// free).  Each wave computes two output rows; a lane keeps its channel's 49 taps in registers and
// slides a 14-wide input row window along W (7 FMAs per input value read from LDS).
//
// The op is HBM-bound (49 FMA per 4-8 bytes moved): per output element it reads the input once
// (+halo re-read ~ (14*14)/(8*8) from LDS, not HBM) and writes the output once.
//
//   fwd          z = b + sum_tap w[tap] * x[p + tap]               (+ LayerNorm via ln_fwd)
//   bwd-data     dx = (acc ? dx : 0) + sum_tap w[48 - tap] * dz[p + tap]   (flipped kernel)
//   bwd-weight   dW[c][tap] = sum_p dz[p,c] * x[p + tap, c],  db[c] = sum_p dz[p,c]
#include "common.h"

extern "C" int sv_layernorm_fwd(const void* x, int32_t x_dtype, const float* w, const float* b, void* y,
                                int32_t y_dtype, float* mean, float* rstd, int64_t rows, int32_t C,
                                float eps, sv_stream_t stream);

namespace sv {

constexpr int TH = 8, TW = 8;            // output tile
constexpr int TR = TH + 6, TC = TW + 6;  // halo tile
constexpr int kDwThreads = 256;          // 4 waves x 2 output rows
constexpr int RPW = TH / 4;

template <typename TIN>
__device__ __forceinline__ void load_halo_tile(float* __restrict__ lds, const TIN* __restrict__ x, int b,
                                               int h0, int w0, int c0, int H, int W, int C) {
  const int sub = threadIdx.x & 15;
  for (int p = threadIdx.x >> 4; p < TR * TC; p += kDwThreads / 16) {
    const int r = p / TC, q = p - r * TC;
    const int h = h0 - 3 + r, w = w0 - 3 + q;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (h >= 0 && h < H && w >= 0 && w < W) v = ld4(x, (((size_t)b * H + h) * W + w) * C + c0 + sub * 4);
    *reinterpret_cast<float4*>(lds + p * 64 + sub * 4) = v;
  }
}

// z (or dx) for one 8x8 tile x 64 channels.  FLIP: use w[48 - tap] (backward-data).
template <typename TIN, typename TOUT, bool FLIP, bool ACCUM>
__global__ void __launch_bounds__(kDwThreads) dwconv7_kernel(const TIN* __restrict__ x,
                                                             const float* __restrict__ wdw,
                                                             const float* __restrict__ bdw,
                                                             TOUT* __restrict__ out,
                                                             uint16_t* __restrict__ out_bf16, int B, int H,
                                                             int W, int C) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [TR*TC][64]
  const int tilesW = (W + TW - 1) / TW, tilesH = (H + TH - 1) / TH;
  int t = blockIdx.x;
  const int tw = t % tilesW;
  t /= tilesW;
  const int th = t % tilesH;
  const int b = t / tilesH;
  const int h0 = th * TH, w0 = tw * TW, c0 = blockIdx.y * 64;
  load_halo_tile(lds, x, b, h0, w0, c0, H, W, C);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = c0 + lane;
  float wk[49];
#pragma unroll
  for (int i = 0; i < 49; ++i) wk[i] = wdw[(size_t)c * 49 + (FLIP ? 48 - i : i)];
  const float bias = bdw ? bdw[c] : 0.f;
  __syncthreads();
#pragma unroll
  for (int rr = 0; rr < RPW; ++rr) {
    const int r = wv * RPW + rr;
    float acc[TW];
#pragma unroll
    for (int o = 0; o < TW; ++o) acc[o] = bias;
#pragma unroll
    for (int kh = 0; kh < 7; ++kh) {
      float in[TC];
#pragma unroll
      for (int j = 0; j < TC; ++j) in[j] = lds[((r + kh) * TC + j) * 64 + lane];
#pragma unroll
      for (int o = 0; o < TW; ++o)
#pragma unroll
        for (int kw = 0; kw < 7; ++kw) acc[o] = fmaf(wk[kh * 7 + kw], in[o + kw], acc[o]);
    }
    const int h = h0 + r;
    if (h < H) {
#pragma unroll
      for (int o = 0; o < TW; ++o) {
        const int w = w0 + o;
        if (w < W) {
          const size_t i = (((size_t)b * H + h) * W + w) * C + c;
          const float v = ACCUM ? ld(out, i) + acc[o] : acc[o];
          st(out, i, v);
          if (out_bf16) out_bf16[i] = f2bf(v);
        }
      }
    }
  }
}

// backward-weight partials.  grid = (nparts, C/64); part p visits tiles p, p+nparts, ...
template <typename TIN>
__global__ void __launch_bounds__(kDwThreads) dwconv7_wgrad_kernel(const float* __restrict__ dz,
                                                                   const TIN* __restrict__ x,
                                                                   float* __restrict__ dw_part,
                                                                   float* __restrict__ db_part, int B,
                                                                   int H, int W, int C) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [TR*TC][64], reused for combine
  const int tilesW = (W + TW - 1) / TW, tilesH = (H + TH - 1) / TH;
  const int ntiles = B * tilesH * tilesW;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c0 = blockIdx.y * 64, c = c0 + lane;
  float acc[49];
#pragma unroll
  for (int i = 0; i < 49; ++i) acc[i] = 0.f;
  float dbacc = 0.f;
  for (int t0 = blockIdx.x; t0 < ntiles; t0 += gridDim.x) {
    int t = t0;
    const int tw = t % tilesW;
    t /= tilesW;
    const int th = t % tilesH;
    const int b = t / tilesH;
    const int h0 = th * TH, w0 = tw * TW;
    __syncthreads();  // previous tile's LDS reads are done
    load_halo_tile(lds, x, b, h0, w0, c0, H, W, C);
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < RPW; ++rr) {
      const int r = wv * RPW + rr;
      const int h = h0 + r;
      float d[TW];
#pragma unroll
      for (int o = 0; o < TW; ++o) {
        const int w = w0 + o;
        d[o] = (h < H && w < W) ? dz[(((size_t)b * H + h) * W + w) * C + c] : 0.f;
        dbacc += d[o];
      }
#pragma unroll
      for (int kh = 0; kh < 7; ++kh) {
        float in[TC];
#pragma unroll
        for (int j = 0; j < TC; ++j) in[j] = lds[((r + kh) * TC + j) * 64 + lane];
#pragma unroll
        for (int kw = 0; kw < 7; ++kw) {
          float s = acc[kh * 7 + kw];
#pragma unroll
          for (int o = 0; o < TW; ++o) s = fmaf(d[o], in[o + kw], s);
          acc[kh * 7 + kw] = s;
        }
      }
    }
  }
  // deterministic combine of the 4 waves through LDS: red[wave][tap][64]
  __syncthreads();
  float* red = lds;
#pragma unroll
  for (int i = 0; i < 49; ++i) red[(wv * 49 + i) * 64 + lane] = acc[i];
  float* redb = lds + 4 * 49 * 64;
  redb[wv * 64 + lane] = dbacc;
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 49; i += kDwThreads) {
    const int ch = i / 49, tap = i - ch * 49;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += red[(k * 49 + tap) * 64 + ch];
    dw_part[(size_t)blockIdx.x * C * 49 + (size_t)(c0 + ch) * 49 + tap] = s;
  }
  if (threadIdx.x < 64) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) s += redb[k * 64 + threadIdx.x];
    db_part[(size_t)blockIdx.x * C + c0 + threadIdx.x] = s;
  }
}

static size_t dw_lds_bytes() {
  size_t a = (size_t)TR * TC * 64 * sizeof(float);
  size_t b = (size_t)(4 * 49 * 64 + 4 * 64) * sizeof(float);
  return a > b ? a : b;
}

static int dw_tiles(int B, int H, int W) { return B * ((H + TH - 1) / TH) * ((W + TW - 1) / TW); }

}  // namespace sv

using namespace sv;

extern "C" {

int sv_dwconv7_ln_fwd(const void* x, int32_t x_dtype, const float* wdw, const float* bdw,
                      const float* lnw, const float* lnb, float eps, void* z, int32_t z_dtype, void* y,
                      int32_t y_dtype, float* mean, float* rstd, int32_t B, int32_t H, int32_t W,
                      int32_t C, sv_stream_t stream) {
  SV_REQUIRE(x && wdw && bdw && lnw && lnb && z && y && mean && rstd, "sv_dwconv7_ln_fwd: null pointer");
  SV_REQUIRE(C % 64 == 0 && C > 0, "sv_dwconv7_ln_fwd: C=%d must be a multiple of 64", C);
  if (B <= 0 || H <= 0 || W <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(dw_tiles(B, H, W), C / 64);
  const size_t lds = dw_lds_bytes();
#define LAUNCH(TI, TO) \
  dwconv7_kernel<TI, TO, false, false><<<grid, kDwThreads, lds, s>>>((const TI*)x, wdw, bdw, (TO*)z, nullptr, B, H, W, C)
  if (x_dtype == SV_F32 && z_dtype == SV_F32) LAUNCH(float, float);
  else if (x_dtype == SV_F32 && z_dtype == SV_BF16) LAUNCH(float, uint16_t);
  else if (x_dtype == SV_BF16 && z_dtype == SV_BF16) LAUNCH(uint16_t, uint16_t);
  else if (x_dtype == SV_BF16 && z_dtype == SV_F32) LAUNCH(uint16_t, float);
  else return set_error(SV_ERR_INVALID_ARG, "sv_dwconv7_ln_fwd: bad dtype");
#undef LAUNCH
  int rc = check_launch("sv_dwconv7_ln_fwd(dwconv)");
  if (rc) return rc;
  return sv_layernorm_fwd(z, z_dtype, lnw, lnb, y, y_dtype, mean, rstd, (int64_t)B * H * W, C, eps, stream);
}

int sv_dwconv7_bwd_data(const float* dz, const float* wdw, float* dx, uint16_t* dx_bf16, int32_t accumulate,
                        int32_t B, int32_t H, int32_t W, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(dz && wdw && dx, "sv_dwconv7_bwd_data: null pointer");
  SV_REQUIRE(C % 64 == 0 && C > 0, "sv_dwconv7_bwd_data: C=%d must be a multiple of 64", C);
  SV_REQUIRE(dz != dx, "sv_dwconv7_bwd_data: dz and dx must not alias");
  if (B <= 0 || H <= 0 || W <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(dw_tiles(B, H, W), C / 64);
  const size_t lds = dw_lds_bytes();
  if (accumulate)
    dwconv7_kernel<float, float, true, true><<<grid, kDwThreads, lds, s>>>(dz, wdw, nullptr, dx, dx_bf16, B, H, W, C);
  else
    dwconv7_kernel<float, float, true, false><<<grid, kDwThreads, lds, s>>>(dz, wdw, nullptr, dx, dx_bf16, B, H, W, C);
  return check_launch("sv_dwconv7_bwd_data");
}

int sv_dwconv7_bwd_weight_nparts(int32_t B, int32_t H, int32_t W, int32_t C) {
  const int tiles = dw_tiles(B, H, W);
  int np = 2048 / (C / 64 > 0 ? C / 64 : 1);
  if (np < 1) np = 1;
  return tiles < np ? tiles : np;
}

int sv_dwconv7_bwd_weight(const float* dz, const void* x, int32_t x_dtype, float* dw_part,
                          float* db_part, int32_t B, int32_t H, int32_t W, int32_t C,
                          sv_stream_t stream) {
  SV_REQUIRE(dz && x && dw_part && db_part, "sv_dwconv7_bwd_weight: null pointer");
  SV_REQUIRE(C % 64 == 0 && C > 0, "sv_dwconv7_bwd_weight: C=%d must be a multiple of 64", C);
  if (B <= 0 || H <= 0 || W <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(sv_dwconv7_bwd_weight_nparts(B, H, W, C), C / 64);
  const size_t lds = dw_lds_bytes();
  if (x_dtype == SV_F32)
    dwconv7_wgrad_kernel<float><<<grid, kDwThreads, lds, s>>>(dz, (const float*)x, dw_part, db_part, B, H, W, C);
  else if (x_dtype == SV_BF16)
    dwconv7_wgrad_kernel<uint16_t><<<grid, kDwThreads, lds, s>>>(dz, (const uint16_t*)x, dw_part, db_part, B, H, W, C);
  else
    return set_error(SV_ERR_INVALID_ARG, "sv_dwconv7_bwd_weight: bad dtype");
  return check_launch("sv_dwconv7_bwd_weight");
}

}  // extern "C"
