// Channels-last LayerNorm family for the ConvNeXt path (gfx950, wave64).
//
//   sv_layernorm_fwd / _bwd           timm LayerNorm on [rows][C]        (one wave per row)
//   sv_stem_patchify_ln_fwd / _bwd    timm stem Conv2d(3,C,4,4)+LayerNorm2d (one wave per pixel)
//   sv_downsample_ln_patch2_fwd/_bwd  timm ConvNeXtStage.downsample[0] LayerNorm2d + 2x2 gather
//   sv_pool_ln_fwd / _bwd             timm NormMlpClassifierHead (avg pool + LayerNorm2d)
//
// All of these are HBM-bound row reductions: one wave owns a whole channel vector, channel c of a
// row is held by lane (c % 64) so every global access is a contiguous 256 B (f32) per wave
// instruction and the row statistics are two wave64 butterfly sums.  Per-channel weight gradients
// are accumulated in registers across the rows a wave visits (grid-stride) and combined per
// workgroup, giving deterministic [nparts][C] partials that sv_reduce_partials folds.
#include "common.h"

namespace sv {

constexpr int kLnThreads = 256;   // 4 waves
constexpr int kMaxCPL = 24;       // channels per lane supported (C <= 1536)

// ------------------------------------------------------------------------------------------
// LayerNorm forward over rows: one wave per row, CPL channels per lane (c = lane + 64*t).
template <typename TX, typename TY, int CPL>
__global__ void __launch_bounds__(kLnThreads) ln_fwd_kernel(const TX* __restrict__ x,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ b,
                                                            TY* __restrict__ y, float* __restrict__ mean,
                                                            float* __restrict__ rstd, int64_t rows, int C,
                                                            float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * (kLnThreads / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (kLnThreads / 64);
  const float invC = 1.0f / (float)C;
  for (int64_t r = wave; r < rows; r += nwaves) {
    const TX* xr = x + (size_t)r * C;
    float v[CPL];
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      v[t] = ld(xr, lane + 64 * t);
      s += v[t];
    }
    const float mu = wave_sum(s) * invC;
    float q = 0.f;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      const float d = v[t] - mu;
      q += d * d;
    }
    const float rs = rsqrtf(wave_sum(q) * invC + eps);
    TY* yr = y + (size_t)r * C;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      const int c = lane + 64 * t;
      st(yr, c, (v[t] - mu) * rs * w[c] + b[c]);
    }
    if (lane == 0) {
      mean[r] = mu;
      rstd[r] = rs;
    }
  }
}

// LayerNorm backward over rows.  dx = rstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*w.
// dy / x / dx may each be f32 or bf16 (bf16 mode: the fc1 dgrad output and the dwconv input
// gradient travel as bf16); statistics and parameter gradients stay f32.
template <typename TDY, typename TX, typename TDX, int CPL>
__global__ void __launch_bounds__(kLnThreads) ln_bwd_kernel(const TDY* __restrict__ dy,
                                                            const TX* __restrict__ x,
                                                            const float* __restrict__ mean,
                                                            const float* __restrict__ rstd,
                                                            const float* __restrict__ w,
                                                            TDX* __restrict__ dx, int accumulate,
                                                            float* __restrict__ dw_part,
                                                            float* __restrict__ db_part, int64_t rows,
                                                            int C) {
  __shared__ float red[kLnThreads / 64][kMaxCPL * 64 > 2048 ? 2048 : kMaxCPL * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wave = (int64_t)blockIdx.x * (kLnThreads / 64) + wid;
  const int64_t nwaves = (int64_t)gridDim.x * (kLnThreads / 64);
  const float invC = 1.0f / (float)C;
  float wr[CPL], adw[CPL], adb[CPL];
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    wr[t] = w[lane + 64 * t];
    adw[t] = 0.f;
    adb[t] = 0.f;
  }
  for (int64_t r = wave; r < rows; r += nwaves) {
    const float mu = mean[r], rs = rstd[r];
    float xh[CPL], g[CPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      const int c = lane + 64 * t;
      const float d = ld(dy, (size_t)r * C + c);
      xh[t] = (ld(x, (size_t)r * C + c) - mu) * rs;
      g[t] = d * wr[t];
      s1 += g[t];
      s2 += g[t] * xh[t];
      adw[t] += d * xh[t];
      adb[t] += d;
    }
    s1 = wave_sum(s1) * invC;
    s2 = wave_sum(s2) * invC;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      const size_t i = (size_t)r * C + lane + 64 * t;
      const float v = rs * (g[t] - s1 - xh[t] * s2);
      st(dx, i, accumulate ? ld(dx, i) + v : v);
    }
  }
  // combine the 4 waves of this workgroup deterministically (fixed order) -> one partial row
#pragma unroll
  for (int t = 0; t < CPL; ++t) red[wid][lane + 64 * t] = adw[t];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kLnThreads) {
    float s = 0.f;
    for (int k = 0; k < kLnThreads / 64; ++k) s += red[k][c];
    dw_part[(size_t)blockIdx.x * C + c] = s;
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < CPL; ++t) red[wid][lane + 64 * t] = adb[t];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kLnThreads) {
    float s = 0.f;
    for (int k = 0; k < kLnThreads / 64; ++k) s += red[k][c];
    db_part[(size_t)blockIdx.x * C + c] = s;
  }
}

static int ln_grid(int64_t rows) {
  const int64_t g = (rows + 3) / 4;
  return (int)(g < 1024 ? (g < 1 ? 1 : g) : 1024);
}

// dispatch helper over supported channel-per-lane counts
#define SV_CPL_SWITCH(CPLV, ...)                                                        \
  switch (CPLV) {                                                                       \
    case 1: { constexpr int CPL = 1; __VA_ARGS__; } break;                              \
    case 2: { constexpr int CPL = 2; __VA_ARGS__; } break;                              \
    case 3: { constexpr int CPL = 3; __VA_ARGS__; } break;                              \
    case 4: { constexpr int CPL = 4; __VA_ARGS__; } break;                              \
    case 6: { constexpr int CPL = 6; __VA_ARGS__; } break;                              \
    case 8: { constexpr int CPL = 8; __VA_ARGS__; } break;                              \
    case 12: { constexpr int CPL = 12; __VA_ARGS__; } break;                            \
    case 16: { constexpr int CPL = 16; __VA_ARGS__; } break;                            \
    case 24: { constexpr int CPL = 24; __VA_ARGS__; } break;                            \
    default: return set_error(SV_ERR_UNSUPPORTED, "channel count %d unsupported", C);   \
  }

static bool cpl_ok(int C) {
  if (C % 64) return false;
  const int k = C / 64;
  return k == 1 || k == 2 || k == 3 || k == 4 || k == 6 || k == 8 || k == 12 || k == 16 || k == 24;
}

// ------------------------------------------------------------------------------------------
// Stem: Conv2d(3, C, 4, 4) + LayerNorm2d.  One wave per output pixel; lane owns channels
// c = lane + 64*t; the 48-value patch is loaded by lanes 0..47 and broadcast with v_readlane
// (scalar operand of the FMAs); weights live in LDS as [48][C] so the per-k reads of consecutive
// channels are bank-conflict free.
constexpr int kStemWaves = 4;

template <typename TY, int CPL>
__global__ void __launch_bounds__(64 * kStemWaves) stem_fwd_kernel(
    const float* __restrict__ img, const float* __restrict__ w, const float* __restrict__ bias,
    const float* __restrict__ lnw, const float* __restrict__ lnb, float eps, TY* __restrict__ y,
    float* __restrict__ mean, float* __restrict__ rstd, int B, int H, int W, int C) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* wl = smem;                       // [48][C]
  for (int i = threadIdx.x; i < 48 * C; i += blockDim.x) {
    const int c = i % C, k = i / C;
    wl[i] = w[(size_t)c * 48 + k];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int Ho = H / 4, Wo = W / 4;
  const int64_t npix = (int64_t)B * Ho * Wo;
  const float invC = 1.0f / (float)C;
  float bb[CPL], gw[CPL], gb[CPL];
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    bb[t] = bias[lane + 64 * t];
    gw[t] = lnw[lane + 64 * t];
    gb[t] = lnb[lane + 64 * t];
  }
  for (int64_t p = (int64_t)blockIdx.x * kStemWaves + wid; p < npix; p += (int64_t)gridDim.x * kStemWaves) {
    const int j = (int)(p % Wo), i = (int)((p / Wo) % Ho), b = (int)(p / ((int64_t)Wo * Ho));
    float pl = 0.f;
    if (lane < 48) {
      const int ci = lane >> 4, kh = (lane >> 2) & 3, kw = lane & 3;
      pl = img[(((size_t)b * 3 + ci) * H + (4 * i + kh)) * W + (4 * j + kw)];
    }
    float z[CPL];
#pragma unroll
    for (int t = 0; t < CPL; ++t) z[t] = bb[t];
#pragma unroll
    for (int k = 0; k < 48; ++k) {
      const float pv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pl), k));
#pragma unroll
      for (int t = 0; t < CPL; ++t) z[t] = fmaf(wl[k * C + lane + 64 * t], pv, z[t]);
    }
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < CPL; ++t) s += z[t];
    const float mu = wave_sum(s) * invC;
    float q = 0.f;
#pragma unroll
    for (int t = 0; t < CPL; ++t) q += (z[t] - mu) * (z[t] - mu);
    const float rs = rsqrtf(wave_sum(q) * invC + eps);
#pragma unroll
    for (int t = 0; t < CPL; ++t) st(y, (size_t)p * C + lane + 64 * t, (z[t] - mu) * rs * gw[t] + gb[t]);
    if (lane == 0) {
      mean[p] = mu;
      rstd[p] = rs;
    }
  }
}

constexpr int kStemBwdBlocks = 256;

template <int CPL>
__global__ void __launch_bounds__(64 * kStemWaves) stem_bwd_kernel(
    const float* __restrict__ img, const float* __restrict__ w, const float* __restrict__ bias,
    const float* __restrict__ lnw, const float* __restrict__ mean, const float* __restrict__ rstd,
    const float* __restrict__ dy, float* __restrict__ dw_part, float* __restrict__ db_part,
    float* __restrict__ dlnw_part, float* __restrict__ dlnb_part, int B, int H, int W, int C) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* wl = smem;                 // [48][C]
  float* comb = smem + 48 * C;      // [48*C + 3*C] combine buffer
  for (int i = threadIdx.x; i < 48 * C; i += blockDim.x) {
    const int c = i % C, k = i / C;
    wl[i] = w[(size_t)c * 48 + k];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int Ho = H / 4, Wo = W / 4;
  const int64_t npix = (int64_t)B * Ho * Wo;
  const float invC = 1.0f / (float)C;
  float bb[CPL], gw[CPL];
  float adw[CPL][48], adb[CPL], adlw[CPL], adlb[CPL];
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    bb[t] = bias[lane + 64 * t];
    gw[t] = lnw[lane + 64 * t];
    adb[t] = adlw[t] = adlb[t] = 0.f;
#pragma unroll
    for (int k = 0; k < 48; ++k) adw[t][k] = 0.f;
  }
  for (int64_t p = (int64_t)blockIdx.x * kStemWaves + wid; p < npix; p += (int64_t)gridDim.x * kStemWaves) {
    const int j = (int)(p % Wo), i = (int)((p / Wo) % Ho), b = (int)(p / ((int64_t)Wo * Ho));
    float pl = 0.f;
    if (lane < 48) {
      const int ci = lane >> 4, kh = (lane >> 2) & 3, kw = lane & 3;
      pl = img[(((size_t)b * 3 + ci) * H + (4 * i + kh)) * W + (4 * j + kw)];
    }
    float pk[48];
#pragma unroll
    for (int k = 0; k < 48; ++k) pk[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pl), k));
    const float mu = mean[p], rs = rstd[p];
    float xh[CPL], g[CPL], d[CPL];
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      float z = bb[t];
#pragma unroll
      for (int k = 0; k < 48; ++k) z = fmaf(wl[k * C + lane + 64 * t], pk[k], z);
      xh[t] = (z - mu) * rs;
      d[t] = dy[(size_t)p * C + lane + 64 * t];
      g[t] = d[t] * gw[t];
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      s1 += g[t];
      s2 += g[t] * xh[t];
    }
    s1 = wave_sum(s1) * invC;
    s2 = wave_sum(s2) * invC;
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      const float dz = rs * (g[t] - s1 - xh[t] * s2);
      adb[t] += dz;
      adlw[t] += d[t] * xh[t];
      adlb[t] += d[t];
#pragma unroll
      for (int k = 0; k < 48; ++k) adw[t][k] = fmaf(dz, pk[k], adw[t][k]);
    }
  }
  // deterministic combine of the 4 waves (fixed order), layout [C][48] + db + dlnw + dlnb
  const int nw = 48 * C + 3 * C;
  for (int wv = 0; wv < kStemWaves; ++wv) {
    if (wid == wv) {
#pragma unroll
      for (int t = 0; t < CPL; ++t) {
        const int c = lane + 64 * t;
#pragma unroll
        for (int k = 0; k < 48; ++k) comb[c * 48 + k] = (wv ? comb[c * 48 + k] : 0.f) + adw[t][k];
        comb[48 * C + c] = (wv ? comb[48 * C + c] : 0.f) + adb[t];
        comb[49 * C + c] = (wv ? comb[49 * C + c] : 0.f) + adlw[t];
        comb[50 * C + c] = (wv ? comb[50 * C + c] : 0.f) + adlb[t];
      }
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < nw; i += blockDim.x) {
    const float v = comb[i];
    if (i < 48 * C) dw_part[(size_t)blockIdx.x * 48 * C + i] = v;
    else if (i < 49 * C) db_part[(size_t)blockIdx.x * C + (i - 48 * C)] = v;
    else if (i < 50 * C) dlnw_part[(size_t)blockIdx.x * C + (i - 49 * C)] = v;
    else dlnb_part[(size_t)blockIdx.x * C + (i - 50 * C)] = v;
  }
}

// ------------------------------------------------------------------------------------------
// Downsample: LayerNorm2d over C of each input pixel, then gather the 2x2/s2 patch into the row
// patches[(b,i,j)][c*4 + kh*2 + kw] (timm conv weight order).  One wave per output patch.
template <typename TP, int CPL>
__global__ void __launch_bounds__(kLnThreads) ds_fwd_kernel(const float* __restrict__ x,
                                                            const float* __restrict__ lnw,
                                                            const float* __restrict__ lnb, float eps,
                                                            TP* __restrict__ patches,
                                                            float* __restrict__ mean,
                                                            float* __restrict__ rstd, int B, int H,
                                                            int W, int C) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * (kLnThreads / 64) + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * (kLnThreads / 64);
  const int Ho = H / 2, Wo = W / 2;
  const int64_t np = (int64_t)B * Ho * Wo;
  const float invC = 1.0f / (float)C;
  for (int64_t p = wave; p < np; p += nwaves) {
    const int j = (int)(p % Wo), i = (int)((p / Wo) % Ho), b = (int)(p / ((int64_t)Wo * Ho));
    float v[4][CPL];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t pix = ((int64_t)b * H + 2 * i + (q >> 1)) * W + 2 * j + (q & 1);
      const float* xr = x + (size_t)pix * C;
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < CPL; ++t) {
        v[q][t] = xr[lane + 64 * t];
        s += v[q][t];
      }
      const float mu = wave_sum(s) * invC;
      float qq = 0.f;
#pragma unroll
      for (int t = 0; t < CPL; ++t) qq += (v[q][t] - mu) * (v[q][t] - mu);
      const float rs = rsqrtf(wave_sum(qq) * invC + eps);
#pragma unroll
      for (int t = 0; t < CPL; ++t) {
        const int c = lane + 64 * t;
        v[q][t] = (v[q][t] - mu) * rs * lnw[c] + lnb[c];
      }
      if (lane == 0) {
        mean[pix] = mu;
        rstd[pix] = rs;
      }
    }
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      const int c = lane + 64 * t;
      st4(patches, (size_t)p * 4 * C + 4 * c, make_float4(v[0][t], v[1][t], v[2][t], v[3][t]));
    }
  }
}

template <int CPL>
__global__ void __launch_bounds__(kLnThreads) ds_bwd_kernel(
    const float* __restrict__ dpatches, const float* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ lnw, float* __restrict__ dx,
    uint16_t* __restrict__ dx_bf16, float* __restrict__ dlnw_part, float* __restrict__ dlnb_part, int B, int H,
    int W, int C) {
  __shared__ float red[kLnThreads / 64][2048];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t wave = (int64_t)blockIdx.x * (kLnThreads / 64) + wid;
  const int64_t nwaves = (int64_t)gridDim.x * (kLnThreads / 64);
  const int Ho = H / 2, Wo = W / 2;
  const int64_t np = (int64_t)B * Ho * Wo;
  const float invC = 1.0f / (float)C;
  float wr[CPL], adw[CPL], adb[CPL];
#pragma unroll
  for (int t = 0; t < CPL; ++t) {
    wr[t] = lnw[lane + 64 * t];
    adw[t] = adb[t] = 0.f;
  }
  for (int64_t p = wave; p < np; p += nwaves) {
    const int j = (int)(p % Wo), i = (int)((p / Wo) % Ho), b = (int)(p / ((int64_t)Wo * Ho));
    float dq[4][CPL];
#pragma unroll
    for (int t = 0; t < CPL; ++t) {
      const float4 d4 = *reinterpret_cast<const float4*>(dpatches + (size_t)p * 4 * C + 4 * (lane + 64 * t));
      dq[0][t] = d4.x; dq[1][t] = d4.y; dq[2][t] = d4.z; dq[3][t] = d4.w;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t pix = ((int64_t)b * H + 2 * i + (q >> 1)) * W + 2 * j + (q & 1);
      const float mu = mean[pix], rs = rstd[pix];
      float xh[CPL], g[CPL], s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int t = 0; t < CPL; ++t) {
        xh[t] = (x[(size_t)pix * C + lane + 64 * t] - mu) * rs;
        g[t] = dq[q][t] * wr[t];
        s1 += g[t];
        s2 += g[t] * xh[t];
        adw[t] += dq[q][t] * xh[t];
        adb[t] += dq[q][t];
      }
      s1 = wave_sum(s1) * invC;
      s2 = wave_sum(s2) * invC;
#pragma unroll
      for (int t = 0; t < CPL; ++t) {
        const size_t i = (size_t)pix * C + lane + 64 * t;
        const float v = rs * (g[t] - s1 - xh[t] * s2);
        dx[i] = v;
        if (dx_bf16) dx_bf16[i] = f2bf(v);
      }
    }
  }
#pragma unroll
  for (int t = 0; t < CPL; ++t) red[wid][lane + 64 * t] = adw[t];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kLnThreads)
    dlnw_part[(size_t)blockIdx.x * C + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
  __syncthreads();
#pragma unroll
  for (int t = 0; t < CPL; ++t) red[wid][lane + 64 * t] = adb[t];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kLnThreads)
    dlnb_part[(size_t)blockIdx.x * C + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c];
}

// ------------------------------------------------------------------------------------------
// Head: global average pool over HW, then LayerNorm over C.  One workgroup per image.
__global__ void __launch_bounds__(kLnThreads) pool_ln_fwd_kernel(const float* __restrict__ x,
                                                                 const float* __restrict__ lnw,
                                                                 const float* __restrict__ lnb,
                                                                 float eps, float* __restrict__ pooled,
                                                                 float* __restrict__ feat,
                                                                 float* __restrict__ mean,
                                                                 float* __restrict__ rstd, int HW,
                                                                 int C) {
  __shared__ float red[kLnThreads / 64];
  const int b = blockIdx.x;
  const float* xb = x + (size_t)b * HW * C;
  const float invHW = 1.0f / (float)HW, invC = 1.0f / (float)C;
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f;
    for (int p = 0; p < HW; ++p) a += xb[(size_t)p * C + c];
    a *= invHW;
    pooled[(size_t)b * C + c] = a;
    s += a;
  }
  const float mu = block_sum(s, red) * invC;
  float q = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float d = pooled[(size_t)b * C + c] - mu;
    q += d * d;
  }
  const float rs = rsqrtf(block_sum(q, red) * invC + eps);
  for (int c = threadIdx.x; c < C; c += blockDim.x)
    feat[(size_t)b * C + c] = (pooled[(size_t)b * C + c] - mu) * rs * lnw[c] + lnb[c];
  if (threadIdx.x == 0) {
    mean[b] = mu;
    rstd[b] = rs;
  }
}

__global__ void __launch_bounds__(kLnThreads) pool_ln_bwd_kernel(
    const float* __restrict__ dfeat, const float* __restrict__ pooled, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ lnw, float* __restrict__ dx,
    uint16_t* __restrict__ dx_bf16, float* __restrict__ dlnw_part, float* __restrict__ dlnb_part, int HW, int C) {
  __shared__ float red[kLnThreads / 64];
  extern __shared__ __attribute__((aligned(16))) float dp[];  // [C]
  const int b = blockIdx.x;
  const float mu = mean[b], rs = rstd[b];
  const float invC = 1.0f / (float)C, invHW = 1.0f / (float)HW;
  float s1 = 0.f, s2 = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float d = dfeat[(size_t)b * C + c];
    const float xh = (pooled[(size_t)b * C + c] - mu) * rs;
    const float g = d * lnw[c];
    s1 += g;
    s2 += g * xh;
    dlnw_part[(size_t)b * C + c] = d * xh;
    dlnb_part[(size_t)b * C + c] = d;
  }
  s1 = block_sum(s1, red) * invC;
  s2 = block_sum(s2, red) * invC;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float xh = (pooled[(size_t)b * C + c] - mu) * rs;
    const float g = dfeat[(size_t)b * C + c] * lnw[c];
    dp[c] = rs * (g - s1 - xh * s2) * invHW;
  }
  __syncthreads();
  float* dxb = dx + (size_t)b * HW * C;
  uint16_t* dbb = dx_bf16 ? dx_bf16 + (size_t)b * HW * C : nullptr;
  for (size_t i = threadIdx.x; i < (size_t)HW * C; i += blockDim.x) {
    dxb[i] = dp[i % C];
    if (dbb) dbb[i] = f2bf(dp[i % C]);
  }
}

}  // namespace sv

using namespace sv;

extern "C" {

int sv_layernorm_fwd(const void* x, int32_t x_dtype, const float* w, const float* b, void* y,
                     int32_t y_dtype, float* mean, float* rstd, int64_t rows, int32_t C, float eps,
                     sv_stream_t stream) {
  SV_REQUIRE(x && w && b && y && mean && rstd, "sv_layernorm_fwd: null pointer");
  SV_REQUIRE(cpl_ok(C), "sv_layernorm_fwd: C=%d must be 64*{1,2,3,4,6,8,12,16,24}", C);
  if (rows <= 0) return SV_OK;
  const int grid = ln_grid(rows);
  hipStream_t s = (hipStream_t)stream;
#define LAUNCH(TX, TY)                                                                            \
  SV_CPL_SWITCH(C / 64, ln_fwd_kernel<TX, TY, CPL><<<grid, kLnThreads, 0, s>>>(                  \
                            (const TX*)x, w, b, (TY*)y, mean, rstd, rows, C, eps))
  if (x_dtype == SV_F32 && y_dtype == SV_F32) { LAUNCH(float, float); }
  else if (x_dtype == SV_F32 && y_dtype == SV_BF16) { LAUNCH(float, uint16_t); }
  else if (x_dtype == SV_BF16 && y_dtype == SV_F32) { LAUNCH(uint16_t, float); }
  else if (x_dtype == SV_BF16 && y_dtype == SV_BF16) { LAUNCH(uint16_t, uint16_t); }
  else return set_error(SV_ERR_INVALID_ARG, "sv_layernorm_fwd: bad dtype");
#undef LAUNCH
  return check_launch("sv_layernorm_fwd");
}

int sv_layernorm_bwd_nparts(int64_t rows, int32_t C) { (void)C; return ln_grid(rows); }

int sv_layernorm_bwd(const void* dy, int32_t dy_dtype, const void* x, int32_t x_dtype, const float* mean,
                     const float* rstd, const float* w, void* dx, int32_t dx_dtype, int32_t accumulate,
                     float* dw_part, float* db_part, int64_t rows, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(dy && x && mean && rstd && w && dx && dw_part && db_part, "sv_layernorm_bwd: null pointer");
  SV_REQUIRE(cpl_ok(C) && C <= 2048, "sv_layernorm_bwd: C=%d unsupported", C);
  if (rows <= 0) return SV_OK;
  const int grid = ln_grid(rows);
  hipStream_t s = (hipStream_t)stream;
#define LNB(TDY, TX, TDX)                                                                              \
  SV_CPL_SWITCH(C / 64, ln_bwd_kernel<TDY, TX, TDX, CPL><<<grid, kLnThreads, 0, s>>>(                 \
                            (const TDY*)dy, (const TX*)x, mean, rstd, w, (TDX*)dx, accumulate, dw_part, \
                            db_part, rows, C))
  if (dy_dtype == SV_F32 && x_dtype == SV_F32 && dx_dtype == SV_F32) {
    LNB(float, float, float);
  } else if (dy_dtype == SV_F32 && x_dtype == SV_BF16 && dx_dtype == SV_F32) {
    LNB(float, uint16_t, float);
  } else if (dy_dtype == SV_BF16 && x_dtype == SV_BF16 && dx_dtype == SV_F32) {
    LNB(uint16_t, uint16_t, float);
  } else if (dy_dtype == SV_BF16 && x_dtype == SV_BF16 && dx_dtype == SV_BF16) {
    LNB(uint16_t, uint16_t, uint16_t);
  } else {
    return set_error(SV_ERR_UNSUPPORTED, "sv_layernorm_bwd: dtype combination (dy %d, x %d, dx %d) unsupported",
                     dy_dtype, x_dtype, dx_dtype);
  }
#undef LNB
  return check_launch("sv_layernorm_bwd");
}

static int stem_grid(int B, int H, int W) {
  const int64_t np = (int64_t)B * (H / 4) * (W / 4);
  const int64_t g = (np + kStemWaves - 1) / kStemWaves;
  return (int)(g < 2048 ? (g < 1 ? 1 : g) : 2048);
}

int sv_stem_patchify_ln_fwd(const float* img, const float* w, const float* b, const float* lnw,
                            const float* lnb, float eps, void* y, int32_t y_dtype, float* mean,
                            float* rstd, int32_t B, int32_t H, int32_t W, int32_t C,
                            sv_stream_t stream) {
  SV_REQUIRE(img && w && b && lnw && lnb && y && mean && rstd, "sv_stem_patchify_ln_fwd: null pointer");
  SV_REQUIRE(H % 4 == 0 && W % 4 == 0, "sv_stem_patchify_ln_fwd: H,W must be multiples of 4");
  SV_REQUIRE(C % 64 == 0 && C <= 256, "sv_stem_patchify_ln_fwd: C=%d unsupported", C);
  if (B <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const size_t lds = (size_t)(48 * C) * sizeof(float);
  const int grid = stem_grid(B, H, W);
#define LAUNCH(TY)                                                                              \
  switch (C / 64) {                                                                             \
    case 1: stem_fwd_kernel<TY, 1><<<grid, 64 * kStemWaves, lds, s>>>(img, w, b, lnw, lnb, eps, (TY*)y, mean, rstd, B, H, W, C); break; \
    case 2: stem_fwd_kernel<TY, 2><<<grid, 64 * kStemWaves, lds, s>>>(img, w, b, lnw, lnb, eps, (TY*)y, mean, rstd, B, H, W, C); break; \
    case 3: stem_fwd_kernel<TY, 3><<<grid, 64 * kStemWaves, lds, s>>>(img, w, b, lnw, lnb, eps, (TY*)y, mean, rstd, B, H, W, C); break; \
    case 4: stem_fwd_kernel<TY, 4><<<grid, 64 * kStemWaves, lds, s>>>(img, w, b, lnw, lnb, eps, (TY*)y, mean, rstd, B, H, W, C); break; \
  }
  if (y_dtype == SV_F32) { LAUNCH(float); }
  else if (y_dtype == SV_BF16) { LAUNCH(uint16_t); }
  else return set_error(SV_ERR_INVALID_ARG, "sv_stem_patchify_ln_fwd: bad dtype");
#undef LAUNCH
  return check_launch("sv_stem_patchify_ln_fwd");
}

int sv_stem_patchify_ln_bwd_nparts(int32_t B, int32_t H, int32_t W, int32_t C) {
  (void)C;
  const int g = stem_grid(B, H, W);
  return g < kStemBwdBlocks ? g : kStemBwdBlocks;
}

int sv_stem_patchify_ln_bwd(const float* img, const float* w, const float* b, const float* lnw,
                            const float* mean, const float* rstd, const float* dy, float* dw_part,
                            float* db_part, float* dlnw_part, float* dlnb_part, int32_t B, int32_t H,
                            int32_t W, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(img && w && b && lnw && mean && rstd && dy && dw_part && db_part && dlnw_part && dlnb_part,
             "sv_stem_patchify_ln_bwd: null pointer");
  SV_REQUIRE(H % 4 == 0 && W % 4 == 0, "sv_stem_patchify_ln_bwd: H,W must be multiples of 4");
  SV_REQUIRE(C % 64 == 0 && C <= 192, "sv_stem_patchify_ln_bwd: C=%d unsupported", C);
  if (B <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const int grid = sv_stem_patchify_ln_bwd_nparts(B, H, W, C);
  const size_t lds = (size_t)(48 * C + 51 * C) * sizeof(float);
  switch (C / 64) {
    case 1: stem_bwd_kernel<1><<<grid, 64 * kStemWaves, lds, s>>>(img, w, b, lnw, mean, rstd, dy, dw_part, db_part, dlnw_part, dlnb_part, B, H, W, C); break;
    case 2: stem_bwd_kernel<2><<<grid, 64 * kStemWaves, lds, s>>>(img, w, b, lnw, mean, rstd, dy, dw_part, db_part, dlnw_part, dlnb_part, B, H, W, C); break;
    case 3: stem_bwd_kernel<3><<<grid, 64 * kStemWaves, lds, s>>>(img, w, b, lnw, mean, rstd, dy, dw_part, db_part, dlnw_part, dlnb_part, B, H, W, C); break;
  }
  return check_launch("sv_stem_patchify_ln_bwd");
}

static int ds_grid(int B, int H, int W) {
  const int64_t np = (int64_t)B * (H / 2) * (W / 2);
  const int64_t g = (np + 3) / 4;
  return (int)(g < 1024 ? (g < 1 ? 1 : g) : 1024);
}

int sv_downsample_ln_patch2_fwd(const float* x, const float* lnw, const float* lnb, float eps,
                                void* patches, int32_t p_dtype, float* mean, float* rstd, int32_t B,
                                int32_t H, int32_t W, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(x && lnw && lnb && patches && mean && rstd, "sv_downsample_ln_patch2_fwd: null pointer");
  SV_REQUIRE(H % 2 == 0 && W % 2 == 0, "sv_downsample_ln_patch2_fwd: H,W must be even");
  SV_REQUIRE(cpl_ok(C) && C <= 1024, "sv_downsample_ln_patch2_fwd: C=%d unsupported", C);
  if (B <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const int grid = ds_grid(B, H, W);
  if (p_dtype == SV_F32) {
    SV_CPL_SWITCH(C / 64, ds_fwd_kernel<float, CPL><<<grid, kLnThreads, 0, s>>>(
                              x, lnw, lnb, eps, (float*)patches, mean, rstd, B, H, W, C));
  } else if (p_dtype == SV_BF16) {
    SV_CPL_SWITCH(C / 64, ds_fwd_kernel<uint16_t, CPL><<<grid, kLnThreads, 0, s>>>(
                              x, lnw, lnb, eps, (uint16_t*)patches, mean, rstd, B, H, W, C));
  } else {
    return set_error(SV_ERR_INVALID_ARG, "sv_downsample_ln_patch2_fwd: bad dtype");
  }
  return check_launch("sv_downsample_ln_patch2_fwd");
}

int sv_downsample_ln_patch2_bwd_nparts(int32_t B, int32_t H, int32_t W, int32_t C) {
  (void)C;
  return ds_grid(B, H, W);
}

int sv_downsample_ln_patch2_bwd(const float* dpatches, const float* x, const float* mean,
                                const float* rstd, const float* lnw, float* dx, uint16_t* dx_bf16, float* dlnw_part,
                                float* dlnb_part, int32_t B, int32_t H, int32_t W, int32_t C,
                                sv_stream_t stream) {
  SV_REQUIRE(dpatches && x && mean && rstd && lnw && dx && dlnw_part && dlnb_part,
             "sv_downsample_ln_patch2_bwd: null pointer");
  SV_REQUIRE(cpl_ok(C) && C <= 1024, "sv_downsample_ln_patch2_bwd: C=%d unsupported", C);
  if (B <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const int grid = ds_grid(B, H, W);
  SV_CPL_SWITCH(C / 64, ds_bwd_kernel<CPL><<<grid, kLnThreads, 0, s>>>(
                            dpatches, x, mean, rstd, lnw, dx, dx_bf16, dlnw_part, dlnb_part, B, H, W, C));
  return check_launch("sv_downsample_ln_patch2_bwd");
}

int sv_pool_ln_fwd(const float* x, const float* lnw, const float* lnb, float eps, float* pooled,
                   float* feat, float* mean, float* rstd, int32_t B, int32_t HW, int32_t C,
                   sv_stream_t stream) {
  SV_REQUIRE(x && lnw && lnb && pooled && feat && mean && rstd, "sv_pool_ln_fwd: null pointer");
  if (B <= 0) return SV_OK;
  pool_ln_fwd_kernel<<<B, kLnThreads, 0, (hipStream_t)stream>>>(x, lnw, lnb, eps, pooled, feat, mean,
                                                                 rstd, HW, C);
  return check_launch("sv_pool_ln_fwd");
}

int sv_pool_ln_bwd(const float* dfeat, const float* pooled, const float* mean, const float* rstd,
                   const float* lnw, float* dx, uint16_t* dx_bf16, float* dlnw_part, float* dlnb_part, int32_t B,
                   int32_t HW, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(dfeat && pooled && mean && rstd && lnw && dx && dlnw_part && dlnb_part,
             "sv_pool_ln_bwd: null pointer");
  if (B <= 0) return SV_OK;
  pool_ln_bwd_kernel<<<B, kLnThreads, C * sizeof(float), (hipStream_t)stream>>>(
      dfeat, pooled, mean, rstd, lnw, dx, dx_bf16, dlnw_part, dlnb_part, HW, C);
  return check_launch("sv_pool_ln_bwd");
}

}  // extern "C"
