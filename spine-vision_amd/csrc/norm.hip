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


// ------------------------------------------------------------------------------------------
// Vectorised LayerNorm for C = 8 * LPR * NV with LPR in {8, 16, 32, 64}: every lane owns NV runs of
// 8 consecutive channels (one 16-B bf16 / two 16-B f32 accesses per run), a row is spread over LPR
// lanes, a wave covers 64/LPR rows at once.  ConvNeXt-base's C = 128/256/512/1024 and ConvNeXt-large's
// 192/384/768/1536 all fit; the per-lane-channel kernels above serve the other widths.
template <typename T>
__device__ __forceinline__ void ld8v(const T* __restrict__ p, float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[2 * j] = __uint_as_float(w[j] << 16);
      v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
    }
  }
}
template <typename T>
__device__ __forceinline__ void st8v(T* __restrict__ p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else {
    *reinterpret_cast<uint4*>(p) =
        make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
  }
}
// the row statistics' butterfly over LPR lanes: from the cross-lane unit for groups of >= 16 lanes (common.h
// xlane_group_sum, bitwise the shuffle form; -DSV_LN_XLANE=0 keeps ds_bpermute shuffles, A/B builds)
#ifndef SV_LN_XLANE
#define SV_LN_XLANE SV_XLANE
#endif
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
  if constexpr (SV_LN_XLANE && LPR >= 16) {
    return xlane_group_sum<LPR>(v);
  } else {
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
  }
}

template <typename TX, typename TY, int LPR, int NV>
__global__ void __launch_bounds__(kLnThreads) ln_fwd_vec_kernel(const TX* __restrict__ x, const float* __restrict__ w,
                                                                const float* __restrict__ b, TY* __restrict__ y,
                                                                float* __restrict__ mean, float* __restrict__ rstd,
                                                                int64_t rows, int C, float eps) {
  constexpr int RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, l = lane % LPR;
  const int64_t r = ((int64_t)blockIdx.x * (kLnThreads / 64) + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const bool ok = r < rows;
  const size_t base = (size_t)(ok ? r : 0) * C;
  float v[NV][8];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    ld8v(x + base + (size_t)(l + LPR * j) * 8, v[j]);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[j][e];
  }
  const float invC = 1.0f / (float)C;
  const float mu = group_sum<LPR>(s) * invC;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) q += (v[j][e] - mu) * (v[j][e] - mu);
  const float rs = rsqrtf(group_sum<LPR>(q) * invC + eps);
  if (!ok) return;  // after the last shuffle
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (l + LPR * j) * 8;
    float wv[8], bv[8], o[8];
    ld8v(w + c, wv);
    ld8v(b + c, bv);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (v[j][e] - mu) * rs * wv[e] + bv[e];
    st8v(y + base + c, o);
  }
  if (l == 0) {
    mean[r] = mu;
    rstd[r] = rs;
  }
}

// backward: grid-stride over row groups with the next group's operands loaded before the current
// one is reduced; dw/db partials per workgroup (lanes of one wave that hold the same channels are
// folded with shuffles, the 4 waves through LDS, fixed order)
template <typename TDY, typename TX, typename TDX, int LPR, int NV>
__global__ void __launch_bounds__(kLnThreads) ln_bwd_vec_kernel(const TDY* __restrict__ dy, const TX* __restrict__ x,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd,
                                                                const float* __restrict__ w, TDX* __restrict__ dx,
                                                                int accumulate, float* __restrict__ dw_part,
                                                                float* __restrict__ db_part, int64_t rows, int C) {
  constexpr int RPW = 64 / LPR;
  __shared__ float red[kLnThreads / 64][2][8 * LPR * NV];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, l = lane % LPR, sub = lane / LPR;
  const int64_t ngroups = (rows + RPW - 1) / RPW;
  const int64_t nw = (int64_t)gridDim.x * (kLnThreads / 64);
  const float invC = 1.0f / (float)C;
  float wr[NV][8], adw[NV][8], adb[NV][8];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    ld8v(w + (l + LPR * j) * 8, wr[j]);
#pragma unroll
    for (int e = 0; e < 8; ++e) adw[j][e] = adb[j][e] = 0.f;
  }
  float nd[NV][8], nx[NV][8], nmu = 0.f, nrs = 0.f;
  auto load = [&](int64_t g) {
    int64_t r = g * RPW + sub;
    const bool ok = g < ngroups && r < rows;
    if (!ok) r = 0;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      ld8v(dy + (size_t)r * C + (l + LPR * j) * 8, nd[j]);
      ld8v(x + (size_t)r * C + (l + LPR * j) * 8, nx[j]);
      if (!ok) {
#pragma unroll
        for (int e = 0; e < 8; ++e) nd[j][e] = 0.f;  // contributes nothing to dw/db
      }
    }
    nmu = mean[r];
    nrs = rstd[r];
  };
  int64_t g = (int64_t)blockIdx.x * (kLnThreads / 64) + wid;
  load(g);
  for (; g < ngroups; g += nw) {
    float d[NV][8], xh[NV][8];
    const float mu = nmu, rs = nrs;
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        d[j][e] = nd[j][e];
        xh[j][e] = (nx[j][e] - mu) * rs;
      }
    load(g + nw);  // next group in flight while this one is reduced
    const int64_t r = g * RPW + sub;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gg = d[j][e] * wr[j][e];
        s1 += gg;
        s2 += gg * xh[j][e];
        adw[j][e] += d[j][e] * xh[j][e];
        adb[j][e] += d[j][e];
      }
    s1 = group_sum<LPR>(s1) * invC;
    s2 = group_sum<LPR>(s2) * invC;
    if (r < rows) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        TDX* p = dx + (size_t)r * C + (l + LPR * j) * 8;
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = rs * (d[j][e] * wr[j][e] - s1 - xh[j][e] * s2);
        if (accumulate) {
          float old[8];
          ld8v(p, old);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] += old[e];
        }
        st8v(p, o);
      }
    }
  }
  // fold the RPW row slots of this wave (lanes l, l+LPR, ... hold the same channels)
#pragma unroll
  for (int o = LPR; o < 64; o <<= 1)
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        adw[j][e] += __shfl_xor(adw[j][e], o, 64);
        adb[j][e] += __shfl_xor(adb[j][e], o, 64);
      }
  if (sub == 0) {
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[wid][0][(l + LPR * j) * 8 + e] = adw[j][e];
        red[wid][1][(l + LPR * j) * 8 + e] = adb[j][e];
      }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kLnThreads) {
    float sw = 0.f, sb = 0.f;
#pragma unroll
    for (int k = 0; k < kLnThreads / 64; ++k) {
      sw += red[k][0][c];
      sb += red[k][1][c];
    }
    dw_part[(size_t)blockIdx.x * C + c] = sw;
    db_part[(size_t)blockIdx.x * C + c] = sb;
  }
}

// fast-path geometry: C = 8 * LPR * NV; returns LPR*16+NV or 0.  ConvNeXt-base 128..1024 (NV 1, 2, 4)
// and ConvNeXt-large 192/384/768/1536 (NV 3 over LPR 8/16/32/64 lanes)
static int ln_vec_kind(int C) {
  if (C % 8) return 0;
  const int u = C / 8;
  if (u == 16 || u == 32 || u == 64) return u * 16 + 1;
  if (u == 128) return 64 * 16 + 2;
  if (u == 256) return 64 * 16 + 4;
  if (u % 3 == 0 && (u / 3 == 8 || u / 3 == 16 || u / 3 == 32 || u / 3 == 64)) return (u / 3) * 16 + 3;
  return 0;
}
#define SV_LNVEC_SWITCH(KIND, ...)                                           \
  switch (KIND) {                                                            \
    case 16 * 16 + 1: { constexpr int LPR = 16, NV = 1; __VA_ARGS__; } break; \
    case 32 * 16 + 1: { constexpr int LPR = 32, NV = 1; __VA_ARGS__; } break; \
    case 64 * 16 + 1: { constexpr int LPR = 64, NV = 1; __VA_ARGS__; } break; \
    case 64 * 16 + 2: { constexpr int LPR = 64, NV = 2; __VA_ARGS__; } break; \
    case 64 * 16 + 4: { constexpr int LPR = 64, NV = 4; __VA_ARGS__; } break; \
    case 8 * 16 + 3: { constexpr int LPR = 8, NV = 3; __VA_ARGS__; } break;   \
    case 16 * 16 + 3: { constexpr int LPR = 16, NV = 3; __VA_ARGS__; } break; \
    case 32 * 16 + 3: { constexpr int LPR = 32, NV = 3; __VA_ARGS__; } break; \
    case 64 * 16 + 3: { constexpr int LPR = 64, NV = 3; __VA_ARGS__; } break; \
    default: break;                                                          \
  }
static int ln_vec_fwd_grid(int64_t rows, int C) {
  const int rpw = 64 / (ln_vec_kind(C) / 16);
  const int64_t waves = (rows + rpw - 1) / rpw;
  return (int)((waves + kLnThreads / 64 - 1) / (kLnThreads / 64));
}
static int ln_vec_bwd_grid(int64_t rows, int C) {
  const int rpw = 64 / (ln_vec_kind(C) / 16);
  const int64_t groups = (rows + rpw - 1) / rpw;
  // ~8 row groups per wave: enough loop trip for the prefetch, partials stay small
  int64_t g = (groups + 8 * (kLnThreads / 64) - 1) / (8 * (kLnThreads / 64));
  if (g > 2048) g = 2048;
  return (int)(g < 1 ? 1 : g);
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
  // C = 128 (the S1 downsample, 32 patches per wave): the next patch's 4 pixels are loaded while this one is
  // normalised (same arithmetic, bit for bit): 157-158 -> 122 us at bs32; for C = 256 it measured 12 % slower
  // (tools/ds_bench.py, profiles/round3/r5g_ds_prefetch.txt), so wider rows keep one patch in flight
  constexpr bool PF = CPL <= 2;
  auto pixel = [&](int64_t pp, int q) {
    const int j = (int)(pp % Wo), i = (int)((pp / Wo) % Ho), b = (int)(pp / ((int64_t)Wo * Ho));
    return ((int64_t)b * H + 2 * i + (q >> 1)) * W + 2 * j + (q & 1);
  };
  float nv[4][CPL];
  auto load = [&](int64_t pp) {
    if (pp >= np) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float* xr = x + (size_t)pixel(pp, q) * C;
#pragma unroll
      for (int t = 0; t < CPL; ++t) nv[q][t] = xr[lane + 64 * t];
    }
  };
  if (PF) load(wave);
  for (int64_t p = wave; p < np; p += nwaves) {
    float v[4][CPL];
    if (!PF) load(p);
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int t = 0; t < CPL; ++t) v[q][t] = nv[q][t];
    if (PF) load(p + nwaves);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t pix = pixel(p, q);
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < CPL; ++t) s += v[q][t];
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
// Head: global average pool over HW, then LayerNorm over C.
//   pool_sum_kernel   grid (C/64, B): 4 waves split the HW rows of one 64-channel group of one
//                     image (256-B coalesced row reads, 8 in flight per lane), LDS fold -> pooled
//   pool_norm_kernel  grid B: LayerNorm of the pooled [C] vector
//   pool_bwd_kernel   grid (HW/kPoolRows, B): every workgroup re-derives the [C] input gradient of
//                     its image (two block sums over C, cheap) and broadcasts it over its rows
constexpr int kPoolRows = 16;

__global__ void __launch_bounds__(kLnThreads) pool_sum_kernel(const float* __restrict__ x, float* __restrict__ pooled,
                                                              int HW, int C) {
  __shared__ float red[kLnThreads / 64][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int b = blockIdx.y, c = blockIdx.x * 64 + lane;
  const float* xb = x + (size_t)b * HW * C + c;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int p = wid;
  for (; p + 28 < HW; p += 32) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += xb[(size_t)(p + 4 * u) * C];
  }
  for (; p < HW; p += 4) acc[0] += xb[(size_t)p * C];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += acc[u];
  red[wid][lane] = s;
  __syncthreads();
  if (wid == 0) pooled[(size_t)b * C + c] = (red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]) / (float)HW;
}

__global__ void __launch_bounds__(kLnThreads) pool_norm_kernel(const float* __restrict__ pooled,
                                                               const float* __restrict__ lnw,
                                                               const float* __restrict__ lnb, float eps,
                                                               float* __restrict__ feat, float* __restrict__ mean,
                                                               float* __restrict__ rstd, int C) {
  __shared__ float red[kLnThreads / 64];
  const int b = blockIdx.x;
  const float* pb = pooled + (size_t)b * C;
  const float invC = 1.0f / (float)C;
  float s = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) s += pb[c];
  const float mu = block_sum(s, red) * invC;
  float q = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) q += (pb[c] - mu) * (pb[c] - mu);
  const float rs = rsqrtf(block_sum(q, red) * invC + eps);
  for (int c = threadIdx.x; c < C; c += blockDim.x) feat[(size_t)b * C + c] = (pb[c] - mu) * rs * lnw[c] + lnb[c];
  if (threadIdx.x == 0) {
    mean[b] = mu;
    rstd[b] = rs;
  }
}

__global__ void __launch_bounds__(kLnThreads) pool_bwd_kernel(
    const float* __restrict__ dfeat, const float* __restrict__ pooled, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ lnw, float* __restrict__ dx,
    uint16_t* __restrict__ dx_bf16, float* __restrict__ dlnw_part, float* __restrict__ dlnb_part, int HW, int C) {
  __shared__ float red[kLnThreads / 64];
  extern __shared__ __attribute__((aligned(16))) float dp[];  // [C]
  const int b = blockIdx.y;
  const float mu = mean[b], rs = rstd[b];
  const float invC = 1.0f / (float)C, invHW = 1.0f / (float)HW;
  const bool first = blockIdx.x == 0;
  float s1 = 0.f, s2 = 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float d = dfeat[(size_t)b * C + c];
    const float xh = (pooled[(size_t)b * C + c] - mu) * rs;
    const float g = d * lnw[c];
    s1 += g;
    s2 += g * xh;
    if (first) {
      dlnw_part[(size_t)b * C + c] = d * xh;
      dlnb_part[(size_t)b * C + c] = d;
    }
  }
  s1 = block_sum(s1, red) * invC;
  s2 = block_sum(s2, red) * invC;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    const float xh = (pooled[(size_t)b * C + c] - mu) * rs;
    const float g = dfeat[(size_t)b * C + c] * lnw[c];
    dp[c] = rs * (g - s1 - xh * s2) * invHW;
  }
  __syncthreads();
  const int p0 = blockIdx.x * kPoolRows;
  const int p1 = p0 + kPoolRows < HW ? p0 + kPoolRows : HW;
  const size_t base = ((size_t)b * HW + p0) * C;
  const size_t n4 = (size_t)(p1 - p0) * C / 4;  // C % 4 == 0
  for (size_t i = threadIdx.x; i < n4; i += blockDim.x) {
    const int c = (int)((i * 4) % C);
    const float4 v = *reinterpret_cast<const float4*>(dp + c);
    *reinterpret_cast<float4*>(dx + base + i * 4) = v;
    if (dx_bf16) st4(dx_bf16, base + i * 4, v);
  }
}

// the two butterfly forms side by side (sv_diag_group_sum: the test of xlane_group_sum's bitwise claim)
template <int LPR>
__global__ void __launch_bounds__(256) diag_group_sum_kernel(const float* __restrict__ in, float* __restrict__ xl,
                                                             float* __restrict__ sh, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // n % 256 == 0: whole waves
  const float v = in[i];
  float t = v;
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  xl[i] = xlane_group_sum<LPR>(v);
  sh[i] = t;
  (void)n;
}

}  // namespace sv

using namespace sv;

extern "C" {

int sv_diag_group_sum(const float* in, float* xlane, float* shuffle, int64_t n, int32_t lanes, sv_stream_t stream) {
  SV_REQUIRE(in && xlane && shuffle && n > 0 && n % 256 == 0, "sv_diag_group_sum: n must be a positive multiple of 256");
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = (unsigned)(n / 256);
  if (lanes == 16) diag_group_sum_kernel<16><<<grid, 256, 0, s>>>(in, xlane, shuffle, n);
  else if (lanes == 32) diag_group_sum_kernel<32><<<grid, 256, 0, s>>>(in, xlane, shuffle, n);
  else if (lanes == 64) diag_group_sum_kernel<64><<<grid, 256, 0, s>>>(in, xlane, shuffle, n);
  else return set_error(SV_ERR_INVALID_ARG, "sv_diag_group_sum: lanes must be 16, 32 or 64");
  return check_launch("sv_diag_group_sum");
}

int sv_layernorm_fwd(const void* x, int32_t x_dtype, const float* w, const float* b, void* y,
                     int32_t y_dtype, float* mean, float* rstd, int64_t rows, int32_t C, float eps,
                     sv_stream_t stream) {
  SV_REQUIRE(x && w && b && y && mean && rstd, "sv_layernorm_fwd: null pointer");
  SV_REQUIRE(ln_vec_kind(C) || cpl_ok(C), "sv_layernorm_fwd: C=%d must be 64*{1,2,3,4,6,8,12,16,24} or 2048", C);
  if (rows <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  if (const int kind = ln_vec_kind(C)) {
    const int vg = ln_vec_fwd_grid(rows, C);
#define LAUNCHV(TX, TY)                                                                                    \
  SV_LNVEC_SWITCH(kind, ln_fwd_vec_kernel<TX, TY, LPR, NV><<<vg, kLnThreads, 0, s>>>((const TX*)x, w, b, (TY*)y, \
                                                                                      mean, rstd, rows, C, eps))
    if (x_dtype == SV_F32 && y_dtype == SV_F32) { LAUNCHV(float, float); }
    else if (x_dtype == SV_F32 && y_dtype == SV_BF16) { LAUNCHV(float, uint16_t); }
    else if (x_dtype == SV_BF16 && y_dtype == SV_F32) { LAUNCHV(uint16_t, float); }
    else if (x_dtype == SV_BF16 && y_dtype == SV_BF16) { LAUNCHV(uint16_t, uint16_t); }
    else return set_error(SV_ERR_INVALID_ARG, "sv_layernorm_fwd: bad dtype");
#undef LAUNCHV
    return check_launch("sv_layernorm_fwd");
  }
  const int grid = ln_grid(rows);
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

int sv_layernorm_bwd_nparts(int64_t rows, int32_t C) {
  return ln_vec_kind(C) ? ln_vec_bwd_grid(rows, C) : ln_grid(rows);
}

int sv_layernorm_bwd(const void* dy, int32_t dy_dtype, const void* x, int32_t x_dtype, const float* mean,
                     const float* rstd, const float* w, void* dx, int32_t dx_dtype, int32_t accumulate,
                     float* dw_part, float* db_part, int64_t rows, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(dy && x && mean && rstd && w && dx && dw_part && db_part, "sv_layernorm_bwd: null pointer");
  SV_REQUIRE(ln_vec_kind(C) || (cpl_ok(C) && C <= 2048), "sv_layernorm_bwd: C=%d unsupported", C);
  if (rows <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  if (const int kind = ln_vec_kind(C)) {
    const int vg = ln_vec_bwd_grid(rows, C);
#define LNBV(TDY, TX, TDX)                                                                                  \
  SV_LNVEC_SWITCH(kind, ln_bwd_vec_kernel<TDY, TX, TDX, LPR, NV><<<vg, kLnThreads, 0, s>>>(                 \
                            (const TDY*)dy, (const TX*)x, mean, rstd, w, (TDX*)dx, accumulate, dw_part, db_part, \
                            rows, C))
    if (dy_dtype == SV_F32 && x_dtype == SV_F32 && dx_dtype == SV_F32) { LNBV(float, float, float); }
    else if (dy_dtype == SV_F32 && x_dtype == SV_BF16 && dx_dtype == SV_F32) { LNBV(float, uint16_t, float); }
    else if (dy_dtype == SV_F32 && x_dtype == SV_BF16 && dx_dtype == SV_BF16) { LNBV(float, uint16_t, uint16_t); }
    else if (dy_dtype == SV_BF16 && x_dtype == SV_BF16 && dx_dtype == SV_F32) { LNBV(uint16_t, uint16_t, float); }
    else if (dy_dtype == SV_BF16 && x_dtype == SV_BF16 && dx_dtype == SV_BF16) { LNBV(uint16_t, uint16_t, uint16_t); }
    else return set_error(SV_ERR_UNSUPPORTED, "sv_layernorm_bwd: dtype combination (dy %d, x %d, dx %d) unsupported",
                          dy_dtype, x_dtype, dx_dtype);
#undef LNBV
    return check_launch("sv_layernorm_bwd");
  }
  const int grid = ln_grid(rows);
#define LNB(TDY, TX, TDX)                                                                              \
  SV_CPL_SWITCH(C / 64, ln_bwd_kernel<TDY, TX, TDX, CPL><<<grid, kLnThreads, 0, s>>>(                 \
                            (const TDY*)dy, (const TX*)x, mean, rstd, w, (TDX*)dx, accumulate, dw_part, \
                            db_part, rows, C))
  if (dy_dtype == SV_F32 && x_dtype == SV_F32 && dx_dtype == SV_F32) {
    LNB(float, float, float);
  } else if (dy_dtype == SV_F32 && x_dtype == SV_BF16 && dx_dtype == SV_F32) {
    LNB(float, uint16_t, float);
  } else if (dy_dtype == SV_F32 && x_dtype == SV_BF16 && dx_dtype == SV_BF16) {
    LNB(float, uint16_t, uint16_t);
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
  SV_REQUIRE(C % 64 == 0, "sv_pool_ln_fwd: C=%d must be a multiple of 64", C);
  if (B <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  pool_sum_kernel<<<dim3(C / 64, B), kLnThreads, 0, s>>>(x, pooled, HW, C);
  pool_norm_kernel<<<B, kLnThreads, 0, s>>>(pooled, lnw, lnb, eps, feat, mean, rstd, C);
  return check_launch("sv_pool_ln_fwd");
}

int sv_pool_ln_bwd(const float* dfeat, const float* pooled, const float* mean, const float* rstd,
                   const float* lnw, float* dx, uint16_t* dx_bf16, float* dlnw_part, float* dlnb_part, int32_t B,
                   int32_t HW, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(dfeat && pooled && mean && rstd && lnw && dx && dlnw_part && dlnb_part,
             "sv_pool_ln_bwd: null pointer");
  SV_REQUIRE(C % 4 == 0, "sv_pool_ln_bwd: C=%d must be a multiple of 4", C);
  if (B <= 0) return SV_OK;
  pool_bwd_kernel<<<dim3(ceil_div(HW, kPoolRows), B), kLnThreads, C * sizeof(float), (hipStream_t)stream>>>(
      dfeat, pooled, mean, rstd, lnw, dx, dx_bf16, dlnw_part, dlnb_part, HW, C);
  return check_launch("sv_pool_ln_bwd");
}

}  // extern "C"
