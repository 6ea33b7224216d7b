// Implicit-GEMM convolution on MFMA for the ResNet-18/50 classification backbone (gfx950).
//
// Replaces the cuDNN convolutions timm's ResNet (BasicBlock / Bottleneck, stem conv7x7/s2, 1x1
// downsample) runs under the reference (spine_vision/training/models/backbone.py:166 ->
// timm/models/resnet.py) and their autograd data / weight gradients.  Nothing is materialised: the
// im2col matrix exists only as the per-chunk address arithmetic of the operand loaders.
//
//   FPROP  y[m = (b,oy,ox)][co]  = sum_{t,c} x[b, oy*s + kh_t - p, ox*s + kw_t - p, c] * wp[co][t][c]
//          A = gathered activations (K-major, k = t*Cs + c), B = packed weight (K-major)
//   DGRAD  dx[b, oy*so+py, ox*so+px][c] = sum_{j,co} dy[b, oy + dy_j, ox + dx_j, co] * wp[co][t_j][c]
//          one launch per output parity class (py, px) of a stride-2 conv: every tap of the class
//          hits a real dy pixel, so no MFMA work is spent on the zeros of the transposed conv;
//          A = gathered gradient (K-major, k = j*Cout + co), B = weight read N-contiguous
//   WGRAD  dw[co][t][c] = sum_pix dy[pix][co] * x[gather(pix, t)][c]
//          A = dy (M-contiguous: the pixel-major NHWC gradient), B = gathered activations
//          (N-contiguous), split-K over pixels into f32 slabs, reduced + permuted to torch layout.
//
// Tiles: the v1 register-staged MFMA structure (mfma_v1.h): 128x128 per 256-thread workgroup,
// 4 waves of 64x64, BK = 32, double-buffered padded LDS images, bf16 (16x16x32) or exact f32
// (16x16x4) MFMA; channel counts are powers of two so tap/channel split of k is a shift and a mask.
// Padding / out-of-image taps are zero-filled in registers.  XCD-aware tile order.
#include "common.h"
#include "gemm_common.h"
#include "mfma_v1.h"

#include <stdlib.h>

#include <type_traits>

namespace sv {
namespace conv {

enum { FPROP = 0, DGRAD = 1, WGRAD = 2 };
constexpr int MAX_TAPS = 64;

// unsigned division by a run-time constant d >= 1 (n < 2^31): q = (umulhi(n, mul) + n) >> shift
struct FastDiv {
  uint32_t d, mul, shift;
};
static FastDiv make_fastdiv(uint32_t d) {
  FastDiv f{d, 0, 0};
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.shift = l;
  f.mul = (uint32_t)((((1ull << l) - d) << 32) / d + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (uint32_t)(((uint64_t)__umulhi(n, f.mul) + n) >> f.shift);
}

struct Args {
  const void* A;
  const void* B;
  int M, N, K;
  int64_t lda, ldb;
  // gather source image [Bn][SH][SW][SC] and the pixel grid the gathered operand is indexed by
  int SH, SW, SC, lsc;  // lsc = log2(SC)
  int GH, GW;           // grid of the decoded index (FPROP/DGRAD: GEMM rows; WGRAD: k)
  FastDiv dGW, dGHW;
  int si;               // source step per grid step
  int ntaps;
  int8_t tdy[MAX_TAPS], tdx[MAX_TAPS];
  uint8_t twt[MAX_TAPS];  // DGRAD: weight tap of gather tap j
  int Tw;                 // DGRAD: taps per output channel in wp
  // epilogue
  void* C;
  int c_dtype;
  int accumulate;
  int so, py, px, DH, DW;  // DGRAD scatter of GEMM row (b,oy,ox) -> pixel (b, oy*so+py, ox*so+px)
  int kper;
};

// ---- operand stages (register-staged, 16-B chunks: 8 bf16 or 4 f32) ----------------------------
template <bool BF16>
struct Chunks {
  static constexpr int EPC = BF16 ? 8 : 4;
  static constexpr int PER_THREAD = BM * BKT / EPC / kGemmThreads;
};

template <typename T>
__device__ __forceinline__ uint4 load16(const T* p) {
  return *reinterpret_cast<const uint4*>(p);
}

// A of FPROP / DGRAD: rows = gathered pixels, K-major.
template <bool BF16, typename T>
struct StageGatherK {
  using CH = Chunks<BF16>;
  uint4 r[CH::PER_THREAD];
  int boff[CH::PER_THREAD], iy0[CH::PER_THREAD], ix0[CH::PER_THREAD];

  __device__ __forceinline__ void init(const Args& a, int m0) {
#pragma unroll
    for (int s = 0; s < CH::PER_THREAD; ++s) {
      const int q = threadIdx.x + kGemmThreads * s;
      const int m = m0 + q / (BKT / CH::EPC);
      if (m < a.M) {
        const uint32_t b = fdiv((uint32_t)m, a.dGHW);
        const uint32_t rem = (uint32_t)m - b * (uint32_t)(a.GH * a.GW);
        const uint32_t oy = fdiv(rem, a.dGW);
        const uint32_t ox = rem - oy * (uint32_t)a.GW;
        boff[s] = (int)b * a.SH;
        iy0[s] = (int)oy * a.si;
        ix0[s] = (int)ox * a.si;
      } else {
        boff[s] = -1;
        iy0[s] = ix0[s] = 0;
      }
    }
  }
  __device__ __forceinline__ void load(const Args& a, int k0) {
    const T* X = reinterpret_cast<const T*>(a.A);
#pragma unroll
    for (int s = 0; s < CH::PER_THREAD; ++s) {
      const int q = threadIdx.x + kGemmThreads * s;
      const int k = k0 + (q % (BKT / CH::EPC)) * CH::EPC;
      const int j = k >> a.lsc, c = k & (a.SC - 1);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (boff[s] >= 0 && k < a.K && j < a.ntaps) {
        const int iy = iy0[s] + a.tdy[j], ix = ix0[s] + a.tdx[j];
        if ((unsigned)iy < (unsigned)a.SH && (unsigned)ix < (unsigned)a.SW)
          v = load16(X + ((int64_t)(boff[s] + iy) * a.SW + ix) * a.SC + c);
      }
      r[s] = v;
    }
  }
};

// B of FPROP: packed weight [N][K] (K-major), or A of WGRAD (dy: [K][M], M-major): plain operands.
template <bool BF16, typename T, bool KMAJ>
struct StagePlain {
  using CH = Chunks<BF16>;
  uint4 r[CH::PER_THREAD];
  __device__ __forceinline__ void load(const T* __restrict__ p, int64_t ld, int row0, int k0, int R, int K) {
#pragma unroll
    for (int s = 0; s < CH::PER_THREAD; ++s) {
      const int q = threadIdx.x + kGemmThreads * s;
      int row, kk;
      if (KMAJ) {
        row = q / (BKT / CH::EPC);
        kk = (q % (BKT / CH::EPC)) * CH::EPC;
      } else {
        kk = q / (BM / CH::EPC);
        row = (q % (BM / CH::EPC)) * CH::EPC;
      }
      const int gr = row0 + row, gk = k0 + kk;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (gr < R && gk < K) v = load16(KMAJ ? p + (int64_t)gr * ld + gk : p + (int64_t)gk * ld + gr);
      r[s] = v;
    }
  }
};

// B of DGRAD: B(k = j*Cout + co, n = c) = wp[(co*Tw + t_j)*N + c]  (N-contiguous)
template <bool BF16, typename T>
struct StageWeightN {
  using CH = Chunks<BF16>;
  uint4 r[CH::PER_THREAD];
  __device__ __forceinline__ void load(const Args& a, int n0, int k0) {
    const T* W = reinterpret_cast<const T*>(a.B);
#pragma unroll
    for (int s = 0; s < CH::PER_THREAD; ++s) {
      const int q = threadIdx.x + kGemmThreads * s;
      const int k = k0 + q / (BN / CH::EPC);
      const int n = n0 + (q % (BN / CH::EPC)) * CH::EPC;
      const int j = k >> a.lsc, co = k & (a.SC - 1);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (k < a.K && n < a.N) v = load16(W + ((int64_t)co * a.Tw + a.twt[j]) * a.N + n);
      r[s] = v;
    }
  }
};

// B of WGRAD: B(k = pix, n = t*SC + c) = x[b, oy*si + dy_t, ox*si + dx_t, c]  (N-contiguous)
template <bool BF16, typename T>
struct StageGatherN {
  using CH = Chunks<BF16>;
  uint4 r[CH::PER_THREAD];
  __device__ __forceinline__ void load(const Args& a, int n0, int k0) {
    const T* X = reinterpret_cast<const T*>(a.B);
#pragma unroll
    for (int s = 0; s < CH::PER_THREAD; ++s) {
      const int q = threadIdx.x + kGemmThreads * s;
      const int k = k0 + q / (BN / CH::EPC);
      const int n = n0 + (q % (BN / CH::EPC)) * CH::EPC;
      const int t = n >> a.lsc, c = n & (a.SC - 1);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (k < a.K && n < a.N && t < a.ntaps) {
        const uint32_t b = fdiv((uint32_t)k, a.dGHW);
        const uint32_t rem = (uint32_t)k - b * (uint32_t)(a.GH * a.GW);
        const uint32_t oy = fdiv(rem, a.dGW);
        const uint32_t ox = rem - oy * (uint32_t)a.GW;
        const int iy = (int)oy * a.si + a.tdy[t], ix = (int)ox * a.si + a.tdx[t];
        if ((unsigned)iy < (unsigned)a.SH && (unsigned)ix < (unsigned)a.SW)
          v = load16(X + (((int64_t)b * a.SH + iy) * a.SW + ix) * a.SC + c);
      }
      r[s] = v;
    }
  }
};

// registers -> LDS image (same images as the v1 GEMM)
template <bool BF16, bool KMAJ, int PT>
__device__ __forceinline__ void store_img(const uint4 (&r)[PT], char* __restrict__ img) {
  constexpr int EPC = BF16 ? 8 : 4, ES = BF16 ? 2 : 4;
  constexpr int LD = Img<BF16, KMAJ>::LD;
#pragma unroll
  for (int s = 0; s < PT; ++s) {
    const int q = threadIdx.x + kGemmThreads * s;
    if (KMAJ) {
      const int row = q / (BKT / EPC), kk = (q % (BKT / EPC)) * EPC;
      *reinterpret_cast<uint4*>(img + ((size_t)row * LD + kk) * ES) = r[s];
    } else {
      const int kk = q / (BM / EPC), row = (q % (BM / EPC)) * EPC;
      *reinterpret_cast<uint4*>(img + ((size_t)kk * LD + row) * ES) = r[s];
    }
  }
}

// ---- epilogue: 16-row LDS slabs re-read as 8-column units (16-B / 32-B row-contiguous stores) ----
template <int MODE>
__device__ __forceinline__ void epilogue(const f32x4 (&acc)[4][4], float* __restrict__ slab, int mb, int nb,
                                         const Args& a, int split) {
  const int l = threadIdx.x & 63;
  const int cu = (l & 7) * 8, r0 = l >> 3;
  const int n = nb + cu;
  const bool okn = n < a.N, okn4 = n + 4 < a.N;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[(4 * (l >> 4) + r) * EPI_LD + j * 16 + (l & 15)] = acc[i][j][r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = r0 + 8 * h;
      const int m = mb + i * 16 + row;
      if (m >= a.M || !okn) continue;
      const float* sp = slab + row * EPI_LD + cu;
      float4 va = make_float4(sp[0], sp[1], sp[2], sp[3]);
      float4 vb = make_float4(sp[4], sp[5], sp[6], sp[7]);
      size_t ci;
      if (MODE == WGRAD) {
        float* C = reinterpret_cast<float*>(a.C) + (size_t)split * a.M * a.N + (size_t)m * a.N + n;
        *reinterpret_cast<float4*>(C) = va;
        if (okn4) *reinterpret_cast<float4*>(C + 4) = vb;
        continue;
      } else if (MODE == FPROP) {
        ci = (size_t)m * a.N + n;
      } else {
        const uint32_t b = fdiv((uint32_t)m, a.dGHW);
        const uint32_t rem = (uint32_t)m - b * (uint32_t)(a.GH * a.GW);
        const uint32_t oy = fdiv(rem, a.dGW);
        const uint32_t ox = rem - oy * (uint32_t)a.GW;
        const size_t pix = ((size_t)b * a.DH + oy * a.so + a.py) * a.DW + ox * a.so + a.px;
        ci = pix * a.N + n;
        if (a.accumulate) {
          float4 xa, xb = make_float4(0.f, 0.f, 0.f, 0.f);
          if (okn4) ld8_any(a.C, a.c_dtype, ci, xa, xb);
          else xa = ld4_any(a.C, a.c_dtype, ci);
          va = add4(va, xa);
          vb = add4(vb, xb);
        }
      }
      if (okn4) st8_any(a.C, a.c_dtype, ci, va, vb);
      else st4_any(a.C, a.c_dtype, ci, va);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
}

template <bool BF16, int MODE>
__global__ void __launch_bounds__(kGemmThreads) conv_kernel(const Args a, int tilesM, int tilesN) {
  using T = typename std::conditional<BF16, uint16_t, float>::type;
  constexpr bool AK = MODE != WGRAD;   // A K-major (gathered pixels) except WGRAD (dy, M-contiguous)
  constexpr bool BKM = MODE == FPROP;  // B K-major only for the packed weight of FPROP
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ABYTES = Img<BF16, AK>::BYTES, BBYTES = Img<BF16, BKM>::BYTES;
  constexpr int STAGE_BYTES = ABYTES + BBYTES;
  constexpr int PT = Chunks<BF16>::PER_THREAD;

  const int nwg = tilesM * tilesN;
  const int pid = blockIdx.x;
  const int xcd = pid & 7, loc = pid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tm = wg / tilesN, tn = wg % tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int split = blockIdx.z;
  const int kbeg = split * a.kper;
  int kend = kbeg + a.kper;
  if (kend > a.K) kend = a.K;
  const int nk = kend > kbeg ? (kend - kbeg + BKT - 1) / BKT : 0;

  const int wid = threadIdx.x >> 6, wm = wid >> 1, wn = wid & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  StageGatherK<BF16, T> ga;      // FPROP / DGRAD A
  StagePlain<BF16, T, false> pa;  // WGRAD A
  StagePlain<BF16, T, true> pb;   // FPROP B
  StageWeightN<BF16, T> wb;       // DGRAD B
  StageGatherN<BF16, T> gb;       // WGRAD B
  if (MODE != WGRAD) ga.init(a, m0);

  auto load = [&](int k0) {
    if constexpr (MODE == WGRAD) {
      pa.load(reinterpret_cast<const T*>(a.A), a.lda, m0, k0, a.M, kend);
      gb.load(a, n0, k0);
    } else {
      ga.load(a, k0);
      if constexpr (MODE == FPROP) pb.load(reinterpret_cast<const T*>(a.B), a.ldb, n0, k0, a.N, a.K);
      else wb.load(a, n0, k0);
    }
  };
  auto store = [&](char* st) {
    if constexpr (MODE == WGRAD) {
      store_img<BF16, AK, PT>(pa.r, st);
      store_img<BF16, BKM, PT>(gb.r, st + ABYTES);
    } else {
      store_img<BF16, AK, PT>(ga.r, st);
      if constexpr (MODE == FPROP) store_img<BF16, BKM, PT>(pb.r, st + ABYTES);
      else store_img<BF16, BKM, PT>(wb.r, st + ABYTES);
    }
  };

  if (nk > 0) {
    load(kbeg);
    store(smem);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE_BYTES;
    char* nxt = smem + ((kt + 1) & 1) * STAGE_BYTES;
    const bool more = kt + 1 < nk;
    if (more) load(kbeg + (kt + 1) * BKT);
    const char* ai = cur;
    const char* bi = cur + ABYTES;
    if constexpr (BF16) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag_bf16<AK>(ai, wm * 64 + i * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag_bf16<BKM>(bi, wn * 64 + j * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < BKT; kk += 4) {
        float af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = frag_f32<AK>(ai, wm * 64 + i * 16, kk);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = frag_f32<BKM>(bi, wn * 64 + j * 16, kk);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) store(nxt);
    __syncthreads();
  }
  epilogue<MODE>(acc, reinterpret_cast<float*>(smem) + wid * 16 * EPI_LD, m0 + wm * 64, n0 + wn * 64, a, split);
}

template <bool BF16, int MODE>
static int launch(const Args& a, int split, hipStream_t s) {
  const int tilesM = ceil_div(a.M, BM), tilesN = ceil_div(a.N, BN);
  constexpr bool AK = MODE != WGRAD, BKM = MODE == FPROP;
  constexpr size_t main_lds = 2 * (size_t)(Img<BF16, AK>::BYTES + Img<BF16, BKM>::BYTES);
  constexpr size_t epi_lds = 4 * 16 * EPI_LD * sizeof(float);
  constexpr size_t lds = main_lds > epi_lds ? main_lds : epi_lds;
  static_assert(lds <= 160 * 1024, "conv kernel LDS");
  if (const int rc_ = ensure_lds_attr(reinterpret_cast<const void*>(&conv_kernel<BF16, MODE>), (int)lds, s)) return rc_;
  dim3 grid(tilesM * tilesN, 1, split);
  conv_kernel<BF16, MODE><<<grid, kGemmThreads, lds, s>>>(a, tilesM, tilesN);
  return check_launch(MODE == FPROP ? "sv_conv_fwd" : MODE == DGRAD ? "sv_conv_bwd_data" : "sv_conv_bwd_weight");
}

template <int MODE>
static int launch_dt(const Args& a, int dtype, int split, hipStream_t s) {
  return dtype == SV_BF16 ? launch<true, MODE>(a, split, s) : launch<false, MODE>(a, split, s);
}

// ---- small helper kernels --------------------------------------------------------------------
template <typename T>
__global__ void weight_pack_kernel(const float* __restrict__ w, T* __restrict__ wp, int Cout, int Cin, int T_,
                                   int Cs) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over wp [Cout][T][Cs]
  const int64_t n = (int64_t)Cout * T_ * Cs;
  if (i >= n) return;
  const int c = (int)(i % Cs);
  const int t = (int)((i / Cs) % T_);
  const int co = (int)(i / ((int64_t)Cs * T_));
  const float v = c < Cin ? w[((int64_t)co * Cin + c) * T_ + t] : 0.f;
  st(wp, (size_t)i, v);
}

template <typename T>
__global__ void image_to_nhwc_kernel(const float* __restrict__ img, T* __restrict__ out, int C, int H, int W, int Cs,
                                     int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over out [B][H][W][Cs]
  if (i >= n) return;
  const int c = (int)(i % Cs);
  const int64_t pix = i / Cs;
  const int64_t hw = pix % ((int64_t)H * W), b = pix / ((int64_t)H * W);
  const float v = c < C ? img[(b * C + c) * H * W + hw] : 0.f;
  st(out, (size_t)i, v);
}

// uint8 HWC crops -> normalised NHWC stem operand: one thread per 4 pixels (12 input bytes as three
// aligned dwords, 4 x Cs output channels as 16-B stores).  Same arithmetic as torchvision's CPU
// ToTensor (x / 255) then Normalize ((x - mean) / std), in f32.
template <typename T, int CS>
__global__ void __launch_bounds__(256) image_u8_hwc_kernel(const uint8_t* __restrict__ img, float m0, float m1,
                                                           float m2, float s0, float s1, float s2,
                                                           T* __restrict__ out, int64_t n4) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= n4) return;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(img) + t * 3;
  const uint32_t w[3] = {src[0], src[1], src[2]};
  const float ms[3] = {m0, m1, m2}, ss[3] = {s0, s1, s2};
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    float v[CS];
#pragma unroll
    for (int c = 0; c < CS; ++c) {
      if (c < 3) {
        const int byte = 3 * p + c;
        const uint32_t u = (w[byte >> 2] >> (8 * (byte & 3))) & 0xffu;
        v[c] = ((float)u / 255.0f - ms[c]) / ss[c];
      } else {
        v[c] = 0.f;
      }
    }
    const size_t o = (size_t)(t * 4 + p) * CS;
#pragma unroll
    for (int c = 0; c < CS; c += 4) st4(out, o + c, make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]));
  }
}

// dw[co][c][t] (+)= sum_s slab[s][co][t*Cs + c]   (c < Cin)
// One thread per slab element, in slab order [Cout][T][Cs] (c fastest): the split x reads -- the bulk
// of the traffic -- are coalesced; only the single write per element is strided (by T, torch layout).
__global__ void wgrad_finish_kernel(const float* __restrict__ slab, int split, int Cout, int Cin, int T_, int Cs,
                                    float* __restrict__ dw, int accumulate) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over slab [Cout][T][Cs]
  const int64_t MN = (int64_t)Cout * T_ * Cs;
  if (i >= MN) return;
  const int c = (int)(i % Cs);
  if (c >= Cin) return;  // padded channels
  const int t = (int)((i / Cs) % T_);
  const int co = (int)(i / ((int64_t)Cs * T_));
  float s = 0.f;
  for (int p = 0; p < split; ++p) s += slab[p * MN + i];
  const int64_t o = ((int64_t)co * Cin + c) * T_ + t;
  dw[o] = accumulate ? dw[o] + s : s;
}

// transposed-slab form (CONV 4): dw[co][c][t] (+)= sum_s slab[s][t*Cs + c][co].  A workgroup owns 64
// consecutive slab elements (lane = element: 256-B coalesced loads) and its 4 waves take every 4th split
// (4 loads in flight each), folded through LDS in a fixed order; the split sums were a serial chain per
// thread over up to ~170 slabs on 100-150 workgroups (42-61 us for 25 MB).
__global__ void __launch_bounds__(256) wgrad_finish_t_kernel(const float* __restrict__ slab, int split, int Cout,
                                                             int Cin, int T_, int Cs, float* __restrict__ dw,
                                                             int accumulate) {
  __shared__ float red[4][64];
  const int64_t n = (int64_t)Cout * T_ * Cs;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (i < n) {
    int q = w;
    for (; q + 12 < split; q += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += slab[(size_t)(q + 4 * u) * n + i];
    }
    for (; q < split; q += 4) a[0] += slab[(size_t)q * n + i];
  }
  red[w][lane] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (w != 0 || i >= n) return;
  const float s = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
  const int co = (int)(i % Cout);
  const int m = (int)(i / Cout);
  const int c = m % Cs, t = m / Cs;
  if (c >= Cin) return;
  float* o = dw + ((size_t)co * Cin + c) * T_ + t;
  *o = accumulate ? *o + s : s;
}

// stride-2 dgrad on the gathered GEMM: each output parity class (py, px) was computed into its own
// compact f32 slab region [split][B*GHc*GWc][Cs]; this pass sums the splits and scatters the rows back
// into dx [B][H][W][Cs] (+= when accumulating).  One thread per 4 channels, dx in natural order.
struct ClassSlabs {
  const float* base[4];  // nullptr: the class receives no gradient (1x1 stride 2: three of the four)
  int GH[4], GW[4];
};
template <typename T>
__global__ void __launch_bounds__(256) dgrad_s2_scatter_kernel(ClassSlabs cs, int split, int B, int H, int W, int Cs,
                                                               T* __restrict__ dx, int accumulate) {
  const int64_t n4 = (int64_t)B * H * W * Cs / 4;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int c = (int)((i * 4) % Cs);
  const int64_t pix = i * 4 / Cs;
  const int x = (int)(pix % W);
  const int64_t by = pix / W;
  const int y = (int)(by % H), b = (int)(by / H);
  const int cls = ((y & 1) << 1) | (x & 1);
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* sb = cs.base[cls];
  if (!sb && accumulate) return;  // a class without taps adds nothing (1x1 stride 2: three of four)
  if (sb) {
    const int64_t rows = (int64_t)B * cs.GH[cls] * cs.GW[cls];
    const int64_t r = ((int64_t)b * cs.GH[cls] + (y >> 1)) * cs.GW[cls] + (x >> 1);
    for (int q = 0; q < split; ++q) {
      const float4 u = *reinterpret_cast<const float4*>(sb + ((size_t)q * rows + r) * Cs + c);
      v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
  }
  const size_t o = (size_t)pix * Cs + c;
  if (accumulate) {
    const float4 d = ld4(dx, o);
    v.x += d.x; v.y += d.y; v.z += d.z; v.w += d.w;
  }
  st4(dx, o, v);
}

// ---- host helpers -----------------------------------------------------------------------------
static bool pow2(int v) { return v > 0 && (v & (v - 1)) == 0; }
static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}
static int out_dim(int in, int k, int s, int p) { return (in + 2 * p - k) / s + 1; }

static int check_shape(const sv_conv_shape* s, int dtype, const char* who) {
  SV_REQUIRE(s, "%s: null shape", who);
  SV_REQUIRE(dtype == SV_BF16 || dtype == SV_F32, "%s: dtype must be SV_BF16 or SV_F32", who);
  const int epc = dtype == SV_BF16 ? 8 : 4;
  SV_REQUIRE(s->B > 0 && s->H > 0 && s->W > 0 && s->KH > 0 && s->KW > 0 && s->stride > 0 && s->pad >= 0,
             "%s: bad geometry", who);
  SV_REQUIRE(pow2(s->Cs) && s->Cs >= epc, "%s: stored channels Cs=%d must be a power of two >= %d", who, s->Cs, epc);
  SV_REQUIRE(s->Cin > 0 && s->Cin <= s->Cs, "%s: Cin=%d must be in [1, Cs=%d]", who, s->Cin, s->Cs);
  SV_REQUIRE(s->Cout > 0 && s->Cout % 8 == 0, "%s: Cout=%d must be a multiple of 8", who, s->Cout);
  SV_REQUIRE(s->KH * s->KW <= MAX_TAPS, "%s: at most %d taps", who, MAX_TAPS);
  SV_REQUIRE(s->stride <= 2, "%s: stride must be 1 or 2", who);
  const int OH = out_dim(s->H, s->KH, s->stride, s->pad), OW = out_dim(s->W, s->KW, s->stride, s->pad);
  SV_REQUIRE(OH > 0 && OW > 0, "%s: empty output", who);
  SV_REQUIRE((int64_t)s->B * s->H * s->W * s->Cs < (1ll << 31) &&
                 (int64_t)s->B * OH * OW * (s->Cout > s->Cs ? s->Cout : s->Cs) < (1ll << 31),
             "%s: tensor too large for 32-bit pixel indexing", who);
  return SV_OK;
}

static void set_grid(Args& a, int GH, int GW) {
  a.GH = GH;
  a.GW = GW;
  a.dGW = make_fastdiv((uint32_t)GW);
  a.dGHW = make_fastdiv((uint32_t)(GH * GW));
}

static int wgrad_split(const sv_conv_shape* s) {
  const int OH = out_dim(s->H, s->KH, s->stride, s->pad), OW = out_dim(s->W, s->KW, s->stride, s->pad);
  const int64_t K = (int64_t)s->B * OH * OW;
  const int tiles = ceil_div(s->Cout, BM) * ceil_div((int64_t)s->KH * s->KW * s->Cs, BN);
  int split = ceil_div(768, tiles);
  const int64_t maxs = K / 256 > 0 ? K / 256 : 1;  // >= 256 pixels (8 k-steps) per split
  if (split > maxs) split = (int)maxs;
  if (split > 256) split = 256;
  return split < 1 ? 1 : split;
}

// the v3 LDS-DMA GEMM with gathered operands (gemm3.hip, CONV modes) for bf16 convolutions whose
// channel count is a power of two >= 32 (every 32-deep k-step inside one tap)
static ConvG make_convg(int SH, int SW, int SC, int GH, int GW, int si) {
  ConvG g{};
  g.SH = SH;
  g.SW = SW;
  g.lsc = ilog2(SC);
  g.GH = GH;
  g.GW = GW;
  g.si = si;
  conv_fastdiv((uint32_t)GW, g.gw_mul, g.gw_shift);
  conv_fastdiv((uint32_t)(GH * GW), g.ghw_mul, g.ghw_shift);
  return g;
}
static sv_gemm_desc conv_desc(const void* A, const void* B, int M, int N, int K, int b_kmajor, int64_t ldb, void* C,
                              int c_dtype, const sv_gemm_policy* pol) {
  sv_gemm_desc d{};
  if (pol) d.policy = *pol;
  d.M = M;
  d.N = N;
  d.K = K;
  d.A = A;
  d.a_dtype = SV_BF16;
  d.a_kmajor = 1;
  d.lda = K;
  d.B = B;
  d.b_dtype = SV_BF16;
  d.b_kmajor = b_kmajor;
  d.ldb = ldb;
  d.epilogue = SV_EPI_STORE;
  d.C = C;
  d.c_dtype = c_dtype;
  d.ldc = N;
  d.split_k = 1;
  d.compute = SV_BF16;
  return d;
}

}  // namespace conv
}  // namespace sv

using namespace sv;
using namespace sv::conv;

extern "C" int sv_conv_weight_pack(const float* w, void* wp, int32_t dtype, const sv_conv_shape* s,
                                   sv_stream_t stream) {
  if (int rc = check_shape(s, dtype, "sv_conv_weight_pack")) return rc;
  SV_REQUIRE(w && wp, "sv_conv_weight_pack: null pointer");
  const int T_ = s->KH * s->KW;
  const int64_t n = (int64_t)s->Cout * T_ * s->Cs;
  const int blocks = (int)((n + 255) / 256);
  if (dtype == SV_BF16)
    weight_pack_kernel<uint16_t><<<blocks, 256, 0, (hipStream_t)stream>>>(w, (uint16_t*)wp, s->Cout, s->Cin, T_, s->Cs);
  else
    weight_pack_kernel<float><<<blocks, 256, 0, (hipStream_t)stream>>>(w, (float*)wp, s->Cout, s->Cin, T_, s->Cs);
  return check_launch("sv_conv_weight_pack");
}

// Several packs in one launch: block ranges per segment (the ResNet forward packs its 7x7 / 3x3 weights,
// 17 launches of 3-6 us each, as one)
struct PackSegs {
  sv_pack_seg s[SV_MAX_PACK_SEGS];
  int64_t first_block[SV_MAX_PACK_SEGS + 1];
  int n;
};

template <typename T>
__global__ void __launch_bounds__(256) weight_pack_multi_kernel(const PackSegs segs) {
  int k = 0;
  while (k + 1 < segs.n && (int64_t)blockIdx.x >= segs.first_block[k + 1]) ++k;  // block-uniform
  const sv_pack_seg& g = segs.s[k];
  const int64_t i = ((int64_t)blockIdx.x - segs.first_block[k]) * 256 + threadIdx.x;
  const int64_t n = (int64_t)g.Cout * g.T * g.Cs;
  if (i >= n) return;
  const int c = (int)(i % g.Cs);
  const int t = (int)((i / g.Cs) % g.T);
  const int co = (int)(i / ((int64_t)g.Cs * g.T));
  const float v = c < g.Cin ? g.w[((int64_t)co * g.Cin + c) * g.T + t] : 0.f;
  st(reinterpret_cast<T*>(g.wp), (size_t)i, v);
}

extern "C" int sv_conv_weight_pack_multi(const sv_pack_seg* segs, int32_t nseg, int32_t dtype, sv_stream_t stream) {
  SV_REQUIRE(segs && nseg >= 1 && nseg <= SV_MAX_PACK_SEGS, "sv_conv_weight_pack_multi: 1..%d segments",
             SV_MAX_PACK_SEGS);
  SV_REQUIRE(dtype == SV_BF16 || dtype == SV_F32, "sv_conv_weight_pack_multi: bad dtype");
  PackSegs a{};
  a.n = nseg;
  int64_t blocks = 0;
  for (int k = 0; k < nseg; ++k) {
    const sv_pack_seg& g = segs[k];
    SV_REQUIRE(g.w && g.wp && g.Cout > 0 && g.Cin > 0 && g.T > 0 && g.Cs >= g.Cin,
               "sv_conv_weight_pack_multi: bad segment %d", k);
    a.s[k] = g;
    a.first_block[k] = blocks;
    blocks += ((int64_t)g.Cout * g.T * g.Cs + 255) / 256;
  }
  a.first_block[nseg] = blocks;
  if (dtype == SV_BF16)
    weight_pack_multi_kernel<uint16_t><<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(a);
  else
    weight_pack_multi_kernel<float><<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(a);
  return check_launch("sv_conv_weight_pack_multi");
}

extern "C" int sv_image_to_nhwc(const float* img, void* out, int32_t dtype, int32_t B, int32_t C, int32_t H, int32_t W,
                                int32_t Cs, sv_stream_t stream) {
  SV_REQUIRE(img && out, "sv_image_to_nhwc: null pointer");
  SV_REQUIRE(B > 0 && C > 0 && H > 0 && W > 0 && Cs >= C, "sv_image_to_nhwc: bad shape");
  SV_REQUIRE(dtype == SV_BF16 || dtype == SV_F32, "sv_image_to_nhwc: bad dtype");
  const int64_t n = (int64_t)B * H * W * Cs;
  const int blocks = (int)((n + 255) / 256);
  if (dtype == SV_BF16)
    image_to_nhwc_kernel<uint16_t><<<blocks, 256, 0, (hipStream_t)stream>>>(img, (uint16_t*)out, C, H, W, Cs, n);
  else
    image_to_nhwc_kernel<float><<<blocks, 256, 0, (hipStream_t)stream>>>(img, (float*)out, C, H, W, Cs, n);
  return check_launch("sv_image_to_nhwc");
}

extern "C" int sv_image_u8_hwc_to_nhwc(const uint8_t* img, const float* norm_mean, const float* norm_std,
                                       void* out, int32_t dtype, int32_t B, int32_t H, int32_t W, int32_t Cs,
                                       sv_stream_t stream) {
  SV_REQUIRE(img && norm_mean && norm_std && out, "sv_image_u8_hwc_to_nhwc: null pointer");
  SV_REQUIRE(B > 0 && H > 0 && W > 0, "sv_image_u8_hwc_to_nhwc: bad shape");
  const int64_t npix = (int64_t)B * H * W;
  SV_REQUIRE(npix % 4 == 0, "sv_image_u8_hwc_to_nhwc: B*H*W must be a multiple of 4");
  SV_REQUIRE(Cs == 4 || Cs == 8, "sv_image_u8_hwc_to_nhwc: Cs must be 4 or 8 (got %d)", Cs);
  SV_REQUIRE(dtype == SV_BF16 || dtype == SV_F32, "sv_image_u8_hwc_to_nhwc: bad dtype");
  SV_REQUIRE(((uintptr_t)img & 3) == 0, "sv_image_u8_hwc_to_nhwc: img must be 4-byte aligned");
  SV_REQUIRE(((uintptr_t)out & (dtype == SV_BF16 ? 7 : 15)) == 0, "sv_image_u8_hwc_to_nhwc: misaligned out");
  const int64_t n4 = npix / 4;
  const int blocks = (int)((n4 + 255) / 256);
  const float* m = norm_mean;
  const float* sd = norm_std;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == SV_BF16 && Cs == 8)
    image_u8_hwc_kernel<uint16_t, 8><<<blocks, 256, 0, st>>>(img, m[0], m[1], m[2], sd[0], sd[1], sd[2], (uint16_t*)out, n4);
  else if (dtype == SV_BF16)
    image_u8_hwc_kernel<uint16_t, 4><<<blocks, 256, 0, st>>>(img, m[0], m[1], m[2], sd[0], sd[1], sd[2], (uint16_t*)out, n4);
  else if (Cs == 8)
    image_u8_hwc_kernel<float, 8><<<blocks, 256, 0, st>>>(img, m[0], m[1], m[2], sd[0], sd[1], sd[2], (float*)out, n4);
  else
    image_u8_hwc_kernel<float, 4><<<blocks, 256, 0, st>>>(img, m[0], m[1], m[2], sd[0], sd[1], sd[2], (float*)out, n4);
  return check_launch("sv_image_u8_hwc_to_nhwc");
}

static int conv_fwd_impl(const void* x, const void* wp, void* y, int32_t y_dtype, int32_t dtype,
                         const sv_conv_shape* s, float* stats, const sv_gemm_policy* pol, sv_stream_t stream,
                         float* slab = nullptr, int split = 1) {
  if (int rc = check_shape(s, dtype, "sv_conv_fwd")) return rc;
  SV_REQUIRE(x && wp && y, "sv_conv_fwd: null pointer");
  SV_REQUIRE(y_dtype == SV_BF16 || y_dtype == SV_F32, "sv_conv_fwd: bad y dtype");
  const int OH = out_dim(s->H, s->KH, s->stride, s->pad), OW = out_dim(s->W, s->KW, s->stride, s->pad);
  Args a{};
  a.A = x;
  a.B = wp;
  a.M = s->B * OH * OW;
  a.N = s->Cout;
  a.K = s->KH * s->KW * s->Cs;
  a.ldb = a.K;
  a.SH = s->H;
  a.SW = s->W;
  a.SC = s->Cs;
  a.lsc = ilog2(s->Cs);
  set_grid(a, OH, OW);
  a.si = s->stride;
  a.ntaps = s->KH * s->KW;
  for (int kh = 0; kh < s->KH; ++kh)
    for (int kw = 0; kw < s->KW; ++kw) {
      a.tdy[kh * s->KW + kw] = (int8_t)(kh - s->pad);
      a.tdx[kh * s->KW + kw] = (int8_t)(kw - s->pad);
    }
  a.C = y;
  a.c_dtype = y_dtype;
  a.kper = ceil_div(a.K, BKT) * BKT;
  // SV_STEM_GATHER=0: the register-staged kernel instead (A/B runs)
  static const bool stem8 = !getenv("SV_STEM_GATHER") || atoi(getenv("SV_STEM_GATHER")) != 0;
  if (stem8 && dtype == SV_BF16 && s->Cs == 8 && !slab && s->KH == s->KW && s->KH <= 7 && a.ntaps <= CONV_MAX_TAPS &&
      a.N % 8 == 0) {
    // 8-channel pixels (the ResNet stem over its zero-padded RGB operand): one tap per 16-B chunk, gathered
    // per lane (mode 6); K padded to whole 32-deep k-steps with zero-page chunks
    ConvG g = make_convg(s->H, s->W, 8, OH, OW, s->stride);
    g.kw = s->KW;
    g.pad = s->pad;
    g.ntaps = a.ntaps;
    g.kw_mul = (65536u + (uint32_t)s->KW - 1) / (uint32_t)s->KW;
    sv_gemm_desc d = conv_desc(x, wp, a.M, a.N, ceil_div(a.K, 32) * 32, 1, a.K, y, y_dtype, pol);
    if (stats) {
      SV_REQUIRE(((uintptr_t)stats & 15) == 0, "sv_conv_fwd_stats: stats alignment");
      d.epilogue = SV_EPI_STORE_STATS;
      d.C2 = stats;
      d.c2_dtype = SV_F32;
    }
    const int rc = launch_gemm3_conv(&d, g, 6, (hipStream_t)stream);
    if (rc != SV_ERR_UNSUPPORTED) return rc;
  }
  if (dtype == SV_BF16 && s->Cs >= 32 && pow2(s->Cs) && a.K % 32 == 0) {
    ConvG g = make_convg(s->H, s->W, s->Cs, OH, OW, s->stride);
    for (int j = 0; j < a.ntaps; ++j) {
      g.tdy[j] = a.tdy[j];
      g.tdx[j] = a.tdx[j];
    }
    sv_gemm_desc d = conv_desc(x, wp, a.M, a.N, a.K, 1, a.K, y, y_dtype, pol);
    if (slab) {
      d.epilogue = SV_EPI_SLAB;
      d.C = slab;
      d.c_dtype = SV_F32;
      d.split_k = split;
      const int rc = launch_gemm3_conv(&d, g, 1, (hipStream_t)stream);
      if (rc) return rc;
      return sv_gemm_slab_finish(slab, split, a.M, a.N, y, y_dtype, a.N, 0, stats, stream);
    }
    if (stats) {
      SV_REQUIRE(a.N % 8 == 0 && ((uintptr_t)stats & 15) == 0, "sv_conv_fwd_stats: Cout %% 8 / stats alignment");
      d.epilogue = SV_EPI_STORE_STATS;
      d.C2 = stats;
      d.c2_dtype = SV_F32;
    }
    const int rc = launch_gemm3_conv(&d, g, 1, (hipStream_t)stream);
    if (rc != SV_ERR_UNSUPPORTED) return rc;
  }
  SV_REQUIRE(!stats, "sv_conv_fwd_stats: shape not on the gathered bf16 GEMM path (use sv_conv_fwd + sv_bn_stats)");
  SV_REQUIRE(!slab, "sv_conv_fwd_split: shape not on the gathered bf16 GEMM path");
  return launch_dt<FPROP>(a, dtype, 1, (hipStream_t)stream);
}

extern "C" int sv_conv_fwd(const void* x, const void* wp, void* y, int32_t y_dtype, int32_t dtype,
                           const sv_conv_shape* s, const sv_gemm_policy* policy, sv_stream_t stream) {
  return conv_fwd_impl(x, wp, y, y_dtype, dtype, s, nullptr, policy, stream);
}

extern "C" int sv_conv_fwd_stats(const void* x, const void* wp, void* y, int32_t y_dtype, int32_t dtype,
                                 const sv_conv_shape* s, float* stats, const sv_gemm_policy* policy,
                                 sv_stream_t stream) {
  SV_REQUIRE(stats, "sv_conv_fwd_stats: null stats");
  return conv_fwd_impl(x, wp, y, y_dtype, dtype, s, stats, policy, stream);
}

extern "C" int sv_conv_fwd_split(const void* x, const void* wp, void* y, int32_t y_dtype, int32_t dtype,
                                 const sv_conv_shape* s, float* stats, float* work, int32_t split,
                                 const sv_gemm_policy* policy, sv_stream_t stream) {
  SV_REQUIRE(work && split >= 1, "sv_conv_fwd_split: need a workspace and split >= 1");
  return conv_fwd_impl(x, wp, y, y_dtype, dtype, s, stats, policy, stream, work, split);
}

// bn != NULL (sv_conv_bwd_data_bn): bf16 dx of the stride-1 gathered path plus the backward statistics of the
// BatchNorm + ReLU whose output the conv read (y = that BatchNorm's input), from the epilogue or the finish
static int conv_bwd_data_impl(const void* dy, const void* wp, void* dx, int32_t dx_dtype, int32_t accumulate,
                              int32_t dtype, const sv_conv_shape* s, const sv_gemm_policy* pol, sv_stream_t stream,
                              float* slab, int split, const void* bny = nullptr, const sv_bn_ref* bn = nullptr, float* bnpart = nullptr) {
  if (int rc = check_shape(s, dtype, "sv_conv_bwd_data")) return rc;
  SV_REQUIRE(dy && wp && dx, "sv_conv_bwd_data: null pointer");
  SV_REQUIRE(dx_dtype == SV_BF16 || dx_dtype == SV_F32, "sv_conv_bwd_data: bad dx dtype");
  SV_REQUIRE(pow2(s->Cout), "sv_conv_bwd_data: Cout=%d must be a power of two", s->Cout);
  const int OH = out_dim(s->H, s->KH, s->stride, s->pad), OW = out_dim(s->W, s->KW, s->stride, s->pad);
  const int st = s->stride;
  const int T_ = s->KH * s->KW;
  if (dtype == SV_BF16 && st == 1 && s->Cout >= 32 && (s->Cs % 8) == 0 &&
      ((int64_t)T_ * s->Cout) % 32 == 0) {
    // stride 1: one gather conv over dy (taps pad - kh, pad - kw) against the weight's rows
    ConvG g = make_convg(OH, OW, s->Cout, s->H, s->W, 1);
    g.lcout = ilog2(s->Cout);
    g.Tw = T_;
    g.Cs = s->Cs;
    for (int kh = 0; kh < s->KH; ++kh)
      for (int kw = 0; kw < s->KW; ++kw) {
        g.tdy[kh * s->KW + kw] = (int8_t)(s->pad - kh);
        g.tdx[kh * s->KW + kw] = (int8_t)(s->pad - kw);
        g.twt[kh * s->KW + kw] = (uint8_t)(kh * s->KW + kw);
      }
    sv_gemm_desc d =
        conv_desc(dy, wp, s->B * s->H * s->W, s->Cs, T_ * s->Cout, 0, (int64_t)T_ * s->Cs, dx, dx_dtype, pol);
    if (slab) {
      d.epilogue = SV_EPI_SLAB;
      d.C = slab;
      d.c_dtype = SV_F32;
      d.split_k = split;
      const int rc = launch_gemm3_conv(&d, g, 2, (hipStream_t)stream);
      if (rc) return rc;
      if (bn) return sv_gemm_slab_finish_bn_bwd(slab, split, d.M, d.N, dx, bny, bn, bnpart, stream);
      return sv_gemm_slab_finish(slab, split, d.M, d.N, dx, dx_dtype, s->Cs, accumulate, nullptr, stream);
    }
    if (bn) {
      d.epilogue = SV_EPI_STORE_BN_BWD;
      d.aux = bny;
      d.aux_dtype = SV_BF16;
      d.ld_aux = s->Cs;
      d.bn = bn;
      d.C2 = bnpart;
      d.c2_dtype = SV_F32;
      return launch_gemm3_conv(&d, g, 2, (hipStream_t)stream);
    }
    if (accumulate) {  // dx += conv^T(dy): residual epilogue with gamma = 1 reading dx in place (f32, or the
      d.epilogue = SV_EPI_BIAS_GAMMA_RES;  // bf16 gradient stream: the sum in f32, stored bf16)
      d.aux = dx;
      d.aux_dtype = dx_dtype;
      d.ld_aux = s->Cs;
    }
    const int rc = launch_gemm3_conv(&d, g, 2, (hipStream_t)stream);
    if (rc != SV_ERR_UNSUPPORTED) return rc;
  }
  // stride 2, even H, W, more than one tap: all four output parity classes share one GH x GW grid
  const bool s2_grid = st == 2 && s->H % 2 == 0 && s->W % 2 == 0;
  const bool s2_even = s2_grid && s->KH * s->KW > 1;
  // ... and without a workspace their rows go straight into dx (plain store, in-place f32 accumulate, or
  // bf16 with the BatchNorm statistics); any kernel size (1x1: only class (0, 0) has a tap)
  const bool s2_direct = s2_grid && !slab && (!bn || dx_dtype == SV_BF16);
  if (dtype == SV_BF16 && st == 2 && (slab || s2_direct) && s->Cout >= 32 && (s->Cs % 8) == 0 && s->Cs >= 8) {
    // stride 2: one gather GEMM per parity class into compact slabs, then one scatter pass.  Even H, W
    // and no split: all four classes run as ONE launch (mode 5) -- the per-class launches are each below
    // one wave of workgroups (64-128 tiles for the ResNet-50 3x3s) -- and with no workspace that launch
    // stores each class's rows at their dx pixels (no slabs, no scatter pass)
    ClassSlabs cs{};
    if (s2_direct || (split == 1 && s2_even)) {
      const int GH = s->H / 2, GW = s->W / 2, M = s->B * GH * GW;
      ConvG g = make_convg(OH, OW, s->Cout, GH, GW, 1);
      g.lcout = ilog2(s->Cout);
      g.Tw = T_;
      g.Cs = s->Cs;
      int nt = 0, maxt = 0;
      for (int cls = 0; cls < 4; ++cls) {
        const int py = cls >> 1, px = cls & 1;
        g.ctap0[cls] = (uint8_t)nt;
        for (int kh = 0; kh < s->KH; ++kh) {
          const int ry = py + s->pad - kh;
          if (ry & 1) continue;
          for (int kw = 0; kw < s->KW; ++kw) {
            const int rx = px + s->pad - kw;
            if (rx & 1) continue;
            g.tdy[nt] = (int8_t)(ry >> 1);
            g.tdx[nt] = (int8_t)(rx >> 1);
            g.twt[nt] = (uint8_t)(kh * s->KW + kw);
            ++nt;
          }
        }
        g.ctaps[cls] = (uint8_t)(nt - g.ctap0[cls]);
        if (g.ctaps[cls] > maxt) maxt = g.ctaps[cls];
        cs.GH[cls] = GH;
        cs.GW[cls] = GW;
        cs.base[cls] = g.ctaps[cls] ? slab + (size_t)cls * M * s->Cs : nullptr;
      }
      if (s2_direct) {
        sv_gemm_desc d = conv_desc(dy, wp, M, s->Cs, maxt * s->Cout, 0, (int64_t)T_ * s->Cs, dx, dx_dtype, pol);
        if (bn) {  // partial rows [4][ceil(M / 64)][2][Cs]: class c's from row c * ceil(M / 64)
          d.epilogue = SV_EPI_STORE_BN_BWD;
          d.aux = bny;
          d.aux_dtype = SV_BF16;
          d.ld_aux = s->Cs;
          d.bn = bn;
          d.C2 = bnpart;
          d.c2_dtype = SV_F32;
        } else if (accumulate) {  // dx += conv^T(dy) in place (gamma = 1; f32 or bf16 dx)
          d.epilogue = SV_EPI_BIAS_GAMMA_RES;
          d.aux = dx;
          d.aux_dtype = dx_dtype;
          d.ld_aux = s->Cs;
        }
        // accumulating: trailing classes without taps would only re-add zero (1x1: one class of four)
        int ncls = 4;
        while (accumulate && ncls > 1 && g.ctaps[ncls - 1] == 0) --ncls;
        d.split_k = ncls;
        return launch_gemm3_conv(&d, g, 5, (hipStream_t)stream);
      }
      sv_gemm_desc d = conv_desc(dy, wp, M, s->Cs, maxt * s->Cout, 0, (int64_t)T_ * s->Cs, slab, SV_F32, pol);
      d.epilogue = SV_EPI_SLAB;
      if (int rc = launch_gemm3_conv(&d, g, 5, (hipStream_t)stream)) return rc;
    } else {
      float* next = slab;
      for (int py = 0; py < 2; ++py)
        for (int px = 0; px < 2; ++px) {
          const int cls = py * 2 + px;
          const int GH = (s->H - py + 1) / 2, GW = (s->W - px + 1) / 2;
          cs.GH[cls] = GH;
          cs.GW[cls] = GW;
          cs.base[cls] = nullptr;
          if (GH <= 0 || GW <= 0) continue;
          ConvG g = make_convg(OH, OW, s->Cout, GH, GW, 1);
          g.lcout = ilog2(s->Cout);
          g.Tw = T_;
          g.Cs = s->Cs;
          int nt = 0;
          for (int kh = 0; kh < s->KH; ++kh) {
            const int ry = py + s->pad - kh;
            if (ry & 1) continue;
            for (int kw = 0; kw < s->KW; ++kw) {
              const int rx = px + s->pad - kw;
              if (rx & 1) continue;
              g.tdy[nt] = (int8_t)(ry >> 1);  // arithmetic shift: floor division of an even value
              g.tdx[nt] = (int8_t)(rx >> 1);
              g.twt[nt] = (uint8_t)(kh * s->KW + kw);
              ++nt;
            }
          }
          if (nt == 0) continue;
          const int M = s->B * GH * GW;
          sv_gemm_desc d = conv_desc(dy, wp, M, s->Cs, nt * s->Cout, 0, (int64_t)T_ * s->Cs, next, SV_F32, pol);
          d.epilogue = SV_EPI_SLAB;
          d.split_k = split;
          if (int rc = launch_gemm3_conv(&d, g, 2, (hipStream_t)stream)) return rc;
          cs.base[cls] = next;
          next += (size_t)split * M * s->Cs;
        }
    }
    const int64_t n4 = (int64_t)s->B * s->H * s->W * s->Cs / 4;
    const int blocks = (int)((n4 + 255) / 256);
    if (dx_dtype == SV_BF16)
      dgrad_s2_scatter_kernel<uint16_t><<<blocks, 256, 0, (hipStream_t)stream>>>(cs, split, s->B, s->H, s->W, s->Cs,
                                                                                 (uint16_t*)dx, accumulate);
    else
      dgrad_s2_scatter_kernel<float><<<blocks, 256, 0, (hipStream_t)stream>>>(cs, split, s->B, s->H, s->W, s->Cs,
                                                                              (float*)dx, accumulate);
    return check_launch("sv_conv_bwd_data(stride-2 scatter)");
  }
  SV_REQUIRE(!slab, "sv_conv_bwd_data_split: shape not on the gathered bf16 GEMM path (Cout >= 32)");
  for (int py = 0; py < st; ++py)
    for (int px = 0; px < st; ++px) {
      Args a{};
      a.A = dy;
      a.B = wp;
      const int GH = (s->H - py + st - 1) / st, GW = (s->W - px + st - 1) / st;
      if (GH <= 0 || GW <= 0) continue;
      a.M = s->B * GH * GW;
      a.N = s->Cs;
      a.SH = OH;
      a.SW = OW;
      a.SC = s->Cout;
      a.lsc = ilog2(s->Cout);
      set_grid(a, GH, GW);
      a.si = 1;
      a.Tw = s->KH * s->KW;
      int nt = 0;
      for (int kh = 0; kh < s->KH; ++kh) {
        const int ry = py + s->pad - kh;
        if (((ry % st) + st) % st) continue;
        for (int kw = 0; kw < s->KW; ++kw) {
          const int rx = px + s->pad - kw;
          if (((rx % st) + st) % st) continue;
          a.tdy[nt] = (int8_t)(ry >= 0 ? ry / st : -((-ry) / st));
          a.tdx[nt] = (int8_t)(rx >= 0 ? rx / st : -((-rx) / st));
          a.twt[nt] = (uint8_t)(kh * s->KW + kw);
          ++nt;
        }
      }
      if (nt == 0 && accumulate) continue;  // this parity class receives no gradient
      a.ntaps = nt;
      a.K = nt * s->Cout;
      a.C = dx;
      a.c_dtype = dx_dtype;
      a.accumulate = accumulate;
      a.so = st;
      a.py = py;
      a.px = px;
      a.DH = s->H;
      a.DW = s->W;
      a.kper = a.K > 0 ? ceil_div(a.K, BKT) * BKT : 0;
      if (int rc = launch_dt<DGRAD>(a, dtype, 1, (hipStream_t)stream)) return rc;
    }
  return SV_OK;
}

extern "C" int sv_conv_bwd_data(const void* dy, const void* wp, void* dx, int32_t dx_dtype, int32_t accumulate,
                                int32_t dtype, const sv_conv_shape* s, const sv_gemm_policy* policy,
                                sv_stream_t stream) {
  return conv_bwd_data_impl(dy, wp, dx, dx_dtype, accumulate, dtype, s, policy, stream, nullptr, 1);
}

extern "C" int sv_conv_bwd_data_split(const void* dy, const void* wp, void* dx, int32_t dx_dtype, int32_t accumulate,
                                      int32_t dtype, const sv_conv_shape* s, float* work, int32_t split,
                                      const sv_gemm_policy* policy, sv_stream_t stream) {
  SV_REQUIRE(work && split >= 1, "sv_conv_bwd_data_split: need a workspace and split >= 1");
  return conv_bwd_data_impl(dy, wp, dx, dx_dtype, accumulate, dtype, s, policy, stream, work, split);
}

extern "C" int sv_conv_bwd_data_bn(const void* dy, const void* wp, void* dx, int32_t dtype, const sv_conv_shape* s,
                                   const void* y, const sv_bn_ref* bn, float* part, float* work, int32_t split,
                                   const sv_gemm_policy* policy, sv_stream_t stream) {
  if (int rc = check_shape(s, dtype, "sv_conv_bwd_data_bn")) return rc;
  SV_REQUIRE(y && bn && part && bn->mean && bn->rstd && bn->gamma && bn->beta && split >= 1 && (split == 1 || work),
             "sv_conv_bwd_data_bn: null pointer / split > 1 without a workspace");
  // stride 2: even H, W, more than one tap, no split (mode 5 straight into dx)
  const bool s2 = s->stride == 2 && s->H % 2 == 0 && s->W % 2 == 0 && s->KH * s->KW > 1 && split == 1;
  SV_REQUIRE(dtype == SV_BF16 && (s->stride == 1 || s2) && s->Cout >= 32 && pow2(s->Cout) && s->Cs % 8 == 0 &&
                 ((int64_t)s->KH * s->KW * s->Cout) % 32 == 0,
             "sv_conv_bwd_data_bn: only the bf16 stride-1 gathered path or stride 2 with even H, W and no split "
             "(Cout >= 32, power of two; Cs %% 8 == 0)");
  return conv_bwd_data_impl(dy, wp, dx, SV_BF16, 0, dtype, s, policy, stream, split > 1 ? work : nullptr, split, y, bn,
                            part);
}

// the transposed wgrad (mode 4: taps*channels on the 256-row side, Cout on the 128-column side) when
// it wastes fewer MFMA rows than mode 3 (Cout on the 256-row side): ResNet layer1/2 3x3 convs and the
// stem (Cout 64 / 128) -- 0.225 -> 0.375 / 0.5 -> 0.9 / 0.19 -> 0.38 of the tile's MFMA work is useful
static bool wgrad_transposed(const sv_conv_shape* s) {
  const int64_t tc = (int64_t)s->KH * s->KW * s->Cs;
  const double e3 = (double)s->Cout / (256.0 * ceil_div(s->Cout, 256)) * (double)tc / (128.0 * ceil_div(tc, 128));
  const double e4 = (double)tc / (256.0 * ceil_div(tc, 256)) * (double)s->Cout / (128.0 * ceil_div(s->Cout, 128));
  return e4 > 1.1 * e3;
}

// split-K depth of the v3 gather wgrad.  Mode 3: ~512 workgroups over its 256x128 tiles, >= 512 pixels
// per slice.  Mode 4 (few output tiles, Cout < 256): 192-256 workgroups with >= 2048 pixels per slice
// where the pixel count allows -- fewer, longer slices halve the slab round trip of the layer1 3x3
// (76 -> 60 us) and the stem (131 -> 119 us) against the 512-workgroup split (tools/conv_bench.py)
// A/B switches (tools/build_ab.sh): the transposed wgrad's workgroup target (and gemm3.hip's SV_CONVW4_STAGES)
#ifndef SV_CONVW4_WGS
#define SV_CONVW4_WGS 256
#endif
static int wgrad_split3(const sv_conv_shape* s) {
  const int OH = out_dim(s->H, s->KH, s->stride, s->pad), OW = out_dim(s->W, s->KW, s->stride, s->pad);
  const int64_t K = (int64_t)s->B * OH * OW;
  const int64_t tc = (int64_t)s->KH * s->KW * s->Cs;
  int64_t split;
  if (wgrad_transposed(s)) {
    const int64_t tiles = ceil_div(tc, 256) * ceil_div(s->Cout, 128);
    const int64_t lo = ceil_div(SV_CONVW4_WGS * 3 / 4, tiles), hi = ceil_div(SV_CONVW4_WGS, tiles);
    split = K / 2048 > lo ? K / 2048 : lo;
    if (split > hi) split = hi;
    const int64_t maxs = K / 512 > 0 ? K / 512 : 1;
    if (split > maxs) split = maxs;
  } else {
    const int64_t tiles = ceil_div(s->Cout, 256) * ceil_div(tc, 128);
    split = ceil_div(512, tiles);
    const int64_t maxs = K / 512 > 0 ? K / 512 : 1;
    if (split > maxs) split = maxs;
  }
  if (split > 256) split = 256;
  return split < 1 ? 1 : (int)split;
}

extern "C" int64_t sv_conv_bwd_weight_work_floats(const sv_conv_shape* s) {
  if (!s) return -1;
  const int sp = wgrad_split(s) > wgrad_split3(s) ? wgrad_split(s) : wgrad_split3(s);
  return (int64_t)sp * s->Cout * s->KH * s->KW * s->Cs;
}

extern "C" int sv_conv_bwd_weight(const void* dy, const void* x, float* work, float* dw, int32_t accumulate,
                                  int32_t dtype, const sv_conv_shape* s, const sv_gemm_policy* policy,
                                  sv_stream_t stream) {
  const sv_gemm_policy* pol = policy;
  if (int rc = check_shape(s, dtype, "sv_conv_bwd_weight")) return rc;
  SV_REQUIRE(dy && x && work && dw, "sv_conv_bwd_weight: null pointer");
  const int OH = out_dim(s->H, s->KH, s->stride, s->pad), OW = out_dim(s->W, s->KW, s->stride, s->pad);
  const int T_ = s->KH * s->KW;
  hipStream_t st = (hipStream_t)stream;
  const int64_t npix = (int64_t)s->B * OH * OW;
  if (dtype == SV_BF16 && s->Cs >= 8 && pow2(s->Cs) && npix % 32 == 0 && s->Cout % 8 == 0) {
    // v3 gather wgrad: A = dy (M-major: [pixel][Cout]), B = gathered x rows, split-K f32 slabs
    const int sp = wgrad_split3(s);
    ConvG g = make_convg(s->H, s->W, s->Cs, OH, OW, s->stride);
    for (int kh = 0; kh < s->KH; ++kh)
      for (int kw = 0; kw < s->KW; ++kw) {
        g.tdy[kh * s->KW + kw] = (int8_t)(kh - s->pad);
        g.tdx[kh * s->KW + kw] = (int8_t)(kw - s->pad);
      }
    const bool tr = wgrad_transposed(s);
    sv_gemm_desc d = tr ? conv_desc(x, dy, T_ * s->Cs, s->Cout, (int)npix, 0, s->Cout, work, SV_F32, pol)
                        : conv_desc(dy, x, s->Cout, T_ * s->Cs, (int)npix, 0, T_ * s->Cs, work, SV_F32, pol);
    d.a_kmajor = 0;
    d.lda = tr ? T_ * s->Cs : s->Cout;
    d.epilogue = SV_EPI_SLAB;
    d.split_k = sp;
    const int rc = launch_gemm3_conv(&d, g, tr ? 4 : 3, st);
    if (rc == SV_OK) {
      const int64_t n = (int64_t)s->Cout * T_ * s->Cs;
      if (tr)
        wgrad_finish_t_kernel<<<(int)((n + 63) / 64), 256, 0, st>>>(work, sp, s->Cout, s->Cin, T_, s->Cs, dw,
                                                                      accumulate);
      else
        wgrad_finish_kernel<<<(int)((n + 255) / 256), 256, 0, st>>>(work, sp, s->Cout, s->Cin, T_, s->Cs, dw,
                                                                      accumulate);
      return check_launch("sv_conv_bwd_weight(finish)");
    }
    if (rc != SV_ERR_UNSUPPORTED) return rc;
  }
  const int split = wgrad_split(s);
  Args a{};
  a.A = dy;
  a.B = x;
  a.M = s->Cout;
  a.N = s->KH * s->KW * s->Cs;
  a.K = s->B * OH * OW;
  a.lda = s->Cout;
  a.SH = s->H;
  a.SW = s->W;
  a.SC = s->Cs;
  a.lsc = ilog2(s->Cs);
  set_grid(a, OH, OW);
  a.si = s->stride;
  a.ntaps = s->KH * s->KW;
  for (int kh = 0; kh < s->KH; ++kh)
    for (int kw = 0; kw < s->KW; ++kw) {
      a.tdy[kh * s->KW + kw] = (int8_t)(kh - s->pad);
      a.tdx[kh * s->KW + kw] = (int8_t)(kw - s->pad);
    }
  a.C = work;
  a.c_dtype = SV_F32;
  a.kper = ceil_div(ceil_div(a.K, split), BKT) * BKT;
  if (int rc = launch_dt<WGRAD>(a, dtype, split, st)) return rc;
  const int64_t n = (int64_t)s->Cout * T_ * s->Cs;
  wgrad_finish_kernel<<<(int)((n + 255) / 256), 256, 0, st>>>(work, split, s->Cout, s->Cin, T_, s->Cs, dw, accumulate);
  return check_launch("sv_conv_bwd_weight(finish)");
}
