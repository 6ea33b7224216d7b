// Depthwise 7x7 convolution (pad 3, stride 1, NHWC) on the matrix cores -- ConvNeXtBlock.conv_dw forward, its
// backward-data and (opt-in) its weight gradient (timm convnext.py via spine_vision/training/models/backbone.py:50;
// round 6).
//
// A depthwise conv has no GEMM across channels: every channel has its own 7x7 filter.  What a channel does have is a
// GEMM along the image ROW: for kernel row kr, the 16 outputs (row m, columns n0 .. n0+15) take
//     out[m][n] += sum_k T_kr[n][k] * x[m + kr - 3][n0 - 3 + k],   T_kr[n][k] = w[kr][k - n]  (0 <= k - n <= 6)
// -- a banded Toeplitz matrix T_kr (16 x 32, 7 diagonals) times 16 input rows x 32 input columns.  One
// v_mfma_f32_16x16x32_bf16 per kernel row computes 256 outputs of one channel; seven of them (kr = 0..6, each reading
// its input rows one lower) finish a 16 x 16 output block.  The k >= 24 quarter of every K window multiplies zero
// taps (its A operand reads a zero region), so the matrix cores do 32/7 x the depthwise FLOPs -- still ~3 us of MFMA
// per ConvNeXt-base S3 layer at bs32, against the VALU kernel's 49 v_fma_f32 per output (dwconv.hip).
//
// Operands are bf16 (the precision torch.autocast gives conv_dw), products exact, sums in f32 by the MFMA.
//
// Workgroup = 4 waves = one image tile of 16 output rows x 16 NB output columns x CG channels (CG = 16 or 32, CG / 4
// per wave; the host picks per pass, launch() below):
//   1. the 22 x (16 NB + 6) input pixels x CG channels are read from HBM (16 B per lane, 32-128-B channel segments),
//      rounded to bf16 and TRANSPOSED into channel planes [c][row][col] in LDS (the MFMA operand wants 8 consecutive
//      columns of one channel per lane; NHWC holds 8 consecutive channels of one column);
//   2. the CG x 7 Toeplitz rows are built once per workgroup as zero-padded tap windows [c][kr][2 parities][24 bf16]:
//      lane (n, q) of the T operand needs taps 8q - n .. 8q - n + 7, a 4-byte-aligned 16-byte read of one parity copy;
//   3. per channel: 7 T operands (28 VGPRs), then per 16-column block 7 MFMAs over LDS reads of the data operand;
//   4. the accumulators (lane: 4 consecutive output columns of one output row, one channel) are staged through LDS as
//      [pixel][channel] and stored 16 B per lane (bf16 z with the bias; or f32 dx accumulated + its bf16 copy).
// Barriers: after the fill, before the staging (the input region is reused), before the read-back.
#include "common.h"
#include "gemm_common.h"

#include <stdlib.h>

namespace sv {
namespace dwm {

constexpr int kCGMin = 16;       // channels per workgroup: CG = 32 (8 per wave) or 16 (4 per wave; less LDS)
constexpr int TH = 16;           // output rows per tile = the MFMA's 16 rows
constexpr int IR = TH + 6;       // input rows per tile
constexpr int kThreads = 256;
constexpr int kTabB = 96;        // bytes per (channel, kernel row) Toeplitz window pair: 2 x 24 bf16
constexpr int kZeroB = 640;      // zero region read by the k >= 24 lanes (<= 6 RS + 32 + 16 bytes)

template <int NB, int CG>
struct Geo {
  static constexpr int TW = 16 * NB;                // output columns per tile
  static constexpr int IC = (TW + 6 + 7) / 8 * 8;   // input columns kept per row (K windows reach column TW + 7)
  static constexpr int RS = IC * 2;                 // bytes per input row of one channel plane
  static constexpr int PS = IR * RS + 16;           // bytes per channel plane (+16: the fill's write banks)
  static constexpr int IN_BYTES = CG * PS + 448;    // + the planes' bank skew (<= 7 x 64 B)
  static constexpr int TAB = CG * 7 * kTabB;
  static constexpr int OP16 = TW * CG * 2 + 16;     // bf16 staging: bytes per output row ([TW pixels][CG ch] + 16)
  static constexpr int OP32 = 16 * CG * 4 + 16;     // f32 staging (one 16-column block at a time)
  static constexpr int LDS = IN_BYTES + TAB + kZeroB;
  static_assert(TH * OP16 <= IN_BYTES && TH * OP32 <= IN_BYTES, "staging reuses the input planes");
  static_assert(6 * RS + 32 * (NB - 1) + 16 <= kZeroB, "zero region");
};

struct DwmGeo {
  int B, H, W, C, tilesW, tilesH, ntiles;
};

// XCD-contiguous order (dwconv.hip xcd_block): each XCD walks a contiguous range of (tile, channel group) pairs, so the
// channel groups of one pixel and the halo rows / columns of neighbouring tiles meet in one L2
__device__ __forceinline__ int xcd_order(int b, int G) { return (G & 7) == 0 ? (b & 7) * (G >> 3) + (b >> 3) : b; }

template <typename T>
__device__ __forceinline__ void to_bf16(const uint4& raw, uint16_t (&o)[16 / sizeof(T)]) {
  if constexpr (sizeof(T) == 4) {
    const uint32_t a = pack2bf(__uint_as_float(raw.x), __uint_as_float(raw.y));
    const uint32_t b = pack2bf(__uint_as_float(raw.z), __uint_as_float(raw.w));
    o[0] = (uint16_t)a, o[1] = (uint16_t)(a >> 16), o[2] = (uint16_t)b, o[3] = (uint16_t)(b >> 16);
  } else {
    const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (uint16_t)(w[i >> 1] >> (16 * (i & 1)));
  }
}

// The input tile -> bf16 channel planes [c][row][col] in LDS (plane c at c PS + ((c / EPC) mod 8) SKEW).  Wave wv loads
// input rows wv, wv + 4, ..: per row NJ instructions of PPI consecutive columns x QPP channel chunks (16 B per lane)
// through a buffer descriptor over the image, so an out-of-image column reads zeros without a branch.  load() issues
// every load, store() converts and writes them (the transpose: EPC 2-byte writes per chunk).  The skew puts the fill's
// lane groups (PPI columns of EPC channels each) on distinct banks instead of PS apart on the same ones (r13h: 11.4 M
// bank-conflict cycles against 9.2 M active LDS cycles at S1 without it).
template <typename TIN, int NB, int CG>
struct XPlanes {
  using G = Geo<NB, CG>;
  static constexpr int EPC = 16 / (int)sizeof(TIN);  // channels per 16-B chunk
  static constexpr int QPP = CG / EPC;               // chunks per pixel
  static constexpr int PPI = 64 / QPP;               // pixels per wave instruction
  static constexpr int NJ = (G::IC + PPI - 1) / PPI;
  static constexpr int NRW = (IR + 3) / 4;
  static constexpr int SKEW = 2 * PPI;
  __device__ __forceinline__ static int plane(int c) { return c * G::PS + ((c / EPC) & 7) * SKEW; }
  uint4 raw[NRW][NJ];
  __device__ __forceinline__ void load(const TIN* x, const DwmGeo& g, int b, int h0, int w0, int c0, int wvu,
                                       int lane) {
    const int fc = lane % PPI, fq = lane / PPI;
    const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<TIN*>(x + (size_t)b * g.H * g.W * g.C), (short)0,
                                                      (int)((size_t)g.H * g.W * g.C * sizeof(TIN)), 0x00020000);
    uint32_t loff[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int col = j * PPI + fc, ww = w0 - 3 + col;
      loff[j] = (col < G::TW + 6 && ww >= 0 && ww < g.W) ? (uint32_t)((ww * g.C + c0 + fq * EPC) * (int)sizeof(TIN))
                                                         : 0x80000000u;
    }
#pragma unroll
    for (int i = 0; i < NRW; ++i) {
      const int row = wvu + 4 * i, hh = h0 - 3 + row;
      const bool okr = row < IR && hh >= 0 && hh < g.H;  // wave-uniform
      const uint32_t ro = okr ? (uint32_t)(hh * g.W * g.C * (int)sizeof(TIN)) : 0u;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rx, loff[j] + ro, 0, 0);
        raw[i][j] = okr ? make_uint4(v[0], v[1], v[2], v[3]) : make_uint4(0u, 0u, 0u, 0u);
      }
    }
  }
  __device__ __forceinline__ void store(char* tin, int wvu, int lane) const {
    const int fc = lane % PPI, fq = lane / PPI;
    char* wb = tin + (fq * EPC) * G::PS + (fq & 7) * SKEW + fc * 2;
#pragma unroll
    for (int i = 0; i < NRW; ++i) {
      const int row = wvu + 4 * i;
      if (row >= IR) break;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (NJ * PPI != G::IC && j * PPI + fc >= G::IC) continue;
        uint16_t e[EPC];
        to_bf16<TIN>(raw[i][j], e);
        char* p = wb + row * G::RS + j * PPI * 2;
#pragma unroll
        for (int t = 0; t < EPC; ++t) *reinterpret_cast<uint16_t*>(p + t * G::PS) = e[t];
      }
    }
  }
};

// MODE 0: z (bf16) = bias + conv(x).  MODE 1: dx (f32) = conv_flipped(dz) [+ bf16 copy].  MODE 2: dx += ...
template <typename TIN, bool FLIP, int MODE, int NB, int CG>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2)))
dw7_mfma_kernel(const TIN* __restrict__ x, const float* __restrict__ wdw, const float* __restrict__ bdw,
                void* __restrict__ out, uint16_t* __restrict__ out_bf16, DwmGeo g) {
  using G = Geo<NB, CG>;
  constexpr int CPW = CG / 4;  // channels per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* tin = smem;
  char* tab = smem + G::IN_BYTES;
  char* zreg = tab + G::TAB;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ncg = g.C / CG;
  const int lb = xcd_order(blockIdx.x, gridDim.x);
  const int cgi = lb % ncg, tile = lb / ncg;
  const int twi = tile % g.tilesW, t2 = tile / g.tilesW, thi = t2 % g.tilesH, b = t2 / g.tilesH;
  const int h0 = thi * TH, w0 = twi * G::TW, c0 = cgi * CG;

  // ---- 1. input tile -> bf16 channel planes (XPlanes): every load now, the LDS writes after the Toeplitz build ----
  using XP = XPlanes<TIN, NB, CG>;
  constexpr int EPC = XP::EPC, SKEW = XP::SKEW;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  XP xp;
  xp.load(x, g, b, h0, w0, c0, wvu, lane);
  // MODE 2: the accumulated gradient's tile is read now, in flight under the fill and the MFMAs, instead of after them
  // (r13h: the backward's waves waited 72 % of their cycles, the read-back's dx loads exposed at every tile's end)
  constexpr int CH32 = CG / 4;  // 16-B chunks of an f32 pixel
  constexpr int NPRE = MODE == 2 ? NB * (TH * 16 * CH32 / kThreads) : 1;
  float4 pre[NPRE];
  if constexpr (MODE == 2) {
    const float* dxo = reinterpret_cast<const float*>(out);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int k = 0; k < TH * 16 * CH32 / kThreads; ++k) {
        const int it = tid + k * kThreads;
        const int ch = it % CH32, pix = it / CH32, row = pix >> 4, col = pix & 15;
        const int hh = h0 + row, ww = w0 + 16 * nb + col;
        pre[nb * (TH * 16 * CH32 / kThreads) + k] =
            hh < g.H && ww < g.W
                ? *reinterpret_cast<const float4*>(dxo + ((size_t)(b * g.H + hh) * g.W + ww) * g.C + c0 + ch * 4)
                : make_float4(0.f, 0.f, 0.f, 0.f);
      }
  }
  // ---- 2. Toeplitz windows: thread (c, kr) packs its 7 taps into the two parity copies of the zero-padded row
  //      Zt[t] = w[kr][t - 8] (t = 8..14), copy 0 = Zt[0..23], copy 1 = Zt[1..24] ----
  if (tid < CG * 7) {
    const int c = tid / 7, kr = tid - 7 * c;
    const float* wp = wdw + (size_t)(c0 + c) * 49 + (FLIP ? 6 - kr : kr) * 7;
    float w7[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) w7[j] = wp[FLIP ? 6 - j : j];
    uint4* d = reinterpret_cast<uint4*>(tab + tid * kTabB);
    const uint4 z4 = make_uint4(0u, 0u, 0u, 0u);
    d[0] = z4;                                                                                   // copy 0 dwords 0-3
    d[1] = make_uint4(pack2bf(w7[0], w7[1]), pack2bf(w7[2], w7[3]), pack2bf(w7[4], w7[5]), pack2bf(w7[6], 0.f));
    d[2] = z4;                                                                                   // dwords 8-11
    d[3] = make_uint4(0u, 0u, 0u, pack2bf(0.f, w7[0]));                                          // copy 1 dwords 0-3
    d[4] = make_uint4(pack2bf(w7[1], w7[2]), pack2bf(w7[3], w7[4]), pack2bf(w7[5], w7[6]), 0u);  // 4-7
    d[5] = z4;
  }
  for (int i = tid; i < kZeroB / 16; i += kThreads) reinterpret_cast<uint4*>(zreg)[i] = make_uint4(0u, 0u, 0u, 0u);
  xp.store(tin, wvu, lane);
  __syncthreads();

  // ---- 3. MFMAs: lane (n = lane & 15, q = lane >> 4) of the T operand takes taps 8q - n .. +7; lane (m, q) of the
  //      data operand columns 8q .. 8q + 7 of input row m + kr (q = 3: the zero region) ----
  const int n = lane & 15, q = lane >> 4;
  int s = 8 * q - n + 8;
  s = s < 0 ? 0 : (s > 16 ? 16 : s);
  const int toff = (s & 1) * 48 + (s >> 1) * 4;
  f32x4 acc[CPW][NB];
#pragma unroll
  for (int t = 0; t < CPW; ++t) {
    const int c = wv * CPW + t;
    const char* tb = tab + c * 7 * kTabB + toff;
    bf16x8 tw[7];
#pragma unroll
    for (int kr = 0; kr < 7; ++kr) {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(tb + kr * kTabB);
      const uint32_t v4[4] = {p[0], p[1], p[2], p[3]};
      tw[kr] = __builtin_bit_cast(bf16x8, v4);
    }
    const char* ab = q < 3 ? tin + c * G::PS + ((c / EPC) & 7) * SKEW + n * G::RS + 16 * q : zreg;
    const float bias = MODE == 0 ? bdw[c0 + c] : 0.f;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      f32x4 a = {bias, bias, bias, bias};
#pragma unroll
      for (int kr = 0; kr < 7; ++kr) {
        const bf16x8 xv = *reinterpret_cast<const bf16x8*>(ab + kr * G::RS + 32 * nb);
        a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tw[kr], xv, a, 0, 0, 0);
      }
      acc[t][nb] = a;
    }
  }
  // lane (m = lane & 15, q) now holds output row h0 + m, columns w0 + 16 nb + 4q + r (r = 0..3), channel CPW wv + t
  __syncthreads();  // every wave is done with the input planes
  const int m = lane & 15;
  if constexpr (MODE == 0) {
    // ---- 4a. bf16 z: stage [row][pixel][32 ch] (16 B per lane: the wave's 8 channels), read back 16 B per lane ----
    uint16_t* z = reinterpret_cast<uint16_t*>(out);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        char* p = smem + m * G::OP16 + (16 * nb + 4 * q + r) * (CG * 2) + wv * (CPW * 2);
        if constexpr (CPW == 8) {
          *reinterpret_cast<uint4*>(p) = make_uint4(pack2bf(acc[0][nb][r], acc[1][nb][r]), pack2bf(acc[2][nb][r], acc[3][nb][r]),
                                                    pack2bf(acc[4][nb][r], acc[5][nb][r]), pack2bf(acc[6][nb][r], acc[7][nb][r]));
        } else {
          *reinterpret_cast<uint2*>(p) = make_uint2(pack2bf(acc[0][nb][r], acc[1][nb][r]), pack2bf(acc[2][nb][r], acc[3][nb][r]));
        }
      }
    __syncthreads();
    constexpr int CH16 = CG / 8;  // 16-B chunks of a bf16 pixel
    constexpr int ITEMS = TH * G::TW * CH16;
#pragma unroll
    for (int k = 0; k < ITEMS / kThreads; ++k) {
      const int it = tid + k * kThreads;
      const int ch = it % CH16, pix = it / CH16, row = pix / G::TW, col = pix - row * G::TW;
      const int hh = h0 + row, ww = w0 + col;
      const uint4 v = *reinterpret_cast<const uint4*>(smem + row * G::OP16 + col * (CG * 2) + ch * 16);
      if (hh < g.H && ww < g.W)
        *reinterpret_cast<uint4*>(z + ((size_t)(b * g.H + hh) * g.W + ww) * g.C + c0 + ch * 8) = v;
    }
  } else {
    // ---- 4b. f32 dx (+= when MODE 2) and its bf16 copy, one 16-column block at a time ----
    float* dx = reinterpret_cast<float*>(out);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      if (nb > 0) __syncthreads();  // the previous block's read-back is done
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float4* p = reinterpret_cast<float4*>(smem + m * G::OP32 + (4 * q + r) * (CG * 4) + wv * (CPW * 4));
        p[0] = make_float4(acc[0][nb][r], acc[1][nb][r], acc[2][nb][r], acc[3][nb][r]);
        if constexpr (CPW == 8) p[1] = make_float4(acc[4][nb][r], acc[5][nb][r], acc[6][nb][r], acc[7][nb][r]);
      }
      __syncthreads();
      constexpr int ITEMS = TH * 16 * CH32;  // 16 x 16 pixels x chunks of 4 channels
#pragma unroll
      for (int k = 0; k < ITEMS / kThreads; ++k) {
        const int it = tid + k * kThreads;
        const int ch = it % CH32, pix = it / CH32, row = pix >> 4, col = pix & 15;
        const int hh = h0 + row, ww = w0 + 16 * nb + col;
        float4 v = *reinterpret_cast<const float4*>(smem + row * G::OP32 + col * (CG * 4) + ch * 16);
        if (hh < g.H && ww < g.W) {
          const size_t o = ((size_t)(b * g.H + hh) * g.W + ww) * g.C + c0 + ch * 4;
          if constexpr (MODE == 2) {
            const float4 old = pre[nb * (ITEMS / kThreads) + k];
            v = make_float4(old.x + v.x, old.y + v.y, old.z + v.z, old.w + v.w);
          }
          *reinterpret_cast<float4*>(dx + o) = v;
          if (out_bf16) *reinterpret_cast<uint2*>(out_bf16 + o) = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
        }
      }
    }
  }
}

// ---- weight gradient --------------------------------------------------------------------------------------------
// dW[c][kr][j] = sum_{m,n} dz[m][n] x[m + kr - 3][n + j - 3].  With n' = n + j (the x column, tile-relative) it is a GEMM
// over the tile's pixels K = (m, n'):
//     D[kr][j] = sum_K P[kr][K] Q[K][j],   P[kr][(m, n')] = x[m + kr][n'],   Q[(m, n')][j] = dz[m][n' - j]
// -- the 7 x 7 taps of one channel are one 16 x 16 MFMA accumulator (rows kr, columns j; 49 of 256 used), summed over
// every pixel of every tile a workgroup visits, so nothing is extracted per tile.  K runs in octs of 8 consecutive
// columns n' of one row m (one 16-B LDS read of the x plane for P); Q's oct starts j columns earlier in the dz row, a
// 4-byte-aligned read of one of two parity copies of the zero-padded row (as the forward's Toeplitz windows).  The bias
// gradient is the tile's plain dz sum, accumulated by the dz fill's threads.  Per workgroup: CG channels, tiles
// part, part + nparts, .. (16 rows x 16 NB columns each), the next tile's loads in flight under this tile's MFMAs.
template <int NB, int CG>
struct WGeo {
  using G = Geo<NB, CG>;
  static constexpr int NO = G::IC / 8;              // 8-column octs per x row (n' in [0, IC))
  static constexpr int NCH = TH * NO / 4;           // K chunks of 32 (4 octs) per tile
  static constexpr int DZC = G::IC + 8;             // dz row: 8 zero columns, the data, zeros to n' - j <= IC
  static constexpr int DZR = 2 * DZC * 2;           // bytes per dz row (two parity copies)
  static constexpr int DZPS = TH * DZR;             // bytes per dz plane
  static constexpr int DZ_BYTES = CG * DZPS;
  static constexpr int LDS = G::IN_BYTES + DZ_BYTES;
  static_assert((TH * NO) % 4 == 0, "whole K chunks");
};

template <typename TIN, int NB, int CG>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2)))
dw7_wgrad_mfma_kernel(const uint16_t* __restrict__ dz, const TIN* __restrict__ x, float* __restrict__ dw_part,
                      float* __restrict__ db_part, int nparts, DwmGeo g) {
  using G = Geo<NB, CG>;
  using WG = WGeo<NB, CG>;
  using XP = XPlanes<TIN, NB, CG>;
  constexpr int CPW = CG / 4, EPC = XP::EPC, SKEW = XP::SKEW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* tin = smem;
  char* tdz = smem + G::IN_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  const int ncg = g.C / CG;
  const int lb = xcd_order(blockIdx.x, gridDim.x);
  const int cgi = lb % ncg, part = lb / ncg, c0 = cgi * CG;
  // the dz planes' padding columns stay zero: every tile rewrites only the data columns
  for (int i = tid; i < WG::DZ_BYTES / 16; i += kThreads) reinterpret_cast<uint4*>(tdz)[i] = make_uint4(0u, 0u, 0u, 0u);

  // dz fill: item = (pixel, 8-channel chunk), 16 B per lane; thread tid always holds chunk tid % (CG / 8)
  constexpr int C8 = CG / 8;
  constexpr int DZN = TH * G::TW * C8 / kThreads;
  static_assert((TH * G::TW * C8) % kThreads == 0, "dz fill");
  const int my_ch = tid % C8;
  float dbs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const auto rdz = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t*>(dz), (short)0, 0x7fffffff, 0x00020000);
  auto tile_of = [&](int t, int& b, int& h0, int& w0) {
    const int twi = t % g.tilesW, t2 = t / g.tilesW;
    b = t2 / g.tilesH;
    h0 = (t2 % g.tilesH) * TH;
    w0 = twi * G::TW;
  };
  uint4 dzr[DZN];
  XP xp;
  auto load_tile = [&](int t) {
    int b, h0, w0;
    tile_of(t, b, h0, w0);
    xp.load(x, g, b, h0, w0, c0, wvu, lane);
#pragma unroll
    for (int k = 0; k < DZN; ++k) {
      const int it = tid + k * kThreads, pix = it / C8, row = pix / G::TW, col = pix - row * G::TW;
      const int hh = h0 + row, ww = w0 + col;
      const uint32_t off = hh < g.H && ww < g.W
                               ? (uint32_t)((((size_t)(b * g.H + hh) * g.W + ww) * g.C + c0 + my_ch * 8) * 2)
                               : 0x80000000u;
      const auto v = __builtin_amdgcn_raw_buffer_load_b128(rdz, off, 0, 0);
      dzr[k] = make_uint4(v[0], v[1], v[2], v[3]);
    }
  };
  auto store_dz = [&]() {
#pragma unroll
    for (int k = 0; k < DZN; ++k) {
      const int it = tid + k * kThreads, pix = it / C8, row = pix / G::TW, col = pix - row * G::TW;
      const uint32_t w4[4] = {dzr[k].x, dzr[k].y, dzr[k].z, dzr[k].w};
      // copy 0 holds padded column col + 8, copy 1 (shifted by one element) col + 7
      char* p = tdz + (my_ch * 8) * WG::DZPS + row * WG::DZR + (col + 8) * 2;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint16_t v = (uint16_t)(w4[e >> 1] >> (16 * (e & 1)));
        *reinterpret_cast<uint16_t*>(p + e * WG::DZPS) = v;
        *reinterpret_cast<uint16_t*>(p + e * WG::DZPS + 2 * WG::DZC - 2) = v;
        dbs[e] += __uint_as_float((uint32_t)v << 16);
      }
    }
  };

  // per-lane operand offsets of every K chunk (the same for every channel and tile): lane (i = lane & 15, q) takes oct
  // o = 4 chunk + q = (row m, column oct co).  P rows i >= 7 repeat kr = 6 (their D rows are discarded); Q columns
  // j >= 7 repeat j = 6
  const int li = lane & 15, q = lane >> 4;
  const int kr = li < 6 ? li : 6, jj = li < 6 ? li : 6;
  uint32_t poff[WG::NCH], qoff[WG::NCH];
  typedef const __attribute__((address_space(3))) char* lds_cptr;
  const uint32_t pbase = (uint32_t)(size_t)(lds_cptr)(tin + XP::plane(wvu * CPW));
  const uint32_t qbase = (uint32_t)(size_t)(lds_cptr)(tdz + (wvu * CPW) * WG::DZPS);
#pragma unroll
  for (int ch = 0; ch < WG::NCH; ++ch) {
    const int o = 4 * ch + q, m = o / WG::NO, co = o - m * WG::NO;
    poff[ch] = pbase + (m + kr) * G::RS + 16 * co;
    const int sc = 8 * co + 8 - jj;  // padded dz column of the oct's first element
    qoff[ch] = qbase + m * WG::DZR + (sc & 1) * (2 * WG::DZC) + (sc >> 1) * 4;
  }
  f32x4 acc[CPW];
#pragma unroll
  for (int t = 0; t < CPW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  int t = part;
  if (t < g.ntiles) load_tile(t);
  for (; t < g.ntiles; t += nparts) {
    __syncthreads();  // the previous tile's MFMAs are done with the planes
    xp.store(tin, wvu, lane);
    store_dz();
    __syncthreads();
    if (t + nparts < g.ntiles) load_tile(t + nparts);  // in flight under this tile's MFMAs
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      // the wave's plane offsets are in poff / qoff; channel c of the wave adds c planes (immediate offsets: a wave's
      // channels start on a skew-group boundary or share one group, so the skew step is c / EPC)
      static_assert(CPW % EPC == 0 || EPC % CPW == 0, "skew groups");
      const uint32_t pc = (uint32_t)(c * G::PS + (CPW % EPC == 0 ? (c / EPC) : 0) * SKEW);
      const uint32_t qc = (uint32_t)(c * WG::DZPS);
#pragma unroll
      for (int ch = 0; ch < WG::NCH; ++ch) {
        typedef const __attribute__((address_space(3))) bf16x8* lds_v8;
        const bf16x8 pv = *(lds_v8)(size_t)(poff[ch] + pc);
        const __attribute__((address_space(3))) uint32_t* qp =
            (const __attribute__((address_space(3))) uint32_t*)(size_t)(qoff[ch] + qc);
        const uint32_t q4[4] = {qp[0], qp[1], qp[2], qp[3]};
        acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pv, __builtin_bit_cast(bf16x8, q4), acc[c], 0, 0, 0);
      }
    }
  }
  // lane (j = lane & 15, q) holds D[4q + r][j] = dW[kr = 4q + r][j] of channel CPW wv + c
#pragma unroll
  for (int c = 0; c < CPW; ++c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int krr = 4 * q + r;
      if (krr < 7 && li < 7) dw_part[(size_t)part * g.C * 49 + (size_t)(c0 + wvu * CPW + c) * 49 + krr * 7 + li] = acc[c][r];
    }
  // bias gradient: the dz sums of the threads holding each 8-channel chunk, in thread order through LDS
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);  // [kThreads][8]
#pragma unroll
  for (int e = 0; e < 8; ++e) red[tid * 8 + e] = dbs[e];
  __syncthreads();
  if (tid < CG) {
    const int chk = tid / 8, e = tid % 8;
    float sum = 0.f;
    for (int u = chk; u < kThreads; u += C8) sum += red[u * 8 + e];
    db_part[(size_t)part * g.C + c0 + tid] = sum;
  }
}

static DwmGeo geo(int B, int H, int W, int C, int tw) {
  DwmGeo g{B, H, W, C, (W + tw - 1) / tw, (H + TH - 1) / TH, 0};
  g.ntiles = B * g.tilesW * g.tilesH;
  return g;
}

template <typename TIN, bool FLIP, int MODE, int NB, int CG>
static int launch1(const void* x, const float* wdw, const float* bdw, void* out, uint16_t* out_bf16, int B, int H,
                   int W, int C, hipStream_t s) {
  using G = Geo<NB, CG>;
  const DwmGeo g = geo(B, H, W, C, G::TW);
  const long long grid = (long long)g.ntiles * (C / CG);
  if (grid > 0x7fffffffLL) return set_error(SV_ERR_INVALID_ARG, "dwconv7 mfma: grid too large");
  auto k = &dw7_mfma_kernel<TIN, FLIP, MODE, NB, CG>;
  if (const int rc = ensure_lds_attr(reinterpret_cast<const void*>(k), G::LDS, s)) return rc;
  k<<<(int)grid, kThreads, G::LDS, s>>>((const TIN*)x, wdw, bdw, out, out_bf16, g);
  return check_launch("sv_dwconv7 (mfma)");
}

// Channels per workgroup: 16 (40 KiB of LDS, 4 workgroups per CU) or 32 (79 KiB, 2).  Measured (r13l, ConvNeXt-base
// bs32 standalone): the forward is faster with 16 at every stage (S3 + LayerNorm 35.3 vs 40.9 us, S1 160 vs 168); the
// backward-data with 16 at C >= 512 (S3 33.3 vs 36.5, S4 19.3 vs 23.8) and with 32 at C = 128 (S1 190 vs 211).
// SV_DW_MFMA_CG=16 / 32 forces one (A/B).
static int cg_choice(int mode, int C) {
  static const int v = getenv("SV_DW_MFMA_CG") ? atoi(getenv("SV_DW_MFMA_CG")) : 0;
  if (v == 16 || v == 32) return v;
  return (mode != 0 && C <= 256) ? 32 : 16;
}

template <typename TIN, bool FLIP, int MODE, int NB>
static int launch(const void* x, const float* wdw, const float* bdw, void* out, uint16_t* out_bf16, int B, int H,
                  int W, int C, hipStream_t s) {
  if (cg_choice(MODE, C) == 16 || C % 32 != 0)
    return launch1<TIN, FLIP, MODE, NB, 16>(x, wdw, bdw, out, out_bf16, B, H, W, C, s);
  return launch1<TIN, FLIP, MODE, NB, 32>(x, wdw, bdw, out, out_bf16, B, H, W, C, s);
}

constexpr int kWgradCG = 16;  // the weight gradient's channels per workgroup (its dz planes double the LDS)

static int wgrad_nparts(int B, int H, int W, int C) {
  const int nb = W > 16 ? 2 : 1;
  const DwmGeo g = geo(B, H, W, C, 16 * nb);
  const int ncg = C / kWgradCG;
  int np = 512 / (ncg > 0 ? ncg : 1);  // ~two workgroups per CU over all channel groups
  if (np > g.ntiles) np = g.ntiles;
  return np < 1 ? 1 : np;
}

template <typename TIN, int NB>
static int launch_wgrad(const uint16_t* dz, const void* x, float* dw_part, float* db_part, int B, int H, int W, int C,
                        hipStream_t s) {
  using WG = WGeo<NB, kWgradCG>;
  const DwmGeo g = geo(B, H, W, C, 16 * NB);
  const int np = wgrad_nparts(B, H, W, C);
  const int grid = np * (C / kWgradCG);
  auto k = &dw7_wgrad_mfma_kernel<TIN, NB, kWgradCG>;
  if (const int rc = ensure_lds_attr(reinterpret_cast<const void*>(k), WG::LDS, s)) return rc;
  k<<<grid, kThreads, WG::LDS, s>>>(dz, (const TIN*)x, dw_part, db_part, np, g);
  return check_launch("sv_dwconv7_bwd_weight_mfma");
}

}  // namespace dwm
}  // namespace sv

using namespace sv;

extern "C" {

int sv_dwconv7_fwd_mfma(const void* x, int32_t x_dtype, const float* wdw, const float* bdw, uint16_t* z, int32_t B,
                        int32_t H, int32_t W, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(x && wdw && bdw && z, "sv_dwconv7_fwd_mfma: null pointer");
  SV_REQUIRE(C % dwm::kCGMin == 0 && C > 0, "sv_dwconv7_fwd_mfma: C=%d must be a multiple of 16", C);
  SV_REQUIRE(x_dtype == SV_F32 || x_dtype == SV_BF16, "sv_dwconv7_fwd_mfma: bad x dtype");
  SV_REQUIRE(x != (const void*)z, "sv_dwconv7_fwd_mfma: x and z must not alias");
  SV_REQUIRE((size_t)H * W * C * (x_dtype == SV_F32 ? 4 : 2) < 0x7fffffffull,
             "sv_dwconv7_fwd_mfma: one image of x over 2 GiB (buffer-descriptor range)");
  if (B <= 0 || H <= 0 || W <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const bool nb2 = W > 16;
  if (x_dtype == SV_F32)
    return nb2 ? dwm::launch<float, false, 0, 2>(x, wdw, bdw, z, nullptr, B, H, W, C, s)
               : dwm::launch<float, false, 0, 1>(x, wdw, bdw, z, nullptr, B, H, W, C, s);
  return nb2 ? dwm::launch<uint16_t, false, 0, 2>(x, wdw, bdw, z, nullptr, B, H, W, C, s)
             : dwm::launch<uint16_t, false, 0, 1>(x, wdw, bdw, z, nullptr, B, H, W, C, s);
}

int sv_dwconv7_bwd_data_mfma(const uint16_t* dz, const float* wdw, float* dx, uint16_t* dx_bf16, int32_t accumulate,
                             int32_t B, int32_t H, int32_t W, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(dz && wdw && dx, "sv_dwconv7_bwd_data_mfma: null pointer");
  SV_REQUIRE(C % dwm::kCGMin == 0 && C > 0, "sv_dwconv7_bwd_data_mfma: C=%d must be a multiple of 16", C);
  SV_REQUIRE((const void*)dz != (const void*)dx && (const void*)dz != (const void*)dx_bf16,
             "sv_dwconv7_bwd_data_mfma: dz must not alias dx / dx_bf16");
  SV_REQUIRE((size_t)H * W * C * 2 < 0x7fffffffull, "sv_dwconv7_bwd_data_mfma: one image of dz over 2 GiB");
  if (B <= 0 || H <= 0 || W <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const bool nb2 = W > 16;
  if (accumulate)
    return nb2 ? dwm::launch<uint16_t, true, 2, 2>(dz, wdw, nullptr, dx, dx_bf16, B, H, W, C, s)
               : dwm::launch<uint16_t, true, 2, 1>(dz, wdw, nullptr, dx, dx_bf16, B, H, W, C, s);
  return nb2 ? dwm::launch<uint16_t, true, 1, 2>(dz, wdw, nullptr, dx, dx_bf16, B, H, W, C, s)
             : dwm::launch<uint16_t, true, 1, 1>(dz, wdw, nullptr, dx, dx_bf16, B, H, W, C, s);
}

int sv_dwconv7_bwd_weight_mfma_nparts(int32_t B, int32_t H, int32_t W, int32_t C) {
  return dwm::wgrad_nparts(B, H, W, C);
}

int sv_dwconv7_bwd_weight_mfma(const uint16_t* dz, const void* x, int32_t x_dtype, float* dw_part, float* db_part,
                               int32_t B, int32_t H, int32_t W, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(dz && x && dw_part && db_part, "sv_dwconv7_bwd_weight_mfma: null pointer");
  SV_REQUIRE(C % dwm::kWgradCG == 0 && C > 0, "sv_dwconv7_bwd_weight_mfma: C=%d must be a multiple of 16", C);
  SV_REQUIRE(x_dtype == SV_F32 || x_dtype == SV_BF16, "sv_dwconv7_bwd_weight_mfma: bad x dtype");
  SV_REQUIRE((size_t)B * H * W * C * 2 < 0x7fffffffull && (size_t)H * W * C * 4 < 0x7fffffffull,
             "sv_dwconv7_bwd_weight_mfma: dz over 2 GiB / one image of x over 2 GiB");
  if (B <= 0 || H <= 0 || W <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const bool nb2 = W > 16;
  if (x_dtype == SV_F32)
    return nb2 ? dwm::launch_wgrad<float, 2>(dz, x, dw_part, db_part, B, H, W, C, s)
               : dwm::launch_wgrad<float, 1>(dz, x, dw_part, db_part, B, H, W, C, s);
  return nb2 ? dwm::launch_wgrad<uint16_t, 2>(dz, x, dw_part, db_part, B, H, W, C, s)
             : dwm::launch_wgrad<uint16_t, 1>(dz, x, dw_part, db_part, B, H, W, C, s);
}

}  // extern "C"
