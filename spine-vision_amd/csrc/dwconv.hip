// Depthwise 7x7 convolution (pad 3, stride 1) on NHWC activations -- ConvNeXtBlock.conv_dw
// (timm convnext.py; HF equivalent transformers/models/convnext/modeling_convnext.py:130,144).
//
// Layout/tiling (gfx950): one WAVE owns a 16-row x 4-column output strip of one image for one
// 64-channel group (lane == channel, so every global access of a wave is 64 consecutive channels:
// 256 B f32 / 128 B bf16, fully coalesced).  The wave streams the 22 input rows of its strip once,
// top to bottom, through a wave-private LDS ring filled by LDS-DMA: each 10-wide input row feeds the
// 7 output rows it touches, with a rolling set of 7 output-row accumulators -- an output row is
// stored as soon as its 7th input row has been consumed.  No barriers: the halo re-reads are row
// re-reads that the CU's L1 / the XCD's L2 absorb, and the HBM traffic is one read of the input and
// one write of the output.
//
// The op is HBM-bound (49 FMA per 4-8 bytes moved).
//
//   fwd          z = b + sum_tap w[tap] * x[p + tap]               (+ LayerNorm via ln_fwd)
//   bwd-data     dx = (acc ? dx : 0) + sum_tap w[48 - tap] * dz[p + tap]   (flipped kernel)
//   bwd-weight   dW[c][tap] = sum_p dz[p,c] * x[p + tap, c],  db[c] = sum_p dz[p,c]
//                (same streaming with a rolling set of 7 dz rows; per-workgroup partials)
#include "common.h"

#include <stdlib.h>

extern "C" int sv_layernorm_fwd(const void* x, int32_t x_dtype, const float* w, const float* b, void* y,
                                int32_t y_dtype, float* mean, float* rstd, int64_t rows, int32_t C,
                                float eps, sv_stream_t stream);

namespace sv {

constexpr int TH = 16;          // output rows per wave strip
constexpr int TR = TH + 6;      // input rows the strip reads
constexpr int kDwThreads = 256;  // 4 independent waves per workgroup

struct DwGeo {
  int B, H, W, C, tw, tilesW, tilesH, ntiles;  // tw = strip width (output columns per lane)
  int xcd;                                      // XCD-contiguous block order (xcd_block)
};

__device__ __forceinline__ void dw_tile(const DwGeo& g, int tile, int& b, int& h0, int& w0) {
  const int tw = tile % g.tilesW;
  const int t = tile / g.tilesW;
  const int th = t % g.tilesH;
  b = t / g.tilesH;
  h0 = th * TH;
  w0 = tw * g.tw;
}

// ---------------------------------------------------------------------------------------------
// Ring kernels: per-wave strip streaming (above); the input rows arrive through a
// wave-private LDS ring filled by LDS-DMA (global_load_lds, one 64-lane column per instruction)
// PF-1 rows ahead of the row being consumed; the prefetch costs no VGPRs.  Everything except the
// channel is wave-uniform, so the strip geometry lives in SGPRs (readfirstlane'd wave id) and every
// global address is an SGPR base + the lane's channel offset: the per-row address arithmetic and the
// bounds checks run on the scalar unit.  Padding costs nothing in the FMA stream: an out-of-image
// column or row is DMA'd from a zero page, so the consumer reads LDS unconditionally.  No barriers:
// each wave only reads rows its own DMA wrote, ordered by a counted `s_waitcnt vmcnt` (the DMA rows
// issued after row ir may stay in flight; stores and loads interleaved with them only make the wait
// conservative).
typedef __attribute__((address_space(3))) void dw_lds_void;

__device__ __attribute__((aligned(256))) float dw_zero_page[64];  // zero-initialised, never written

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until only the DMA rows issued after the current one (`younger` rows of NL instructions) may
// still be outstanding
template <int PF, int NL>
__device__ __forceinline__ void wait_rows(int younger) {
  static_assert((PF - 1) * NL <= 63, "vmcnt immediate");
  if (PF > 3 && younger >= 3) vm_wait<(PF > 3 ? 3 * NL : 0)>();
  else if (PF > 2 && younger >= 2) vm_wait<(PF > 2 ? 2 * NL : 0)>();
  else if (younger >= 1) vm_wait<NL>();
  else vm_wait<0>();
}

__device__ __forceinline__ int wave_id_uniform() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// XCD-contiguous block order: blocks are dealt round-robin over the 8 XCDs (b, b + 8, ... share one), so
// consecutive block indices -- neighbouring strips, whose 3-pixel halos overlap -- would land on different XCDs
// and each XCD's L2 would fetch the shared halo rows / columns again.  Block b works on logical block
// (b % 8) * (G / 8) + b / 8 instead: each XCD walks a contiguous range of strips and the halo re-reads hit its
// own L2 (G % 8 == 0; otherwise the identity).  `xcd` = 0 disables it (A/B).
__device__ __forceinline__ int xcd_block(int b, int G, int xcd) {
  return (xcd && (G & 7) == 0) ? (b & 7) * (G >> 3) + (b >> 3) : b;
}

// LDS image of one input row: NCOL columns x the wave's 64 channels, packed ([column][channel], 64 *
// sizeof(T) bytes per column).  DMA'd 16 B per lane (global_load_lds_dwordx4): one instruction moves
// 1 KiB = CPD columns (4 f32 / 8 bf16), lane L fetching channels (L % LPC) * EPL .. of column L / LPC.
// Round 1 moved one 4-B dword per lane per column (10 DMAs per f32 or bf16 row of a 4-wide strip,
// 256 B each): the kernels took the same time for bf16 and f32 inputs, i.e. they were DMA-issue-bound.
template <typename T>
struct DwRow {
  static constexpr int CB = 64 * (int)sizeof(T);  // bytes per column
  static constexpr int CPD = 1024 / CB;           // columns per DMA instruction
  static constexpr int LPC = 64 / CPD;            // lanes per column
  static constexpr int EPL = 16 / (int)sizeof(T);  // elements per lane chunk
  template <int NCOL>
  static constexpr int nd() { return (NCOL + CPD - 1) / CPD; }  // DMA instructions per row
  template <int NCOL>
  static constexpr int bytes() { return nd<NCOL>() * 1024; }
};

// DMA the NCOL columns wstart .. wstart+NCOL-1 of row h of the wave's channel group (xg = x + c0,
// uniform) into dst.  Out-of-image rows / columns, and the columns past NCOL that fill the last
// instruction, read the zero page, so every row costs the same fixed number of DMAs.
template <int NCOL, typename T>
__device__ __forceinline__ void dma_row(const T* __restrict__ xg, const DwGeo& g, int b, int h, int wstart, int lane,
                                        char* dst) {
  using R = DwRow<T>;
  const bool okh = h >= 0 && h < g.H;
  const T* rowp = xg + (size_t)((b * g.H + (okh ? h : 0)) * g.W) * g.C;
  const T* zero = reinterpret_cast<const T*>(dw_zero_page);
  const int jl = lane / R::LPC, ch = (lane % R::LPC) * R::EPL;
#pragma unroll
  for (int d = 0; d < R::template nd<NCOL>(); ++d) {
    const int j = d * R::CPD + jl, w = wstart + j;
    const bool ok = okh && j < NCOL && w >= 0 && w < g.W;
    const T* src = ok ? rowp + (size_t)w * g.C + ch : zero + ch;
    __builtin_amdgcn_global_load_lds((const void*)src, (dw_lds_void*)(dst + d * 1024), 16, 0, 0);
  }
}
template <typename T>
__device__ __forceinline__ float lds_ld(const char* row, int j, int lane) {
  if constexpr (sizeof(T) == 4) return *reinterpret_cast<const float*>(row + j * DwRow<T>::CB + lane * 4);
  else return bf2f(*reinterpret_cast<const uint16_t*>(row + j * DwRow<T>::CB + lane * 2));
}

template <int PF, int TW, typename TIN>
constexpr size_t dw_ring_lds() {
  return (size_t)(kDwThreads / 64) * PF * DwRow<TIN>::template bytes<TW + 6>();
}

template <int PF, int TW, typename TIN, typename TOUT, bool FLIP, bool ACCUM>
__global__ void __launch_bounds__(kDwThreads) dwconv7_ring_kernel(const TIN* __restrict__ x,
                                                                  const float* __restrict__ wdw,
                                                                  const float* __restrict__ bdw,
                                                                  TOUT* __restrict__ out,
                                                                  uint16_t* __restrict__ out_bf16, DwGeo g) {
  extern __shared__ __attribute__((aligned(16))) char dw_smem[];
  constexpr int TC = TW + 6;
  constexpr int ROWB = DwRow<TIN>::template bytes<TC>();
  constexpr int NL = DwRow<TIN>::template nd<TC>();  // DMA instructions per row
  const int lane = threadIdx.x & 63, wv = wave_id_uniform();
  const int gw = xcd_block(blockIdx.x, gridDim.x, g.xcd) * (kDwThreads / 64) + wv;
  const int ncg = g.C / 64;
  if (gw >= g.ntiles * ncg) return;  // whole wave; no barriers below
  char* ring = dw_smem + wv * PF * ROWB;
  const int tile = gw % g.ntiles, c0 = (gw / g.ntiles) * 64, c = c0 + lane;
  int b, h0, w0;
  dw_tile(g, tile, b, h0, w0);
  const TIN* xg = x + c0;
  TOUT* og = out + c0;
  uint16_t* obg = out_bf16 ? out_bf16 + c0 : nullptr;
  float wk[49];
#pragma unroll
  for (int i = 0; i < 49; ++i) wk[i] = wdw[(size_t)c * 49 + (FLIP ? 48 - i : i)];
  const float bias = bdw ? bdw[c] : 0.f;
  float acc[7][TW];
#pragma unroll
  for (int r = 0; r < 7; ++r)
#pragma unroll
    for (int o = 0; o < TW; ++o) acc[r][o] = bias;
  float in[TC];
  float pcur[TW], pnew[TW];
#pragma unroll
  for (int o = 0; o < TW; ++o) pcur[o] = pnew[o] = 0.f;
#pragma unroll
  for (int p = 0; p < PF - 1; ++p) dma_row<TC>(xg, g, b, h0 - 3 + p, w0 - 3, lane, ring + p * ROWB);
#pragma nounroll
  for (int ib = 0; ib < TR; ib += 7) {
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int ir = ib + u;
      if (ir >= TR) break;
      if (ir + PF - 1 < TR) dma_row<TC>(xg, g, b, h0 - 3 + ir + PF - 1, w0 - 3, lane, ring + ((ir + PF - 1) % PF) * ROWB);
      const int rem = TR - 1 - ir;
      wait_rows<PF, NL>(rem < PF - 1 ? rem : PF - 1);
      const char* row = ring + (ir % PF) * ROWB;
#pragma unroll
      for (int j = 0; j < TC; ++j) in[j] = lds_ld<TIN>(row, j, lane);
      if (ACCUM && ir >= 5 && ir - 5 < TH) {
        const int h = h0 + ir - 5;
        if (h < g.H) {
          const TOUT* prow = og + ((size_t)b * g.H + h) * g.W * g.C;
#pragma unroll
          for (int o = 0; o < TW; ++o) pnew[o] = (w0 + o < g.W) ? ld(prow + (size_t)(w0 + o) * g.C, lane) : 0.f;
        }
      }
#pragma unroll
      for (int kh = 0; kh < 7; ++kh) {
        const int orow = ir - kh;
        if (orow < 0 || orow >= TH) continue;
        const int sl = (u - kh + 7) % 7;
#pragma unroll
        for (int o = 0; o < TW; ++o)
#pragma unroll
          for (int kw = 0; kw < 7; ++kw) acc[sl][o] = fmaf(wk[kh * 7 + kw], in[o + kw], acc[sl][o]);
      }
      if (ir >= 6) {
        const int orow = ir - 6;
        const int sl = (u + 1) % 7;
        const int h = h0 + orow;
        if (h < g.H) {
          const size_t rbase = ((size_t)b * g.H + h) * g.W;
#pragma unroll
          for (int o = 0; o < TW; ++o) {
            if (w0 + o < g.W) {
              const size_t i = (rbase + w0 + o) * g.C;
              const float v = ACCUM ? pcur[o] + acc[sl][o] : acc[sl][o];
              st(og + i, lane, v);
              if (obg) obg[i + lane] = f2bf(v);
            }
          }
        }
#pragma unroll
        for (int o = 0; o < TW; ++o) acc[sl][o] = bias;
      }
      if (ACCUM) {
#pragma unroll
        for (int o = 0; o < TW; ++o) pcur[o] = pnew[o];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// backward-weight with the ring: per input row ir the wave DMAs the TC-wide x row h0-3+ir and the
// TW-wide dz row h0+ir (rows past the strip's TH read the zero page, which keeps the per-row
// instruction count fixed and contributes nothing)
template <int PF, int TW, typename TDZ, typename TIN>
constexpr size_t dw_wgrad_ring_lds() {
  return (size_t)(kDwThreads / 64) * PF * (DwRow<TIN>::template bytes<TW + 6>() + DwRow<TDZ>::template bytes<TW>());
}

template <int PF, int TW, typename TDZ, typename TIN>
__global__ void __launch_bounds__(kDwThreads) dwconv7_wgrad_ring_kernel(const TDZ* __restrict__ dz,
                                                                        const TIN* __restrict__ x,
                                                                        float* __restrict__ dw_part,
                                                                        float* __restrict__ db_part, DwGeo g) {
  extern __shared__ __attribute__((aligned(16))) char dw_smem[];
  constexpr int TC = TW + 6;
  constexpr int XB = DwRow<TIN>::template bytes<TC>();  // x part of a ring slot; the dz row follows
  constexpr int ROWB = XB + DwRow<TDZ>::template bytes<TW>();
  constexpr int NL = DwRow<TIN>::template nd<TC>() + DwRow<TDZ>::template nd<TW>();
  const int lane = threadIdx.x & 63, wv = wave_id_uniform();
  const int c0 = blockIdx.y * 64;
  const TIN* xg = x + c0;
  const TDZ* dg = dz + c0;
  char* ring = dw_smem + wv * PF * ROWB;
  float acc[49];
#pragma unroll
  for (int i = 0; i < 49; ++i) acc[i] = 0.f;
  float dbacc = 0.f;
  const int lb = xcd_block(blockIdx.x, gridDim.x, g.xcd);  // logical block: its tiles AND its partial row
  for (int tile = lb * 4 + wv; tile < g.ntiles; tile += gridDim.x * 4) {
    int b, h0, w0;
    dw_tile(g, tile, b, h0, w0);
    auto issue = [&](int ir) {
      char* slot = ring + (ir % PF) * ROWB;
      dma_row<TC>(xg, g, b, h0 - 3 + ir, w0 - 3, lane, slot);
      dma_row<TW>(dg, g, b, ir < TH ? h0 + ir : -1, w0, lane, slot + XB);
    };
    float dzb[7][TW];
    float in[TC];
#pragma unroll
    for (int p = 0; p < PF - 1; ++p) issue(p);
#pragma nounroll
    for (int ib = 0; ib < TR; ib += 7) {
#pragma unroll
      for (int u = 0; u < 7; ++u) {
        const int ir = ib + u;
        if (ir >= TR) break;
        if (ir + PF - 1 < TR) issue(ir + PF - 1);
        const int rem = TR - 1 - ir;
        wait_rows<PF, NL>(rem < PF - 1 ? rem : PF - 1);
        const char* row = ring + (ir % PF) * ROWB;
#pragma unroll
        for (int j = 0; j < TC; ++j) in[j] = lds_ld<TIN>(row, j, lane);
        if (ir < TH) {
#pragma unroll
          for (int o = 0; o < TW; ++o) {
            const float v = lds_ld<TDZ>(row + XB, o, lane);
            dzb[u][o] = v;
            dbacc += v;
          }
        }
#pragma unroll
        for (int kh = 0; kh < 7; ++kh) {
          const int orow = ir - kh;
          if (orow < 0 || orow >= TH) continue;
          const int sl = (u - kh + 7) % 7;
#pragma unroll
          for (int kw = 0; kw < 7; ++kw) {
            float s = acc[kh * 7 + kw];
#pragma unroll
            for (int o = 0; o < TW; ++o) s = fmaf(dzb[sl][o], in[o + kw], s);
            acc[kh * 7 + kw] = s;
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  // every wave's DMAs have landed (its last row waited with vmcnt(0)); reuse LDS as the combine
  // buffer [49 taps][64] + [64], the 4 waves adding in turn (fixed order, 12.8 KiB)
  float* red = reinterpret_cast<float*>(dw_smem);
  float* redb = red + 49 * 64;
  __syncthreads();
  for (int k = 0; k < 4; ++k) {
    if (wv == k) {
#pragma unroll
      for (int i = 0; i < 49; ++i) red[i * 64 + lane] = (k ? red[i * 64 + lane] : 0.f) + acc[i];
      redb[lane] = (k ? redb[lane] : 0.f) + dbacc;
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < 64 * 49; i += kDwThreads) {
    const int ch = i / 49, tap = i - ch * 49;
    dw_part[(size_t)lb * g.C * 49 + (size_t)(c0 + ch) * 49 + tap] = red[tap * 64 + ch];
  }
  if (threadIdx.x < 64) db_part[(size_t)lb * g.C + c0 + threadIdx.x] = redb[threadIdx.x];
}

// ring depths: f32 input rows (3 KiB for a 4-wide strip) 3 deep, so four workgroups fit a CU as with bf16
// rows (2 KiB) 4 deep (measured, f32 4 -> 3: S3 bwd-data over an f32 gradient 57-64 -> 46-51 us, the step
// unchanged within noise; bf16 4 -> 5 or 6 slower); the wgrad ring holds x AND dz rows (14 columns), so
// depth 2 keeps 4 workgroups per CU (measured: 2 >= 3, 4 on the S1/S3 shapes).  Strip width 4 keeps a lane
// within 3 waves/SIMD; the register-prefetch (no ring) kernels and 8-wide strips measured slower (round 1).
constexpr int DW_PF_F32 = 3, DW_PF_BF16 = 4, DW_WGRAD_PF = 2, DW_TW = 4;
template <typename T>
constexpr int dw_pf() { return sizeof(T) == 4 ? DW_PF_F32 : DW_PF_BF16; }

static DwGeo dw_geo(int B, int H, int W, int C) {
  static const int xcd = getenv("SV_DW_XCD") ? atoi(getenv("SV_DW_XCD")) : 1;  // A/B runs: 0 = dispatch order
  DwGeo g{B, H, W, C, DW_TW, (W + DW_TW - 1) / DW_TW, (H + TH - 1) / TH, 0, xcd};
  g.ntiles = B * g.tilesW * g.tilesH;
  return g;
}

static int dw_blocks(const DwGeo& g) { return ceil_div((long long)g.ntiles * (g.C / 64), kDwThreads / 64); }

// ---------------------------------------------------------------------------------------------
// Depthwise conv + LayerNorm in ONE pass (timm ConvNeXtBlock: conv_dw -> norm): one workgroup per strip with one wave
// per 64-channel group (C / 64 waves), so every output row of the strip holds all C channels of its TW pixels inside
// the workgroup.  Per output row the waves park the values as stored (z rounded to its dtype) in an LDS tile [TW][C];
// the first TW * LPR lanes then reduce each pixel exactly as ln_fwd_vec_kernel<LPR, NV> (norm.hip) does -- lane l sums
// channels 8 (l + LPR j) .. +7 in order, then the LPR-lane butterfly, then the centred second pass -- and every wave
// normalises its own channel.  y, mean and rstd are bit for bit the two-launch result (dwconv ring kernel, then the
// vectorised LayerNorm over z), without z's HBM round trip, and without z at all when the caller keeps none (the eval
// forward).  Two workgroup barriers per output row; the LDS tile is accessed through inline asm so the compiler's
// LDS-DMA alias tracking does not drain the ring's prefetches (vmcnt(0)) before each access.
__device__ __forceinline__ void lds_st_f32(float* p, float v) {
  const uint32_t a = (uint32_t)(size_t)(__attribute__((address_space(3))) char*)(p);
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_ld8_f32(const float* p, float (&v)[8]) {
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t a, b;
  const uint32_t o = (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p);
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(a), "=v"(b)
               : "v"(o)
               : "memory");
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ float2 lds_ld2_f32(const float* p) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  f32x2_t a;
  const uint32_t o = (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p);
  asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(a) : "v"(o) : "memory");
  return make_float2(a.x, a.y);
}
// workgroup barrier that waits for this wave's LDS operations only (not for the ring's DMAs in flight)
__device__ __forceinline__ void wg_bar_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <typename T>
__device__ __forceinline__ float as_stored(float v) {
  if constexpr (sizeof(T) == 4) return v;
  else return bf2f(f2bf(v));
}
// norm.hip group_sum<LPR>'s butterfly, bitwise, from the cross-lane unit (common.h)
template <int LPR>
__device__ __forceinline__ float dw_group_sum(float v) {
  return xlane_group_sum<LPR>(v);
}

template <int PF, int TW, typename TIN, typename TOUT, int NWV, int LPR, int NV>
constexpr size_t dw_ln_lds() {
  return (size_t)NWV * PF * DwRow<TIN>::template bytes<TW + 6>() + (size_t)TW * 64 * NWV * 4;
}

template <int PF, int TW, typename TIN, typename TOUT, int NWV, int LPR, int NV>
__global__ void __launch_bounds__(64 * NWV) dwconv7_ln_ring_kernel(const TIN* __restrict__ x,
                                                                   const float* __restrict__ wdw,
                                                                   const float* __restrict__ bdw,
                                                                   const float* __restrict__ lnw,
                                                                   const float* __restrict__ lnb, float eps,
                                                                   TOUT* __restrict__ z, TOUT* __restrict__ y,
                                                                   float* __restrict__ mean, float* __restrict__ rstd,
                                                                   DwGeo g) {
  constexpr int C = 64 * NWV;
  static_assert(8 * LPR * NV == C, "LayerNorm lane geometry (norm.hip ln_vec_kind)");
  static_assert((TW * LPR) % 64 == 0 && TW * LPR <= 64 * NWV, "the statistics lanes are whole waves");
  extern __shared__ __attribute__((aligned(16))) char dw_smem[];
  constexpr int TC = TW + 6;
  constexpr int ROWB = DwRow<TIN>::template bytes<TC>();
  constexpr int NL = DwRow<TIN>::template nd<TC>();  // DMA instructions per row
  const int lane = threadIdx.x & 63, wv = wave_id_uniform();
  int b, h0, w0;
  dw_tile(g, xcd_block(blockIdx.x, gridDim.x, g.xcd), b, h0, w0);
  const int c0 = wv * 64, c = c0 + lane;
  char* ring = dw_smem + wv * PF * ROWB;
  // [TW][C]: the output row as stored; after the statistics pass, pixel p's mean / rstd in its first two slots, so the
  // whole LDS is 80 KiB at C = 512 (two workgroups per CU; a separate statistics array would push it past 160 KiB per
  // two).  Every wave reads those slots after the second barrier of the row and wave 0 overwrites them with its next
  // row's channel-0/1 values: a third barrier after the reads orders the reuse
  float* zt = reinterpret_cast<float*>(dw_smem + NWV * PF * ROWB);
  const TIN* xg = x + c0;
  float wk[49];
#pragma unroll
  for (int i = 0; i < 49; ++i) wk[i] = wdw[(size_t)c * 49 + i];
  const float bias = bdw[c], lw = lnw[c], lb = lnb[c];
  const float invC = 1.0f / (float)C;
  float acc[7][TW];
#pragma unroll
  for (int r = 0; r < 7; ++r)
#pragma unroll
    for (int o = 0; o < TW; ++o) acc[r][o] = bias;
  float in[TC];
#pragma unroll
  for (int p = 0; p < PF - 1; ++p) dma_row<TC>(xg, g, b, h0 - 3 + p, w0 - 3, lane, ring + p * ROWB);
#pragma nounroll
  for (int ib = 0; ib < TR; ib += 7) {
#pragma unroll
    for (int u = 0; u < 7; ++u) {
      const int ir = ib + u;
      if (ir >= TR) break;
      if (ir + PF - 1 < TR) dma_row<TC>(xg, g, b, h0 - 3 + ir + PF - 1, w0 - 3, lane, ring + ((ir + PF - 1) % PF) * ROWB);
      const int rem = TR - 1 - ir;
      wait_rows<PF, NL>(rem < PF - 1 ? rem : PF - 1);
      const char* row = ring + (ir % PF) * ROWB;
#pragma unroll
      for (int j = 0; j < TC; ++j) in[j] = lds_ld<TIN>(row, j, lane);
#pragma unroll
      for (int kh = 0; kh < 7; ++kh) {
        const int orow = ir - kh;
        if (orow < 0 || orow >= TH) continue;
        const int sl = (u - kh + 7) % 7;
#pragma unroll
        for (int o = 0; o < TW; ++o)
#pragma unroll
          for (int kw = 0; kw < 7; ++kw) acc[sl][o] = fmaf(wk[kh * 7 + kw], in[o + kw], acc[sl][o]);
      }
      if (ir >= 6) {  // output row ir - 6 is complete (workgroup-uniform)
        const int sl = (u + 1) % 7;
        const int h = h0 + ir - 6;
        const bool okh = h < g.H;
        const size_t rbase = ((size_t)b * g.H + (okh ? h : 0)) * g.W;
        float zq[TW];
#pragma unroll
        for (int o = 0; o < TW; ++o) {
          zq[o] = as_stored<TOUT>(acc[sl][o]);
          if (z && okh && w0 + o < g.W) st(z + (rbase + w0 + o) * C + c0, lane, acc[sl][o]);
          lds_st_f32(zt + o * C + c, zq[o]);
          acc[sl][o] = bias;
        }
        wg_bar_lds();
        if (threadIdx.x < TW * LPR) {  // whole waves: pixel p, LayerNorm lane l (ln_fwd_vec_kernel's reduction)
          const int p = threadIdx.x / LPR, l = threadIdx.x % LPR;
          float v[NV][8];
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < NV; ++j) {
            lds_ld8_f32(zt + p * C + (l + LPR * j) * 8, v[j]);
#pragma unroll
            for (int e = 0; e < 8; ++e) s += v[j][e];
          }
          const float mu = dw_group_sum<LPR>(s) * invC;
          // the centred second pass as norm.hip's build of ln_fwd_vec_kernel evaluates it (its SLP-packed
          // v_pk_mul_f32 rounds each square before the add; the variance's scale and eps are one fma)
          float q = 0.f;
          {
#pragma clang fp contract(off)
#pragma unroll
            for (int j = 0; j < NV; ++j)
#pragma unroll
              for (int e = 0; e < 8; ++e) {
                const float d = v[j][e] - mu;
                q += d * d;
              }
          }
          const float rs = rsqrtf(fmaf(dw_group_sum<LPR>(q), invC, eps));
          if (l == 0) {
            lds_st_f32(zt + p * C, mu);
            lds_st_f32(zt + p * C + 1, rs);
            if (okh && w0 + p < g.W) {
              mean[rbase + w0 + p] = mu;
              rstd[rbase + w0 + p] = rs;
            }
          }
        }
        wg_bar_lds();
#pragma unroll
        for (int o = 0; o < TW; ++o) {
          const float2 m = lds_ld2_f32(zt + o * C);
          if (okh && w0 + o < g.W) st(y + (rbase + w0 + o) * C + c0, lane, (zq[o] - m.x) * m.y * lw + lb);
        }
        wg_bar_lds();  // every wave has read the statistics slots before any wave stores the next row into zt
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// the one-pass form: C = 128 / 256 / 512 (the C / 64 waves of a strip fit one workgroup with two or more workgroups per
// CU), an f32 input (the residual stream) and z / y of one dtype.  It runs where the caller keeps no z (z == NULL: the
// eval forward), and there measured +2.4 % (3485 / 3467 vs 3390 / 3400 img/s interleaved); where z is kept (training) it
// measured no faster than the two launches (1092.9 / 1089.5 vs 1096.4 / 1092.0 img/s): the two barriers per output row
// tie the strip's waves together, which costs what the z re-read saves (profiles/round5/r11z_dw_ln_fused_ab.txt).
// SV_DW_LN_FUSED: unset = that split, 1 = the one-pass form whenever it applies, 0 = never (z required; A/B runs)
static int dw_ln_mode() {
  static const int m = getenv("SV_DW_LN_FUSED") ? atoi(getenv("SV_DW_LN_FUSED")) : -1;
  return m;
}
static bool dw_ln_fusable(int C, int x_dtype, int z_dtype, int y_dtype) {
  return (C == 128 || C == 256 || C == 512) && x_dtype == SV_F32 && z_dtype == y_dtype &&
         (y_dtype == SV_F32 || y_dtype == SV_BF16);
}
static bool dw_ln_fused(int C, int x_dtype, int z_dtype, int y_dtype, bool keep_z) {
  const int m = dw_ln_mode();
  return dw_ln_fusable(C, x_dtype, z_dtype, y_dtype) && (m == 1 || (m < 0 && !keep_z));
}

}  // namespace sv

using namespace sv;

extern "C" {

int sv_dwconv7_ln_fwd(const void* x, int32_t x_dtype, const float* wdw, const float* bdw,
                      const float* lnw, const float* lnb, float eps, void* z, int32_t z_dtype, void* y,
                      int32_t y_dtype, float* mean, float* rstd, int32_t B, int32_t H, int32_t W,
                      int32_t C, sv_stream_t stream) {
  SV_REQUIRE(x && wdw && bdw && lnw && lnb && y && mean && rstd, "sv_dwconv7_ln_fwd: null pointer");
  SV_REQUIRE(C % 64 == 0 && C > 0, "sv_dwconv7_ln_fwd: C=%d must be a multiple of 64", C);
  if (B <= 0 || H <= 0 || W <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const DwGeo g = dw_geo(B, H, W, C);
  if (dw_ln_fused(C, x_dtype, z_dtype, y_dtype, z != nullptr)) {
    const int grid = g.ntiles;
#define FLAUNCH(TI, TO, NWV, LPR, NV)                                                                               \
  dwconv7_ln_ring_kernel<dw_pf<TI>(), DW_TW, TI, TO, NWV, LPR, NV>                                                  \
      <<<grid, 64 * NWV, dw_ln_lds<dw_pf<TI>(), DW_TW, TI, TO, NWV, LPR, NV>(), s>>>(                               \
          (const TI*)x, wdw, bdw, lnw, lnb, eps, (TO*)z, (TO*)y, mean, rstd, g)
#define FLAUNCH_C(TI, TO)                                                      \
  if (C == 128) FLAUNCH(TI, TO, 2, 16, 1);                                     \
  else if (C == 256) FLAUNCH(TI, TO, 4, 32, 1);                                \
  else FLAUNCH(TI, TO, 8, 64, 1);
    if (y_dtype == SV_F32) { FLAUNCH_C(float, float) }
    else { FLAUNCH_C(float, uint16_t) }
#undef FLAUNCH_C
#undef FLAUNCH
    return check_launch("sv_dwconv7_ln_fwd(fused)");
  }
  SV_REQUIRE(z, "sv_dwconv7_ln_fwd: z == NULL needs the fused form (sv_dwconv7_ln_fused_ok)");
  const int grid = dw_blocks(g);
#define RLAUNCH(TI, TO)                                                                                       \
  dwconv7_ring_kernel<dw_pf<TI>(), DW_TW, TI, TO, false, false><<<grid, kDwThreads, dw_ring_lds<dw_pf<TI>(), DW_TW, TI>(), s>>>( \
      (const TI*)x, wdw, bdw, (TO*)z, nullptr, g)
  if (x_dtype == SV_F32 && z_dtype == SV_F32) RLAUNCH(float, float);
  else if (x_dtype == SV_F32 && z_dtype == SV_BF16) RLAUNCH(float, uint16_t);
  else if (x_dtype == SV_BF16 && z_dtype == SV_BF16) RLAUNCH(uint16_t, uint16_t);
  else if (x_dtype == SV_BF16 && z_dtype == SV_F32) RLAUNCH(uint16_t, float);
  else return set_error(SV_ERR_INVALID_ARG, "sv_dwconv7_ln_fwd: bad dtype");
#undef RLAUNCH
  int rc = check_launch("sv_dwconv7_ln_fwd(dwconv)");
  if (rc) return rc;
  return sv_layernorm_fwd(z, z_dtype, lnw, lnb, y, y_dtype, mean, rstd, (int64_t)B * H * W, C, eps, stream);
}

int sv_dwconv7_ln_fused_ok(int32_t B, int32_t H, int32_t W, int32_t C, int32_t x_dtype, int32_t z_dtype,
                           int32_t y_dtype) {
  (void)B; (void)H; (void)W;
  return dw_ln_fusable(C, x_dtype, z_dtype, y_dtype) && dw_ln_mode() != 0 ? 1 : 0;
}

int sv_dwconv7_bwd_data(const void* dz, int32_t dz_dtype, const float* wdw, float* dx, uint16_t* dx_bf16,
                        int32_t accumulate, int32_t B, int32_t H, int32_t W, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(dz && wdw && dx, "sv_dwconv7_bwd_data: null pointer");
  SV_REQUIRE(C % 64 == 0 && C > 0, "sv_dwconv7_bwd_data: C=%d must be a multiple of 64", C);
  SV_REQUIRE(dz != (const void*)dx, "sv_dwconv7_bwd_data: dz and dx must not alias");
  SV_REQUIRE(dz_dtype == SV_F32 || dz_dtype == SV_BF16, "sv_dwconv7_bwd_data: bad dz dtype");
  if (B <= 0 || H <= 0 || W <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const DwGeo g = dw_geo(B, H, W, C);
  const int grid = dw_blocks(g);
#define RBWD(TD, ACC)                                                                                             \
  dwconv7_ring_kernel<dw_pf<TD>(), DW_TW, TD, float, true, ACC><<<grid, kDwThreads, dw_ring_lds<dw_pf<TD>(), DW_TW, TD>(), s>>>( \
      (const TD*)dz, wdw, nullptr, dx, dx_bf16, g)
  if (dz_dtype == SV_F32) {
    if (accumulate) RBWD(float, true); else RBWD(float, false);
  } else {
    if (accumulate) RBWD(uint16_t, true); else RBWD(uint16_t, false);
  }
#undef RBWD
  return check_launch("sv_dwconv7_bwd_data");
}

int sv_dwconv7_bwd_weight_nparts(int32_t B, int32_t H, int32_t W, int32_t C) {
  const DwGeo g = dw_geo(B, H, W, C);
  const int ncg = C / 64 > 0 ? C / 64 : 1;
  // ~1024 workgroups (4096 waves, about 4 workgroups per CU) over all channel groups: with the 2-row ring a
  // wave has only ~6 KiB in flight, so the HBM latency is hidden by waves per CU (round 3, tools/dw_bench.py:
  // 512 -> 1024 workgroups S1 143 -> 129 us, S2 72 -> 62, S3 37.7 -> 33.2 (bf16 dz), S4 equal; 2048 no
  // better; step 1052-1054 -> 1059-1060 img/s, profiles/round3/r4i_*).  SV_DW_WGRAD_WGS overrides.
  static int wgs = -1;
  if (wgs < 0) {
    const char* v = getenv("SV_DW_WGRAD_WGS");
    wgs = v ? atoi(v) : 1024;
    if (wgs < 64) wgs = 64;
  }
  int np = wgs / ncg;
  if (np < 1) np = 1;
  const int need = ceil_div(g.ntiles, 4);
  return need < np ? need : np;
}

int sv_dwconv7_bwd_weight(const void* dz, int32_t dz_dtype, const void* x, int32_t x_dtype, float* dw_part,
                          float* db_part, int32_t B, int32_t H, int32_t W, int32_t C,
                          sv_stream_t stream) {
  SV_REQUIRE(dz && x && dw_part && db_part, "sv_dwconv7_bwd_weight: null pointer");
  SV_REQUIRE(C % 64 == 0 && C > 0, "sv_dwconv7_bwd_weight: C=%d must be a multiple of 64", C);
  SV_REQUIRE((dz_dtype == SV_F32 || dz_dtype == SV_BF16) && (x_dtype == SV_F32 || x_dtype == SV_BF16),
             "sv_dwconv7_bwd_weight: bad dtype");
  if (B <= 0 || H <= 0 || W <= 0) return SV_OK;
  hipStream_t s = (hipStream_t)stream;
  const DwGeo g = dw_geo(B, H, W, C);
  const dim3 grid(sv_dwconv7_bwd_weight_nparts(B, H, W, C), C / 64);
  constexpr size_t red_bytes = (49 * 64 + 64) * sizeof(float);
#define RWG(TD, TX)                                                                                            \
  {                                                                                                            \
    constexpr size_t ring = dw_wgrad_ring_lds<DW_WGRAD_PF, DW_TW, TD, TX>();                                   \
    dwconv7_wgrad_ring_kernel<DW_WGRAD_PF, DW_TW, TD, TX><<<grid, kDwThreads, ring > red_bytes ? ring : red_bytes, s>>>( \
        (const TD*)dz, (const TX*)x, dw_part, db_part, g);                                                     \
  }
  if (dz_dtype == SV_F32 && x_dtype == SV_F32) RWG(float, float)
  else if (dz_dtype == SV_F32) RWG(float, uint16_t)
  else if (x_dtype == SV_F32) RWG(uint16_t, float)
  else RWG(uint16_t, uint16_t)
#undef RWG
  return check_launch("sv_dwconv7_bwd_weight");
}

}  // extern "C"
