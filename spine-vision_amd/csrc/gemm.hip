// MFMA GEMM family for the ConvNeXt hot path (gfx950 / CDNA4, wave64).
//
// Replaces the cuBLAS GEMMs that timm's Mlp.fc1 / Mlp.fc2 / downsample Conv2d(k2,s2) launch under
// the reference (spine_vision/training/models/backbone.py:166 -> timm convnext.py) and their
// autograd dgrad/wgrad, with the elementwise neighbours fused into the epilogue:
//   fc1 fwd   h = y_ln W1^T + b1, a = GELU(h)                 (SV_EPI_BIAS_GELU2, both stored bf16)
//   fc2 fwd   out = x + gamma * (a W2^T + b2)                 (SV_EPI_BIAS_GAMMA_RES)
//   fc2 dgrad dh = ((d_out * gamma) W2) * GELU'(h)            (a_scale_k = gamma, SV_EPI_GELU_GRAD)
//   wgrads    split-K over the pixel dimension into f32 slabs (SV_EPI_SLAB)
//
// Structure: 128x128 output tile per 256-thread workgroup (4 waves in 2x2, 64x64 per wave = 4x4
// v_mfma_f32_16x16x32_bf16 fragments, or 16x16x4_f32 for the exact-f32 parity mode), BK = 32,
// register-staged double-buffered LDS (global loads for tile k+1 are issued before the MFMAs of
// tile k; one barrier per k-step).  Operands may be K-contiguous ("k-major": torch Linear weights,
// activations as the reduction operand) or M/N-contiguous (activations as the wgrad operand);
// k-major tiles are read with ds_read_b128, M/N-contiguous tiles are kept in their natural
// [k][m] image and turned into MFMA fragments by the gfx950 LDS transpose read
// ds_read_b64_tr_b16 -- no transposed copies of activations ever go through HBM.
// f32 operands (the f32 gradient stream) are rounded to bf16 while staging.
// Epilogue: the 64x64 f32 accumulator of each wave is staged through LDS in 16-row slabs and
// re-read row-contiguous, so every global load/store of the epilogue is a 16-B vector access.
// The blockIdx -> tile map is XCD-aware (each XCD gets a contiguous run of tiles, which share
// A row panels in its private L2).
#include "common.h"
#include "gemm_common.h"
#include "mfma_v1.h"

#include <stdlib.h>

namespace sv {


// Global -> register stage of one operand tile (rows = M or N extent of the tile, BKT deep).
// Chunk = 16 B of the LDS image: 8 bf16 or 4 f32 compute elements.
template <bool BF16, typename T, bool KMAJ>
struct Stage {
  static constexpr int EPC = BF16 ? 8 : 4;                       // elements per chunk
  static constexpr int CHUNKS = BM * BKT / EPC;                  // per tile
  static constexpr int PER_THREAD = CHUNKS / kGemmThreads;       // 2 (bf16) or 4 (f32)
  uint4 r[PER_THREAD];

  // p: operand base; ld: leading dim; row0: tile offset along M/N; k0: k offset;
  // R: M/N bound; K: k bound; scale: optional per-k scale (A operand only)
  __device__ __forceinline__ void load(const T* __restrict__ p, int64_t ld, int row0, int k0, int R, int K,
                                       const float* __restrict__ scale) {
#pragma unroll
    for (int s = 0; s < PER_THREAD; ++s) {
      const int q = threadIdx.x + kGemmThreads * s;
      int row, kk;  // position of the chunk's first element: (row along M/N, k)
      if (KMAJ) {
        constexpr int CPR = BKT / EPC;  // chunks per row
        row = q / CPR;
        kk = (q % CPR) * EPC;
      } else {
        constexpr int CPR = BM / EPC;
        kk = q / CPR;
        row = (q % CPR) * EPC;
      }
      const int gr = row0 + row, gk = k0 + kk;
      const bool ok = gr < R && gk < K;
      const T* src = KMAJ ? p + (size_t)gr * ld + gk : p + (size_t)gk * ld + gr;
      if (BF16) {
        if constexpr (sizeof(T) == 2) {
          uint4 v = make_uint4(0, 0, 0, 0);
          if (ok) v = *reinterpret_cast<const uint4*>(src);
          if (scale && ok) {
            // rare path (only f32 operands carry a scale in practice) -- keep it exact anyway
            const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
            float f[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = bf2f(e[j]) * scale[KMAJ ? gk + j : gk];
            v = make_uint4(pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7]));
          }
          r[s] = v;
        } else {
          float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a;
          if (ok) {
            a = *reinterpret_cast<const float4*>(src);
            b = *reinterpret_cast<const float4*>(src + 4);
            if (scale) {
              if (KMAJ) {
                const float4 sa = *reinterpret_cast<const float4*>(scale + gk);
                const float4 sb = *reinterpret_cast<const float4*>(scale + gk + 4);
                a.x *= sa.x; a.y *= sa.y; a.z *= sa.z; a.w *= sa.w;
                b.x *= sb.x; b.y *= sb.y; b.z *= sb.z; b.w *= sb.w;
              } else {
                const float sc = scale[gk];
                a.x *= sc; a.y *= sc; a.z *= sc; a.w *= sc;
                b.x *= sc; b.y *= sc; b.z *= sc; b.w *= sc;
              }
            }
          }
          r[s] = make_uint4(pack2bf(a.x, a.y), pack2bf(a.z, a.w), pack2bf(b.x, b.y), pack2bf(b.z, b.w));
        }
      } else {
        float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
        if (ok) {
          a = *reinterpret_cast<const float4*>(src);
          if (scale) {
            if (KMAJ) {
              const float4 sa = *reinterpret_cast<const float4*>(scale + gk);
              a.x *= sa.x; a.y *= sa.y; a.z *= sa.z; a.w *= sa.w;
            } else {
              const float sc = scale[gk];
              a.x *= sc; a.y *= sc; a.z *= sc; a.w *= sc;
            }
          }
        }
        r[s] = make_uint4(__float_as_uint(a.x), __float_as_uint(a.y), __float_as_uint(a.z), __float_as_uint(a.w));
      }
    }
  }

  __device__ __forceinline__ void store(char* __restrict__ img) const {
    constexpr int ES = BF16 ? 2 : 4;
    constexpr int LD = Img<BF16, KMAJ>::LD;
#pragma unroll
    for (int s = 0; s < PER_THREAD; ++s) {
      const int q = threadIdx.x + kGemmThreads * s;
      int row, kk;
      if (KMAJ) {
        constexpr int CPR = BKT / EPC;
        row = q / CPR;
        kk = (q % CPR) * EPC;
        *reinterpret_cast<uint4*>(img + ((size_t)row * LD + kk) * ES) = r[s];
      } else {
        constexpr int CPR = BM / EPC;
        kk = q / CPR;
        row = (q % CPR) * EPC;
        *reinterpret_cast<uint4*>(img + ((size_t)kk * LD + row) * ES) = r[s];
      }
    }
  }
};

// sum over the BKT k of A(row, k) from the staged A image (row = one of the BM tile rows)
template <bool BF16, bool KMAJ>
__device__ __forceinline__ float colsum_tile(const char* __restrict__ img, int row) {
  constexpr int LD = Img<BF16, KMAJ>::LD;
  float s = 0.f;
  if constexpr (BF16) {
    const uint16_t* h = reinterpret_cast<const uint16_t*>(img);
    if (KMAJ) {
#pragma unroll
      for (int c = 0; c < BKT; c += 8) {
        const uint4 v = *reinterpret_cast<const uint4*>(h + (size_t)row * LD + c);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) s += __uint_as_float(w[j] << 16) + __uint_as_float(w[j] & 0xffff0000u);
      }
    } else {
#pragma unroll
      for (int k = 0; k < BKT; ++k) s += bf2f(h[(size_t)k * LD + row]);
    }
  } else {
    const float* f = reinterpret_cast<const float*>(img);
#pragma unroll
    for (int k = 0; k < BKT; ++k) s += KMAJ ? f[(size_t)row * LD + k] : f[(size_t)k * LD + row];
  }
  return s;
}

template <bool BF16, typename TA, typename TB, bool AK, bool BKM>
__global__ void __launch_bounds__(kGemmThreads) gemm_kernel(const TA* __restrict__ A, int64_t lda,
                                                            const TB* __restrict__ B, int64_t ldb,
                                                            const float* __restrict__ a_scale, int K,
                                                            int kper, int tilesM, int tilesN, EpiArgs e,
                                                            float* __restrict__ colsum) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int ABYTES = Img<BF16, AK>::BYTES, BBYTES = Img<BF16, BKM>::BYTES;
  constexpr int STAGE_BYTES = ABYTES + BBYTES;

  // ---- XCD-aware tile map: blocks b, b+8, ... share an XCD; give each XCD a contiguous run of
  //      tiles (tn fastest) so the tiles co-resident in one L2 share their A row panel.
  const int nwg = tilesM * tilesN;
  const int pid = blockIdx.x;
  const int xcd = pid & 7, loc = pid >> 3, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tm = wg / tilesN, tn = wg % tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int split = blockIdx.z;
  const int kbeg = split * kper;
  int kend = kbeg + kper;
  if (kend > K) kend = K;
  const int nk = kend > kbeg ? (kend - kbeg + BKT - 1) / BKT : 0;

  const int wid = threadIdx.x >> 6, wm = wid >> 1, wn = wid & 1;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fused bias gradient of a wgrad GEMM: sum over this split's k of A(m,k), from the staged tile
  const bool do_cs = colsum != nullptr && tn == 0;
  float csum = 0.f;

  Stage<BF16, TA, AK> sa;
  Stage<BF16, TB, BKM> sb;
  if (nk > 0) {
    sa.load(A, lda, m0, kbeg, e.M, kend, a_scale);
    sb.load(B, ldb, n0, kbeg, e.N, kend, nullptr);
    sa.store(smem);
    sb.store(smem + ABYTES);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * STAGE_BYTES;
    char* nxt = smem + ((kt + 1) & 1) * STAGE_BYTES;
    const bool more = kt + 1 < nk;
    if (more) {
      const int k0 = kbeg + (kt + 1) * BKT;
      sa.load(A, lda, m0, k0, e.M, kend, a_scale);
      sb.load(B, ldb, n0, k0, e.N, kend, nullptr);
    }
    const char* ai = cur;
    const char* bi = cur + ABYTES;
    if (do_cs && threadIdx.x < BM) csum += colsum_tile<BF16, AK>(ai, threadIdx.x);
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
    if (more) {
      sa.store(nxt);
      sb.store(nxt + ABYTES);
    }
    __syncthreads();
  }

  if (do_cs && threadIdx.x < BM && m0 + (int)threadIdx.x < e.M) colsum[(size_t)split * e.M + m0 + threadIdx.x] = csum;

  // ---- epilogue: per wave, 16-row slabs staged through its private LDS region
  wave_tile_epilogue(acc, reinterpret_cast<float*>(smem) + wid * 16 * EPI_LD, m0 + wm * 64, n0 + wn * 64, e, split);
}

template <bool BF16, typename TA, typename TB, bool AK, bool BKM>
static int launch(const sv_gemm_desc* d, hipStream_t s) {
  const int tilesM = ceil_div(d->M, BM), tilesN = ceil_div(d->N, BN);
  int split = d->epilogue == SV_EPI_SLAB ? (d->split_k < 1 ? 1 : d->split_k) : 1;
  int kper = ceil_div(ceil_div(d->K, split), BKT) * BKT;
  EpiArgs e{d->M, d->N, d->epilogue, d->C, d->c_dtype, d->ldc, d->C2, d->c2_dtype, d->bias, d->gamma,
            d->aux, d->aux_dtype, d->ld_aux};
  constexpr size_t main_lds = 2 * (size_t)(Img<BF16, AK>::BYTES + Img<BF16, BKM>::BYTES);
  constexpr size_t epi_lds = 4 * 16 * EPI_LD * sizeof(float);
  constexpr size_t lds = main_lds > epi_lds ? main_lds : epi_lds;
  dim3 grid(tilesM * tilesN, 1, split);
  if (const int rc_ = ensure_lds_attr(reinterpret_cast<const void*>(&gemm_kernel<BF16, TA, TB, AK, BKM>), (int)lds, s)) return rc_;
  gemm_kernel<BF16, TA, TB, AK, BKM><<<grid, kGemmThreads, lds, s>>>(
      reinterpret_cast<const TA*>(d->A), d->lda, reinterpret_cast<const TB*>(d->B), d->ldb, d->a_scale_k, d->K,
      kper, tilesM, tilesN, e, d->epilogue == SV_EPI_SLAB ? reinterpret_cast<float*>(d->C2) : nullptr);
  return check_launch("sv_gemm");
}

template <bool BF16, typename TA, typename TB>
static int launch_layout(const sv_gemm_desc* d, hipStream_t s) {
  if (d->a_kmajor && d->b_kmajor) return launch<BF16, TA, TB, true, true>(d, s);
  if (d->a_kmajor && !d->b_kmajor) return launch<BF16, TA, TB, true, false>(d, s);
  if (!d->a_kmajor && d->b_kmajor) return launch<BF16, TA, TB, false, true>(d, s);
  return launch<BF16, TA, TB, false, false>(d, s);
}

static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace sv

using namespace sv;

extern "C" int sv_gemm(const sv_gemm_desc* d, sv_stream_t stream) {
  SV_REQUIRE(d, "sv_gemm: null descriptor");
  SV_REQUIRE(d->A && d->B && d->C, "sv_gemm: null operand");
  SV_REQUIRE(d->M >= 0 && d->N >= 0 && d->K >= 0, "sv_gemm: negative size");
  SV_REQUIRE(d->epilogue >= SV_EPI_STORE && d->epilogue <= SV_EPI_LN_BWD, "sv_gemm: bad epilogue %d", d->epilogue);
  SV_REQUIRE(d->policy.impl == 0 || d->policy.impl == 2 || d->policy.impl == 3 || d->policy.impl == 8 || d->policy.impl == 9,
             "sv_gemm: policy.impl must be 0, 2, 3, 8 or 9 (got %d)", d->policy.impl);
  SV_REQUIRE(d->policy.grid_cap >= 0 && d->policy.wg_per_cu >= 0 && d->policy.wg_per_cu <= 2 &&
                 (d->policy.priority == 0 || d->policy.priority == 1),
             "sv_gemm: bad policy (grid_cap >= 0, wg_per_cu 0..2, priority 0/1)");
  if (d->M == 0 || d->N == 0) return SV_OK;
  const bool bf = d->compute == SV_BF16;
  SV_REQUIRE(bf || d->compute == SV_F32, "sv_gemm: bad compute type");
  SV_REQUIRE(bf || (d->a_dtype == SV_F32 && d->b_dtype == SV_F32), "sv_gemm: f32 compute needs f32 operands");
  const int vec = bf ? 8 : 4;
  // contiguous dims must hold whole 16-B chunks; leading dims keep every chunk 16-B aligned
  SV_REQUIRE((d->a_kmajor ? d->K : d->M) % vec == 0, "sv_gemm: A contiguous dim not a multiple of %d", vec);
  SV_REQUIRE((d->b_kmajor ? d->K : d->N) % vec == 0, "sv_gemm: B contiguous dim not a multiple of %d", vec);
  SV_REQUIRE(d->lda % vec == 0 && d->ldb % vec == 0, "sv_gemm: lda/ldb must be multiples of %d", vec);
  SV_REQUIRE(al16(d->A) && al16(d->B) && al16(d->C), "sv_gemm: operands must be 16-byte aligned");
  SV_REQUIRE(d->N % 4 == 0, "sv_gemm: N must be a multiple of 4");
  if (d->epilogue == SV_EPI_SLAB) {
    SV_REQUIRE(d->c_dtype == SV_F32 || (bf && d->c_dtype == SV_BF16 && !d->fold_out && d->N % 8 == 0),
               "sv_gemm: slab epilogue writes f32 (bf16 slabs: bf16 compute, N %% 8 == 0, no in-kernel fold)");
    SV_REQUIRE(!d->C2 || d->c2_dtype == SV_F32, "sv_gemm: slab colsum output is f32");
  } else {
    SV_REQUIRE(d->ldc % 4 == 0, "sv_gemm: ldc must be a multiple of 4");
  }
  if (d->epilogue == SV_EPI_BIAS_GELU2 || d->epilogue == SV_EPI_BIAS_GELU_DUAL)
    SV_REQUIRE(d->C2 && al16(d->C2), "sv_gemm: GELU epilogue needs an aligned C2");
  if (d->epilogue == SV_EPI_BIAS_GAMMA_RES) SV_REQUIRE(d->gamma && d->aux, "sv_gemm: gamma/residual missing");
  if (d->epilogue == SV_EPI_STORE_STATS)
    SV_REQUIRE(bf && d->C2 && al16(d->C2) && d->N % 8 == 0, "sv_gemm: STORE_STATS needs bf16, an aligned C2, N %% 8 == 0");
  if (d->epilogue == SV_EPI_GELU_GRAD || d->epilogue == SV_EPI_MUL_AUX) SV_REQUIRE(d->aux, "sv_gemm: aux missing");
  if (d->epilogue == SV_EPI_STORE_BN_BWD)
    SV_REQUIRE(bf && d->c_dtype == SV_BF16 && d->C2 && d->N % 8 == 0 && d->aux && d->aux_dtype == SV_BF16 && !d->bias &&
                   d->bn && d->bn->mean && d->bn->rstd && d->bn->gamma && d->bn->beta,
               "sv_gemm: STORE_BN_BWD needs bf16 C and aux, C2, N %% 8 == 0, no bias and the bn parameters");
  if (d->epilogue == SV_EPI_LN_BWD)
    SV_REQUIRE(bf && d->c_dtype == SV_BF16 && d->C2 && al16(d->C2) && d->aux && d->aux_dtype == SV_BF16 && d->bn &&
                   d->bn->mean && d->bn->rstd && d->bn->gamma && d->fold_out && d->fold_counters && al16(d->fold_out),
               "sv_gemm: LN_BWD needs bf16 C and aux (z), C2, the bn mean / rstd / gamma and the exchange workspace");
  if (d->aux) SV_REQUIRE(d->ld_aux % 4 == 0 && al16(d->aux), "sv_gemm: aux must be aligned");
  if (d->fold_out && d->epilogue != SV_EPI_LN_BWD)
    SV_REQUIRE(d->epilogue == SV_EPI_SLAB && bf && d->fold_counters && d->fold_ld == d->N && al16(d->fold_out),
               "sv_gemm: fold_out needs SV_EPI_SLAB (bf16), fold_counters, fold_ld == N and a 16-byte aligned output");
  if (d->a_scale_k) SV_REQUIRE(al16(d->a_scale_k), "sv_gemm: a_scale_k must be aligned");
  hipStream_t s = (hipStream_t)stream;
  if (!bf) return launch_layout<false, float, float>(d, s);
  // bf16 operands: the LDS-DMA pipelined v2 kernel when the shape fits its contract (K % 64 == 0)
  const int impl = d->policy.impl;
  const int wpc = d->policy.wg_per_cu;
  if (d->epilogue == SV_EPI_STORE_BN_BWD) {  // the v3 kernels carry the BatchNorm-backward epilogue
    const int rc = launch_gemm3(d, s);
    SV_REQUIRE(rc != SV_ERR_UNSUPPORTED, "sv_gemm: STORE_BN_BWD needs K %% 32 == 0, bf16 operands, k-major A, m-major B");
    return rc;
  }
  if (d->epilogue == SV_EPI_LN_BWD) return launch_gemm9(d, s);  // v9 only; SV_ERR_UNSUPPORTED -> the caller's two passes
  if (d->epilogue == SV_EPI_STORE_STATS) {  // the v3 and v9 kernels carry the statistics epilogue
    const long t9 = (long)ceil_div(d->M, 256) * ceil_div(d->N, 256);
    if ((impl == 0 || impl == 9) && d->N >= 256 && t9 >= 256 && d->a_kmajor) {
      const int rc9 = launch_gemm9(d, s);
      if (rc9 != SV_ERR_UNSUPPORTED) return rc9;
    }
    const int rc = launch_gemm3(d, s);
    SV_REQUIRE(rc != SV_ERR_UNSUPPORTED, "sv_gemm: STORE_STATS needs K %% 32 == 0 and bf16 operands");
    return rc;
  }
  {
    // Measured per ConvNeXt shape (tools/gemm_bench.py, profiles/r1s2_gemm_cfg.txt):
    //   v3 32x3 (two workgroups per CU, one's epilogue beside the other's MFMAs): VALU-heavy and
    //     operand-reading epilogues and plain stores with K <= 2048 (fc1 fwd, fc2 dgrad, fc1 dgrad);
    //   v3 32x4 (one workgroup per CU, two tiles in flight): the split-K wgrads (-10..25% vs v2);
    //   v2 (BK 64, 3 stages): long-K residual epilogue (fc2 fwd).
    const bool heavy_epi = d->epilogue == SV_EPI_BIAS_GELU2 || d->epilogue == SV_EPI_BIAS_GELU_DUAL ||
                           d->epilogue == SV_EPI_GELU_GRAD || d->epilogue == SV_EPI_MUL_AUX ||
                           d->epilogue == SV_EPI_BIAS_GELU;
    // v8 (256x256, one workgroup per CU) where it measured faster and the chip holds >= one full wave
    // of its tiles: the fc1 forward (GELU dual epilogue) and the long-K forward GEMMs (fc2 residual,
    // K >= 2048); never beside the side-stream GEMMs (128 KiB of LDS leaves no room for a co-resident
    // workgroup).  tools/gemm_bench.py, gpurun_out g8a.
    const long tiles8 = (long)ceil_div(d->M, 256) * ceil_div(d->N, 256);
    const bool v8_shape = tiles8 >= 256 && (d->epilogue == SV_EPI_BIAS_GELU_DUAL || d->epilogue == SV_EPI_BIAS_GELU ||
                                            ((d->epilogue == SV_EPI_BIAS_GAMMA_RES) && d->K >= 2048));
    // v9 (persistent 256x256, BK 64 phase-interleaved, register-direct epilogue) where the chip holds
    // a full wave of its tiles and N fills the 256-wide tile
    const int split9 = d->epilogue == SV_EPI_SLAB ? (d->split_k < 1 ? 1 : d->split_k) : 1;
    // (weight gradients: outputs of at least 128 x 256 in either orientation, the split-K factor sized
    // for one tile per CU by kernels._wgrad_split_for)
    const bool v9_slab = d->epilogue == SV_EPI_SLAB && (d->M < d->N ? d->M : d->N) >= 128 &&
                         (d->M > d->N ? d->M : d->N) >= 256 && tiles8 * split9 >= 128;
    const bool v9_shape = v9_slab || (d->epilogue != SV_EPI_SLAB && d->epilogue != SV_EPI_BIAS_GELU2 && d->N >= 256 &&
                                      tiles8 >= 256);
    const bool v9_pick = impl == 0 && v9_shape;
    int rc = SV_ERR_UNSUPPORTED;
    if (d->epilogue == SV_EPI_SLAB && d->c_dtype == SV_BF16) {  // bf16 slabs: the v9 weight-gradient kernel only
      rc = launch_gemm9(d, s);
      SV_REQUIRE(rc != SV_ERR_UNSUPPORTED, "sv_gemm: bf16 slabs need the v9 weight-gradient layout (N/M-major A)");
      return rc;
    }
    if (impl == 9 || v9_pick) rc = launch_gemm9(d, s);  // shapes outside v9's contract take the dispatch below
    if (rc != SV_ERR_UNSUPPORTED) return rc;
    if (d->fold_out) {  // another family: the slabs, then the fold as its own pass (bitwise v9's in-kernel fold)
      sv_gemm_desc dd = *d;
      dd.fold_out = nullptr;
      dd.fold_counters = nullptr;
      if (int r = sv_gemm(&dd, stream)) return r;
      const int split = d->split_k < 1 ? 1 : d->split_k;
      return sv_reduce_partials(reinterpret_cast<const float*>(d->C), split, split, (int64_t)d->M * d->N, d->fold_out,
                                1.0f, d->fold_accumulate, stream);
    }
    if ((impl == 0 || impl == 9) && !wpc && v8_shape) rc = launch_gemm8(d, s);
    else if (impl == 8) rc = launch_gemm8(d, s);
    else if (impl == 2) rc = launch_gemm2(d, s);
    else if (impl == 3) rc = launch_gemm3(d, s);
    else if (d->epilogue == SV_EPI_SLAB) rc = launch_gemm3(d, s, wpc ? "32x3" : "32x4");
    else if (heavy_epi || (d->epilogue == SV_EPI_STORE && d->K <= 2048)) rc = launch_gemm3(d, s);
    else if (wpc) rc = launch_gemm3(d, s);  // v2's 144 KiB would not share a CU
    else rc = launch_gemm2(d, s);
    if (rc != SV_ERR_UNSUPPORTED) return rc;
  }
  const bool a32 = d->a_dtype == SV_F32, b32 = d->b_dtype == SV_F32;
  SV_REQUIRE((a32 || d->a_dtype == SV_BF16) && (b32 || d->b_dtype == SV_BF16), "sv_gemm: bad operand dtype");
  if (!a32 && !b32) return launch_layout<true, uint16_t, uint16_t>(d, s);
  if (a32 && !b32) return launch_layout<true, float, uint16_t>(d, s);
  if (!a32 && b32) return launch_layout<true, uint16_t, float>(d, s);
  return launch_layout<true, float, float>(d, s);
}

// ---- split-K finish ------------------------------------------------------------------------------
// C = (accumulate ? C : 0) + sum_s slab[s] over the f32 slabs of a split-K GEMM (SV_EPI_SLAB), slices
// summed in order s = 0, 1, ... (deterministic), and optionally the SV_EPI_STORE_STATS partials of
// the stored values.  Block = 256 threads over a 64-row x 64-column tile: thread (ph, q) owns columns
// n0 + 4q .. +3 of rows m0 + ph + 16 i, i < 4 (16-B slab reads; every slab load of a thread is
// independent, so the split slices stream in parallel); the 16 row phases are folded through LDS into
// the 64-row group's statistics row.  Small grids are the point of split-K, so the tile is small.
namespace sv {
namespace {
constexpr int SF_THREADS = 256;
__global__ void __launch_bounds__(SF_THREADS) slab_finish_kernel(const float* __restrict__ slab, int split, int M, int N,
                                                                 void* __restrict__ C, int c_dtype, int64_t ldc,
                                                                 int accumulate, float* __restrict__ stats) {
  const int q = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int n = blockIdx.x * 64 + q * 4, m0 = blockIdx.y * 64;
  const size_t sstride = (size_t)M * N;
  float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f), s2 = s1;
  if (n < N) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + ph + 16 * i;
      if (m >= M) break;
      const float* p = slab + (size_t)m * N + n;
      float4 v = *reinterpret_cast<const float4*>(p);
      for (int sl = 1; sl < split; ++sl) {
        const float4 w = *reinterpret_cast<const float4*>(p + sl * sstride);
        v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
      }
      const size_t ci = (size_t)m * ldc + n;
      if (c_dtype == SV_F32) {
        float4* cp = reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + ci);
        if (accumulate) {
          const float4 o = *cp;
          v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        *cp = v;
      } else {
        uint2* cp = reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(C) + ci);
        if (accumulate) {  // the bf16 gradient stream: the sum in f32, stored bf16
          const uint2 o = *cp;
          v.x += __uint_as_float(o.x << 16); v.y += __uint_as_float(o.x & 0xffff0000u);
          v.z += __uint_as_float(o.y << 16); v.w += __uint_as_float(o.y & 0xffff0000u);
        }
        const uint2 u = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
        *cp = u;
        // statistics of the values as stored
        v = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                        __uint_as_float(u.y & 0xffff0000u));
      }
      if (stats) {
        s1.x += v.x; s1.y += v.y; s1.z += v.z; s1.w += v.w;
        s2.x = fmaf(v.x, v.x, s2.x); s2.y = fmaf(v.y, v.y, s2.y); s2.z = fmaf(v.z, v.z, s2.z); s2.w = fmaf(v.w, v.w, s2.w);
      }
    }
  }
  if (!stats) return;  // grid-uniform
  __shared__ float4 red[2][SF_THREADS];
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  if (ph == 0 && n < N) {
    for (int k = 1; k < 16; ++k) {
      const float4 a = red[0][k * 16 + q], b = red[1][k * 16 + q];
      s1.x += a.x; s1.y += a.y; s1.z += a.z; s1.w += a.w;
      s2.x += b.x; s2.y += b.y; s2.z += b.z; s2.w += b.w;
    }
    float* o = stats + (size_t)blockIdx.y * 2 * N;
    *reinterpret_cast<float4*>(o + n) = s1;
    *reinterpret_cast<float4*>(o + N + n) = s2;
  }
}

// the same finish into bf16 C plus the BatchNorm + ReLU backward statistics of the values as stored (the
// split-K data gradient at a BatchNorm + ReLU output): g = C * (fmaf(gamma rstd, y - mean, beta) > 0), the
// mask and products of sv_bn_relu_bwd_stats; sums of g and g * xhat per 64-row group
__global__ void __launch_bounds__(SF_THREADS) slab_finish_bnb_kernel(const float* __restrict__ slab, int split, int M,
                                                                     int N, uint16_t* __restrict__ C,
                                                                     const uint16_t* __restrict__ y, sv_bn_ref bn,
                                                                     float* __restrict__ part) {
  const int q = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const int n = blockIdx.x * 64 + q * 4, m0 = blockIdx.y * 64;
  const size_t sstride = (size_t)M * N;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    const float4 mu4 = *reinterpret_cast<const float4*>(bn.mean + n), rs4 = *reinterpret_cast<const float4*>(bn.rstd + n);
    const float4 ga4 = *reinterpret_cast<const float4*>(bn.gamma + n), be4 = *reinterpret_cast<const float4*>(bn.beta + n);
    const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, rs[4] = {rs4.x, rs4.y, rs4.z, rs4.w};
    const float ga[4] = {ga4.x, ga4.y, ga4.z, ga4.w}, be[4] = {be4.x, be4.y, be4.z, be4.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + ph + 16 * i;
      if (m >= M) break;
      const float* p = slab + (size_t)m * N + n;
      float4 v = *reinterpret_cast<const float4*>(p);
      for (int sl = 1; sl < split; ++sl) {
        const float4 w = *reinterpret_cast<const float4*>(p + sl * sstride);
        v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
      }
      const size_t ci = (size_t)m * N + n;
      const uint2 u = make_uint2(pack2bf(v.x, v.y), pack2bf(v.z, v.w));
      *reinterpret_cast<uint2*>(C + ci) = u;
      const uint2 yu = *reinterpret_cast<const uint2*>(y + ci);
      const float o[4] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                          __uint_as_float(u.y & 0xffff0000u)};
      const float yv[4] = {__uint_as_float(yu.x << 16), __uint_as_float(yu.x & 0xffff0000u),
                           __uint_as_float(yu.y << 16), __uint_as_float(yu.y & 0xffff0000u)};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float g = fmaf(ga[j] * rs[j], yv[j] - mu[j], be[j]) > 0.f ? o[j] : 0.f;
        s1[j] += g;
        s2[j] = fmaf(g, (yv[j] - mu[j]) * rs[j], s2[j]);
      }
    }
  }
  __shared__ float4 red[2][SF_THREADS];
  red[0][threadIdx.x] = make_float4(s1[0], s1[1], s1[2], s1[3]);
  red[1][threadIdx.x] = make_float4(s2[0], s2[1], s2[2], s2[3]);
  __syncthreads();
  if (ph == 0 && n < N) {
    float4 a1 = red[0][q], a2 = red[1][q];
    for (int k = 1; k < 16; ++k) {
      const float4 a = red[0][k * 16 + q], b = red[1][k * 16 + q];
      a1.x += a.x; a1.y += a.y; a1.z += a.z; a1.w += a.w;
      a2.x += b.x; a2.y += b.y; a2.z += b.z; a2.w += b.w;
    }
    float* o = part + (size_t)blockIdx.y * 2 * N;
    *reinterpret_cast<float4*>(o + n) = a1;
    *reinterpret_cast<float4*>(o + N + n) = a2;
  }
}
}  // namespace
}  // namespace sv

extern "C" int sv_gemm_slab_finish_bn_bwd(const float* slab, int32_t split, int32_t M, int32_t N, void* C, const void* y,
                                          const sv_bn_ref* bn, float* part, sv_stream_t stream) {
  SV_REQUIRE(slab && C && y && bn && part && bn->mean && bn->rstd && bn->gamma && bn->beta,
             "sv_gemm_slab_finish_bn_bwd: null pointer");
  SV_REQUIRE(split >= 1 && M >= 0 && N >= 0 && N % 4 == 0, "sv_gemm_slab_finish_bn_bwd: bad sizes (N multiple of 4)");
  SV_REQUIRE(al16(slab) && al16(C) && al16(y) && al16(part) && al16(bn->mean) && al16(bn->rstd) && al16(bn->gamma) &&
                 al16(bn->beta),
             "sv_gemm_slab_finish_bn_bwd: operands must be 16-byte aligned");
  if (M == 0 || N == 0) return SV_OK;
  const dim3 grid((unsigned)ceil_div(N, 64), (unsigned)ceil_div(M, 64));
  sv::slab_finish_bnb_kernel<<<grid, sv::SF_THREADS, 0, (hipStream_t)stream>>>(
      slab, split, M, N, reinterpret_cast<uint16_t*>(C), reinterpret_cast<const uint16_t*>(y), *bn, part);
  return check_launch("sv_gemm_slab_finish_bn_bwd");
}

extern "C" int sv_gemm_slab_finish(const float* slab, int32_t split, int32_t M, int32_t N, void* C, int32_t c_dtype,
                                   int64_t ldc, int32_t accumulate, float* stats, sv_stream_t stream) {
  SV_REQUIRE(slab && C, "sv_gemm_slab_finish: null pointer");
  SV_REQUIRE(split >= 1 && M >= 0 && N >= 0 && N % 4 == 0 && ldc % 4 == 0 && ldc >= N,
             "sv_gemm_slab_finish: bad sizes (N, ldc multiples of 4)");
  SV_REQUIRE(c_dtype == SV_F32 || c_dtype == SV_BF16, "sv_gemm_slab_finish: bad C dtype");
  SV_REQUIRE(!stats || c_dtype == SV_BF16, "sv_gemm_slab_finish: statistics are of bf16 outputs");
  SV_REQUIRE(al16(slab) && al16(C) && (!stats || al16(stats)), "sv_gemm_slab_finish: operands must be 16-byte aligned");
  if (M == 0 || N == 0) return SV_OK;
  const dim3 grid((unsigned)ceil_div(N, 64), (unsigned)ceil_div(M, 64));
  sv::slab_finish_kernel<<<grid, sv::SF_THREADS, 0, (hipStream_t)stream>>>(slab, split, M, N, C, c_dtype, ldc,
                                                                           accumulate, stats);
  return check_launch("sv_gemm_slab_finish");
}
