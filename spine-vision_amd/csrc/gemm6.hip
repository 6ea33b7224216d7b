// MFMA GEMM v6 (bf16 operands, f32 accumulate): 256x256 output tile per 256-thread workgroup, one
// workgroup per CU, each of the 4 waves owns a 128x128 quadrant (8x8 v_mfma_f32_16x16x32_bf16
// fragments, 256 f32 accumulators per lane in the unified VGPR/AGPR file at one wave per SIMD).
//
// Why: the 256x128 tiles of v2/v3 move (256+128)/(256*128) = 11.7 mB of L2->LDS operand traffic per
// FLOP (47 B/clk/CU at the bf16 MFMA peak), above what one CU's LDS-DMA sustains (~33 B/clk measured
// for 128-B rows out of L2, MI355X_MICROARCH.md "Indexed rows"), and every wave re-reads 64x64
// operand fragments from LDS for 64x64 outputs.  256x256 tiles halve the DMA bytes per FLOP
// (7.8 mB/FLOP) and the 128x128 wave quadrant halves the LDS fragment bytes per MFMA.
//
//   * BK = 32, 4-stage LDS ring (4 x 32 KiB = 128 KiB)
//     filled by LDS-DMA (global_load_lds_dwordx4) with XOR-swizzled SOURCE addresses (v2/v3
//     layouts); counted `s_waitcnt vmcnt` keeps S-2 younger tiles in flight, one s_barrier per tile;
//   * k-major operands read with ds_read_b128, m-major with ds_read_b64_tr_b16 (no transposed HBM
//     copies), XCD-aware tile order, split-K slabs + fused bias column sum for the wgrads;
//   * epilogue: the shared LDS-slab 16-B-store path (gemm_common.h), 64x64 groups.
#include "common.h"
#include "gemm_common.h"

#include <stdlib.h>

namespace sv {
namespace g6 {

constexpr int BM = 256, BN = 256, THREADS = 256, NW = 4;
constexpr int FM = 8, FN = 8;  // 16x16 fragments per wave (128 x 128)
constexpr size_t LDS = 128 * 1024;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int mswz(int r) { return ((r & 3) << 1) ^ (((r >> 3) & 1) << 3); }
// k-major rows: BK 64 -> 128-B rows, chunk ^= row & 7;  BK 32 -> 64-B rows, chunk ^= 2((row >> 3) & 1)
template <int BKT>
__device__ __forceinline__ int kswz(int row) {
  if constexpr (BKT == 64) return row & 7;
  else return ((row >> 3) & 1) << 1;
}

template <int BKT>
struct Cfg {
  static constexpr int A_BYTES = BM * BKT * 2, B_BYTES = BN * BKT * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int A_PER_WAVE = A_BYTES / 1024 / NW, B_PER_WAVE = B_BYTES / 1024 / NW;
  static constexpr int LOADS = A_PER_WAVE + B_PER_WAVE;  // LDS-DMA instructions per wave per stage
  static constexpr int STAGES = (int)(LDS / STAGE_BYTES);
};

// LDS-DMA pieces of one operand tile (ROWS x BKT).  KMAJ: X(row,k) = X[row*ld + k] -> image
// [ROWS][BKT];  !KMAJ: X(row,k) = X[k*ld + row] -> image [BKT][ROWS].
template <bool KMAJ, int ROWS, int BKT, int PER_WAVE>
__device__ __forceinline__ void issue_tile(const uint16_t* __restrict__ X, int64_t ld, int row0, int k0, int R,
                                           char* lds_tile, int wid) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int piece = wid + NW * j;
    const int byte = piece * 1024 + lane * 16;
    const uint16_t* src;
    if constexpr (KMAJ) {
      constexpr int RB = BKT * 2;
      const int row = byte / RB, ch = (byte % RB) >> 4;
      const int gc = ch ^ kswz<BKT>(row);
      int grow = row0 + row;
      if (grow >= R) grow = 0;  // clamped; the result row is never stored
      src = X + (size_t)grow * ld + k0 + gc * 8;
    } else {
      constexpr int RB = ROWS * 2;
      const int krow = byte / RB, ch = (byte % RB) >> 4;
      const int gc = ch ^ mswz(krow);
      int gcol = row0 + gc * 8;
      if (gcol >= R) gcol = 0;
      src = X + (size_t)(k0 + krow) * ld + gcol;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds_tile + piece * 1024), 16, 0, 0);
  }
}

// MFMA fragment: lane l holds X[row = base + (l&15)][k = 32*kk + 8*(l>>4) + j], j = 0..7
template <bool KMAJ, int ROWS, int BKT>
__device__ __forceinline__ bf16x8 frag(const char* __restrict__ img, int base, int kk) {
  const int l = threadIdx.x & 63;
  if constexpr (KMAJ) {
    constexpr int RB = BKT * 2;
    const int row = base + (l & 15);
    const int gc = kk * 4 + (l >> 4);
    return *reinterpret_cast<const bf16x8*>(img + row * RB + ((gc ^ kswz<BKT>(row)) << 4));
  } else {
    constexpr int RB = ROWS * 2;
    const int g = l >> 4, q = (l >> 2) & 3, p = l & 3;
    const int gc = (base >> 3) + (p >> 1);
    const int r0 = kk * 32 + 8 * g + q, r1 = r0 + 4;
    const char* a0 = img + r0 * RB + ((gc ^ mswz(r0)) << 4) + (p & 1) * 8;
    const char* a1 = img + r1 * RB + ((gc ^ mswz(r1)) << 4) + (p & 1) * 8;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// wgrad bias gradient (column sums of A over k).  k-major A image: thread t < BM sums its row.
template <int BKT>
__device__ __forceinline__ float colsum_kmajor(const char* __restrict__ img, int row) {
  constexpr int RB = BKT * 2;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < BKT / 8; ++c) {
    const uint4 v = *reinterpret_cast<const uint4*>(img + row * RB + ((c ^ kswz<BKT>(row)) << 4));
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) s += __uint_as_float(w[j] << 16) + __uint_as_float(w[j] & 0xffff0000u);
  }
  return s;
}
// m-major A image [BKT][256]: thread t owns chunk t&31 (8 m) of k rows (t>>5)*BKT/8 ..+BKT/8-1
template <int BKT>
__device__ __forceinline__ void colsum_mmajor(const char* __restrict__ img, float (&cs)[8]) {
  constexpr int RB = BM * 2, RPG = BKT / 8;
  const int gc = threadIdx.x & 31, kg = threadIdx.x >> 5;
#pragma unroll
  for (int j = 0; j < RPG; ++j) {
    const int r = kg * RPG + j;
    const uint4 v = *reinterpret_cast<const uint4*>(img + r * RB + ((gc ^ mswz(r)) << 4));
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      cs[2 * q] += __uint_as_float(w[q] << 16);
      cs[2 * q + 1] += __uint_as_float(w[q] & 0xffff0000u);
    }
  }
}
__device__ __forceinline__ float colsum_fold(const float (&cs)[8], float* red) {
  const int gc = threadIdx.x & 31, kg = threadIdx.x >> 5;
#pragma unroll
  for (int q = 0; q < 8; ++q) red[kg * BM + gc * 8 + q] = cs[q];
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int g = 0; g < THREADS / 32; ++g) s += red[g * BM + threadIdx.x];
  __syncthreads();
  return s;
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// DBG (measurement builds only, SV_GEMM6_DBG): 1 = MFMAs on fragments read once (no ring traffic),
// 2 = skip the epilogue stores, 3 = both
template <bool AK, bool BKM, int BKT, int DBG = 0>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(1, 1)))
gemm6_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb, int K,
             int kper, int tilesM, int tilesN, EpiArgs e, float* __restrict__ colsum) {
  using C = Cfg<BKT>;
  constexpr int S = C::STAGES;
  static_assert(S >= 2 && (S - 2) * C::LOADS <= 63, "ring / vmcnt");
  extern __shared__ __attribute__((aligned(16))) char smem[];
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
  const int nk = kend > kbeg ? (kend - kbeg) / BKT : 0;

  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wm = wid >> 1, wn = wid & 1;
  const bool do_cs = colsum != nullptr && tn == 0;
  float csum = 0.f;
  float cs8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt) {
    char* st = smem + (kt % S) * C::STAGE_BYTES;
    const int k0 = kbeg + kt * BKT;
    issue_tile<AK, BM, BKT, C::A_PER_WAVE>(A, lda, m0, k0, e.M, st, wid);
    issue_tile<BKM, BN, BKT, C::B_PER_WAVE>(B, ldb, n0, k0, e.N, st + C::A_BYTES, wid);
  };

#pragma unroll
  for (int p = 0; p < S - 1; ++p)
    if (p < nk) issue(p);
  // Software pipeline (one wave per SIMD, so the wave must hide its own LDS latency): iteration kt
  // reads tile kt's fragments into F[kt & 1] while the MFMAs consume tile kt-1's fragments from
  // F[(kt - 1) & 1].  The lgkmcnt(0) before the barrier retires tile kt-1's reads before any wave
  // re-fills its ring slot.  BKT = 32 only (one k32 step per tile).
  static_assert(BKT == 32, "pipelined loop is written for one k32 step per tile");
  bf16x8 fa[2][FM], fb[2][FN];
  auto load_frags = [&](int kt, int buf) {
    if ((DBG & 1) && kt > 1) return;
    const char* ai = smem + (kt % S) * C::STAGE_BYTES;
    const char* bi = ai + C::A_BYTES;
#pragma unroll
    for (int i = 0; i < FM; ++i) fa[buf][i] = frag<AK, BM, BKT>(ai, wm * 128 + i * 16, 0);
#pragma unroll
    for (int j = 0; j < FN; ++j) fb[buf][j] = frag<BKM, BN, BKT>(bi, wn * 128 + j * 16, 0);
  };
  auto mfmas = [&](int buf) {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[buf][i], fb[buf][j], acc[i][j], 0, 0, 0);
  };
  auto sync_tile = [&](int kt) {
    // tile kt must have landed; the min(S-2, nk-1-kt) younger tiles may stay in flight
    const int younger = nk - 1 - kt < S - 2 ? nk - 1 - kt : S - 2;
    if (S > 3 && younger >= 2) vm_wait<(S > 3 ? 2 * C::LOADS : 0)>();
    else if (S > 2 && younger >= 1) vm_wait<(S > 2 ? C::LOADS : 0)>();
    else vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (!(DBG & 1) && kt + S - 1 < nk) issue(kt + S - 1);  // into the slot of tile kt-1
  };
  auto colsums = [&](int kt) {
    if (do_cs) {
      const char* ai = smem + (kt % S) * C::STAGE_BYTES;
      if constexpr (AK) csum += colsum_kmajor<BKT>(ai, threadIdx.x);
      else colsum_mmajor<BKT>(ai, cs8);
    }
  };
  if (nk > 0) {
    sync_tile(0);
    load_frags(0, 0);
    colsums(0);
  }
  int kt = 1;
  for (; kt + 1 < nk; kt += 2) {  // two tiles per trip keep the fragment buffers compile-time
    sync_tile(kt);
    load_frags(kt, 1);
    mfmas(0);
    colsums(kt);
    sync_tile(kt + 1);
    load_frags(kt + 1, 0);
    mfmas(1);
    colsums(kt + 1);
  }
  if (kt < nk) {  // nk even: one tile left, its fragments go to buffer 1
    sync_tile(kt);
    load_frags(kt, 1);
    mfmas(0);
    colsums(kt);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    mfmas(1);
  } else if (nk > 0) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    mfmas(0);
  }
  vm_wait<0>();
  __syncthreads();
  if constexpr (!AK) {
    if (do_cs) csum = colsum_fold(cs8, reinterpret_cast<float*>(smem));  // block-uniform branch
  }
  if (do_cs && m0 + (int)threadIdx.x < e.M) colsum[(size_t)split * e.M + m0 + threadIdx.x] = csum;
  if constexpr (DBG & 2) {
    if (e.M < 0) wave_tile_epilogue_wide<FM, FN, 1>(acc, reinterpret_cast<float*>(smem) + wid * 16 * EPI_LD,
                                                      m0 + wm * 128, n0 + wn * 128, e, split);  // never taken
    return;
  }
  wave_tile_epilogue_wide<FM, FN, 1>(acc, reinterpret_cast<float*>(smem) + wid * 16 * EPI_LD, m0 + wm * 128,
                                        n0 + wn * 128, e, split);
}

template <bool AK, bool BKM, int BKT, int DBG>
static void launch_dbg(const sv_gemm_desc* d, int split, int kper, hipStream_t s, const EpiArgs& e, int tilesM,
                       int tilesN) {
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm6_kernel<AK, BKM, BKT, DBG>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS);
    attr_set = true;
  }
  dim3 grid(tilesM * tilesN, 1, split);
  gemm6_kernel<AK, BKM, BKT, DBG><<<grid, THREADS, LDS, s>>>(
      reinterpret_cast<const uint16_t*>(d->A), d->lda, reinterpret_cast<const uint16_t*>(d->B), d->ldb, d->K, kper,
      tilesM, tilesN, e, d->epilogue == SV_EPI_SLAB ? reinterpret_cast<float*>(d->C2) : nullptr);
}

template <bool AK, bool BKM, int BKT>
static int launch(const sv_gemm_desc* d, int split, int kper, hipStream_t s) {
  const int tilesM = ceil_div(d->M, BM), tilesN = ceil_div(d->N, BN);
  EpiArgs e{d->M, d->N, d->epilogue, d->C, d->c_dtype, d->ldc, d->C2, d->c2_dtype, d->bias, d->gamma,
            d->aux, d->aux_dtype, d->ld_aux};
  static const int dbg = getenv("SV_GEMM6_DBG") ? atoi(getenv("SV_GEMM6_DBG")) : 0;
  if (dbg) {
    if (dbg == 1) launch_dbg<AK, BKM, BKT, 1>(d, split, kper, s, e, tilesM, tilesN);
    else if (dbg == 2) launch_dbg<AK, BKM, BKT, 2>(d, split, kper, s, e, tilesM, tilesN);
    else launch_dbg<AK, BKM, BKT, 3>(d, split, kper, s, e, tilesM, tilesN);
    return check_launch("sv_gemm(v6 dbg)");
  }
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm6_kernel<AK, BKM, BKT>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS);
    attr_set = true;
  }
  dim3 grid(tilesM * tilesN, 1, split);
  gemm6_kernel<AK, BKM, BKT><<<grid, THREADS, LDS, s>>>(
      reinterpret_cast<const uint16_t*>(d->A), d->lda, reinterpret_cast<const uint16_t*>(d->B), d->ldb, d->K, kper,
      tilesM, tilesN, e, d->epilogue == SV_EPI_SLAB ? reinterpret_cast<float*>(d->C2) : nullptr);
  return check_launch("sv_gemm(v6)");
}

template <int BKT>
static int launch_bk(const sv_gemm_desc* d, int split, int kper, hipStream_t s) {
  if (d->a_kmajor && d->b_kmajor) return launch<true, true, BKT>(d, split, kper, s);
  if (d->a_kmajor && !d->b_kmajor) return launch<true, false, BKT>(d, split, kper, s);
  if (!d->a_kmajor && d->b_kmajor) return launch<false, true, BKT>(d, split, kper, s);
  return launch<false, false, BKT>(d, split, kper, s);
}

}  // namespace g6

int launch_gemm6(const sv_gemm_desc* d, hipStream_t s) {
  using namespace g6;
  if (d->compute != SV_BF16 || d->a_dtype != SV_BF16 || d->b_dtype != SV_BF16 || d->a_scale_k)
    return SV_ERR_UNSUPPORTED;
  constexpr int bk = 32;
  if (d->K % bk != 0 || d->K < bk) return SV_ERR_UNSUPPORTED;
  const int split = d->epilogue == SV_EPI_SLAB ? (d->split_k < 1 ? 1 : d->split_k) : 1;
  const int kper = ceil_div(ceil_div(d->K, split), bk) * bk;
  return launch_bk<bk>(d, split, kper, s);
}

}  // namespace sv
