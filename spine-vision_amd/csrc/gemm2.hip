// MFMA GEMM v2 (bf16 operands, f32 accumulate) -- the pipelined kernel behind sv_gemm for the
// ConvNeXt MLP GEMMs and their dgrad/wgrad (see gemm.hip for the epilogue contract).
//
// gfx950 design:
//   * 256x128 output tile per 512-thread workgroup, 8 waves in 4(M) x 2(N), 64x64 per wave
//     (4x4 v_mfma_f32_16x16x32_bf16 fragments, 64 f32 accumulators per lane);
//   * BK = 64; a 3-stage LDS ring (3 x 48 KiB) filled by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
//     wave-instruction, 6 per wave per stage) so tiles k+1 and k+2 are in flight while tile k is
//     multiplied: counted `s_waitcnt vmcnt(6)` + raw s_barrier, never vmcnt(0) in the loop;
//   * LDS-DMA writes lane-linearly, so bank-conflict avoidance is done by XOR-swizzling the per-lane
//     SOURCE address and reading back through the same involution:
//       k-major tile  [rows][64 k]  (128-B rows):  LDS chunk = k-chunk ^ (row & 7)      -> ds_read_b128
//       m-major tile  [64 k][rows]  (row = tile width): LDS chunk = m-chunk ^ f(k-row),
//       f(r) = 2(r&3) ^ 8((r>>3)&1)  -> conflict-free ds_read_b64_tr_b16 transposed fragment reads;
//   * XCD-aware tile order (tiles sharing an A row panel run on one XCD's L2);
//   * out-of-range rows/columns read a clamped (valid) address and are discarded at the store;
//     K (per split slice) must be a multiple of 64 -- other shapes go to the v1 kernel.
#include "common.h"
#include "gemm_common.h"

#include <stdlib.h>

namespace sv {
namespace g2 {

constexpr int BM = 256, BK = 64, THREADS = 512;
constexpr int A_BYTES = BM * BK * 2;
constexpr int A_PER_WAVE = A_BYTES / 1024 / 8;  // 1 KiB LDS-DMA pieces per wave per stage

// Tile configurations: BN = 128 -> 8 waves as 4(M) x 2(N) of 64x64, 3-stage ring (144 KiB);
//                      BN = 256 -> 8 waves as 2(M) x 4(N) of 128x64, 2-stage ring (128 KiB): half the
//                      L2->LDS bytes per FLOP, used when the grid still fills the chip.
template <int BN>
struct Cfg {
  static constexpr int B_BYTES = BN * BK * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int B_PER_WAVE = B_BYTES / 1024 / 8;
  static constexpr int LOADS = A_PER_WAVE + B_PER_WAVE;  // LDS-DMA instructions per wave per stage
  static constexpr int STAGES = BN == 128 ? 3 : 2;
  static constexpr int WAVES_N = BN / 64, WAVES_M = 8 / WAVES_N;
  static constexpr int FM = BM / WAVES_M / 16;  // fragment rows per wave (4 or 8)
  static constexpr size_t LDS = (size_t)STAGES * STAGE_BYTES;
};

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int mswz(int r) { return ((r & 3) << 1) ^ (((r >> 3) & 1) << 3); }

// Issue the LDS-DMA pieces of one operand tile.
//   KMAJ: global X(row, k) = X[row*ld + k]; tile = ROWS rows x 64 k  -> image [ROWS][64]
//  !KMAJ: global X(row, k) = X[k*ld + row]; tile = 64 k x ROWS rows  -> image [64][ROWS]
template <bool KMAJ, int ROWS, int PER_WAVE>
__device__ __forceinline__ void issue_tile(const uint16_t* __restrict__ X, int64_t ld, int row0, int k0, int R,
                                           char* lds_tile) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int piece = wid + 8 * j;
    const int byte = piece * 1024 + lane * 16;
    const uint16_t* src;
    if constexpr (KMAJ) {
      const int row = byte >> 7, ch = (byte >> 4) & 7;
      const int gc = ch ^ (row & 7);
      int grow = row0 + row;
      if (grow >= R) grow = 0;  // clamped; the result row is never stored
      src = X + (size_t)grow * ld + k0 + gc * 8;
    } else {
      constexpr int RB = ROWS * 2;  // bytes per k-row of the image
      const int krow = byte / RB, ch = (byte % RB) >> 4;
      const int gc = ch ^ mswz(krow);
      int gcol = row0 + gc * 8;
      if (gcol >= R) gcol = 0;
      src = X + (size_t)(k0 + krow) * ld + gcol;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds_tile + piece * 1024), 16, 0, 0);
  }
}

// MFMA fragment (lane l holds X[row = base + (l&15)][k = 32*kk + 8*(l>>4) + j], j = 0..7)
template <bool KMAJ, int ROWS>
__device__ __forceinline__ bf16x8 frag(const char* __restrict__ img, int base, int kk) {
  const int l = threadIdx.x & 63;
  if constexpr (KMAJ) {
    const int row = base + (l & 15);
    const int gc = kk * 4 + (l >> 4);
    return *reinterpret_cast<const bf16x8*>(img + row * 128 + ((gc ^ (row & 7)) << 4));
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

// column sum over the 64 k of the A image for tile row `row` (wgrad bias gradient)
template <bool KMAJ>
__device__ __forceinline__ float colsum64(const char* __restrict__ img, int row) {
  float s = 0.f;
  if constexpr (KMAJ) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint4 v = *reinterpret_cast<const uint4*>(img + row * 128 + (c << 4));
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) s += __uint_as_float(w[j] << 16) + __uint_as_float(w[j] & 0xffff0000u);
    }
  } else {
    constexpr int RB = BM * 2;
    const int gc = row >> 3, within = (row & 7) * 2;
#pragma unroll 16
    for (int r = 0; r < BK; ++r) {
      const uint16_t h = *reinterpret_cast<const uint16_t*>(img + r * RB + ((gc ^ mswz(r)) << 4) + within);
      s += bf2f(h);
    }
  }
  return s;
}

// wgrad bias gradient for an m-major A image [64 k][BM m]: thread t owns the 16-B chunk t&31 (8 m)
// of k rows 4(t>>5)..+3, accumulated over the k-steps with ds_read_b128 (4 per k-step); the 16
// k-groups are folded through LDS once after the main loop (colsum_fold).
__device__ __forceinline__ void colsum_mmajor(const char* __restrict__ img, float (&cs)[8]) {
  constexpr int RB = BM * 2;
  const int gc = threadIdx.x & 31, kg = threadIdx.x >> 5;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = kg * 4 + j;
    const uint4 v = *reinterpret_cast<const uint4*>(img + r * RB + ((gc ^ mswz(r)) << 4));
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      cs[2 * q] += __uint_as_float(w[q] << 16);
      cs[2 * q + 1] += __uint_as_float(w[q] & 0xffff0000u);
    }
  }
}
// after the main loop (LDS free): fold the 16 k-groups, thread m < BM returns the sum for row m
__device__ __forceinline__ float colsum_fold(const float (&cs)[8], float* red) {
  const int gc = threadIdx.x & 31, kg = threadIdx.x >> 5;
#pragma unroll
  for (int q = 0; q < 8; ++q) red[kg * BM + gc * 8 + q] = cs[q];
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x < BM)
    for (int g = 0; g < 16; ++g) s += red[g * BM + threadIdx.x];
  __syncthreads();
  return s;
}

template <bool AK, bool BKM, int BN>
__global__ void __launch_bounds__(THREADS) gemm2_kernel(const uint16_t* __restrict__ A, int64_t lda,
                                                       const uint16_t* __restrict__ B, int64_t ldb, int K,
                                                       int kper, int tilesM, int tilesN, EpiArgs e,
                                                       float* __restrict__ colsum) {
  using C = Cfg<BN>;
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
  const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;

  const int wid = threadIdx.x >> 6, wm = wid / C::WAVES_N, wn = wid % C::WAVES_N;
  const bool do_cs = colsum != nullptr && tn == 0;
  float csum = 0.f;
  float cs8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x4 acc[C::FM][4];
#pragma unroll
  for (int i = 0; i < C::FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt) {
    char* st = smem + (kt % C::STAGES) * C::STAGE_BYTES;
    const int k0 = kbeg + kt * BK;
    issue_tile<AK, BM, A_PER_WAVE>(A, lda, m0, k0, e.M, st);
    issue_tile<BKM, BN, C::B_PER_WAVE>(B, ldb, n0, k0, e.N, st + A_BYTES);
  };

  for (int p = 0; p < C::STAGES - 1 && p < nk; ++p) issue(p);
  for (int kt = 0; kt < nk; ++kt) {
    // tile kt must have landed; the (STAGES - 2) younger tiles may stay in flight
    if constexpr (C::STAGES == 3) {
      static_assert(C::LOADS == 6, "vmcnt immediate below assumes 6 LDS-DMA pieces per wave per stage");
      if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // into the slot of tile kt-1, which every wave has finished reading
    if (kt + C::STAGES - 1 < nk) issue(kt + C::STAGES - 1);
    const char* ai = smem + (kt % C::STAGES) * C::STAGE_BYTES;
    const char* bi = ai + A_BYTES;
    if constexpr (AK) {
      if (do_cs && threadIdx.x < BM) csum += colsum64<AK>(ai, threadIdx.x);
    } else {
      static_assert(THREADS == 512 && BK == 64, "colsum_mmajor thread map");
      if (do_cs) colsum_mmajor(ai, cs8);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 af[C::FM], bfr[4];
#pragma unroll
      for (int i = 0; i < C::FM; ++i) af[i] = frag<AK, BM>(ai, wm * (16 * C::FM) + i * 16, kk);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BKM, BN>(bi, wn * 64 + j * 16, kk);
#pragma unroll
      for (int i = 0; i < C::FM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if constexpr (!AK) {
    if (do_cs) csum = colsum_fold(cs8, reinterpret_cast<float*>(smem));  // block-uniform branch
  }
  if (do_cs && threadIdx.x < BM && m0 + (int)threadIdx.x < e.M) colsum[(size_t)split * e.M + m0 + threadIdx.x] = csum;
  wave_tile_epilogue<C::FM>(acc, reinterpret_cast<float*>(smem) + wid * 16 * EPI_LD, m0 + wm * (16 * C::FM),
                            n0 + wn * 64, e, split);
}

template <bool AK, bool BKM, int BN>
static int launch(const sv_gemm_desc* d, int split, int kper, hipStream_t s) {
  const int tilesM = ceil_div(d->M, BM), tilesN = ceil_div(d->N, BN);
  EpiArgs e{d->M, d->N, d->epilogue, d->C, d->c_dtype, d->ldc, d->C2, d->c2_dtype, d->bias, d->gamma,
            d->aux, d->aux_dtype, d->ld_aux};
  constexpr size_t lds = Cfg<BN>::LDS;
  if (const int rc_ = ensure_lds_attr(reinterpret_cast<const void*>(&gemm2_kernel<AK, BKM, BN>), (int)lds, s)) return rc_;
  dim3 grid(tilesM * tilesN, 1, split);
  gemm2_kernel<AK, BKM, BN><<<grid, THREADS, lds, s>>>(
      reinterpret_cast<const uint16_t*>(d->A), d->lda, reinterpret_cast<const uint16_t*>(d->B), d->ldb, d->K, kper,
      tilesM, tilesN, e, d->epilogue == SV_EPI_SLAB ? reinterpret_cast<float*>(d->C2) : nullptr);
  return check_launch("sv_gemm(v2)");
}

template <bool AK, bool BKM>
static int launch_bn(const sv_gemm_desc* d, int split, int kper, hipStream_t s) {
  // 256-wide tiles (half the L2->LDS bytes per FLOP) measured slower than 128-wide on every ConvNeXt
  // shape (the 2-stage ring exposes the DMA latency at one workgroup per CU), round 1
  return launch<AK, BKM, 128>(d, split, kper, s);
}

}  // namespace g2

int launch_gemm2(const sv_gemm_desc* d, hipStream_t s) {
  using namespace g2;
  if (d->compute != SV_BF16 || d->a_dtype != SV_BF16 || d->b_dtype != SV_BF16 || d->a_scale_k)
    return SV_ERR_UNSUPPORTED;
  const int split = d->epilogue == SV_EPI_SLAB ? (d->split_k < 1 ? 1 : d->split_k) : 1;
  const int kper = ceil_div(ceil_div(d->K, split), BK) * BK;
  if (d->K % BK != 0 || d->K < BK) return SV_ERR_UNSUPPORTED;
  // m-major operands need whole 16-B chunks along the tile width: M/N multiples of 8 (checked by
  // sv_gemm); k-major need K multiple of 64 (above)
  if (d->a_kmajor && d->b_kmajor) return launch_bn<true, true>(d, split, kper, s);
  if (d->a_kmajor && !d->b_kmajor) return launch_bn<true, false>(d, split, kper, s);
  if (!d->a_kmajor && d->b_kmajor) return launch_bn<false, true>(d, split, kper, s);
  return launch_bn<false, false>(d, split, kper, s);
}

}  // namespace sv
