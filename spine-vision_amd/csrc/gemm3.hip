// MFMA GEMM v3 (bf16 operands, f32 accumulate): the v2 LDS-DMA pipeline re-cut so that TWO
// workgroups fit on every CU, and one workgroup's epilogue (GELU / GELU' / residual math and the
// output stores, which on the ConvNeXt fc1/fc2 shapes take as long as the MFMA main loop) runs
// while the other workgroup's waves keep the matrix cores busy.
//
//   * 256x128 output tile per 512-thread workgroup, 8 waves in 4(M) x 2(N), 64x64 per wave;
//   * BK = 32, 3-stage LDS ring of 24 KiB stages (72 KiB per workgroup, 144 KiB per CU), filled by
//     LDS-DMA (global_load_lds_dwordx4): 3 wave-instructions per wave per stage, counted
//     `s_waitcnt vmcnt(3)` keeps the next tile in flight;
//   * <= 128 VGPRs per lane (amdgpu_waves_per_eu 4): 16 waves per CU = 2 workgroups;
//   * LDS-DMA writes lane-linearly, so bank conflicts are avoided by XOR-swizzling the SOURCE:
//       k-major tile [rows][32 k] (64-B rows): LDS chunk = k-chunk ^ 2((row>>3)&1)
//         -> every 16-lane group of a ds_read_b128 fragment read hits 16 distinct bank quads;
//       m-major tile [32 k][rows]: LDS chunk = m-chunk ^ (2(r&3) ^ 8((r>>3)&1)) as in v2
//         -> conflict-free ds_read_b64_tr_b16;
//   * one kernel per epilogue kind; bf16 epilogue operands (GELU'(h)) are prefetched packed for a
//     whole 64-row group before its first store (a per-slab load would drain all earlier stores).
#include "common.h"
#include "gemm_common.h"

namespace sv {
namespace g3 {

constexpr int BM = 256, BN = 128, BK = 32, STAGES = 3, THREADS = 512;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE_BYTES = A_BYTES + B_BYTES;
constexpr int A_PER_WAVE = A_BYTES / 1024 / 8, B_PER_WAVE = B_BYTES / 1024 / 8;  // 2 + 1
constexpr size_t LDS = (size_t)STAGES * STAGE_BYTES;                             // 72 KiB

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int kswz(int row) { return ((row >> 3) & 1) << 1; }
__device__ __forceinline__ int mswz(int r) { return ((r & 3) << 1) ^ (((r >> 3) & 1) << 3); }

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
      const int row = byte >> 6, ch = (byte >> 4) & 3;
      const int gc = ch ^ kswz(row);
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

template <bool KMAJ, int ROWS>
__device__ __forceinline__ bf16x8 frag(const char* __restrict__ img, int base) {
  const int l = threadIdx.x & 63;
  if constexpr (KMAJ) {
    const int row = base + (l & 15);
    const int c = (l >> 4) ^ kswz(row);
    return *reinterpret_cast<const bf16x8*>(img + row * 64 + (c << 4));
  } else {
    constexpr int RB = ROWS * 2;
    const int g = l >> 4, q = (l >> 2) & 3, p = l & 3;
    const int gc = (base >> 3) + (p >> 1);
    const int r0 = 8 * g + q, r1 = r0 + 4;
    const char* a0 = img + r0 * RB + ((gc ^ mswz(r0)) << 4) + (p & 1) * 8;
    const char* a1 = img + r1 * RB + ((gc ^ mswz(r1)) << 4) + (p & 1) * 8;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// sum over the 32 k of the A image for tile row `row` (wgrad bias gradient)
template <bool KMAJ>
__device__ __forceinline__ float colsum32(const char* __restrict__ img, int row) {
  float s = 0.f;
  if constexpr (KMAJ) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint4 v = *reinterpret_cast<const uint4*>(img + row * 64 + (c << 4));
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) s += __uint_as_float(w[j] << 16) + __uint_as_float(w[j] & 0xffff0000u);
    }
  } else {
    constexpr int RB = BM * 2;
    const int gc = row >> 3, within = (row & 7) * 2;
#pragma unroll 8
    for (int r = 0; r < BK; ++r) {
      const uint16_t h = *reinterpret_cast<const uint16_t*>(img + r * RB + ((gc ^ mswz(r)) << 4) + within);
      s += bf2f(h);
    }
  }
  return s;
}

template <bool AK, bool BKM, int EPI>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(4, 4)))
gemm3_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb, int K, int kper,
             int tilesM, int tilesN, int nsplit, int stagger, EpiArgs e, float* __restrict__ colsum) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // Persistent: gridDim.x workgroups (two per CU) walk the tiles t = blockIdx.x, + gridDim.x, ...
  // The second workgroup of every CU starts `stagger` cycles late, so the two co-resident
  // workgroups stay out of phase and one's epilogue (VALU + stores) runs beside the other's MFMAs.
  const int nwg = tilesM * tilesN, total = nwg * nsplit;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wm = wid >> 1, wn = wid & 1;
  if (stagger > 0 && blockIdx.x >= gridDim.x / 2) {
    for (int c = 0; c < stagger; c += 2048) __builtin_amdgcn_s_sleep(32);
  }
  for (int t = blockIdx.x; t < total; t += gridDim.x) {
    // XCD-aware order: tiles t = x (mod 8) run on XCD x; each XCD walks a contiguous tile range so
    // concurrently resident tiles share A row panels in that XCD's L2
    const int xcd = t & 7, loc = t >> 3, q8 = total >> 3, r8 = total & 7;
    const int wgi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    const int split = wgi / nwg, wg = wgi - split * nwg;
    const int tm = wg / tilesN, tn = wg % tilesN;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = split * kper;
    int kend = kbeg + kper;
    if (kend > K) kend = K;
    const int nk = kend > kbeg ? (kend - kbeg) / BK : 0;

    const bool do_cs = colsum != nullptr && tn == 0;
    float csum = 0.f;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto issue = [&](int kt) {
      char* st = smem + (kt % STAGES) * STAGE_BYTES;
      const int k0 = kbeg + kt * BK;
      issue_tile<AK, BM, A_PER_WAVE>(A, lda, m0, k0, e.M, st);
      issue_tile<BKM, BN, B_PER_WAVE>(B, ldb, n0, k0, e.N, st + A_BYTES);
    };

    __syncthreads();  // the previous tile's epilogue slabs overlap the ring
    if (nk > 0) issue(0);
    if (nk > 1) issue(1);
    for (int kt = 0; kt < nk; ++kt) {
      static_assert(A_PER_WAVE + B_PER_WAVE == 3, "vmcnt immediate below assumes 3 LDS-DMA pieces per wave per stage");
      if (kt + 1 < nk) {
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // tile kt landed, tile kt+1 stays in flight
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + 2 < nk) issue(kt + 2);  // into the slot of tile kt-1, which every wave has finished
      const char* ai = smem + (kt % STAGES) * STAGE_BYTES;
      const char* bi = ai + A_BYTES;
      if (do_cs && threadIdx.x < BM) csum += colsum32<AK>(ai, threadIdx.x);
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<AK, BM>(ai, wm * 64 + i * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BKM, BN>(bi, wn * 64 + j * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (do_cs && threadIdx.x < BM && m0 + (int)threadIdx.x < e.M) colsum[(size_t)split * e.M + m0 + threadIdx.x] = csum;
    wave_tile_epilogue<4, 2, EPI>(acc, reinterpret_cast<float*>(smem) + wid * 16 * EPI_LD, m0 + wm * 64,
                                  n0 + wn * 64, e, split);
  }
}

static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <bool AK, bool BKM, int EPI>
static int launch(const sv_gemm_desc* d, int split, int kper, hipStream_t s) {
  const int tilesM = ceil_div(d->M, BM), tilesN = ceil_div(d->N, BN);
  EpiArgs e{d->M, d->N, d->epilogue, d->C, d->c_dtype, d->ldc, d->C2, d->c2_dtype, d->bias, d->gamma,
            d->aux, d->aux_dtype, d->ld_aux};
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm3_kernel<AK, BKM, EPI>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS);
    attr_set = true;
  }
  // SV_GEMM3_PERSIST=0: one workgroup per tile (no stagger); default persistent, 2 per CU
  static const int persist = getenv("SV_GEMM3_PERSIST") ? atoi(getenv("SV_GEMM3_PERSIST")) : 1;
  static const int stag_env = getenv("SV_GEMM3_STAGGER") ? atoi(getenv("SV_GEMM3_STAGGER")) : -1;
  const int total = tilesM * tilesN * split;
  int grid = total, stagger = 0;
  if (persist) {
    const int slots = 2 * num_cus();
    if (total > slots) {
      grid = slots;
      const int nk = kper / BK;
      stagger = stag_env >= 0 ? stag_env * nk : 384 * nk;  // ~half a tile's main loop
    }
  }
  gemm3_kernel<AK, BKM, EPI><<<grid, THREADS, LDS, s>>>(
      reinterpret_cast<const uint16_t*>(d->A), d->lda, reinterpret_cast<const uint16_t*>(d->B), d->ldb, d->K, kper,
      tilesM, tilesN, split, stagger, e, d->epilogue == SV_EPI_SLAB ? reinterpret_cast<float*>(d->C2) : nullptr);
  return check_launch("sv_gemm(v3)");
}

// one kernel per epilogue kind: each carries only its own epilogue's registers
template <bool AK, bool BKM>
static int launch_epi(const sv_gemm_desc* d, int split, int kper, hipStream_t s) {
  switch (d->epilogue) {
    case SV_EPI_STORE: return launch<AK, BKM, SV_EPI_STORE>(d, split, kper, s);
    case SV_EPI_BIAS_GELU2: return launch<AK, BKM, SV_EPI_BIAS_GELU2>(d, split, kper, s);
    case SV_EPI_BIAS_GAMMA_RES: return launch<AK, BKM, SV_EPI_BIAS_GAMMA_RES>(d, split, kper, s);
    case SV_EPI_GELU_GRAD: return launch<AK, BKM, SV_EPI_GELU_GRAD>(d, split, kper, s);
    case SV_EPI_SLAB: return launch<AK, BKM, SV_EPI_SLAB>(d, split, kper, s);
    case SV_EPI_BIAS_GELU_DUAL: return launch<AK, BKM, SV_EPI_BIAS_GELU_DUAL>(d, split, kper, s);
    case SV_EPI_MUL_AUX: return launch<AK, BKM, SV_EPI_MUL_AUX>(d, split, kper, s);
    default: return SV_ERR_UNSUPPORTED;
  }
}

}  // namespace g3

int launch_gemm3(const sv_gemm_desc* d, hipStream_t s) {
  using namespace g3;
  if (d->compute != SV_BF16 || d->a_dtype != SV_BF16 || d->b_dtype != SV_BF16 || d->a_scale_k)
    return SV_ERR_UNSUPPORTED;
  const int split = d->epilogue == SV_EPI_SLAB ? (d->split_k < 1 ? 1 : d->split_k) : 1;
  const int kper = ceil_div(ceil_div(d->K, split), BK) * BK;
  if (d->K % BK != 0 || d->K < BK) return SV_ERR_UNSUPPORTED;
  if (d->a_kmajor && d->b_kmajor) return launch_epi<true, true>(d, split, kper, s);
  if (d->a_kmajor && !d->b_kmajor) return launch_epi<true, false>(d, split, kper, s);
  if (!d->a_kmajor && d->b_kmajor) return launch_epi<false, true>(d, split, kper, s);
  return launch_epi<false, false>(d, split, kper, s);
}

}  // namespace sv
