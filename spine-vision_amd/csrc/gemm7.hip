// MFMA GEMM v7 (bf16 operands, f32 accumulate): the v3 tile (256x128 per 512-thread workgroup,
// 8 waves of 64x64 = 4x4 v_mfma_f32_16x16x32_bf16 fragments, BK 32) with REGISTER-STAGED operand
// loads instead of LDS-DMA: every wave fetches its 3 KiB share of tile kt+3 with global_load_dwordx4
// into VGPRs while tile kt is multiplied, and writes tile kt+1 into the LDS double buffer with
// ds_write_b128.  An LDS-DMA piece costs its wave 60-185 issue cycles beside MFMAs
// (MI355X_MICROARCH.md, cycle constants), a global_load + ds_write_b128 pair a fraction of that.
//
//   * two tiles in flight in registers (2 x 12 VGPRs), LDS 2 x 24 KiB, one s_barrier per tile;
//   * OCC 4: 128 VGPRs, two workgroups per CU; OCC 2: one workgroup per CU;
//   * the LDS image is written lane-linearly, so bank conflicts are avoided by XOR-swizzling the SOURCE:
//       k-major [rows][BK]: LDS chunk = k-chunk ^ (row & 7) (BK 64) / ^ 2((row>>3)&1) (BK 32)
//         -> conflict-free ds_read_b128 fragment reads;
//       m-major [BK][rows]: LDS chunk = m-chunk ^ (2(r&3) ^ 8((r>>3)&1))
//         -> conflict-free ds_read_b64_tr_b16 (no transposed copies in HBM);
//   * persistent: gridDim.x = slots (two per CU at 72 KiB), tile t = blockIdx.x + k gridDim.x in an
//     XCD-aware order; the second workgroup of each CU starts `stagger` cycles late;
//   * one kernel per epilogue kind; bf16 epilogue operands (GELU'(h)) are fetched one slab ahead so
//     their wait never drains the stores issued before them.
#include "common.h"
#include "gemm_common.h"

#include <stdlib.h>
#include <string.h>

namespace sv {
namespace g7 {

constexpr int BM = 256, BN = 128, THREADS = 512, NW = 8;

typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <int BKT>
__device__ __forceinline__ int kswz(int row) {
  if constexpr (BKT == 64) return row & 7;
  else return ((row >> 3) & 1) << 1;
}
__device__ __forceinline__ int mswz(int r) { return ((r & 3) << 1) ^ (((r >> 3) & 1) << 3); }

template <int BKT, int S = 2>
struct Cfg {
  static constexpr int A_BYTES = BM * BKT * 2, B_BYTES = BN * BKT * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int A_PER_WAVE = A_BYTES / 1024 / NW, B_PER_WAVE = B_BYTES / 1024 / NW;
  static constexpr int LOADS = A_PER_WAVE + B_PER_WAVE;  // global_load_dwordx4 per wave per tile
  static constexpr size_t LDS = (size_t)S * STAGE_BYTES > 36 * 1024 ? (size_t)S * STAGE_BYTES : 36 * 1024;
};

// Global -> register half of a tile load: the lane's 16 B of 1-KiB LDS piece `piece`, read from the
// XOR-swizzled SOURCE address so the linear LDS image it lands in is the bank-conflict-free layout
// the fragment reads expect (the v2/v3 LDS-DMA layout).
template <bool KMAJ, int ROWS, int BKT>
__device__ __forceinline__ uint4 fetch_piece(const uint16_t* __restrict__ X, int64_t ld, int row0, int k0, int R,
                                             int piece) {
  const int lane = threadIdx.x & 63;
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
  return *reinterpret_cast<const uint4*>(src);
}
__device__ __forceinline__ void store_piece(char* lds_tile, const uint4& r, int piece) {
  *reinterpret_cast<uint4*>(lds_tile + piece * 1024 + (threadIdx.x & 63) * 16) = r;
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

// wgrad bias gradient = column sums of A over k.  k-major image: thread t < BM sums its row;
// m-major image [BK][256]: thread t owns 16-B chunk t&31 (8 m) of k rows (t>>5)*BK/16 .. +BK/16-1,
// folded through LDS after the main loop.
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
template <int BKT>
__device__ __forceinline__ void colsum_mmajor(const char* __restrict__ img, float (&cs)[8]) {
  constexpr int RB = BM * 2, RPG = BKT / 16;
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
  if (threadIdx.x < BM)
    for (int g = 0; g < THREADS / 32; ++g) s += red[g * BM + threadIdx.x];
  __syncthreads();
  return s;
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <bool AK, bool BKM, int EPI, int BKT, int OCC>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(OCC, OCC)))
gemm7_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb, int K, int kper,
             int tilesM, int tilesN, int nsplit, int stagger, EpiArgs e, float* __restrict__ colsum) {
  using C = Cfg<BKT>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nwg = tilesM * tilesN, total = nwg * nsplit;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wm = wid >> 1, wn = wid & 1;
  if (stagger > 0 && blockIdx.x >= gridDim.x / 2) {
    for (int c = 0; c < stagger; c += 2048) __builtin_amdgcn_s_sleep(32);
  }
  for (int t = blockIdx.x; t < total; t += gridDim.x) {
    // XCD-aware order: tiles t = x (mod 8) run on XCD x, each XCD walks a contiguous tile range so
    // concurrently resident tiles share A row panels in that XCD's L2
    const int xcd = t & 7, loc = t >> 3, q8 = total >> 3, r8 = total & 7;
    const int wgi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    const int split = wgi / nwg, wg = wgi - split * nwg;
    const int tm = wg / tilesN, tn = wg % tilesN;
    const int m0 = tm * BM, n0 = tn * BN;
    const int kbeg = split * kper;
    int kend = kbeg + kper;
    if (kend > K) kend = K;
    const int nk = kend > kbeg ? (kend - kbeg) / BKT : 0;

    const bool do_cs = EPI == SV_EPI_SLAB && colsum != nullptr && tn == 0;  // compile-time off otherwise
    float csum = 0.f;
    float cs8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // staging sets: tile t lives in set t & 1; 2 A + 1 B uint4 per lane each (BK 32), kept as
    // scalars so they stay in VGPRs
    static_assert(C::A_PER_WAVE == 2 && C::B_PER_WAVE == 1, "staging written for BK 32");
    uint4 x0a, x0b, x0c, x1a, x1b, x1c;
#define SV7_GLOAD(kt, ra, rb, rc)                                                         \
    {                                                                                     \
      const int k0_ = kbeg + (kt) * BKT;                                                  \
      ra = fetch_piece<AK, BM, BKT>(A, lda, m0, k0_, e.M, wid);                           \
      rb = fetch_piece<AK, BM, BKT>(A, lda, m0, k0_, e.M, wid + NW);                      \
      rc = fetch_piece<BKM, BN, BKT>(B, ldb, n0, k0_, e.N, wid);                          \
    }
#define SV7_SWRITE(kt, ra, rb, rc)                                                        \
    {                                                                                     \
      char* st_ = smem + ((kt) & 1) * C::STAGE_BYTES;                                     \
      store_piece(st_, ra, wid);                                                          \
      store_piece(st_, rb, wid + NW);                                                     \
      store_piece(st_ + C::A_BYTES, rc, wid);                                             \
    }
    auto compute = [&](int kt) __attribute__((always_inline)) {
      const char* ai = smem + (kt & 1) * C::STAGE_BYTES;
      const char* bi = ai + C::A_BYTES;
      if (do_cs) {
        if constexpr (AK) {
          if (threadIdx.x < BM) csum += colsum_kmajor<BKT>(ai, threadIdx.x);
        } else {
          colsum_mmajor<BKT>(ai, cs8);
        }
      }
#pragma unroll
      for (int kk = 0; kk < BKT / 32; ++kk) {
        bf16x8 af[4], bfr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = frag<AK, BM, BKT>(ai, wm * 64 + i * 16, kk);
#pragma unroll
        for (int j = 0; j < 4; ++j) bfr[j] = frag<BKM, BN, BKT>(bi, wn * 64 + j * 16, kk);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    };
    // one pipeline step: tile kt+1 (staged two steps ago) goes to LDS, tile kt+3 is fetched into the
    // freed set, tile kt is multiplied.  (ra, rb, rc) = set (kt+1) & 1.
#define SV7_STEP(kt, ra, rb, rc)                                                               \
    {                                                                                          \
      if ((kt) + 2 < nk) vm_wait<C::LOADS>(); /* tile kt+1 arrived, kt+2 may stay in flight */ \
      else vm_wait<0>();                                                                       \
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); /* my part of tile kt is in LDS */    \
      __builtin_amdgcn_s_barrier();                      /* everyone's; slot (kt+1)&1 free */  \
      asm volatile("" ::: "memory");                                                           \
      if ((kt) + 1 < nk) SV7_SWRITE((kt) + 1, ra, rb, rc);                                     \
      if ((kt) + 3 < nk) SV7_GLOAD((kt) + 3, ra, rb, rc);                                      \
      compute(kt);                                                                             \
    }

    __syncthreads();  // the previous tile's epilogue slabs overlap the LDS buffers
    if (nk > 0) SV7_GLOAD(0, x0a, x0b, x0c);
    if (nk > 1) SV7_GLOAD(1, x1a, x1b, x1c);
    if (nk > 0) {
      if (nk > 1) vm_wait<C::LOADS>();
      else vm_wait<0>();
      SV7_SWRITE(0, x0a, x0b, x0c);
      if (nk > 2) SV7_GLOAD(2, x0a, x0b, x0c);
    }
    int kt = 0;
    for (; kt + 1 < nk; kt += 2) {  // two steps per trip: the staging set stays compile-time
      SV7_STEP(kt, x1a, x1b, x1c);
      SV7_STEP(kt + 1, x0a, x0b, x0c);
    }
    if (kt < nk) SV7_STEP(kt, x1a, x1b, x1c);
#undef SV7_STEP
#undef SV7_SWRITE
#undef SV7_GLOAD
    vm_wait<0>();
    __syncthreads();
    if constexpr (!AK) {
      if (do_cs) csum = colsum_fold(cs8, reinterpret_cast<float*>(smem));  // block-uniform branch
    }
    if (do_cs && threadIdx.x < BM && m0 + (int)threadIdx.x < e.M) colsum[(size_t)split * e.M + m0 + threadIdx.x] = csum;
    // the epilogue operand is bf16 (GELU'(h), pre-activation) or the f32 residual stream
    constexpr int AUXT = (EPI == SV_EPI_MUL_AUX || EPI == SV_EPI_GELU_GRAD) ? SV_BF16
                         : EPI == SV_EPI_BIAS_GAMMA_RES ? SV_F32 : -1;
    wave_tile_epilogue<4, 2, EPI, AUXT>(acc, reinterpret_cast<float*>(smem) + wid * 16 * EPI_LD, m0 + wm * 64,
                                  n0 + wn * 64, e, split);
  }
}

static int num_cus() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  }
  return n;
}

template <bool AK, bool BKM, int EPI, int BKT, int OCC>
static int launch(const sv_gemm_desc* d, int split, hipStream_t s) {
  using C = Cfg<BKT>;
  if ((EPI == SV_EPI_MUL_AUX || EPI == SV_EPI_GELU_GRAD) && d->aux_dtype != SV_BF16) return SV_ERR_UNSUPPORTED;
  if (EPI == SV_EPI_BIAS_GAMMA_RES && d->aux_dtype != SV_F32) return SV_ERR_UNSUPPORTED;
  const int kper = ceil_div(ceil_div(d->K, split), BKT) * BKT;
  const int tilesM = ceil_div(d->M, BM), tilesN = ceil_div(d->N, BN);
  EpiArgs e{d->M, d->N, d->epilogue, d->C, d->c_dtype, d->ldc, d->C2, d->c2_dtype, d->bias, d->gamma,
            d->aux, d->aux_dtype, d->ld_aux};
  const int total = tilesM * tilesN * split;
  const int slots = (OCC == 4 ? 2 : 1) * num_cus();
  const int grid = total > slots ? slots : total;
  static const int stag_env = getenv("SV_GEMM3_STAGGER") ? atoi(getenv("SV_GEMM3_STAGGER")) : -1;
  const int stagger = (OCC == 4 && total > slots) ? (stag_env >= 0 ? stag_env : 384) * (kper / 32) : 0;
  gemm7_kernel<AK, BKM, EPI, BKT, OCC><<<grid, THREADS, C::LDS, s>>>(
      reinterpret_cast<const uint16_t*>(d->A), d->lda, reinterpret_cast<const uint16_t*>(d->B), d->ldb, d->K, kper,
      tilesM, tilesN, split, stagger, e, d->epilogue == SV_EPI_SLAB ? reinterpret_cast<float*>(d->C2) : nullptr);
  return check_launch("sv_gemm(v7)");
}

template <bool AK, bool BKM, int OCC>
static int launch_epi(const sv_gemm_desc* d, int split, hipStream_t s) {
  switch (d->epilogue) {
    case SV_EPI_STORE: return launch<AK, BKM, SV_EPI_STORE, 32, OCC>(d, split, s);
    case SV_EPI_BIAS_GELU2: return launch<AK, BKM, SV_EPI_BIAS_GELU2, 32, OCC>(d, split, s);
    case SV_EPI_BIAS_GAMMA_RES: return launch<AK, BKM, SV_EPI_BIAS_GAMMA_RES, 32, OCC>(d, split, s);
    case SV_EPI_GELU_GRAD: return launch<AK, BKM, SV_EPI_GELU_GRAD, 32, OCC>(d, split, s);
    case SV_EPI_SLAB: return launch<AK, BKM, SV_EPI_SLAB, 32, OCC>(d, split, s);
    case SV_EPI_BIAS_GELU_DUAL: return launch<AK, BKM, SV_EPI_BIAS_GELU_DUAL, 32, OCC>(d, split, s);
    case SV_EPI_MUL_AUX: return launch<AK, BKM, SV_EPI_MUL_AUX, 32, OCC>(d, split, s);
    case SV_EPI_BIAS_GELU: return launch<AK, BKM, SV_EPI_BIAS_GELU, 32, OCC>(d, split, s);
    default: return SV_ERR_UNSUPPORTED;
  }
}

template <int OCC>
static int launch_occ(const sv_gemm_desc* d, int split, hipStream_t s) {
  if (d->K % 32 != 0 || d->K < 32) return SV_ERR_UNSUPPORTED;
  if (d->a_kmajor && d->b_kmajor) return launch_epi<true, true, OCC>(d, split, s);
  if (d->a_kmajor && !d->b_kmajor) return launch_epi<true, false, OCC>(d, split, s);
  if (!d->a_kmajor && d->b_kmajor) return launch_epi<false, true, OCC>(d, split, s);
  return launch_epi<false, false, OCC>(d, split, s);
}

}  // namespace g7

int launch_gemm7(const sv_gemm_desc* d, hipStream_t s, int occ) {
  using namespace g7;
  if (d->compute != SV_BF16 || d->a_dtype != SV_BF16 || d->b_dtype != SV_BF16 || d->a_scale_k)
    return SV_ERR_UNSUPPORTED;
  const int split = d->epilogue == SV_EPI_SLAB ? (d->split_k < 1 ? 1 : d->split_k) : 1;
  static const int occ_env = getenv("SV_GEMM7_OCC") ? atoi(getenv("SV_GEMM7_OCC")) : 0;
  if (occ_env) occ = occ_env;
  return occ == 2 ? launch_occ<2>(d, split, s) : launch_occ<4>(d, split, s);
}

}  // namespace sv
