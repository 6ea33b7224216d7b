// MFMA GEMM v8 (bf16 operands, f32 accumulate): 256x256 output tile per 512-thread workgroup, one
// workgroup per CU; 8 waves in 2(M) x 4(N), 128x64 per wave = 8x4 v_mfma_f32_16x16x32_bf16 fragments
// (128 accumulator VGPRs, ~210 VGPRs at two waves per SIMD).
//
// Why: the 256x128 tile of v2/v3 moves (256+128)/(256*128) operand bytes per MAC through LDS-DMA --
// at the bf16 MFMA peak 47 B/clk/CU, above what one CU's LDS-DMA sustains from L2 (~33 B/clk) -- so
// the long-K GEMMs (fc2 fwd, fc1 dgrad, the wgrads: K >= 1024) are ingest-bound.  256x256 needs
// 32 B/clk at the peak and halves the fragment reads per MFMA of the M side.  Everything else is v3:
// LDS-DMA ring (BK 32 x 4 stages = 128 KiB) from XOR-swizzled SOURCE addresses, counted vmcnt with two
// k-tiles in flight, raw s_barrier, ds_read_b128 / ds_read_b64_tr_b16 fragments, XCD-aware tile order,
// one kernel per epilogue kind, split-K slabs with the fused bias column sum.
#include "common.h"
#include "gemm_common.h"

#include <stdlib.h>
#include <string.h>

namespace sv {
namespace g8 {

constexpr int BM = 256, BN = 256, THREADS = 512, NW = 8;
constexpr int FM = 8, FN = 4;  // 16x16 fragments per wave (128 x 64)

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <int BKT>
__device__ __forceinline__ int kswz(int row) {
  if constexpr (BKT == 64) return row & 7;
  else return ((row >> 3) & 1) << 1;
}
__device__ __forceinline__ int mswz(int r) { return ((r & 3) << 1) ^ (((r >> 3) & 1) << 3); }

template <int BKT, int S>
struct Cfg {
  static constexpr int A_BYTES = BM * BKT * 2, B_BYTES = BN * BKT * 2, STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int A_PER_WAVE = A_BYTES / 1024 / NW, B_PER_WAVE = B_BYTES / 1024 / NW;
  static constexpr int LOADS = A_PER_WAVE + B_PER_WAVE;  // LDS-DMA instructions per wave per stage
  static constexpr size_t LDS = (size_t)S * STAGE_BYTES;
  static constexpr bool TWO_PER_CU = LDS <= 80 * 1024;
};

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

template <bool AK, bool BKM, int EPI, int BKT, int S, int OCC>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(OCC, OCC)))
gemm8_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb, int K, int kper,
             int tilesM, int tilesN, int nsplit, int stagger, EpiArgs e, float* __restrict__ colsum) {
  using C = Cfg<BKT, S>;
  static_assert(S >= 2 && (S - 2) * C::LOADS <= 63, "ring / vmcnt");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nwg = tilesM * tilesN, total = nwg * nsplit;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wm = wid >> 2, wn = wid & 3;
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

    __syncthreads();  // the previous tile's epilogue slabs overlap the ring
#pragma unroll
    for (int p = 0; p < S - 1; ++p)
      if (p < nk) issue(p);
    for (int kt = 0; kt < nk; ++kt) {
      // tile kt must have landed; the min(S-2, nk-1-kt) younger tiles may stay in flight
      const int younger = nk - 1 - kt < S - 2 ? nk - 1 - kt : S - 2;
      if (S > 3 && younger >= 2) vm_wait<(S > 3 ? 2 * C::LOADS : 0)>();
      else if (S > 2 && younger >= 1) vm_wait<(S > 2 ? C::LOADS : 0)>();
      else vm_wait<0>();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + S - 1 < nk) issue(kt + S - 1);  // into the slot of tile kt-1, which every wave has finished
      const char* ai = smem + (kt % S) * C::STAGE_BYTES;
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
        bf16x8 af[FM], bfr[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) bfr[j] = frag<BKM, BN, BKT>(bi, wn * 64 + j * 16, kk);
#pragma unroll
        for (int i = 0; i < FM; ++i) af[i] = frag<AK, BM, BKT>(ai, wm * 128 + i * 16, kk);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    vm_wait<0>();
    __syncthreads();
    if constexpr (!AK) {
      if (do_cs) csum = colsum_fold(cs8, reinterpret_cast<float*>(smem));  // block-uniform branch
    }
    if (do_cs && threadIdx.x < BM && m0 + (int)threadIdx.x < e.M) colsum[(size_t)split * e.M + m0 + threadIdx.x] = csum;
    // the epilogue operand is bf16 (GELU'(h), pre-activation) or the f32 residual stream
    constexpr int AUXT = (EPI == SV_EPI_MUL_AUX || EPI == SV_EPI_GELU_GRAD) ? SV_BF16
                         : EPI == SV_EPI_BIAS_GAMMA_RES ? SV_F32 : -1;
    wave_tile_epilogue<FM, 2, EPI, AUXT>(acc, reinterpret_cast<float*>(smem) + wid * 16 * EPI_LD, m0 + wm * 128,
                                         n0 + wn * 64, e, split);
  }
}

template <bool AK, bool BKM, int EPI, int BKT, int S>
static int launch(const sv_gemm_desc* d, int split, hipStream_t s) {
  using C = Cfg<BKT, S>;
  if ((EPI == SV_EPI_MUL_AUX || EPI == SV_EPI_GELU_GRAD) && d->aux_dtype != SV_BF16) return SV_ERR_UNSUPPORTED;
  if (EPI == SV_EPI_BIAS_GAMMA_RES && d->aux_dtype != SV_F32) return SV_ERR_UNSUPPORTED;
  constexpr int OCC = 2;  // two waves per SIMD: one 512-thread workgroup per CU
  const int kper = ceil_div(ceil_div(d->K, split), BKT) * BKT;
  const int tilesM = ceil_div(d->M, BM), tilesN = ceil_div(d->N, BN);
  EpiArgs e{d->M, d->N, d->epilogue, d->C, d->c_dtype, d->ldc, d->C2, d->c2_dtype, d->bias, d->gamma,
            d->aux, d->aux_dtype, d->ld_aux};
  if (const int rc_ = ensure_lds_attr(reinterpret_cast<const void*>(&gemm8_kernel<AK, BKM, EPI, BKT, S, OCC>), (int)C::LDS, s)) return rc_;
  const int total = tilesM * tilesN * split;
  gemm8_kernel<AK, BKM, EPI, BKT, S, OCC><<<total, THREADS, C::LDS, s>>>(
      reinterpret_cast<const uint16_t*>(d->A), d->lda, reinterpret_cast<const uint16_t*>(d->B), d->ldb, d->K, kper,
      tilesM, tilesN, split, 0, e, d->epilogue == SV_EPI_SLAB ? reinterpret_cast<float*>(d->C2) : nullptr);
  return check_launch("sv_gemm(v8)");
}

// one kernel per epilogue kind: each carries only its own epilogue's registers
template <bool AK, bool BKM, int BKT, int S>
static int launch_epi(const sv_gemm_desc* d, int split, hipStream_t s) {
  switch (d->epilogue) {
    case SV_EPI_STORE: return launch<AK, BKM, SV_EPI_STORE, BKT, S>(d, split, s);
    case SV_EPI_BIAS_GELU2: return launch<AK, BKM, SV_EPI_BIAS_GELU2, BKT, S>(d, split, s);
    case SV_EPI_BIAS_GAMMA_RES: return launch<AK, BKM, SV_EPI_BIAS_GAMMA_RES, BKT, S>(d, split, s);
    case SV_EPI_GELU_GRAD: return launch<AK, BKM, SV_EPI_GELU_GRAD, BKT, S>(d, split, s);
    case SV_EPI_SLAB: return launch<AK, BKM, SV_EPI_SLAB, BKT, S>(d, split, s);
    case SV_EPI_BIAS_GELU_DUAL: return launch<AK, BKM, SV_EPI_BIAS_GELU_DUAL, BKT, S>(d, split, s);
    case SV_EPI_MUL_AUX: return launch<AK, BKM, SV_EPI_MUL_AUX, BKT, S>(d, split, s);
    case SV_EPI_BIAS_GELU: return launch<AK, BKM, SV_EPI_BIAS_GELU, BKT, S>(d, split, s);
    default: return SV_ERR_UNSUPPORTED;
  }
}

template <int BKT, int S>
static int launch_cfg(const sv_gemm_desc* d, int split, hipStream_t s) {
  if (d->K % BKT != 0 || d->K < BKT) return SV_ERR_UNSUPPORTED;
  if (d->a_kmajor && d->b_kmajor) return launch_epi<true, true, BKT, S>(d, split, s);
  if (d->a_kmajor && !d->b_kmajor) return launch_epi<true, false, BKT, S>(d, split, s);
  if (!d->a_kmajor && d->b_kmajor) return launch_epi<false, true, BKT, S>(d, split, s);
  return launch_epi<false, false, BKT, S>(d, split, s);
}

}  // namespace g8

int launch_gemm8(const sv_gemm_desc* d, hipStream_t s) {
  using namespace g8;
  if (d->compute != SV_BF16 || d->a_dtype != SV_BF16 || d->b_dtype != SV_BF16 || d->a_scale_k)
    return SV_ERR_UNSUPPORTED;
  const int split = d->epilogue == SV_EPI_SLAB ? (d->split_k < 1 ? 1 : d->split_k) : 1;
  return launch_cfg<32, 4>(d, split, s);
}

}  // namespace sv
