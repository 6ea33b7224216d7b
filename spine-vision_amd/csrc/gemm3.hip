// MFMA GEMM v3 (bf16 operands, f32 accumulate): 256x128 output tile per 512-thread workgroup
// (8 waves in 4(M) x 2(N), 64x64 per wave = 4x4 v_mfma_f32_16x16x32_bf16 fragments), LDS ring of S
// stages of BK k, filled by LDS-DMA (global_load_lds_dwordx4), persistent over the tiles.
//
//   * configurations: BK 32 x 3 stages = 72 KiB (two workgroups per CU: one's epilogue runs beside
//     the other's MFMAs; default) and BK 32 x 4 = 96 KiB (one workgroup per CU, the split-K wgrads).
//     BK 64 x 2/3, a persistent grid and a staggered second workgroup measured no faster (round 1);
//   * counted `s_waitcnt vmcnt` keeps the S-2 younger tiles in flight, one s_barrier per tile;
//   * LDS-DMA writes lane-linearly, so bank conflicts are avoided by XOR-swizzling the SOURCE:
//       k-major [rows][BK]: LDS chunk = k-chunk ^ (row & 7) (BK 64) / ^ 2((row>>3)&1) (BK 32)
//         -> conflict-free ds_read_b128 fragment reads;
//       m-major [BK][rows]: LDS chunk = m-chunk ^ (2(r&3) ^ 8((r>>3)&1))
//         -> conflict-free ds_read_b64_tr_b16 (no transposed copies in HBM);
//   * one workgroup per tile (the grid is capped at the co-resident slots only under
//     sv_gemm_set_workgroups_per_cu), tile t = blockIdx.x + k gridDim.x in an XCD-aware order;
//   * one kernel per epilogue kind; bf16 epilogue operands (GELU'(h)) are fetched one slab ahead so
//     their wait never drains the stores issued before them.
#include "common.h"
#include "gemm_common.h"

#include <stdlib.h>
#include <string.h>

namespace sv {
namespace g3 {

constexpr int BM = 256, BN = 128, THREADS = 512, NW = 8;

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

// implicit-GEMM A operand (CONV 1/2): 16-B chunks of gathered pixels; out-of-image taps and rows
// past M read this zero page, so the MFMA consumer never branches
__device__ __attribute__((aligned(64))) uint16_t g_conv_zero[64];

template <int BKT, int PER_WAVE>
__device__ __forceinline__ void issue_gather(const uint16_t* __restrict__ X, const ConvG& g, const int (&gb)[PER_WAVE],
                                             const int (&gy)[PER_WAVE], const int (&gx)[PER_WAVE], int ty, int tx,
                                             int cb, char* lds_tile, int wid) {
  const int lane = threadIdx.x & 63;
  constexpr int RB = BKT * 2;
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int piece = wid + NW * j;
    const int byte = piece * 1024 + lane * 16;
    const int row = byte / RB, ch = (byte % RB) >> 4;
    const int gc = ch ^ kswz<BKT>(row);
    const int iy = gy[j] + ty, ix = gx[j] + tx;
    const uint16_t* src = g_conv_zero;
    if (gb[j] >= 0 && (unsigned)iy < (unsigned)g.SH && (unsigned)ix < (unsigned)g.SW)
      src = X + ((((size_t)(gb[j] + iy) * g.SW + ix) << g.lsc) + cb + gc * 8);
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds_tile + piece * 1024), 16, 0, 0);
  }
}

// implicit-GEMM A operand over 8-channel pixels (CONV 6, the ResNet stem's Cs = 8): each lane's 16-B chunk
// is one whole tap of its pixel, so the tap is decoded per lane (taps past ntaps read the zero page)
template <int BKT, int PER_WAVE>
__device__ __forceinline__ void issue_gather8(const uint16_t* __restrict__ X, const ConvG& g, const int (&gb)[PER_WAVE],
                                              const int (&gy)[PER_WAVE], const int (&gx)[PER_WAVE], int k0,
                                              char* lds_tile, int wid) {
  const int lane = threadIdx.x & 63;
  constexpr int RB = BKT * 2;
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int piece = wid + NW * j;
    const int byte = piece * 1024 + lane * 16;
    const int row = byte / RB, ch = (byte % RB) >> 4;
    const int t = (k0 >> 3) + (ch ^ kswz<BKT>(row));
    const uint16_t* src = g_conv_zero;
    if (t < g.ntaps && gb[j] >= 0) {
      const int q = (int)(((uint32_t)t * g.kw_mul) >> 16);
      const int iy = gy[j] + q - g.pad, ix = gx[j] + (t - q * g.kw) - g.pad;
      if ((unsigned)iy < (unsigned)g.SH && (unsigned)ix < (unsigned)g.SW)
        src = X + ((size_t)(gb[j] + iy) * g.SW + ix) * 8;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds_tile + piece * 1024), 16, 0, 0);
  }
}
// its B operand: the packed weight [N][ntaps * 8] k-major, columns past ntaps * 8 (the K padding to a whole
// k-step) read the zero page instead of the next row
template <int BKT, int PER_WAVE>
__device__ __forceinline__ void issue_tile_kclamp(const uint16_t* __restrict__ X, int64_t ld, int row0, int k0, int R,
                                                  int kreal, char* lds_tile, int wid) {
  const int lane = threadIdx.x & 63;
  constexpr int RB = BKT * 2;
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int piece = wid + NW * j;
    const int byte = piece * 1024 + lane * 16;
    const int row = byte / RB, ch = (byte % RB) >> 4;
    const int k = k0 + (ch ^ kswz<BKT>(row)) * 8;
    int grow = row0 + row;
    if (grow >= R) grow = 0;
    const uint16_t* src = k < kreal ? X + (size_t)grow * ld + k : g_conv_zero;
    __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(lds_tile + piece * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ uint32_t cg_div(uint32_t n, uint32_t mul, uint32_t shift) {
  return (uint32_t)(((uint64_t)__umulhi(n, mul) + n) >> shift);
}

// implicit-GEMM B operand of the weight gradient (CONV 3): B(k = pixel, n = t*SC + c) =
// x[b, oy*si + tdy[t], ox*si + tdx[t], c], M-major image [BK][BN].  A lane's k-row and 8-column chunk
// are fixed for the whole tile (so its tap / channel offset is precomputed: bc, by, bx); per k-step
// only the pixel k0 + krow is decoded.
template <int BKT, int PER_WAVE>
__device__ __forceinline__ void issue_gather_n(const uint16_t* __restrict__ X, const ConvG& g, int K, int k0,
                                               const int (&bk)[PER_WAVE], const int (&bc)[PER_WAVE],
                                               const int (&by)[PER_WAVE], const int (&bx)[PER_WAVE],
                                               char* lds_tile, int wid) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < PER_WAVE; ++j) {
    const int piece = wid + NW * j;
    const int pix = k0 + bk[j];
    const uint16_t* src = g_conv_zero;
    if (bc[j] >= 0 && pix < K) {
      const uint32_t b = cg_div((uint32_t)pix, g.ghw_mul, g.ghw_shift);
      const uint32_t rem = (uint32_t)pix - b * (uint32_t)(g.GH * g.GW);
      const uint32_t oy = cg_div(rem, g.gw_mul, g.gw_shift);
      const uint32_t ox = rem - oy * (uint32_t)g.GW;
      const int iy = (int)oy * g.si + by[j], ix = (int)ox * g.si + bx[j];
      if ((unsigned)iy < (unsigned)g.SH && (unsigned)ix < (unsigned)g.SW)
        src = X + (((((size_t)b * g.SH + iy) * g.SW + ix) << g.lsc) + bc[j]);
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

// wait until at most min(younger, S-2) younger tiles' LOADS-per-tile DMAs are outstanding
template <int LOADS, int S>
__device__ __forceinline__ void ring_wait(int younger) {
  if constexpr (S > 2) {
    if (younger >= S - 2) vm_wait<(S - 2) * LOADS>();
    else ring_wait<LOADS, S - 1>(younger);
  } else {
    vm_wait<0>();
  }
}

// AUXO >= 0: the epilogue operand's dtype, overriding the one the epilogue kind implies (the bf16 gradient stream's
// in-place accumulate: SV_EPI_BIAS_GAMMA_RES over a bf16 dx)
template <bool AK, bool BKM, int EPI, int BKT, int S, int OCC, int CONV = 0, int AUXO = -1>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(OCC, OCC)))
gemm3_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb, int K, int kper,
             int tilesM, int tilesN, int nsplit, EpiArgs e, float* __restrict__ colsum, ConvG cg) {
  using C = Cfg<BKT, S>;
  static_assert(S >= 2 && (S - 2) * C::LOADS <= 63, "ring / vmcnt");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nwg = tilesM * tilesN, total = nwg * nsplit;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wm = wid >> 1, wn = wid & 1;
  // a critical-path GEMM sharing its CUs with a concurrent stream's kernels issues first
  if (e.prio) __builtin_amdgcn_s_setprio(2);
  for (int t = blockIdx.x; t < total; t += gridDim.x) {
    // XCD-aware order: tiles t = x (mod 8) run on XCD x, each XCD walks a contiguous tile range so
    // concurrently resident tiles share A row panels in that XCD's L2
    const int xcd = t & 7, loc = t >> 3, q8 = total >> 3, r8 = total & 7;
    const int wgi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    const int split = wgi / nwg, wg = wgi - split * nwg;
    const int tm = wg / tilesN, tn = wg % tilesN;
    const int m0 = tm * BM, n0 = tn * BN;
    int kbeg = split * kper;
    int kend = kbeg + kper;
    if (kend > K) kend = K;
    if constexpr (CONV == 5) {  // "split" = the parity class: its own tap run, its own slab
      kbeg = 0;
      kend = (int)cg.ctaps[split] << cg.lsc;
    }
    const int nk = kend > kbeg ? (kend - kbeg) / BKT : 0;

    const bool do_cs = EPI == SV_EPI_SLAB && colsum != nullptr && tn == 0;  // compile-time off otherwise
    float csum = 0.f;
    float cs8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // implicit-GEMM rows: the pixel of each of this lane's A rows, decoded once per tile
    int gb[C::A_PER_WAVE], gy[C::A_PER_WAVE], gx[C::A_PER_WAVE];
    if constexpr (CONV > 0) {
      const int lane = threadIdx.x & 63;
#pragma unroll
      for (int j = 0; j < C::A_PER_WAVE; ++j) {
        const int row = ((wid + NW * j) * 1024 + lane * 16) / (BKT * 2);
        const int m = m0 + row;
        gb[j] = -1;
        gy[j] = gx[j] = 0;
        if (m < e.M) {
          const uint32_t b = cg_div((uint32_t)m, cg.ghw_mul, cg.ghw_shift);
          const uint32_t rem = (uint32_t)m - b * (uint32_t)(cg.GH * cg.GW);
          const uint32_t oy = cg_div(rem, cg.gw_mul, cg.gw_shift);
          const uint32_t ox = rem - oy * (uint32_t)cg.GW;
          gb[j] = (int)b * cg.SH;
          gy[j] = (int)oy * cg.si;
          gx[j] = (int)ox * cg.si;
        }
      }
    }
    // weight-gradient gather (CONV 3): this lane's B k-row and (tap, channel) per DMA piece
    int bk[C::B_PER_WAVE], bc[C::B_PER_WAVE], by[C::B_PER_WAVE], bx[C::B_PER_WAVE];
    if constexpr (CONV == 3) {
      const int lane = threadIdx.x & 63;
#pragma unroll
      for (int j = 0; j < C::B_PER_WAVE; ++j) {
        const int byte = (wid + NW * j) * 1024 + lane * 16;
        const int krow = byte / (BN * 2), ch = (byte % (BN * 2)) >> 4;
        const int n = n0 + (ch ^ mswz(krow)) * 8;
        const int t = n >> cg.lsc;
        bk[j] = krow;
        bc[j] = n < e.N ? n & ((1 << cg.lsc) - 1) : -1;
        by[j] = n < e.N ? cg.tdy[t] : 0;
        bx[j] = n < e.N ? cg.tdx[t] : 0;
      }
    }
    // transposed weight-gradient gather (CONV 4, small Cout): A(m = t*SC + c, k = pixel) gathered
    // M-major, this lane's k-row and (tap, channel) per DMA piece; B = dy [pixel][Cout] N-contiguous
    int ak[C::A_PER_WAVE], ac[C::A_PER_WAVE], ay[C::A_PER_WAVE], ax[C::A_PER_WAVE];
    if constexpr (CONV == 4) {
      const int lane = threadIdx.x & 63;
#pragma unroll
      for (int j = 0; j < C::A_PER_WAVE; ++j) {
        const int byte = (wid + NW * j) * 1024 + lane * 16;
        const int krow = byte / (BM * 2), ch = (byte % (BM * 2)) >> 4;
        const int m = m0 + (ch ^ mswz(krow)) * 8;
        const int t = m >> cg.lsc;
        ak[j] = krow;
        ac[j] = m < e.M ? m & ((1 << cg.lsc) - 1) : -1;
        ay[j] = m < e.M ? cg.tdy[t] : 0;
        ax[j] = m < e.M ? cg.tdx[t] : 0;
      }
    }
    auto issue = [&](int kt) {
      char* st = smem + (kt % S) * C::STAGE_BYTES;
      const int k0 = kbeg + kt * BKT;
      if constexpr (CONV == 4) {
        issue_gather_n<BKT, C::A_PER_WAVE>(A, cg, K, k0, ak, ac, ay, ax, st, wid);
        issue_tile<false, BN, BKT, C::B_PER_WAVE>(B, ldb, n0, k0, e.N, st + C::A_BYTES, wid);
      } else if constexpr (CONV == 3) {
        issue_tile<AK, BM, BKT, C::A_PER_WAVE>(A, lda, m0, k0, e.M, st, wid);
        issue_gather_n<BKT, C::B_PER_WAVE>(B, cg, K, k0, bk, bc, by, bx, st + C::A_BYTES, wid);
      } else if constexpr (CONV == 0) {
        issue_tile<AK, BM, BKT, C::A_PER_WAVE>(A, lda, m0, k0, e.M, st, wid);
        issue_tile<BKM, BN, BKT, C::B_PER_WAVE>(B, ldb, n0, k0, e.N, st + C::A_BYTES, wid);
      } else if constexpr (CONV == 6) {
        issue_gather8<BKT, C::A_PER_WAVE>(A, cg, gb, gy, gx, k0, st, wid);
        issue_tile_kclamp<BKT, C::B_PER_WAVE>(B, ldb, n0, k0, e.N, cg.ntaps * 8, st + C::A_BYTES, wid);
      } else {
        const int jt = (CONV == 5 ? (int)cg.ctap0[split] : 0) + (k0 >> cg.lsc);  // wave-uniform tap
        const int cb = k0 & ((1 << cg.lsc) - 1);                                  // and channel base
        issue_gather<BKT, C::A_PER_WAVE>(A, cg, gb, gy, gx, cg.tdy[jt], cg.tdx[jt], cb, st, wid);
        if constexpr (CONV == 1) {
          issue_tile<BKM, BN, BKT, C::B_PER_WAVE>(B, ldb, n0, k0, e.N, st + C::A_BYTES, wid);
        } else {  // dgrad: k = j*Cout + co -> weight rows (co*Tw + twt[j])*Cs, i.e. rows co of stride Tw*Cs
          issue_tile<false, BN, BKT, C::B_PER_WAVE>(B + (size_t)cg.twt[jt] * cg.Cs, (int64_t)cg.Tw * cg.Cs, n0, cb,
                                                    e.N, st + C::A_BYTES, wid);
        }
      }
    };

    __syncthreads();  // the previous tile's epilogue slabs overlap the ring
#pragma unroll
    for (int p = 0; p < S - 1; ++p)
      if (p < nk) issue(p);
    for (int kt = 0; kt < nk; ++kt) {
      // tile kt must have landed; the min(S-2, nk-1-kt) younger tiles may stay in flight
      ring_wait<C::LOADS, S>(nk - 1 - kt);
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
    }
    vm_wait<0>();
    __syncthreads();
    if constexpr (!AK) {
      if (do_cs) csum = colsum_fold(cs8, reinterpret_cast<float*>(smem));  // block-uniform branch
    }
    if (do_cs && threadIdx.x < BM && m0 + (int)threadIdx.x < e.M) colsum[(size_t)split * e.M + m0 + threadIdx.x] = csum;
    // the epilogue operand is bf16 (GELU'(h), pre-activation) or the f32 residual stream
    constexpr int AUXT = AUXO >= 0 ? AUXO
                         : (EPI == SV_EPI_MUL_AUX || EPI == SV_EPI_GELU_GRAD || EPI == SV_EPI_STORE_BN_BWD) ? SV_BF16
                         : EPI == SV_EPI_BIAS_GAMMA_RES ? SV_F32 : -1;
    // mode 5 with a non-slab epilogue: each class's rows go straight to their dx pixels
    constexpr bool REMAP = CONV == 5 && EPI != SV_EPI_SLAB;
    wave_tile_epilogue<4, 2, EPI, AUXT, REMAP>(acc, reinterpret_cast<float*>(smem) + wid * 16 * EPI_LD, m0 + wm * 64,
                                  n0 + wn * 64, e, split);
  }
}

template <bool AK, bool BKM, int EPI, int BKT, int S, int CONV = 0, int AUXO = -1>
static int launch(const sv_gemm_desc* d, int split, hipStream_t s, const ConvG* cg = nullptr) {
  using C = Cfg<BKT, S>;
  // the kernels are specialised for the operand dtype each epilogue carries in the bf16 model
  if ((EPI == SV_EPI_MUL_AUX || EPI == SV_EPI_GELU_GRAD) && d->aux_dtype != SV_BF16) return SV_ERR_UNSUPPORTED;
  if (EPI == SV_EPI_BIAS_GAMMA_RES && d->aux_dtype != (AUXO >= 0 ? AUXO : SV_F32)) return SV_ERR_UNSUPPORTED;
  if (EPI == SV_EPI_STORE_BN_BWD && (d->aux_dtype != SV_BF16 || !d->bn || d->c_dtype != SV_BF16)) return SV_ERR_UNSUPPORTED;
  constexpr int OCC = C::TWO_PER_CU ? 4 : 2;
  const int kper = ceil_div(ceil_div(d->K, split), BKT) * BKT;
  const int tilesM = ceil_div(d->M, BM), tilesN = ceil_div(d->N, BN);
  EpiArgs e{d->M, d->N, d->epilogue, d->C, d->c_dtype, d->ldc, d->C2, d->c2_dtype, d->bias, d->gamma,
            d->aux, d->aux_dtype, d->ld_aux};
  e.prio = d->policy.priority;
  if (EPI == SV_EPI_STORE_BN_BWD) {
    e.bn_mu = d->bn->mean;
    e.bn_rs = d->bn->rstd;
    e.bn_be = d->bn->beta;
    e.gamma = d->bn->gamma;
  }
  if constexpr (CONV == 5 && EPI != SV_EPI_SLAB) {  // rows remapped to dx pixels (even H, W: 2GH x 2GW)
    e.rm_gh = cg->GH;
    e.rm_gw = cg->GW;
    e.rm_gw_mul = cg->gw_mul;
    e.rm_gw_shift = cg->gw_shift;
    e.rm_ghw_mul = cg->ghw_mul;
    e.rm_ghw_shift = cg->ghw_shift;
    e.rm_prow = ceil_div(d->M, 64);
  }
  if (const int rc_ = ensure_lds_attr(reinterpret_cast<const void*>(&gemm3_kernel<AK, BKM, EPI, BKT, S, OCC, CONV, AUXO>), (int)C::LDS, s)) return rc_;
  // one workgroup per tile, which lets kernels of the side stream take CUs as tiles retire
  const int total = tilesM * tilesN * split;
  // (policy.wg_per_cu: co-residency with a concurrent GEMM; policy.grid_cap: persistent over the rest)
  const int grid = policy_grid(&d->policy, total, 0, s);
  gemm3_kernel<AK, BKM, EPI, BKT, S, OCC, CONV, AUXO><<<grid, THREADS, C::LDS, s>>>(
      reinterpret_cast<const uint16_t*>(d->A), d->lda, reinterpret_cast<const uint16_t*>(d->B), d->ldb, d->K, kper,
      tilesM, tilesN, split, e, d->epilogue == SV_EPI_SLAB ? reinterpret_cast<float*>(d->C2) : nullptr,
      cg ? *cg : ConvG{});
  return check_launch("sv_gemm(v3)");
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
    case SV_EPI_STORE_STATS: return launch<AK, BKM, SV_EPI_STORE_STATS, BKT, S>(d, split, s);
    case SV_EPI_STORE_BN_BWD:  // data gradients into a BatchNorm + ReLU (A k-major = dy rows)
      if constexpr (AK && !BKM) return launch<AK, BKM, SV_EPI_STORE_BN_BWD, BKT, S>(d, split, s);
      return SV_ERR_UNSUPPORTED;
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

}  // namespace g3

namespace g3 {
// gathered fprop / dgrad (modes 1, 2, 5) at S ring stages
template <int S>
static int conv_fd(const sv_gemm_desc* d, const ConvG& g, int mode, hipStream_t s) {
  if (mode == 1 && d->epilogue == SV_EPI_STORE) return launch<true, true, SV_EPI_STORE, 32, S, 1>(d, 1, s, &g);
  if (mode == 1 && d->epilogue == SV_EPI_STORE_STATS)
    return launch<true, true, SV_EPI_STORE_STATS, 32, S, 1>(d, 1, s, &g);
  if (mode == 2 && d->epilogue == SV_EPI_STORE) return launch<true, false, SV_EPI_STORE, 32, S, 2>(d, 1, s, &g);
  if (mode == 2 && d->epilogue == SV_EPI_BIAS_GAMMA_RES)  // in-place accumulate into an f32 or a bf16 dx
    return d->aux_dtype == SV_BF16 ? launch<true, false, SV_EPI_BIAS_GAMMA_RES, 32, S, 2, SV_BF16>(d, 1, s, &g)
                                   : launch<true, false, SV_EPI_BIAS_GAMMA_RES, 32, S, 2>(d, 1, s, &g);
  if (mode == 2 && d->epilogue == SV_EPI_STORE_BN_BWD)
    return launch<true, false, SV_EPI_STORE_BN_BWD, 32, S, 2>(d, 1, s, &g);
  // split-K fprop / dgrad for grids below one workgroup per CU: f32 slabs, summed by sv_gemm_slab_finish
  if (mode == 1 && d->epilogue == SV_EPI_SLAB)
    return launch<true, true, SV_EPI_SLAB, 32, S, 1>(d, d->split_k < 1 ? 1 : d->split_k, s, &g);
  if (mode == 2 && d->epilogue == SV_EPI_SLAB)
    return launch<true, false, SV_EPI_SLAB, 32, S, 2>(d, d->split_k < 1 ? 1 : d->split_k, s, &g);
  if (mode == 5 && d->epilogue == SV_EPI_SLAB) return launch<true, false, SV_EPI_SLAB, 32, S, 5>(d, 4, s, &g);
  // mode 5 straight into dx (no split): plain store, in-place accumulate, or with the BatchNorm statistics;
  // split_k = the number of classes launched (classes 0 .. split_k - 1; an accumulate skips trailing classes
  // without taps)
  const int ncls = d->split_k >= 1 && d->split_k <= 4 ? d->split_k : 4;
  if (mode == 5 && d->epilogue == SV_EPI_STORE) return launch<true, false, SV_EPI_STORE, 32, S, 5>(d, ncls, s, &g);
  if (mode == 5 && d->epilogue == SV_EPI_BIAS_GAMMA_RES)
    return d->aux_dtype == SV_BF16 ? launch<true, false, SV_EPI_BIAS_GAMMA_RES, 32, S, 5, SV_BF16>(d, ncls, s, &g)
                                   : launch<true, false, SV_EPI_BIAS_GAMMA_RES, 32, S, 5>(d, ncls, s, &g);
  if (mode == 5 && d->epilogue == SV_EPI_STORE_BN_BWD)
    return launch<true, false, SV_EPI_STORE_BN_BWD, 32, S, 5>(d, 4, s, &g);
  // 8-channel pixels (the ResNet stem), plain store or with the BatchNorm statistics
  if (mode == 6 && d->epilogue == SV_EPI_STORE) return launch<true, true, SV_EPI_STORE, 32, S, 6>(d, 1, s, &g);
  if (mode == 6 && d->epilogue == SV_EPI_STORE_STATS)
    return launch<true, true, SV_EPI_STORE_STATS, 32, S, 6>(d, 1, s, &g);
  return SV_ERR_UNSUPPORTED;
}
// gathered weight gradients (modes 3, 4) at S ring stages
template <int S>
static int conv_w(const sv_gemm_desc* d, const ConvG& g, int mode, hipStream_t s) {
  if (mode == 3 && d->epilogue == SV_EPI_SLAB && !d->a_kmajor && !d->b_kmajor)
    return launch<false, false, SV_EPI_SLAB, 32, S, 3>(d, d->split_k < 1 ? 1 : d->split_k, s, &g);
  if (mode == 4 && d->epilogue == SV_EPI_SLAB && !d->a_kmajor && !d->b_kmajor)
    return launch<false, false, SV_EPI_SLAB, 32, S, 4>(d, d->split_k < 1 ? 1 : d->split_k, s, &g);
  return SV_ERR_UNSUPPORTED;
}
}  // namespace g3

// ring depth of the transposed gather wgrad (mode 4): 4 stages (96 KiB, one workgroup per CU); A/B builds try 3
// (72 KiB, two per CU) with conv.hip's SV_CONVW4_WGS doubled
#ifndef SV_CONVW4_STAGES
#define SV_CONVW4_STAGES 4
#endif
int launch_gemm3_conv(const sv_gemm_desc* d, const ConvG& g, int mode, hipStream_t s) {
  using namespace g3;
  if (d->compute != SV_BF16 || d->a_dtype != SV_BF16 || d->b_dtype != SV_BF16 || d->K % 32 ||
      (mode != 3 && mode != 4 && mode != 6 && g.lsc < 5) || (mode == 6 && (g.lsc != 3 || g.ntaps * 8 > d->K)))
    return SV_ERR_UNSUPPORTED;
  // ring depth: 3 stages (fprop / dgrad, two workgroups per CU) and 4 (wgrads); 6 stages (144 KiB, five
  // tiles in flight) measured no faster for any ResNet-50 conv pass (profiles/round3/r6b_conv_ring_depth.txt)
  if (mode == 4) return conv_w<SV_CONVW4_STAGES>(d, g, mode, s);
  if (mode == 3) return conv_w<4>(d, g, mode, s);
  return conv_fd<3>(d, g, mode, s);
}

int launch_gemm3(const sv_gemm_desc* d, hipStream_t s, const char* cfg) {
  using namespace g3;
  if (d->compute != SV_BF16 || d->a_dtype != SV_BF16 || d->b_dtype != SV_BF16 || d->a_scale_k)
    return SV_ERR_UNSUPPORTED;
  const int split = d->epilogue == SV_EPI_SLAB ? (d->split_k < 1 ? 1 : d->split_k) : 1;
  // BKxSTAGES: 32x3 (default: two workgroups per CU) or 32x4
  if (cfg && !strcmp(cfg, "32x4")) return launch_cfg<32, 4>(d, split, s);
  return launch_cfg<32, 3>(d, split, s);
}

}  // namespace sv
