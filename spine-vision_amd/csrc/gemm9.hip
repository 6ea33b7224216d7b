// MFMA GEMM v9 (bf16 operands, f32 accumulate): persistent 256x256 tiles, BK 64, one 512-thread
// workgroup per CU, 8 waves in 2(M) x 4(N) (128 x 64 per wave = 8 x 4 v_mfma_f32_16x16x32_bf16
// fragments).  What is different from v3/v8:
//
//  * phase-interleaved K loop: a 64-deep K-tile is four phases, each {read a register subtile from
//    LDS, issue part of the LDS-DMA of the K-tile TWO ahead, barrier, 16 MFMAs on one quadrant of the
//    wave tile, barrier}; waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave reads
//    while its partner multiplies;
//  * two LDS buffers (2 x 64 KiB), each refilled region by region as soon as every wave has read it
//    (A rows of quadrant 0 after phase 0, B after phase 1, A rows of quadrant 1 after phase 2): about
//    1.5 K-tiles of DMA in flight, retired by counted `s_waitcnt vmcnt` (never 0 in the loop); an
//    N/M-major A (weight gradients) cannot be refilled by quadrant, so it gets a third buffer;
//  * persistent over the tiles with ONE K-tile stream: the DMA of the next tile's first K-tiles is
//    issued during the current tile's last ones, and the epilogue's stores stay in flight while the
//    next tile starts (the vmcnt counts include them);
//  * register-direct epilogue: the MFMA runs with the operands swapped (D^T = B^T A^T), so a lane
//    holds 4 consecutive OUTPUT COLUMNS of one row; for bf16 outputs the B rows are permuted inside
//    each 32-column group (at DMA time for K-major B, in the fragment address for N-major B) so that
//    a lane holds 8 consecutive columns -> one 16-B buffer store per 8 outputs, no LDS round trip,
//    out-of-range rows/columns dropped by the buffer descriptor's range check (no branches, so every
//    wave issues a fixed number of memory instructions per tile, which the vmcnt counts rely on).
#include "common.h"
#include "gemm_common.h"

#include <stdlib.h>

namespace sv {
namespace g9 {

#ifdef SV_CLOCK_STAMPS
// diagnostic build only (tools/build_stamp.sh, MI355X_MICROARCH.md "DVFS give-back" item 6): per workgroup
// s_memtime / s_memrealtime at the start and the end of the launch, in a buffer of their own that no other
// code reads; the in-kernel clock is d(memtime) / d(memrealtime) x 100 MHz.  Not part of libsv_kernels.so.
__device__ unsigned long long g_stamps[1024][4];
__device__ __forceinline__ void stamp(int slot) {
  const unsigned long long t = __builtin_amdgcn_s_memtime(), r = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0 && blockIdx.x < 1024) {
    volatile unsigned long long* p = g_stamps[blockIdx.x];
    p[2 * slot] = t;
    p[2 * slot + 1] = r;
  }
}
#else
__device__ __forceinline__ void stamp(int) {}
#endif

// wave priority in the K loop: 0 = s_setprio 1 around each MFMA quadrant; 1 = static priority 1 for
// waves 4-7 (the second-dispatched half), no per-segment flips; 2 = none (A/B builds only)
#ifndef SV_G9_PRIO
#define SV_G9_PRIO 0
#endif

constexpr int BM = 256, BN = 256, BK = 64, THREADS = 512, NW = 8;
constexpr int FM = 8, FN = 4;
constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, BUF_BYTES = A_BYTES + B_BYTES;
// LDS: K-major A: two buffers of {A, B} (128 KiB); N/M-major A: A triple-buffered (it is refilled
// only after the last phase that reads it), B double-buffered (160 KiB)
template <bool AK>
constexpr int lds_bytes() { return AK ? 2 * BUF_BYTES : 3 * A_BYTES + 2 * B_BYTES; }
template <bool AK>
__device__ __forceinline__ int a_off(int g) { return AK ? (g & 1) * BUF_BYTES : (g % 3) * A_BYTES; }
template <bool AK>
__device__ __forceinline__ int b_off(int g) { return AK ? (g & 1) * BUF_BYTES + A_BYTES : 3 * A_BYTES + (g & 1) * B_BYTES; }
constexpr uint32_t OOB = 0x80000000u;     // buffer offset past every descriptor's range

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// K-major image [rows][64] bf16 (128-B rows): 16-B chunk c of row r stored at c ^ ((r >> 1) & 7), so
// the 16 rows x one chunk of every ds_read_b128 lane group land on 16 distinct bank slots
__device__ __forceinline__ int kswz(int row) { return (row >> 1) & 7; }
// N/M-major image [64 k][256] bf16 (512-B rows), read with ds_read_b64_tr_b16
__device__ __forceinline__ int mswz(int r) { return ((r & 3) << 1) ^ (((r >> 3) & 1) << 3); }
// bf16-output column permutation inside a 32-row group of B: LDS row 16h + 4g + r holds column
// 8g + 4h + r, so fragment pair (2q, 2q+1) gives lane group g the 8 consecutive columns 32q + 8g ..
__device__ __forceinline__ int perm8(int rho) {
  return (rho & ~31) | (((rho & 15) >> 2) << 3) | (((rho >> 4) & 1) << 2) | (rho & 3);
}

// LDS-DMA by buffer_load ... lds: the per-lane byte offset of each of a wave's pieces is computed
// once per tile (voffset), the K position is the uniform soffset, rows / columns past the matrix get
// an offset past the descriptor's range and land as zeros (their results are never stored)
template <int CPOL = 0>
__device__ __forceinline__ void dma(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, char* dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)dst, 16, voff, soff, 0, CPOL);
}
// A/B switches (tools/build_ab.sh): cache policy of the epilogue's bf16 operand loads (GELU'(h): its last read) and
// of a weight gradient's B operand DMA (the saved activation: its last read).  nt on either measured no better
// (profiles/round4/r8h_nt_loads_rejected.txt: the wgrad's B panel is re-read by every M tile of its K slice)
#ifndef SV_G9_AUXBF_CPOL
#define SV_G9_AUXBF_CPOL 0
#endif
#ifndef SV_G9_SLAB_B_CPOL
#define SV_G9_SLAB_B_CPOL 0
#endif
// A wave's DMA pieces of one operand differ only by whole rows (K-major: 64 rows; N/M-major: 16 k-rows)
// and the source swizzle does not depend on the piece, so each operand needs ONE per-lane byte offset
// (per tile) plus a uniform piece offset in soffset.  Rows / columns past the matrix read past the
// descriptor's range (zeros) or garbage that only reaches outputs that are never stored.
// K-major: piece wid + 8j covers rows 64j + 8wid + lane/8, 16-B chunk lane%8 (swizzled)
template <bool PERM>
__device__ __forceinline__ uint32_t vbase_k(int64_t ld, int row0, int wid) {
  const int lane = threadIdx.x & 63;
  const int row = 8 * wid + (lane >> 3), ch = lane & 7;
  return (uint32_t)(((int64_t)(row0 + (PERM ? perm8(row) : row)) * ld + ((ch ^ kswz(row)) << 3)) * 2);
}
// N/M-major: piece wid + 8j covers k-rows 16j + 2wid + lane/32, 16-B chunk lane%32 (swizzled)
__device__ __forceinline__ uint32_t vbase_m(int64_t ld, int col0, int wid) {
  const int lane = threadIdx.x & 63;
  const int krow = 2 * wid + (lane >> 5), ch = lane & 31;
  return (uint32_t)(((int64_t)krow * ld + col0 + ((ch ^ mswz(krow)) << 3)) * 2);
}

// fragment: lane l holds X[row = base + (l & 15)][k = 32 kh + 8 (l >> 4) + 0..7]
__device__ __forceinline__ bf16x8 frag_k(const char* __restrict__ region, int base, int kh) {
  const int l = threadIdx.x & 63;
  const int row = base + (l & 15), ch = kh * 4 + (l >> 4);
  return *reinterpret_cast<const bf16x8*>(region + row * 128 + ((ch ^ kswz(row)) << 4));
}
// N/M-major fragment through the transposing read; lanes p = l & 3 fetch the 4-column run that
// becomes fragment rows 4p .. 4p+3: run start chunk `ch(p)` and half `hf(p)`
__device__ __forceinline__ bf16x8 frag_tr(const char* __restrict__ region, int ch, int hf, int kh) {
  const int l = threadIdx.x & 63;
  const int g = l >> 4, q = (l >> 2) & 3;
  const int r0 = kh * 32 + 8 * g + q, r1 = r0 + 4;
  const char* a0 = region + r0 * 512 + ((ch ^ mswz(r0)) << 4) + hf * 8;
  const char* a1 = region + r1 * 512 + ((ch ^ mswz(r1)) << 4) + hf * 8;
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a0);
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)a1);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// natural 16-row fragment at `base` (runs base + 4p)
__device__ __forceinline__ bf16x8 frag_m(const char* __restrict__ region, int base, int kh) {
  const int p = threadIdx.x & 3;
  return frag_tr(region, (base >> 3) + (p >> 1), p & 1, kh);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

struct Geo {
  int m0, n0, kbeg, split;
};

// descriptor extents (bytes) of the epilogue's buffers; a byte offset >= extent is dropped / reads 0
struct Ext {
  uint32_t c, c2, aux, a, b;
};

// in-kernel split-K fold (SV_EPI_SLAB with sv_gemm_desc.fold_out), write-through (sc1) slab stores and sc1 loads --
// the hand-off of MI355X_MICROARCH.md's inter-workgroup table, row 1 (every storing wave vmcnt(0), a workgroup
// barrier, ONE agent-scope atomic add per workgroup).  Two forms, two int32 counters per tile (arrivals,
// departures), zero between launches:
//   kFoldLast   the workgroup whose add returns split - 1 sums the whole tile.  No workgroup waits for another,
//               so any grid, cap or co-scheduling is deadlock-free; but one CU then streams split x 256 KiB
//               (round 4: the one-CU tail cost the step 1-6 %).
//   kFoldSpread every workgroup of the tile polls the arrival counter (sc1 loads) until all split slices have
//               landed, then sums its own 1/split of the tile's rows; the last to leave re-arms both counters.
//               Needs every slice of a tile resident at once: the host picks it only when the grid holds every
//               (tile, slice) unit, one per workgroup, within the chip's CUs.
struct Fold {
  float* out;
  int64_t ld;
  int acc;
  int* cnt;
};
constexpr int kFoldNone = 0, kFoldLast = 1, kFoldSpread = 2;
constexpr int kSC1 = 16;  // buffer instruction cache policy: sc1 (write-through store / L1-bypassing load)
// cache policy of the GELU'(h) store of the dual epilogue: nt (2).  That tensor is read only by the backward,
// ~20 ms and tens of GB of traffic later, so keeping its lines in L2 / the Infinity Cache only evicts the GELU(h)
// the next GEMM reads at once: step 1072.9-1073.7 -> 1083.4-1084.2 img/s interleaved (profiles/round4/
// r8g_gelu_grad_nt_ab.txt).  -DSV_G9_GRAD_CPOL=0 restores the default policy (tools/build_ab.sh)
#ifndef SV_G9_GRAD_CPOL
#define SV_G9_GRAD_CPOL 2
#endif
// ... and of its GELU(h) store (C2, read by the fc2 forward at once and the fc2 weight gradient in the backward);
// A/B builds only (-DSV_G9_C2_CPOL=2: nt)
// GELU epilogues two elements at a time in packed f32 (bitwise the scalar form; -DSV_GELU_PK=0: scalar, A/B)
#ifndef SV_GELU_PK
#define SV_GELU_PK 1
#endif
#ifndef SV_G9_C2_CPOL
#define SV_G9_C2_CPOL 0
#endif

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  // built from kernel arguments only: wave-uniform, so no waterfall loop around the buffer ops
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// LDS read the compiler does not see: its alias analysis would otherwise drain every LDS-DMA in flight
// (vmcnt(0)) before an LDS read it cannot prove disjoint from them; the data is ordered by the K
// loop's own waits and barriers
__device__ __forceinline__ float4 lds_f4(const float* p) {
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t v;
  const uint32_t a = (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p);
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
  return make_float4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ u32x4 pack8(const float (&v)[8]) {
  return u32x4{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
}

// vector-memory instructions one wave issues in an epilogue (all unconditional): the vmcnt counts of
// the K loop's waits include them when an epilogue lies between a DMA and its wait
template <int EPI, bool P8>
struct EpiCount {
  static constexpr int CH = P8 ? 2 : 4;  // column chunks per 16-row group
  static constexpr int OUTS = (EPI == SV_EPI_BIAS_GELU_DUAL) ? 2 : 1;
  static constexpr int AUX = (EPI == SV_EPI_MUL_AUX || EPI == SV_EPI_GELU_GRAD) ? CH
                             : EPI == SV_EPI_BIAS_GAMMA_RES ? (P8 ? 2 * CH : CH)
                                                            : 0;
#ifdef SV_DIAG_NOSTORE
  static constexpr int E = 0;  // diagnostic build: the epilogue issues no memory instruction
#else
  static constexpr int E = FM * (CH * OUTS + AUX);
#endif
};

// Epilogue of one wave tile: rows m_w + 16 i + (l & 15), columns per chunk c:
//   P8: n_w + 32c + 8(l >> 4) .. +7  (acc[i][2c][0..3], acc[i][2c+1][0..3]),
//   P4: n_w + 16c + 4(l >> 4) .. +3  (acc[i][c][0..3]).
// Arithmetic identical to wave_group_epilogue (gemm_common.h).
template <int EPI, bool P8, bool AK, int FOLD = kFoldNone>
__device__ __forceinline__ void epilogue(const f32x4 (&acc)[FM][FN], const EpiArgs& e, const Ext& x, int m_w, int n_w,
                                         int split, const float* lbias) {
#ifdef SV_DIAG_NOSTORE
  // diagnostic build (tools/build_diag.sh): the K loop alone -- keep the accumulators live, store nothing
  float sink = 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) sink += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  asm volatile("" ::"v"(sink));
  return;
#endif
  // lbias: the tile's bias[256] and gamma[256] staged in LDS (K loop, first K-tile), or nullptr
  constexpr int CH = P8 ? 2 : 4, CW = P8 ? 8 : 4;
  const int l = threadIdx.x & 63, ml = l & 15, gq = l >> 4;
  int n[CH];
  bool okn[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    n[c] = n_w + (P8 ? 32 * c + 8 * gq : 16 * c + 4 * gq);
    okn[c] = n[c] < e.N;
  }
  const bool slab = EPI == SV_EPI_SLAB;
  const bool has_bias = !slab && EPI != SV_EPI_GELU_GRAD && EPI != SV_EPI_MUL_AUX;
  float bias[CH][CW], gam[CH][CW];
#pragma unroll
  for (int c = 0; c < CH; ++c)
#pragma unroll
    for (int w = 0; w < CW; ++w) bias[c][w] = 0.f, gam[c][w] = 1.f;
  const int wcol = n_w & 255;  // the wave's first column inside the tile
  auto ld_vec = [&](const float* g, int lo, int c, float (&dst)[CH][CW]) {
#pragma unroll
    for (int w = 0; w < CW; w += 4) {
      float4 b;
      if (lbias) b = lds_f4(lbias + lo + wcol + (n[c] - n_w) + w);
      else b = okn[c] ? *reinterpret_cast<const float4*>(g + n[c] + w) : make_float4(0.f, 0.f, 0.f, 0.f);
      dst[c][w] = b.x, dst[c][w + 1] = b.y, dst[c][w + 2] = b.z, dst[c][w + 3] = b.w;
    }
  };
  if (has_bias && e.bias) {
#pragma unroll
    for (int c = 0; c < CH; ++c) ld_vec(e.bias, 0, c, bias);
  }
  if (EPI == SV_EPI_BIAS_GAMMA_RES && e.gamma) {
#pragma unroll
    for (int c = 0; c < CH; ++c) ld_vec(e.gamma, 256, c, gam);
  }
  const int64_t ldc = slab ? e.N : e.ldc;
  const char* cbase = reinterpret_cast<const char*>(e.C);
  if (slab) cbase += (size_t)split * e.M * e.N * (P8 ? 2 : 4);  // f32 slabs, or bf16 (P8)
  const auto rc = rsrc(cbase, x.c);
  const auto rc2 = rsrc(e.C2 ? e.C2 : e.C, x.c2);
  constexpr int CS = P8 ? 2 : 4;  // output element bytes: P8 <=> bf16 outputs (bf16 slabs included)
  constexpr bool AUXBF = EPI == SV_EPI_MUL_AUX || EPI == SV_EPI_GELU_GRAD;
  constexpr bool AUXF = EPI == SV_EPI_BIAS_GAMMA_RES;
  const auto ra = rsrc(e.aux ? e.aux : e.C, x.aux);
  // epilogue operands of HALF row groups at a time: the bf16 operand in ONE batch per tile (64 VGPRs), the f32
  // residual in two (64); the K loop's fragment registers are dead by then (212-251 VGPRs, no scratch).  Round 3:
  // step 1048 -> 1055-1056 img/s interleaved against two / four batches (-DSV_G9_AUXB=0, 32 VGPRs per batch;
  // standalone shapes within noise, profiles/round3/r5e_g9_aux_batch.txt)
#ifndef SV_G9_AUXB
#define SV_G9_AUXB 1
#endif
  constexpr int HALF = AUXF ? (SV_G9_AUXB && AK ? FM / 2 : FM / 4) : (AUXBF && SV_G9_AUXB ? FM : FM / 2);
  // SV_EPI_STORE_STATS: per-lane column sums of one 64-row group (4 row groups = one HALF batch)
  constexpr bool kStats = EPI == SV_EPI_STORE_STATS;
  static_assert(!kStats || (P8 && HALF == 4), "statistics need bf16 output and 64-row batches");
  float st1[kStats ? CH : 1][kStats ? 8 : 1], st2[kStats ? CH : 1][kStats ? 8 : 1];
#pragma unroll
  for (int hb = 0; hb < FM / HALF; ++hb) {
    if constexpr (kStats) {
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int w = 0; w < 8; ++w) st1[c][w] = st2[c][w] = 0.f;
    }
    u32x4 raw[HALF][CH][AUXF && P8 ? 2 : 1];
    if constexpr (AUXBF || AUXF) {
#pragma unroll
      for (int ii = 0; ii < HALF; ++ii) {
        const int m = m_w + 16 * (hb * HALF + ii) + ml;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
          const uint32_t base = okn[c] && m < e.M ? (uint32_t)((m * e.ld_aux + n[c]) * (AUXF ? 4 : 2)) : OOB;
          if constexpr (AUXBF && P8) {
            raw[ii][c][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, base, 0, SV_G9_AUXBF_CPOL);
          } else if constexpr (AUXBF) {
            const u32x2 t = __builtin_amdgcn_raw_buffer_load_b64(ra, base, 0, SV_G9_AUXBF_CPOL);
            raw[ii][c][0] = u32x4{t.x, t.y, 0u, 0u};
          } else if constexpr (P8) {
            raw[ii][c][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, base, 0, 0);
            raw[ii][c][AUXF && P8 ? 1 : 0] = __builtin_amdgcn_raw_buffer_load_b128(ra, base + 16, 0, 0);
          } else {
            raw[ii][c][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, base, 0, 0);
          }
        }
      }
    }
#pragma unroll
    for (int ii = 0; ii < HALF; ++ii) {
      const int i = hb * HALF + ii;
      const int m = m_w + 16 * i + ml;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        float v[CW];
        if constexpr (P8) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = acc[i][2 * c][r], v[4 + r] = acc[i][2 * c + 1][r];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = acc[i][c][r];
        }
        const uint32_t off = okn[c] && m < e.M ? (uint32_t)((m * ldc + n[c]) * CS) : OOB;
        float o[CW], o2[CW];
        if (!slab) {
#pragma unroll
          for (int w = 0; w < CW; ++w) v[w] += bias[c][w];
        }
        float xa[CW];
        if constexpr (AUXBF) {
          const uint32_t wd[4] = {raw[ii][c][0].x, raw[ii][c][0].y, raw[ii][c][0].z, raw[ii][c][0].w};
#pragma unroll
          for (int w = 0; w < CW; w += 2) {
            xa[w] = __uint_as_float(wd[w >> 1] << 16);
            xa[w + 1] = __uint_as_float(wd[w >> 1] & 0xffff0000u);
          }
        } else if constexpr (AUXF) {
#pragma unroll
          for (int w = 0; w < CW; ++w) {
            const u32x4 t = raw[ii][c][w >> 2];
            const uint32_t wd = (w & 3) == 0 ? t.x : (w & 3) == 1 ? t.y : (w & 3) == 2 ? t.z : t.w;
            xa[w] = __uint_as_float(wd);
          }
        }
#if SV_GELU_PK
        if constexpr (EPI == SV_EPI_BIAS_GELU_DUAL || EPI == SV_EPI_BIAS_GELU) {  // pairs in packed f32
#pragma unroll
          for (int w = 0; w < CW; w += 2) {
            const gelu_f2 h = {v[w], v[w + 1]};
            gelu_f2 ph, de;
            gelu_parts2(h, ph, de);
            const gelu_f2 g = h * ph;
            if constexpr (EPI == SV_EPI_BIAS_GELU_DUAL) {
              const gelu_f2 dg = __builtin_elementwise_fma(h, de, ph);
              o[w] = dg.x, o[w + 1] = dg.y, o2[w] = g.x, o2[w + 1] = g.y;  // C = GELU'(h), C2 = GELU(h)
            } else {
              o[w] = g.x, o[w + 1] = g.y;
            }
          }
        } else
#endif
#pragma unroll
        for (int w = 0; w < CW; ++w) {
          if constexpr (EPI == SV_EPI_SLAB || EPI == SV_EPI_STORE || EPI == SV_EPI_STORE_STATS) {
            o[w] = v[w];
          } else if constexpr (EPI == SV_EPI_BIAS_GELU_DUAL) {
            gelu_and_grad(v[w], o2[w], o[w]);  // C = GELU'(h), C2 = GELU(h)
          } else if constexpr (EPI == SV_EPI_BIAS_GELU) {
            o[w] = gelu_f(v[w]);
          } else if constexpr (EPI == SV_EPI_MUL_AUX) {
            o[w] = v[w] * xa[w];
          } else if constexpr (EPI == SV_EPI_GELU_GRAD) {
            o[w] = v[w] * gelu_grad_f(xa[w]);
          } else {  // SV_EPI_BIAS_GAMMA_RES
            o[w] = fmaf(gam[c][w], v[w], xa[w]);
          }
        }
        if constexpr (P8) {
          const u32x4 pk = pack8(o);
          __builtin_amdgcn_raw_buffer_store_b128(pk, rc, off, 0,
                                                 EPI == SV_EPI_BIAS_GELU_DUAL ? SV_G9_GRAD_CPOL : 0);
          if constexpr (EPI == SV_EPI_BIAS_GELU_DUAL) __builtin_amdgcn_raw_buffer_store_b128(pack8(o2), rc2, off, 0, SV_G9_C2_CPOL);
          if constexpr (EPI == SV_EPI_STORE_STATS) {
            // statistics of the values AS STORED (bf16), rows past M excluded
            if (m < e.M) {
              const uint32_t wd[4] = {pk.x, pk.y, pk.z, pk.w};
#pragma unroll
              for (int w = 0; w < 8; ++w) {
                const float q = __uint_as_float((w & 1) ? (wd[w >> 1] & 0xffff0000u) : (wd[w >> 1] << 16));
                st1[c][w] += q;
                st2[c][w] = fmaf(q, q, st2[c][w]);
              }
            }
          }
        } else {
          const u32x4 d = {__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]), __float_as_uint(o[3])};
          __builtin_amdgcn_raw_buffer_store_b128(d, rc, off, 0, FOLD ? kSC1 : 0);  // fold: write-through slab
          if constexpr (EPI == SV_EPI_BIAS_GELU_DUAL) {
            const u32x4 d2 = {__float_as_uint(o2[0]), __float_as_uint(o2[1]), __float_as_uint(o2[2]),
                              __float_as_uint(o2[3])};
            __builtin_amdgcn_raw_buffer_store_b128(d2, rc2, off, 0, 0);
          }
        }
      }
    }
    if constexpr (kStats) {
      // the 16 lanes l & 15 hold the group's 64 rows 4 at a time: fold them (fixed order), then lane
      // group gq writes its 8 columns of the group's partial row [mb / 64][2][N] (one writer each)
      const int mb = m_w + 64 * hb;
#pragma unroll
      for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int w = 0; w < 8; ++w) {
#if SV_STATS_XLANE
          // the same partners from the cross-lane unit (bitwise the shuffle form): xor 1 / 2 / 8 exact, xor 4 through
          // the half-row mirror once the quads are uniform
          st1[c][w] += xlane_xor<1>(st1[c][w]);
          st2[c][w] += xlane_xor<1>(st2[c][w]);
          st1[c][w] += xlane_xor<2>(st1[c][w]);
          st2[c][w] += xlane_xor<2>(st2[c][w]);
          st1[c][w] += xlane_xor<4, true>(st1[c][w]);
          st2[c][w] += xlane_xor<4, true>(st2[c][w]);
          st1[c][w] += xlane_xor<8>(st1[c][w]);
          st2[c][w] += xlane_xor<8>(st2[c][w]);
#else
#pragma unroll
          for (int off = 1; off < 16; off <<= 1) {
            st1[c][w] += __shfl_xor(st1[c][w], off);
            st2[c][w] += __shfl_xor(st2[c][w], off);
          }
#endif
        }
      if (ml == 0 && mb < e.M) {
        float* P = reinterpret_cast<float*>(e.C2) + (size_t)(mb >> 6) * 2 * e.N;
#pragma unroll
        for (int c = 0; c < CH; ++c)
          if (okn[c]) {
            *reinterpret_cast<float4*>(P + n[c]) = make_float4(st1[c][0], st1[c][1], st1[c][2], st1[c][3]);
            *reinterpret_cast<float4*>(P + n[c] + 4) = make_float4(st1[c][4], st1[c][5], st1[c][6], st1[c][7]);
            *reinterpret_cast<float4*>(P + e.N + n[c]) = make_float4(st2[c][0], st2[c][1], st2[c][2], st2[c][3]);
            *reinterpret_cast<float4*>(P + e.N + n[c] + 4) = make_float4(st2[c][4], st2[c][5], st2[c][6], st2[c][7]);
          }
      }
    }
  }
}

// The last-arriving workgroup's fold of tile (m0, n0): out[m][n] = (acc ? out : 0) + sum_s slab_s[m][n], the
// slices added in order s = 0, 1, ... exactly as sv_reduce_partials' wide body (bitwise its result).  Every
// lane owns whole 16-B column chunks; FB chunks at a time, each with its 8 slice loads in flight (sc1: the
// slabs of other XCDs were written through and are read past this CU's L1).
template <int FB>
__device__ __forceinline__ void fold_tile(const EpiArgs& e, const Ext& x, const Fold& f, int m0, int n0, int nsplit,
                                          int r_lo = 0, int r_hi = BM) {
  // a spread slice's range may run past the tile when nsplit does not divide BM: never fold the next tile's rows
  if (r_hi > BM) r_hi = BM;
  if (e.M - m0 < r_hi) r_hi = e.M - m0;
  m0 += r_lo;
  const int rows = r_hi - r_lo;
  if (rows <= 0) return;
  const int c4 = (e.N - n0 < BN ? e.N - n0 : BN) / 4;
  const auto rs = rsrc(e.C, (uint32_t)((size_t)nsplit * e.M * e.N * 4 > 0x7fffffffu ? 0x7fffffffu
                                                                                    : (size_t)nsplit * e.M * e.N * 4));
  const uint32_t sstride = (uint32_t)((size_t)e.M * e.N * 4);
  const int nq = rows * 64;
  for (int q0 = threadIdx.x; q0 < nq; q0 += THREADS * FB) {
    float4 acc[FB];
    uint32_t off[FB];
    bool ok[FB];
#pragma unroll
    for (int b = 0; b < FB; ++b) {
      const int q = q0 + b * THREADS, r = q >> 6, c = q & 63;
      ok[b] = q < nq && c < c4;
      off[b] = ok[b] ? (uint32_t)(((size_t)(m0 + r) * e.N + n0 + 4 * c) * 4) : OOB;
      acc[b] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    int sl = 0;
    for (; sl + 8 <= nsplit; sl += 8) {
      u32x4 v[FB][8];
#pragma unroll
      for (int b = 0; b < FB; ++b)
#pragma unroll
        for (int u = 0; u < 8; ++u)
          v[b][u] = __builtin_amdgcn_raw_buffer_load_b128(rs, off[b], (sl + u) * sstride, kSC1);
#pragma unroll
      for (int b = 0; b < FB; ++b)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          acc[b].x += __uint_as_float(v[b][u].x); acc[b].y += __uint_as_float(v[b][u].y);
          acc[b].z += __uint_as_float(v[b][u].z); acc[b].w += __uint_as_float(v[b][u].w);
        }
    }
    for (; sl < nsplit; ++sl) {
#pragma unroll
      for (int b = 0; b < FB; ++b) {
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, off[b], sl * sstride, kSC1);
        acc[b].x += __uint_as_float(v.x); acc[b].y += __uint_as_float(v.y);
        acc[b].z += __uint_as_float(v.z); acc[b].w += __uint_as_float(v.w);
      }
    }
#pragma unroll
    for (int b = 0; b < FB; ++b) {
      if (!ok[b]) continue;
      const int q = q0 + b * THREADS, r = q >> 6, c = q & 63;
      float4* o = reinterpret_cast<float4*>(f.out + (size_t)(m0 + r) * f.ld + n0 + 4 * c);
      float4 a = acc[b];
      if (f.acc) {
        const float4 p = *o;
        a.x += p.x; a.y += p.y; a.z += p.z; a.w += p.w;
      }
      *o = a;
    }
  }
  (void)x;
}

// ---- SV_EPI_LN_BWD (round 6): the LayerNorm backward in the fc1 data gradient's epilogue.  The
// unfused block stores dy = bf16(dh W1) and sv_layernorm_bwd reads it back with z / mean / rstd; here dy stays in the
// accumulators.  Its row sums (sum dy w, sum dy w x^) span all N columns while a 256x256 tile holds a quarter / half of
// a row: every wave sums its 64 columns (lane groups by shuffles), the 4 column waves of the tile through LDS (fixed
// order), and the tiles of one 256-row block through a global workspace -- each stores its 256 partial row sums
// write-through (sc1), every storing wave waits for its stores, one lane adds to the block's arrival counter and polls
// it (sc1 loads) until all N / 256 tiles have arrived (MI355X_MICROARCH.md inter-workgroup table, row 1); every tile
// then adds the N / 256 partials in tile order, so the tiles of a row use the same sums bit for bit.  The last tile out
// re-arms both counters.  The host takes this form only when every tile has a workgroup of its own, all resident at
// once (grid == tiles <= the stream's CUs): a tile waits only for its row-block partners.  A poll that outlasts ~2^26
// sleeps gives up and poisons its rows (NaN dz) instead of hanging the chip.
constexpr int kLnRed = 2 * 4 * 128 * 2 * 4;  // LDS: [wm][wn][128 rows][s1, s2] f32 = 8 KiB

__device__ __forceinline__ void ln_bwd_epilogue(const f32x4 (&acc)[FM][FN], const EpiArgs& e, const Ext& x,
                                                const Fold& f, int m0, int n0, int tilesN, const float* lw_lds,
                                                float* lred, char* dyl) {
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wm = wid >> 2, wn = wid & 3;
  const int l = threadIdx.x & 63, ml = l & 15, gq = l >> 4;
  const int m_w = m0 + 128 * wm, n_w = n0 + 64 * wn;
  constexpr int CH = 2;  // 32-column chunks of the wave; lane group gq: columns n_w + 32 c + 8 gq .. + 7
  const float invC = 1.0f / (float)e.N;
  auto lw_of = [&](int c, float (&lw)[8]) {  // this lane's 8 LayerNorm weights of chunk c (staged in LDS)
    const float4 a = lds_f4(lw_lds + 64 * wn + 32 * c + 8 * gq), b = lds_f4(lw_lds + 64 * wn + 32 * c + 8 * gq + 4);
    lw[0] = a.x, lw[1] = a.y, lw[2] = a.z, lw[3] = a.w, lw[4] = b.x, lw[5] = b.y, lw[6] = b.z, lw[7] = b.w;
  };
  const auto rz = rsrc(e.aux, x.aux);
  const auto rmu = rsrc(e.bn_mu, (uint32_t)e.M * 4), rrs = rsrc(e.bn_rs, (uint32_t)e.M * 4);
  float mu[FM], rs[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int m = m_w + 16 * i + ml;
    const uint32_t o = m < e.M ? (uint32_t)m * 4 : OOB;
    mu[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rmu, o, 0, 0));
    rs[i] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rrs, o, 0, 0));
  }
  // dy = bf16(acc) (the unfused path's stored dy) parks in the K loop's LDS buffers between the passes, so the 128
  // accumulators are dead during the exchange: a lane's 16 B per (row fragment, chunk), lane-linear (conflict-free)
  vm_wait<0>();  // the K loop's DMAs past the end of its stream have landed in those buffers ...
  bar();         // ... in every wave
  auto dy_slot = [&](int i, int c) { return dyl + (((wid * FM + i) * 2 + c) * 64 + l) * 16; };
  auto unpack = [](const u32x4& pk, float (&d)[8]) {
    const uint32_t wd[4] = {pk.x, pk.y, pk.z, pk.w};
#pragma unroll
    for (int w = 0; w < 8; ++w) d[w] = __uint_as_float((w & 1) ? (wd[w >> 1] & 0xffff0000u) : (wd[w >> 1] << 16));
  };
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float v[8];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][2 * c][r], v[4 + r] = acc[i][2 * c + 1][r];
      *reinterpret_cast<u32x4*>(dy_slot(i, c)) = pack8(v);
    }
  asm volatile("" ::: "memory");  // the accumulators are dead from here on
  auto dy_back = [&](int i, int c, float (&d)[8]) { unpack(*reinterpret_cast<const u32x4*>(dy_slot(i, c)), d); };
  auto z_of = [&](const u32x4& raw, int i, float (&xh)[8]) {
    const uint32_t wd[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      const float zz = __uint_as_float((w & 1) ? (wd[w >> 1] & 0xffff0000u) : (wd[w >> 1] << 16));
      xh[w] = (zz - mu[i]) * rs[i];
    }
  };
  auto zoff = [&](int i, int c) {
    const int m = m_w + 16 * i + ml, n = n_w + 32 * c + 8 * gq;
    return m < e.M ? (uint32_t)(((size_t)m * e.ld_aux + n) * 2) : OOB;
  };
  // pass 1, one 32-column chunk at a time (registers: the 128 accumulators stay live throughout): per-row partials
  // over this lane's columns; per-column partials over the wave's 128 rows (16 lanes ml by shuffles, then lane ml == 0
  // stores them into [2][ceil(M / 128)][N])
  const int P = (e.M + 127) / 128, prow = m_w / 128;
  float s1[FM], s2[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) s1[i] = s2[i] = 0.f;
#pragma nounroll
  for (int c = 0; c < CH; ++c) {  // a loop, not unrolled: both chunks' state at once would spill
    float lw[8], pw[8], pb[8];
    lw_of(c, lw);
#pragma unroll
    for (int w = 0; w < 8; ++w) pw[w] = pb[w] = 0.f;
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      asm volatile("" ::: "memory");  // one batch of z loads at a time (hoisting them all would spill)
      u32x4 zr[FM / 2];
#pragma unroll
      for (int ii = 0; ii < FM / 2; ++ii) zr[ii] = __builtin_amdgcn_raw_buffer_load_b128(rz, zoff(hb * FM / 2 + ii, c), 0, 0);
#pragma unroll
      for (int ii = 0; ii < FM / 2; ++ii) {
        const int i = hb * FM / 2 + ii;
        float d[8], xh[8];
        dy_back(i, c, d);
        z_of(zr[ii], i, xh);
#pragma unroll
        for (int w = 0; w < 8; ++w) {
          const float g = d[w] * lw[w];
          s1[i] += g;
          s2[i] += g * xh[w];
          pw[w] += d[w] * xh[w];
          pb[w] += d[w];
        }
      }
    }
#pragma unroll
    for (int w = 0; w < 8; ++w)
#pragma unroll
      for (int sh = 1; sh < 16; sh <<= 1) {
        pw[w] += __shfl_xor(pw[w], sh);
        pb[w] += __shfl_xor(pb[w], sh);
      }
    if (ml == 0 && m_w < e.M) {
      float* C2 = reinterpret_cast<float*>(e.C2);
      const int n = n_w + 32 * c + 8 * gq;
      float4* qw = reinterpret_cast<float4*>(C2 + ((size_t)prow) * e.N + n);
      float4* qb = reinterpret_cast<float4*>(C2 + ((size_t)P + prow) * e.N + n);
      qw[0] = make_float4(pw[0], pw[1], pw[2], pw[3]);
      qw[1] = make_float4(pw[4], pw[5], pw[6], pw[7]);
      qb[0] = make_float4(pb[0], pb[1], pb[2], pb[3]);
      qb[1] = make_float4(pb[4], pb[5], pb[6], pb[7]);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  // the wave's 64 columns of a row: the 4 lane groups (xor 16, 32)
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    s1[i] += __shfl_xor(s1[i], 16);
    s1[i] += __shfl_xor(s1[i], 32);
    s2[i] += __shfl_xor(s2[i], 16);
    s2[i] += __shfl_xor(s2[i], 32);
  }
  // the tile's 4 column waves through LDS (fixed order wn = 0..3)
  if (gq == 0) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      float* q = lred + ((wm * 4 + wn) * 128 + 16 * i + ml) * 2;
      q[0] = s1[i], q[1] = s2[i];
    }
  }
  lgkm0();
  bar();
  // the tile's partial row sums -> the workspace, by the wn == 0 wave of each row half (write-through)
  const int tile_m = m0 / BM, half = n0 / BN;
  const uint32_t xbytes = (uint32_t)(((size_t)((e.M + BM - 1) / BM) * tilesN * BM * 2) * 4);
  const auto rx = rsrc(f.out, xbytes);
  auto xoff = [&](int h, int row) { return (uint32_t)((((size_t)tile_m * tilesN + h) * BM + row) * 8); };
  if (wn == 0 && gq == 0) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = 16 * i + ml;
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w4 = 0; w4 < 4; ++w4) {
        const float* q = lred + ((wm * 4 + w4) * 128 + row) * 2;
        t1 += q[0];
        t2 += q[1];
      }
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(t1), __float_as_uint(t2)}, rx,
                                            xoff(half, 128 * wm + row), 0, kSC1);
    }
  }
  vm_wait<0>();  // every storing wave's stores complete before the workgroup's arrival
  bar();
  int* arrive = f.cnt + 2 * tile_m;
  int* depart = arrive + 1;
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    for (int spin = 0; __hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < tilesN; ++spin) {
      if (spin > (1 << 26)) {  // a partner never arrived: give up rather than hang the chip
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    s_ok = ok;
  }
  bar();
  const bool ok = s_ok != 0;
  // the row's sums: every tile's partial in tile order (the same additions in every tile of the row block)
  float S1[FM], S2[FM];
#pragma unroll
  for (int i = 0; i < FM; ++i) S1[i] = S2[i] = 0.f;
  for (int h = 0; h < tilesN; ++h) {
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rx, xoff(h, 128 * wm + 16 * i + ml), 0, kSC1);
      S1[i] += __uint_as_float(v.x);
      S2[i] += __uint_as_float(v.y);
    }
  }
  vm_wait<0>();
  bar();
  if (threadIdx.x == 0 && __hip_atomic_fetch_add(depart, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == tilesN - 1) {
    __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(depart, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // pass 2: dz = rstd (dy w - s1 / N - x^ s2 / N)  (sv_layernorm_bwd's arithmetic), stored bf16
  const auto rc = rsrc(e.C, x.c);
#pragma unroll
  for (int hb = 0; hb < 2; ++hb) {
    asm volatile("" ::: "memory");
    u32x4 zr[FM / 2][CH];
#pragma unroll
    for (int ii = 0; ii < FM / 2; ++ii)
#pragma unroll
      for (int c = 0; c < CH; ++c) zr[ii][c] = __builtin_amdgcn_raw_buffer_load_b128(rz, zoff(hb * FM / 2 + ii, c), 0, 0);
#pragma unroll
    for (int ii = 0; ii < FM / 2; ++ii) {
      const int i = hb * FM / 2 + ii;
      const int m = m_w + 16 * i + ml;
      const float a1 = ok ? S1[i] * invC : __builtin_nanf(""), a2 = S2[i] * invC;
#pragma unroll
      for (int c = 0; c < CH; ++c) {
        float d[8], xh[8], o[8], lw[8];
        lw_of(c, lw);
        dy_back(i, c, d);
        z_of(zr[ii][c], i, xh);
#pragma unroll
        for (int w = 0; w < 8; ++w) o[w] = rs[i] * (d[w] * lw[w] - a1 - xh[w] * a2);
        const int n = n_w + 32 * c + 8 * gq;
        const uint32_t off = m < e.M ? (uint32_t)(((size_t)m * e.ldc + n) * 2) : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(pack8(o), rc, off, 0, 0);
      }
    }
  }
  vm_wait<0>();
}

template <bool AK, bool BKM, int EPI, bool P8, int FOLD = kFoldNone>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(2, 2)))
gemm9_kernel(const uint16_t* __restrict__ A, int64_t lda, const uint16_t* __restrict__ B, int64_t ldb, int nk, int tilesM,
             int tilesN, int nsplit, EpiArgs e, Ext x, Fold fold) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), wm = wid >> 2, wn = wid & 3;
  const int nwg = tilesM * tilesN, total = nwg * nsplit;
  const int my_tiles = (total - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;  // >= 1 (grid <= total)
  const int kper = nk * BK;

  auto geo = [&](int it) {
    const int t = blockIdx.x + it * gridDim.x;
    // XCD-aware order: tiles t = x (mod 8) run on XCD x, each XCD walks a contiguous range of tiles
    const int xcd = t & 7, loc = t >> 3, q8 = total >> 3, r8 = total & 7;
    const int wgi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    const int split = wgi / nwg, wg = wgi - split * nwg;
    Geo gg;
    gg.m0 = (wg / tilesN) * BM;
    gg.n0 = (wg % tilesN) * BN;
    gg.split = split;
    gg.kbeg = split * kper;
    return gg;
  };

  // ---- DMA stream: K-tile l_g = (l_it, l_kt), two K-tiles ahead of the MFMAs.  Past the end of the
  // stream it re-reads the last K-tile's data into the regions K-tile l_g would use (freed by the
  // same schedule and never read again), so every phase issues the same number of DMAs.
  const auto ra = rsrc(A, x.a), rb = rsrc(B, x.b);
  int l_it = 0, l_kt = 0, l_g = 0;
  Geo lg = geo(0);
  uint32_t va = 0, vb = 0;  // this wave's per-lane DMA offsets for the load pointer's tile
  auto set_voffs = [&]() {
    va = AK ? vbase_k<false>(lda, lg.m0, wid) : vbase_m(lda, lg.m0, wid);
    vb = BKM ? vbase_k<P8>(ldb, lg.n0, wid) : vbase_m(ldb, lg.n0, wid);
  };
  set_voffs();
  // K-major A: part 1 = A rows of quadrant 0, part 2 = B, part 3 = A rows of quadrant 1.
  // N/M-major A (a DMA piece spans both quadrants): part 1 = all of A (triple-buffered), part 2 = B.
  auto issue_part = [&](int part) {
    const int k0 = lg.kbeg + l_kt * BK;
    if (part == 2) {
      char* bb = smem + b_off<AK>(l_g);
      const uint32_t so = BKM ? (uint32_t)k0 * 2 : (uint32_t)((int64_t)k0 * ldb * 2);
      const uint32_t step = (uint32_t)((BKM ? 64 : 16) * ldb * 2);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        dma<EPI == SV_EPI_SLAB ? SV_G9_SLAB_B_CPOL : 0>(rb, vb, so + j * step, bb + (wid + 8 * j) * 1024);
      SV_VMTAG("p2");
    } else if constexpr (AK) {
      char* ab = smem + a_off<AK>(l_g);
      const int h = part == 1 ? 0 : 1;  // pieces h*8 + wid (rows 64h + ..) and h*8 + 16 + wid (+128 rows)
      const uint32_t so = (uint32_t)k0 * 2 + (uint32_t)(64 * h * lda * 2);
      dma(ra, va, so, ab + (h * 8 + wid) * 1024);
      dma(ra, va, so + (uint32_t)(128 * lda * 2), ab + (h * 8 + 16 + wid) * 1024);
      if (part == 1) SV_VMTAG("p1");
      else SV_VMTAG("p3");
    } else if (part == 1) {
      char* ab = smem + a_off<AK>(l_g);
      const uint32_t so = (uint32_t)((int64_t)k0 * lda * 2), step = (uint32_t)(16 * lda * 2);
#pragma unroll
      for (int j = 0; j < 4; ++j) dma(ra, va, so + j * step, ab + (wid + 8 * j) * 1024);
      SV_VMTAG("p1");
    }
  };
  auto advance = [&]() {
    ++l_g;
    if (++l_kt == nk) {
      if (l_it + 1 < my_tiles) {
        ++l_it;
        l_kt = 0;
        lg = geo(l_it);
        set_voffs();
      } else {
        l_kt = nk - 1;  // past the end: repeat the last K-tile's data
      }
    }
  };

  constexpr int E = EpiCount<EPI, P8>::E;
  // forward epilogues read the tile's bias (and gamma) from LDS, staged by DMA: a plain global load
  // in the epilogue would make the compiler drain every DMA in flight (vmcnt(0)) at each tile's end
  constexpr bool LBIAS = AK && (EPI == SV_EPI_STORE || EPI == SV_EPI_BIAS_GELU_DUAL || EPI == SV_EPI_BIAS_GELU ||
                                EPI == SV_EPI_BIAS_GAMMA_RES || EPI == SV_EPI_STORE_STATS || EPI == SV_EPI_LN_BWD);
  // DMAs younger than the W1 / W2 targets in steady state (see the phase comments below)
  constexpr int W1 = AK ? 10 : 8, W2 = 10;
  constexpr int W1E = W1 + E > 63 ? 63 : W1 + E, W2E = W2 + E > 63 ? 63 : W2 + E;
  // SV_EPI_SLAB with C2: the bias gradient sum_k A(m, k) of a weight-gradient GEMM (N/M-major A) from
  // the A fragments this wave already holds: wave (wm, wn) sums fragment rows wn (quadrant 0) and
  // 4 + wn (quadrant 1) of its 128 rows, so the 8 waves cover the tile's 256 rows once
  const bool do_cs = EPI == SV_EPI_SLAB && !AK && e.C2 != nullptr;
  float cs[2] = {0.f, 0.f};
  auto colsum_frag = [&](const bf16x8 (&af)[4][2], float& acc_cs) {
    // fragment wn of the quadrant, chosen by a wave-uniform branch (a dynamic index would spill af)
    bf16x8 f0 = af[0][0], f1 = af[0][1];
    if (wn == 1) f0 = af[1][0], f1 = af[1][1];
    else if (wn == 2) f0 = af[2][0], f1 = af[2][1];
    else if (wn == 3) f0 = af[3][0], f1 = af[3][1];
    const bf16x8 f[2] = {f0, f1};
    // one v_dot2_f32_bf16 against (1, 1) per bf16 pair (f32 accumulation, fixed order)
    typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
    const bf16x2_t ones = {(__bf16)1.0f, (__bf16)1.0f};
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bf16x2_t pr = {f[kh][2 * q], f[kh][2 * q + 1]};
        acc_cs = __builtin_amdgcn_fdot2_f32_bf16(pr, ones, acc_cs, false);
      }
  };

  stamp(0);
  // prologue: K-tiles 0 and 1, then K-tile 0 landed everywhere
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    issue_part(1);
    issue_part(2);
    if constexpr (AK) issue_part(3);
    advance();
  }
  vm_wait<8>();
  bar();
  if (wm == 1) bar();  // waves 4-7 run one barrier behind
  if constexpr (SV_G9_PRIO == 1) {
    if (wm == 1) __builtin_amdgcn_s_setprio(1);  // static priority for the second-dispatched half
  }

  int g = 0;  // the MFMAs' K-tile in the stream
  for (int it = 0; it < my_tiles; ++it) {
    const Geo cg = geo(it);
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    cs[0] = cs[1] = 0.f;
    for (int kt = 0; kt < nk; ++kt, ++g) {
      const char* Ab = smem + a_off<AK>(g);
      const char* Bb = smem + b_off<AK>(g);
      bf16x8 af[4][2], bq[2][2][2];
      auto read_a = [&](int qm) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kh = 0; kh < 2; ++kh)
            af[i][kh] = AK ? frag_k(Ab, wm * 128 + 64 * qm + 16 * i, kh) : frag_m(Ab, wm * 128 + 64 * qm + 16 * i, kh);
      };
      auto read_b = [&](int qn) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
#pragma unroll
          for (int kh = 0; kh < 2; ++kh) {
            const int j = 2 * qn + jj;
            if constexpr (BKM) {
              bq[qn][jj][kh] = frag_k(Bb, wn * 64 + 16 * j, kh);
            } else if constexpr (P8) {
              const int p = threadIdx.x & 3;
              bq[qn][jj][kh] = frag_tr(Bb, wn * 8 + 4 * qn + p, jj, kh);
            } else {
              bq[qn][jj][kh] = frag_m(Bb, wn * 64 + 16 * j, kh);
            }
          }
      };
      auto quad = [&](int qm, int qn) {
        if constexpr (SV_G9_PRIO == 0) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int kh = 0; kh < 2; ++kh)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj)
              acc[4 * qm + i][2 * qn + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  bq[qn][jj][kh], af[i][kh], acc[4 * qm + i][2 * qn + jj], 0, 0, 0);
        if constexpr (SV_G9_PRIO == 0) __builtin_amdgcn_s_setprio(0);
      };
      // phase 0: A quadrant-0 rows and B columns 0-31 of the wave
      read_a(0);
      read_b(0);
      if constexpr (LBIAS) {
        // the tile's bias / gamma columns into LDS (slot by tile parity: the other group may still be
        // in the previous tile's epilogue); retired by the W1 wait of the next K-tile (nk >= 2) or
        // by the wait before the epilogue
        if (kt == 0 && wid < 2) {
          const float* src = wid == 0 ? e.bias : e.gamma;
          if (src && (wid == 0 || EPI == SV_EPI_BIAS_GAMMA_RES))
            dma(rsrc(src, (uint32_t)e.N * 4), (uint32_t)(cg.n0 + (threadIdx.x & 63) * 4) * 4, 0,
                smem + lds_bytes<AK>() + (it & 1) * 2048 + wid * 1024);
          SV_VMTAG("bias");
        }
      }
      lgkm0();
      bar();
      quad(0, 0);
      bar();
      // phase 1: B columns 32-63; the first DMA part of K-tile g+2 into its freed region.  K-major A:
      // the A quadrant-1 rows of THIS K-tile (issued in phase 3 two K-tiles back) must have landed:
      // younger DMAs = 2 + 4 + 2 (previous K-tile's phases 1-3) + 2 (this phase) [+ an epilogue]
      read_b(1);
      issue_part(1);
      if (do_cs) colsum_frag(af, cs[0]);
      if (AK) {
        // the A quadrant-1 rows of THIS K-tile: the part-3 DMA two K-tiles back
        if (it > 0 && kt <= 1) SV_VMWAIT(W2E, "p3:2@epi");  // the previous tile's epilogue lies between
        else SV_VMWAIT(W2, "p3:2");
      }
      lgkm0();
      bar();
      quad(0, 1);
      bar();
      // phase 2: A quadrant-1 rows; B of K-tile g+2
      read_a(1);
      issue_part(2);
      lgkm0();
      bar();
      quad(1, 1);
      bar();
      // phase 3: (K-major A) the A quadrant-1 rows of K-tile g+2; then A quadrant-0 rows and B of
      // K-tile g+1 must have landed: younger DMAs = 2 + (2 + 4 + 2) (K-major A) / 4 + 4 (N-major A:
      // all of A in phase 1, B in phase 2) [+ an epilogue]
      if constexpr (AK) issue_part(3);
      advance();
      if (do_cs) colsum_frag(af, cs[1]);
      // parts 1 and 2 of K-tile g+1: issued one K-tile back (this K-tile's phases 1-2 issued K-tile g+2's)
      if (it > 0 && kt == 0) SV_VMWAIT(W1E, "p1:2@epi p2:2@epi");
      else SV_VMWAIT(W1, "p1:2 p2:2");
      lgkm0();
      bar();
      quad(1, 0);
      bar();
    }
    if (do_cs) {
      // the 4 lane groups hold partial sums of the same row over different k: fold in a fixed order
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        cs[h] += __shfl_xor(cs[h], 16);
        cs[h] += __shfl_xor(cs[h], 32);
        const int m = cg.m0 + wm * 128 + 64 * h + 16 * wn + (threadIdx.x & 15);
        if ((threadIdx.x & 63) < 16 && m < e.M) reinterpret_cast<float*>(e.C2)[(size_t)cg.split * e.M + m] = cs[h];
      }
    }
    if (LBIAS && nk < 2) {  // the bias DMA was issued in this tile's only K-tile
      vm_wait<0>();
      bar();
    }
    if constexpr (FOLD) {
      if (wm == 0) bar();  // align the two wave halves (waves 4-7 run one barrier behind in the K loop)
    }
    if constexpr (EPI == SV_EPI_LN_BWD) {
      // one tile per workgroup (the host's contract): align the staggered wave halves, the epilogue with its
      // workgroup barriers and the row-block exchange, then re-stagger for the kernel's closing barrier
      if (wm == 0) bar();
      ln_bwd_epilogue(acc, e, x, fold, cg.m0, cg.n0, tilesN, reinterpret_cast<const float*>(smem + lds_bytes<AK>()),
                      reinterpret_cast<float*>(smem + lds_bytes<AK>() + 4096), smem);
      if (wm == 1) bar();
    } else {
      epilogue<EPI, P8, AK, FOLD>(acc, e, x, cg.m0 + wm * 128, cg.n0 + wn * 64, cg.split,
                        LBIAS ? reinterpret_cast<const float*>(smem + lds_bytes<AK>() + (it & 1) * 2048) : nullptr);
    }
    SV_VMTAG("epi");  // after the epilogue's fixed EpiCount memory instructions (the E in W1E / W2E)
    if constexpr (FOLD) {
      // arrival: every wave's slab stores complete (this also drains the next tile's first DMAs: the K loop's
      // counted waits then find fewer in flight, which they allow), one ticket per workgroup
      vm_wait<0>();
      bar();
      // the flag word: the A slot of the tile's last K-tile, g - 1 (N/M-major A is triple-buffered: every wave
      // has read it -- the barrier above -- and the next DMA into it is K-tile g + 2's, issued in the next
      // tile's first K-tile, after the barriers below)
      static_assert(!AK, "the in-kernel fold is for the weight-gradient layout (N/M-major A)");
      volatile int* flag = reinterpret_cast<volatile int*>(smem + a_off<AK>(g - 1));
      const int tile = (cg.m0 / BM) * tilesN + cg.n0 / BN;
      int* arrive = fold.cnt + 2 * tile;
      int* depart = arrive + 1;
      if constexpr (FOLD == kFoldLast) {
        if (threadIdx.x == 0)
          *flag = __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsplit - 1;
        lgkm0();  // the flag's LDS write before the barrier (s_barrier waits for no memory operation on gfx950)
        bar();
        if (*flag) {  // workgroup-uniform: the last slice of this tile landed -- fold it
          fold_tile<2>(e, x, fold, cg.m0, cg.n0, nsplit);
          if (threadIdx.x == 0) __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        // arrive, then poll (one lane, sc1 loads, s_sleep between) until every slice of the tile has landed;
        // the other waves load after the barrier the polling wave joins
        if (threadIdx.x == 0) {
          __hip_atomic_fetch_add(arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          while (__hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < nsplit)
            __builtin_amdgcn_s_sleep(4);
        }
        bar();
        const int per = (BM + nsplit - 1) / nsplit;
        fold_tile<2>(e, x, fold, cg.m0, cg.n0, nsplit, cg.split * per, cg.split * per + per);
        // departure: the last workgroup out re-arms both counters (nobody polls them any more)
        if (threadIdx.x == 0 &&
            __hip_atomic_fetch_add(depart, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsplit - 1) {
          __hip_atomic_store(arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(depart, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      bar();  // the flag word is rewritten by the next tile
      if (wm == 1) bar();  // re-stagger for the next tile's K loop
    }
  }
  vm_wait<0>();  // no LDS-DMA may land after the workgroup's LDS is released
  if (wm == 0) bar();
  stamp(1);
}

template <bool AK, int EPI, int FOLD = kFoldNone>
constexpr int lds_total() {
  return lds_bytes<AK>() + ((AK && (EPI == SV_EPI_STORE || EPI == SV_EPI_BIAS_GELU_DUAL || EPI == SV_EPI_BIAS_GELU ||
                                   EPI == SV_EPI_BIAS_GAMMA_RES || EPI == SV_EPI_STORE_STATS || EPI == SV_EPI_LN_BWD))
                                ? 4096 : 0) +
         (EPI == SV_EPI_LN_BWD ? kLnRed : 0);
}

template <bool AK, bool BKM, int EPI, bool P8, int FOLD = kFoldNone>
static int launch(const sv_gemm_desc* d, int split, hipStream_t s) {
  const int nk = d->K / split / BK;
  const int tilesM = ceil_div(d->M, BM), tilesN = ceil_div(d->N, BN);
  EpiArgs e{d->M, d->N, d->epilogue, d->C, d->c_dtype, d->ldc, d->C2, d->c2_dtype, d->bias, d->gamma,
            d->aux, d->aux_dtype, d->ld_aux};
  if constexpr (EPI == SV_EPI_LN_BWD) {  // LayerNorm weight staged through the bias slot; mean / rstd per row
    e.bias = d->bn->gamma;
    e.bn_mu = d->bn->mean;
    e.bn_rs = d->bn->rstd;
  }
  const int cs = d->c_dtype == SV_F32 ? 4 : 2;
  Ext x;
  if (EPI == SV_EPI_SLAB) {
    x.c = (uint32_t)((size_t)d->M * d->N * (P8 ? 2 : 4));
  } else {
    x.c = (uint32_t)(((size_t)(d->M - 1) * d->ldc + d->N) * cs);
  }
  x.c2 = d->C2 ? (uint32_t)(((size_t)(d->M - 1) * d->ldc + d->N) * (d->c2_dtype == SV_F32 ? 4 : 2)) : 0u;
  x.aux = d->aux ? (uint32_t)(((size_t)(d->M - 1) * d->ld_aux + d->N) * (d->aux_dtype == SV_F32 ? 4 : 2)) : 0u;
  x.a = (uint32_t)((AK ? (size_t)(d->M - 1) * d->lda + d->K : (size_t)(d->K - 1) * d->lda + d->M) * 2);
  x.b = (uint32_t)((BKM ? (size_t)(d->N - 1) * d->ldb + d->K : (size_t)(d->K - 1) * d->ldb + d->N) * 2);
  constexpr int LDS = lds_total<AK, EPI, FOLD>();
  if (const int rc_ = ensure_lds_attr(reinterpret_cast<const void*>(&gemm9_kernel<AK, BKM, EPI, P8, FOLD>), LDS, s)) return rc_;
  const int total = tilesM * tilesN * split;
  const int grid = policy_grid(&d->policy, total, 1, s);  // persistent: one workgroup per CU (or the cap)
  const Fold fold{d->fold_out, d->fold_ld, d->fold_accumulate, d->fold_counters};
  if constexpr (EPI == SV_EPI_LN_BWD) {
    // the row-block exchange waits for partner tiles: every tile a workgroup of its own, all of them resident at
    // once on the CUs this stream may use (its CU mask, the policy's cap)
    int usable = stream_cus(s);
    if (d->policy.grid_cap > 0 && d->policy.grid_cap < usable) usable = d->policy.grid_cap;
    if (grid != total || total > usable) return SV_ERR_UNSUPPORTED;
  }
  if constexpr (FOLD != kFoldNone) {
    // the spread fold waits for a tile's other slices: only when every (tile, slice) unit has a workgroup of its
    // own and the grid is at most half the chip (one workgroup per CU): then two such launches on two streams
    // can never hold every CU with partly-resident grids, so a waiting workgroup's peers always find a CU.
    // "The chip" is the CUs this stream may use: a CU-masked stream (training/cumask.py) or a grid cap
    // (sv_gemm_policy.grid_cap, which also marks a launch that shares the chip by design) shrinks it.
    // Otherwise the wait-free last-arriver form.
    int usable = stream_cus(s);
    if (d->policy.grid_cap > 0 && d->policy.grid_cap < usable) usable = d->policy.grid_cap;
    if (grid == total && 2 * total <= usable) {
      constexpr int LDS2 = lds_total<AK, EPI, kFoldSpread>();
      if (const int rc_ = ensure_lds_attr(reinterpret_cast<const void*>(&gemm9_kernel<AK, BKM, EPI, P8, kFoldSpread>), LDS2, s)) return rc_;
      gemm9_kernel<AK, BKM, EPI, P8, kFoldSpread><<<grid, THREADS, LDS2, s>>>(
          reinterpret_cast<const uint16_t*>(d->A), d->lda, reinterpret_cast<const uint16_t*>(d->B), d->ldb, nk, tilesM,
          tilesN, split, e, x, fold);
      return check_launch("sv_gemm(v9, spread fold)");
    }
  }
  gemm9_kernel<AK, BKM, EPI, P8, FOLD><<<grid, THREADS, LDS, s>>>(reinterpret_cast<const uint16_t*>(d->A), d->lda,
                                                                 reinterpret_cast<const uint16_t*>(d->B), d->ldb, nk,
                                                                 tilesM, tilesN, split, e, x, fold);
  return check_launch("sv_gemm(v9)");
}

template <bool AK, bool BKM>
static int launch_epi(const sv_gemm_desc* d, int split, hipStream_t s) {
  const bool bf_out = d->c_dtype == SV_BF16;
  switch (d->epilogue) {
    case SV_EPI_STORE:
      return bf_out ? launch<AK, BKM, SV_EPI_STORE, true>(d, split, s) : launch<AK, BKM, SV_EPI_STORE, false>(d, split, s);
    case SV_EPI_BIAS_GELU_DUAL:
      if (!bf_out || d->c2_dtype != SV_BF16) return SV_ERR_UNSUPPORTED;
      return launch<AK, BKM, SV_EPI_BIAS_GELU_DUAL, true>(d, split, s);
    case SV_EPI_BIAS_GELU:
      if (!bf_out) return SV_ERR_UNSUPPORTED;
      return launch<AK, BKM, SV_EPI_BIAS_GELU, true>(d, split, s);
    case SV_EPI_BIAS_GAMMA_RES:
      if (d->aux_dtype != SV_F32) return SV_ERR_UNSUPPORTED;
      return bf_out ? launch<AK, BKM, SV_EPI_BIAS_GAMMA_RES, true>(d, split, s)
                    : launch<AK, BKM, SV_EPI_BIAS_GAMMA_RES, false>(d, split, s);
    case SV_EPI_MUL_AUX:
      if (d->aux_dtype != SV_BF16) return SV_ERR_UNSUPPORTED;
      return bf_out ? launch<AK, BKM, SV_EPI_MUL_AUX, true>(d, split, s)
                    : launch<AK, BKM, SV_EPI_MUL_AUX, false>(d, split, s);
    case SV_EPI_GELU_GRAD:
      if (d->aux_dtype != SV_BF16) return SV_ERR_UNSUPPORTED;
      return bf_out ? launch<AK, BKM, SV_EPI_GELU_GRAD, true>(d, split, s)
                    : launch<AK, BKM, SV_EPI_GELU_GRAD, false>(d, split, s);
    case SV_EPI_STORE_STATS:
      if (!bf_out || !AK || d->N % 8) return SV_ERR_UNSUPPORTED;
      return launch<AK, BKM, SV_EPI_STORE_STATS, true>(d, split, s);
    case SV_EPI_LN_BWD:
      if constexpr (!AK) {
        return SV_ERR_UNSUPPORTED;
      } else {
        if (!bf_out || d->aux_dtype != SV_BF16 || d->N % BN || d->N > 4 * BN || split != 1 || !d->bn || !d->C2 ||
            !d->fold_out || !d->fold_counters)
          return SV_ERR_UNSUPPORTED;
        return launch<AK, BKM, SV_EPI_LN_BWD, true>(d, split, s);
      }
    case SV_EPI_SLAB:
      if (d->C2 && (AK || d->c2_dtype != SV_F32)) return SV_ERR_UNSUPPORTED;  // fused column sum: N/M-major A
      if (d->c_dtype == SV_BF16) {  // bf16 slabs (the weight-gradient layout, folded in a separate pass)
        if constexpr (AK) {
          return SV_ERR_UNSUPPORTED;
        } else {
          if (d->fold_out || d->N % 8) return SV_ERR_UNSUPPORTED;
          return launch<AK, BKM, SV_EPI_SLAB, true>(d, split, s);
        }
      }
      if (d->fold_out) {  // (the weight-gradient layout only: N/M-major A; others fold in a separate pass)
        if constexpr (AK) return SV_ERR_UNSUPPORTED;
        else return launch<AK, BKM, SV_EPI_SLAB, false, kFoldLast>(d, split, s);
      }
      return launch<AK, BKM, SV_EPI_SLAB, false>(d, split, s);
    default:
      return SV_ERR_UNSUPPORTED;
  }
}

}  // namespace g9

#ifdef SV_CLOCK_STAMPS
extern "C" int sv_diag_clock_stamps(unsigned long long* host, int n) {
  if (n > 1024) n = 1024;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g9::g_stamps), (size_t)n * 4 * sizeof(unsigned long long), 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#endif

int launch_gemm9(const sv_gemm_desc* d, hipStream_t s) {
  using namespace g9;
  if (d->compute != SV_BF16 || d->a_dtype != SV_BF16 || d->b_dtype != SV_BF16 || d->a_scale_k)
    return SV_ERR_UNSUPPORTED;
  const int split = d->epilogue == SV_EPI_SLAB ? (d->split_k < 1 ? 1 : d->split_k) : 1;
  // uniform K-tiles per split, the epilogue's 8-column (bf16) / 4-column (f32) chunks whole, every
  // buffer offset inside 31 bits
  if (d->K % (split * BK) != 0 || d->N % 8 != 0) return SV_ERR_UNSUPPORTED;
  if (d->epilogue != SV_EPI_SLAB && d->ldc % 8 != 0) return SV_ERR_UNSUPPORTED;
  if (d->aux && d->ld_aux % 8 != 0) return SV_ERR_UNSUPPORTED;
  const size_t lim = (size_t)1 << 31;
  const size_t rows = (size_t)ceil_div(d->M, BM) * BM;
  if (rows * (size_t)(d->epilogue == SV_EPI_SLAB ? d->N : d->ldc) * 4 * (size_t)split >= lim) return SV_ERR_UNSUPPORTED;
  if (d->aux && rows * (size_t)d->ld_aux * 4 >= lim) return SV_ERR_UNSUPPORTED;
  // operand extents: the DMA offsets (voffset + soffset) stay below the 0x7fffffff descriptor range
  const size_t a_ext = d->a_kmajor ? (size_t)d->M * d->lda : (size_t)d->K * d->lda;
  const size_t b_ext = d->b_kmajor ? (size_t)d->N * d->ldb : (size_t)d->K * d->ldb;
  if ((a_ext + 4096) * 2 >= lim || (b_ext + 4096) * 2 >= lim) return SV_ERR_UNSUPPORTED;
  if (d->a_kmajor && d->b_kmajor) return launch_epi<true, true>(d, split, s);
  if (d->a_kmajor && !d->b_kmajor) return launch_epi<true, false>(d, split, s);
  if (!d->a_kmajor && d->b_kmajor) return launch_epi<false, true>(d, split, s);
  return launch_epi<false, false>(d, split, s);
}

}  // namespace sv
