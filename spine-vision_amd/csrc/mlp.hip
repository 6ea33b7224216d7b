// Fused ConvNeXt MLP forward for the narrow stages (C = 128 / 192 / 256: S1 / S2 of ConvNeXt-base, S1 of -large):
//     h = y W1^T + b1,  [gh = GELU'(h), a = GELU(h) stored bf16 for the backward],  x_out = gamma (.) (a W2^T + b2) + x
// in ONE persistent kernel, so the 4C-wide hidden activation a never makes the HBM round trip fc1 -> fc2 (VERDICT r4,
// missing 1 / next 3: the FlashAttention shape -- stream the hidden dimension in chunks, keep the C-wide fc2
// accumulator in registers).  Reference: timm ConvNeXtBlock.mlp + gamma + shortcut, via
// spine_vision/training/models/backbone.py:50,164-170.
//
// Layout of the work (512 threads = 8 waves, one workgroup per CU, persistent over 8*RW-row tiles):
//  * wave w owns rows [16 RF w, +16 RF) of the tile (RF 16-row fragments); its y rows live in REGISTERS for the
//    whole tile (the second MFMA operand of fc1), loaded once;
//  * the hidden dimension streams through LDS in chunks of HC = 64 units: W1 rows [j0, j0+64) and W2 columns
//    [j0, j0+64), double-buffered by LDS-DMA (buffer_load ... lds), the next chunk's DMA in flight while this one
//    computes;
//  * fc1 runs with the operands swapped as in v9 (D^T = W1 . y^T: a lane holds 4 consecutive hidden units of one
//    row), the W1 rows permuted inside each 32-group at DMA time (perm8), so after bias + GELU a lane holds 8
//    CONSECUTIVE hidden units of its row: that is both the 16-B store of the dual epilogue and, packed to bf16,
//    exactly the second MFMA operand of fc2 (lane l: row l & 15, k = 8 (l >> 4) .. +7) -- P never leaves the
//    registers;
//  * fc2 accumulates D^T = W2 . P^T into C/16 x RF fragments per wave across all chunks; the epilogue applies
//    gamma (.) (acc + b2) + x and stores f32 rows (4 consecutive channels per lane, 16 B).
// Every accumulator sees the same MFMA instruction with the same operands in the same k order as the unfused v9
// pair (fc1 GELU-dual epilogue, fc2 gamma-residual epilogue), and the epilogue arithmetic is v9's, so the outputs
// are bit for bit the unfused path's (tests/test_mlp_fused_gpu.py).
#include "common.h"
#include "gemm_common.h"

#include <stdlib.h>

namespace sv {
namespace mlp {

constexpr int HC = 64;
// diagnostic builds only (tools/sessions): 1 = no GELU arithmetic, 2 = no weight DMA after chunk 0, 4 = no chunk
// barriers, 8 = weight fragments from registers instead of LDS (results wrong)
#ifndef SV_MLP_DIAG
#define SV_MLP_DIAG 0
#endif
constexpr uint32_t OOB = 0x80000000u;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
// K-major LDS image [rows][64] bf16 (128-B rows), 16-B chunk c of row r at c ^ ((r >> 1) & 7) (as v9)
__device__ __forceinline__ int kswz(int row) { return (row >> 1) & 7; }
// bf16-output row permutation inside a 32-row group (as v9): LDS row 16h + 4g + r holds hidden unit 8g + 4h + r
__device__ __forceinline__ int perm8(int rho) {
  return (rho & ~31) | (((rho & 15) >> 2) << 3) | (((rho >> 4) & 1) << 2) | (rho & 3);
}
__device__ __forceinline__ void dma(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, char* dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)dst, 16, voff, soff, 0, 0);
}
// fragment of a K-major image: lane l holds X[row = base + (l & 15)][k = 32 kh + 8 (l >> 4) + 0..7]
__device__ __forceinline__ bf16x8 frag_k(const char* __restrict__ region, int base, int kh) {
  const int l = threadIdx.x & 63;
  const int row = base + (l & 15), ch = kh * 4 + (l >> 4);
  return *reinterpret_cast<const bf16x8*>(region + row * 128 + ((ch ^ kswz(row)) << 4));
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
// LDS reads of the per-channel vectors the compiler does not see: its alias analysis would otherwise drain every
// LDS-DMA in flight (vmcnt(0)) before a plain LDS read it cannot prove disjoint from them (as v9's lds_f4); two
// 16-B reads, then lgkmcnt(0)
__device__ __forceinline__ void lds_f8(const float* p, float (&v)[8]) {
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t u, w;
  const uint32_t ad = (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p);
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %2 offset:16\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(u), "=v"(w)
               : "v"(ad)
               : "memory");
  v[0] = u.x, v[1] = u.y, v[2] = u.z, v[3] = u.w, v[4] = w.x, v[5] = w.y, v[6] = w.z, v[7] = w.w;
}
__device__ __forceinline__ void lds_f4x2(const float* p0, const float* p1, float (&v0)[4], float (&v1)[4]) {
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t u, w;
  const uint32_t a0 = (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p0);
  const uint32_t a1 = (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p1);
  asm volatile("ds_read_b128 %0, %2\n\tds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)"
               : "=v"(u), "=v"(w)
               : "v"(a0), "v"(a1)
               : "memory");
  v0[0] = u.x, v0[1] = u.y, v0[2] = u.z, v0[3] = u.w, v1[0] = w.x, v1[1] = w.y, v1[2] = w.z, v1[3] = w.w;
}
__device__ __forceinline__ void lds_f4(const float* p, float (&v)[4]) {
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t u;
  const uint32_t ad = (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p);
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(u) : "v"(ad) : "memory");
  v[0] = u.x, v[1] = u.y, v[2] = u.z, v[3] = u.w;
}
__device__ __forceinline__ u32x4 pack8(const float (&v)[8]) {
  return u32x4{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
}
// cache policy of the GELU'(h) store: nt, as the v9 dual epilogue (read only by the backward, much later)
constexpr int kGradCpol = 2;

template <int C>
struct Cfg {
  static constexpr int H = 4 * C;              // hidden units
  static constexpr int NCH = H / HC;            // chunks per tile
  static constexpr int KB = C / 64;             // 64-deep k-blocks of fc1
  static constexpr int KS = C / 32;             // 32-deep MFMA k-steps of fc1
  static constexpr int CF = C / 16;             // 16-channel fragments of the fc2 output
  static constexpr int RF = C == 128 ? 2 : 1;   // 16-row fragments per wave (C = 192 at 2 spills)
  // waves per workgroup: C = 128 runs two 4-wave workgroups per CU (67 KiB of LDS each), which desynchronise -- one
  // computes while the other streams its tile's y / x / x_out; the wider C need one 8-wave workgroup per CU (the
  // second group staggered half a chunk behind)
  static constexpr int NW = C == 128 ? 4 : 8;
  static constexpr int THREADS = 64 * NW;
  static constexpr int WG_PER_CU = NW == 4 ? 2 : 1;
  static constexpr int R = NW * 16 * RF;        // rows per tile
  static constexpr int W1B = HC * C * 2;        // W1 chunk image bytes (KB k-blocks of [HC][64])
  static constexpr int W2B = C * HC * 2;        // W2 chunk image bytes ([C][64])
  static constexpr int PERSIST = (H + 2 * C) * 4;  // b1 [H], b2 [C], gamma [C] (f32)
  static constexpr int LDS = 2 * (W1B + W2B) + PERSIST;
};

template <int C, bool TRAIN>
__global__ void __launch_bounds__(Cfg<C>::THREADS) __attribute__((amdgpu_waves_per_eu(2, 2)))
mlp_fwd_kernel(const uint16_t* __restrict__ y, const uint16_t* __restrict__ w1, const float* __restrict__ b1,
               const uint16_t* __restrict__ w2, const float* __restrict__ b2, const float* __restrict__ gamma,
               const float* __restrict__ x, float* __restrict__ xo, uint16_t* __restrict__ gh, uint16_t* __restrict__ a,
               int M) {
  using K = Cfg<C>;
  constexpr int RF = K::RF, KS = K::KS, CF = K::CF, KB = K::KB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* lb1 = reinterpret_cast<float*>(smem + 2 * (K::W1B + K::W2B));
  float* lb2 = lb1 + K::H;
  float* lgam = lb2 + C;
  const int lane = threadIdx.x & 63, ml = lane & 15, gq = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles = (M + K::R - 1) / K::R;
  const int my_tiles = (tiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;  // >= 1 (grid <= tiles)
  const int total = my_tiles * K::NCH;

  // the per-channel vectors once into LDS (plain loads / stores, before any DMA)
  for (int i = threadIdx.x; i < K::H; i += K::THREADS) lb1[i] = b1[i];
  for (int i = threadIdx.x; i < C; i += K::THREADS) lb2[i] = b2[i], lgam[i] = gamma[i];

  // ---- two wave groups, B (waves 4-7) one barrier = half a chunk behind A (waves 0-3): on every SIMD one wave's
  // GELU (VALU) runs beside its partner's MFMAs (MI355X_MICROARCH.md "Two waves per SIMD", item 9: stagger waves
  // 4-7).  Chunk q is two halves: X_q [fc1, bias + GELU, the dual epilogue's stores] Y_q [fc2].  W1 and W2 chunks live
  // in separate 2-slot rings; only group A issues their DMA: W1(q+1) right after its X_q barrier (B is then at Y_{q-1},
  // done with W1(q-1), whose slot it takes), W2(q+1) right after its Y_q barrier (B at X_q: done with W2(q-1)); each
  // lands within a chunk -- A waits for it before its next barrier of the same kind, which B passes only later.
  const int grp = wid >> 2, wa = wid & 3;
  const auto rw1 = rsrc(w1, (uint32_t)(K::H * C * 2)), rw2 = rsrc(w2, (uint32_t)(C * K::H * 2));
  // a DMA piece = 8 rows x 128 B; A-wave wa issues pieces wa and wa + 4 of every 64-row block (+32 rows via soffset:
  // perm8 and the swizzle commute with it)
  const int prow = 8 * wa + (lane >> 3), pch = lane & 7;
  const uint32_t v1 = (uint32_t)((perm8(prow) * C + ((pch ^ kswz(prow)) << 3)) * 2);
  const uint32_t v2 = (uint32_t)((prow * K::H + ((pch ^ kswz(prow)) << 3)) * 2);
  char* w1r = smem;                 // W1 ring: 2 x [KB][HC][64]
  char* w2r = smem + 2 * K::W1B;    // W2 ring: 2 x [C][64]
  auto issue_w1 = [&](int q) {
    const int j0 = (q % K::NCH) * HC;
    char* st = w1r + (q & 1) * K::W1B;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        dma(rw1, v1, (uint32_t)(((j0 + 32 * h) * C + 64 * kb) * 2), st + kb * (HC * 128) + (wa + 4 * h) * 1024);
    SV_VMTAG("w1");
  };
  auto issue_w2 = [&](int q) {
    const int j0 = (q % K::NCH) * HC;
    char* st = w2r + (q & 1) * K::W2B;
#pragma unroll
    for (int j = 0; j < KB; ++j)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        dma(rw2, v2, (uint32_t)(((64 * j + 32 * h) * K::H + j0) * 2), st + (8 * j + wa + 4 * h) * 1024);
    SV_VMTAG("w2");
  };
  // vector-memory instructions of group A younger than the DMA each wait retires: the dual epilogue's S stores per
  // chunk, the other ring's N1 pieces (the counts allow them to stay in flight)
  constexpr int S = TRAIN ? RF * (HC / 32) * 2 : 0;
  constexpr int N1 = 2 * KB;

  const auto ry = rsrc(y, (uint32_t)((size_t)M * C * 2));
  const auto rx = rsrc(x, (uint32_t)((size_t)M * C * 4));
  const auto rxo = rsrc(xo, (uint32_t)((size_t)M * C * 4));
  const auto rgh = rsrc(TRAIN ? gh : nullptr, TRAIN ? (uint32_t)((size_t)M * K::H * 2) : 0u);
  const auto ra = rsrc(TRAIN ? a : nullptr, TRAIN ? (uint32_t)((size_t)M * K::H * 2) : 0u);

  if (grp == 0) {
    issue_w1(0);
    issue_w2(0);
    vm_wait<0>();
  }
  __syncthreads();  // the per-channel vectors and chunk 0
  if (K::NW == 8 && grp == 1) bar();  // group B one barrier behind
  int q = 0;
  for (int it = 0; it < my_tiles; ++it) {
    const int row0 = ((int)blockIdx.x + it * (int)gridDim.x) * K::R + wid * 16 * RF;
    // this wave's y rows: lane holds row row0 + 16 rf + ml, k = 32 ks + 8 gq .. +7
    bf16x8 yf[RF][KS];
#pragma unroll
    for (int rf = 0; rf < RF; ++rf) {
      const int m = row0 + 16 * rf + ml;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const uint32_t off = m < M ? (uint32_t)((m * C + 32 * ks + 8 * gq) * 2) : OOB;
        yf[rf][ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0));
      }
    }
    f32x4 acc2[CF][RF];
#pragma unroll
    for (int cf = 0; cf < CF; ++cf)
#pragma unroll
      for (int rf = 0; rf < RF; ++rf) acc2[cf][rf] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int ch = 0; ch < K::NCH; ++ch, ++q) {
      // X_q: W1(q) landed (A: issued after X_{q-1}; younger: chunk q-1's stores, W2(q)'s pieces)
      if (grp == 0) SV_VMWAIT(S + N1, "w1:1");
      lgkm0();
      if (!(SV_MLP_DIAG & 4)) bar();
      // unconditional (past the end: a harmless re-load of chunk 0 into the free slot): every chunk issues the same
      // vector-memory instructions, which the counted waits assume.  Round 5 skipped it for q + 1 == total, which left
      // the last chunk's Y wait with fewer younger instructions than its count: W2 of a workgroup's last chunk was not
      // covered (tools/check_vmcnt.py found it)
      if (grp == 0 && !(SV_MLP_DIAG & 2)) issue_w1(q + 1);
      const char* st = w1r + (q & 1) * K::W1B;
      const int j0 = ch * HC;
      // this lane's fc1 bias: hidden units j0 + 32 qq + 8 gq .. +7
      float bia[2][8];
      lds_f8(lb1 + j0 + 8 * gq, bia[0]);
      lds_f8(lb1 + j0 + 32 + 8 * gq, bia[1]);
      // fc1: h^T chunk [64 hidden (4 fragments, perm8 rows)] x [16 RF rows], k ascending
      f32x4 acc1[4][RF];
#pragma unroll
      for (int hf = 0; hf < 4; ++hf)
#pragma unroll
        for (int rf = 0; rf < RF; ++rf) acc1[hf][rf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const char* img = st + (ks >> 1) * (HC * 128);
#pragma unroll
        for (int hf = 0; hf < 4; ++hf) {
          const bf16x8 wf = (SV_MLP_DIAG & 8) ? yf[0][(ks + hf) % KS] : frag_k(img, 16 * hf, ks & 1);
#pragma unroll
          for (int rf = 0; rf < RF; ++rf)
            acc1[hf][rf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, yf[rf][ks], acc1[hf][rf], 0, 0, 0);
        }
      }
      // bias + GELU pair (v9's packed form, same operations and order); P = bf16 GELU(h), the fc2 operand
      bf16x8 pf[2][RF];
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
#pragma unroll
        for (int rf = 0; rf < RF; ++rf) {
          float v[8], o[8], o2[8];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = acc1[2 * qq][rf][r], v[4 + r] = acc1[2 * qq + 1][rf][r];
#pragma unroll
          for (int w = 0; w < 8; ++w) v[w] += bia[qq][w];
#pragma unroll
          for (int w = 0; w < 8; w += 2) {
            const gelu_f2 hh = {v[w], v[w + 1]};
            gelu_f2 ph, de;
#if SV_MLP_DIAG & 1
            ph = (gelu_f2){1.0f, 1.0f}, de = hh;  // diagnostic: no GELU arithmetic (results wrong)
#else
            gelu_parts2(hh, ph, de);
#endif
            const gelu_f2 g = hh * ph;
            o2[w] = g.x, o2[w + 1] = g.y;
            if constexpr (TRAIN) {
              const gelu_f2 dg = __builtin_elementwise_fma(hh, de, ph);
              o[w] = dg.x, o[w + 1] = dg.y;
            }
          }
          const u32x4 pk = pack8(o2);
          pf[qq][rf] = __builtin_bit_cast(bf16x8, pk);
          if constexpr (TRAIN) {
            const int m = row0 + 16 * rf + ml;
            const uint32_t off = m < M ? (uint32_t)(((size_t)m * K::H + j0 + 32 * qq + 8 * gq) * 2) : OOB;
            __builtin_amdgcn_raw_buffer_store_b128(pack8(o), rgh, off, 0, kGradCpol);
            __builtin_amdgcn_raw_buffer_store_b128(pk, ra, off, 0, 0);
          } else {
            (void)o;
          }
        }
      }
      // Y_q: W2(q) landed (A: issued after Y_{q-1}; younger: W1(q+1)'s pieces, this chunk's stores)
      if (grp == 0) SV_VMWAIT(N1 + S, "w2:1");
      lgkm0();
      if (!(SV_MLP_DIAG & 4)) bar();
      if (grp == 0 && !(SV_MLP_DIAG & 2)) issue_w2(q + 1);
      // fc2: acc2 += W2[:, chunk] . P^T, k (hidden) ascending
      const char* img2 = w2r + (q & 1) * K::W2B;
#pragma unroll
      for (int qq = 0; qq < 2; ++qq)
#pragma unroll
        for (int cf = 0; cf < CF; ++cf) {
          const bf16x8 wf = (SV_MLP_DIAG & 8) ? yf[0][(cf + qq) % KS] : frag_k(img2, 16 * cf, qq);
#pragma unroll
          for (int rf = 0; rf < RF; ++rf)
            acc2[cf][rf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, pf[qq][rf], acc2[cf][rf], 0, 0, 0);
        }
    }
    // epilogue: x_out = gamma (.) (acc + b2) + x   (v9's gamma-residual arithmetic); lane: row m, channels 16 cf + 4 gq
#pragma unroll
    for (int rf = 0; rf < RF; ++rf) {
      const int m = row0 + 16 * rf + ml;
      u32x4 xr[CF];
#pragma unroll
      for (int cf = 0; cf < CF; ++cf) {
        const uint32_t off = m < M ? (uint32_t)(((size_t)m * C + 16 * cf + 4 * gq) * 4) : OOB;
        xr[cf] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
      }
#pragma unroll
      for (int cf = 0; cf < CF; ++cf) {
        const int c = 16 * cf + 4 * gq;
        float bv[4], gv[4];
        lds_f4x2(lb2 + c, lgam + c, bv, gv);
        const uint32_t xw[4] = {xr[cf].x, xr[cf].y, xr[cf].z, xr[cf].w};
        float o[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) o[w] = fmaf(gv[w], acc2[cf][rf][w] + bv[w], __uint_as_float(xw[w]));
        const uint32_t off = m < M ? (uint32_t)(((size_t)m * C + c) * 4) : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(o[0]), __float_as_uint(o[1]),
                                                     __float_as_uint(o[2]), __float_as_uint(o[3])},
                                               rxo, off, 0, 0);
      }
    }
  }
  if (K::NW == 8 && grp == 0) bar();  // the barrier group B is behind
  vm_wait<0>();  // no LDS-DMA may land after the workgroup's LDS is released
}

// ---- C = 128 (ConvNeXt-base S1, the largest fused shape: 3 blocks of 524288 rows at bs32): two 4-wave workgroups
// per CU, hidden chunks of 32 units, and nothing waits on HBM at a tile boundary -- each wave DMAs its NEXT tile's y
// fragments into its own LDS region at the start of the current tile (64 lanes x 16 B per fragment: the LDS image IS
// the register image), and loads the tile's residual x at the start of its last chunk, a chunk ahead of the epilogue.
// The W2 chunk image has 64-B rows ([128][32]); 16-B chunk c of row r sits at c ^ {0,2,3,1}[(r >> 2) & 3], which
// keeps the fragment reads (16 rows x one 16-B chunk per lane group of ds_read_b128) conflict-free.
namespace c128 {
constexpr int C = 128, H = 512, HC = 32, NCH = H / HC, KB = 2, KS = 4, CF = 8, RF = 2, NW = 4, THREADS = 256;
constexpr int R = NW * 16 * RF;                 // 128 rows per tile
constexpr int W1B = KB * HC * 128;              // [KB][32][64] bf16 = 8 KiB
constexpr int W2B = C * HC * 2;                 // [128][32] bf16 = 8 KiB
constexpr int YB = RF * KS * 1024;              // one wave's y fragments, 8 KiB
constexpr int OFF_W1 = 0, OFF_W2 = 2 * W1B, OFF_Y = OFF_W2 + 2 * W2B, OFF_P = OFF_Y + NW * YB;
constexpr int LDS = OFF_P + (H + 2 * C) * 4;    // 67 KiB: two workgroups per CU
constexpr int LDS_BWD = OFF_P + (C + NW * 2 * C) * 4;  // the backward: LayerNorm weight + per-wave partials
// vector-memory instructions per wave: W1 / W2 pieces per chunk, y fragments per tile, x loads and x_out stores per tile
constexpr int N1 = KB, N2 = 2, YP = RF * KS, XL = RF * CF, XO = RF * CF;

__device__ __forceinline__ int w2swz(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }  // {0,2,3,1}
__device__ __forceinline__ bf16x8 frag64(const char* __restrict__ region, int base) {
  const int l = threadIdx.x & 63;
  const int row = base + (l & 15);
  return *reinterpret_cast<const bf16x8*>(region + row * 64 + (((l >> 4) ^ w2swz(row)) << 4));
}
__device__ __forceinline__ bf16x8 lds_frag(const char* p) {  // ds_read_b128 the compiler does not see (see lds_f8)
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t u;
  const uint32_t ad = (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p);
  asm volatile("ds_read_b128 %0, %1" : "=v"(u) : "v"(ad) : "memory");
  return __builtin_bit_cast(bf16x8, u);
}

template <bool TRAIN>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(2, 2)))
mlp128_kernel(const uint16_t* __restrict__ y, const uint16_t* __restrict__ w1, const float* __restrict__ b1,
              const uint16_t* __restrict__ w2, const float* __restrict__ b2, const float* __restrict__ gamma,
              const float* __restrict__ x, float* __restrict__ xo, uint16_t* __restrict__ gh, uint16_t* __restrict__ a,
              int M) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* lb1 = reinterpret_cast<float*>(smem + OFF_P);
  float* lb2 = lb1 + H;
  float* lgam = lb2 + C;
  const int lane = threadIdx.x & 63, ml = lane & 15, gq = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles = (M + R - 1) / R;
  const int my_tiles = (tiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;  // >= 1 (grid <= tiles)
  for (int i = threadIdx.x; i < H; i += THREADS) lb1[i] = b1[i];
  for (int i = threadIdx.x; i < C; i += THREADS) lb2[i] = b2[i], lgam[i] = gamma[i];

  const auto rw1 = rsrc(w1, (uint32_t)(H * C * 2)), rw2 = rsrc(w2, (uint32_t)(C * H * 2));
  const auto ry = rsrc(y, (uint32_t)((size_t)M * C * 2));
  const auto rx = rsrc(x, (uint32_t)((size_t)M * C * 4));
  const auto rxo = rsrc(xo, (uint32_t)((size_t)M * C * 4));
  const auto rgh = rsrc(TRAIN ? gh : nullptr, TRAIN ? (uint32_t)((size_t)M * H * 2) : 0u);
  const auto ra = rsrc(TRAIN ? a : nullptr, TRAIN ? (uint32_t)((size_t)M * H * 2) : 0u);
  // W1 chunk: rows [j0, j0 + 32) permuted (perm8), two k-blocks [32][64]; wave wid's piece = rows 8 wid .. + 7
  const int p1 = 8 * wid + (lane >> 3);
  const uint32_t v1 = (uint32_t)((perm8(p1) * C + (((lane & 7) ^ kswz(p1)) << 3)) * 2);
  // W2 chunk: columns [j0, j0 + 32) of the 128 channel rows; wave wid's pieces = rows 16 wid + 64 h .. + 15
  const int p2 = 16 * wid + (lane >> 2);
  const uint32_t v2 = (uint32_t)((p2 * H + (((lane & 3) ^ w2swz(p2)) << 3)) * 2);
  auto issue_w1 = [&](int q) {
    const int j0 = (q % NCH) * HC;
    char* st = smem + OFF_W1 + (q & 1) * W1B;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) dma(rw1, v1, (uint32_t)((j0 * C + 64 * kb) * 2), st + kb * (HC * 128) + wid * 1024);
    SV_VMTAG("w1");
  };
  auto issue_w2 = [&](int q) {
    const int j0 = (q % NCH) * HC;
    char* st = smem + OFF_W2 + (q & 1) * W2B;
#pragma unroll
    for (int h = 0; h < 2; ++h) dma(rw2, v2, (uint32_t)((64 * h * H + j0) * 2), st + (wid + 4 * h) * 1024);
    SV_VMTAG("w2");
  };
  // this wave's y fragments of tile t into its own region (rows past M, and tiles past the end, read as zeros)
  char* ybuf = smem + OFF_Y + wid * YB;
  auto issue_y = [&](int it) {
    const int wrow = ((int)blockIdx.x + it * (int)gridDim.x) * R + wid * 16 * RF;
#pragma unroll
    for (int rf = 0; rf < RF; ++rf) {
      const int m = wrow + 16 * rf + ml;
      const uint32_t vy = (it < my_tiles && m < M) ? (uint32_t)((m * C + 8 * gq) * 2) : OOB;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) dma(ry, vy, (uint32_t)(64 * ks), ybuf + (rf * KS + ks) * 1024);
    }
    SV_VMTAG("y");
  };
  constexpr int S = TRAIN ? RF * 2 : 0;  // the dual epilogue's stores per chunk

  issue_w1(0);
  issue_w2(0);
  issue_y(0);
  vm_wait<0>();
  __syncthreads();  // the per-channel vectors, chunk 0 and every wave's y of its first tile
  int q = 0;
  for (int it = 0; it < my_tiles; ++it) {
    const int row0 = ((int)blockIdx.x + it * (int)gridDim.x) * R + wid * 16 * RF;
    // y of this tile landed (issued at the previous tile's start: a whole tile of vector-memory instructions -- at
    // least 16 chunks x (N1 + N2) -- is younger)
    SV_VMWAIT(32, "y:1");
    bf16x8 yf[RF][KS];
#pragma unroll
    for (int rf = 0; rf < RF; ++rf)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) yf[rf][ks] = lds_frag(ybuf + (rf * KS + ks) * 1024 + lane * 16);
    lgkm0();
    issue_y(it + 1);
    f32x4 acc2[CF][RF];
#pragma unroll
    for (int cf = 0; cf < CF; ++cf)
#pragma unroll
      for (int rf = 0; rf < RF; ++rf) acc2[cf][rf] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x4 xr[RF][CF];

    for (int ch = 0; ch < NCH; ++ch, ++q) {
      // X_q: W1(q) landed.  Younger than it (issued after the previous X barrier): that chunk's stores and W2(q);
      // across a tile boundary also the x loads, the x_out stores and this tile's y prefetch
      if (ch == 0) SV_VMWAIT(XL + S + N2 + XO + YP, "w1:1");
      else SV_VMWAIT(S + N2, "w1:1");
      lgkm0();
      bar();
      issue_w1(q + 1);  // past the end: a harmless re-load of chunk 0 into the free slot (uniform counts)
      if (ch == NCH - 1) {  // the epilogue's residual, a chunk ahead
#pragma unroll
        for (int rf = 0; rf < RF; ++rf) {
          const int m = row0 + 16 * rf + ml;
#pragma unroll
          for (int cf = 0; cf < CF; ++cf) {
            const uint32_t off = m < M ? (uint32_t)(((size_t)m * C + 16 * cf + 4 * gq) * 4) : OOB;
            xr[rf][cf] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
          }
        }
      }
      const char* st1 = smem + OFF_W1 + (q & 1) * W1B;
      const int j0 = ch * HC;
      float bia[8];
      lds_f8(lb1 + j0 + 8 * gq, bia);
      // fc1: h^T chunk [32 hidden (2 fragments, perm8 rows)] x [32 rows], k ascending
      f32x4 acc1[2][RF];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int rf = 0; rf < RF; ++rf) acc1[hf][rf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const char* img = st1 + (ks >> 1) * (HC * 128);
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const bf16x8 wf = frag_k(img, 16 * hf, ks & 1);
#pragma unroll
          for (int rf = 0; rf < RF; ++rf)
            acc1[hf][rf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, yf[rf][ks], acc1[hf][rf], 0, 0, 0);
        }
      }
      // bias + GELU pair (v9's packed form); P = bf16 GELU(h), fc2's operand; both stored nt (read only by the backward)
      bf16x8 pf[RF];
#pragma unroll
      for (int rf = 0; rf < RF; ++rf) {
        float v[8], o[8], o2[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc1[0][rf][r], v[4 + r] = acc1[1][rf][r];
#pragma unroll
        for (int w = 0; w < 8; ++w) v[w] += bia[w];
#pragma unroll
        for (int w = 0; w < 8; w += 2) {
          const gelu_f2 hh = {v[w], v[w + 1]};
          gelu_f2 ph, de;
          gelu_parts2(hh, ph, de);
          const gelu_f2 g = hh * ph;
          o2[w] = g.x, o2[w + 1] = g.y;
          if constexpr (TRAIN) {
            const gelu_f2 dg = __builtin_elementwise_fma(hh, de, ph);
            o[w] = dg.x, o[w + 1] = dg.y;
          }
        }
        const u32x4 pk = pack8(o2);
        pf[rf] = __builtin_bit_cast(bf16x8, pk);
        if constexpr (TRAIN) {
          const int m = row0 + 16 * rf + ml;
          const uint32_t off = m < M ? (uint32_t)(((size_t)m * H + j0 + 8 * gq) * 2) : OOB;
          __builtin_amdgcn_raw_buffer_store_b128(pack8(o), rgh, off, 0, kGradCpol);
          __builtin_amdgcn_raw_buffer_store_b128(pk, ra, off, 0, kGradCpol);
        } else {
          (void)o;
        }
      }
      // Y_q: W2(q) landed.  Younger (issued after the previous Y barrier): W1(q+1) and this chunk's stores; in a
      // tile's first chunk also the x_out stores and the y prefetch, in its last the x loads
      if (ch == 0) SV_VMWAIT(XO + YP + N1 + S, "w2:1");
      else if (ch == NCH - 1) SV_VMWAIT(N1 + XL + S, "w2:1");
      else SV_VMWAIT(N1 + S, "w2:1");
      lgkm0();
      bar();
      issue_w2(q + 1);
      // fc2: acc2 += W2[:, chunk] . P^T, k (hidden) ascending
      const char* st2 = smem + OFF_W2 + (q & 1) * W2B;
#pragma unroll
      for (int cf = 0; cf < CF; ++cf) {
        const bf16x8 wf = frag64(st2, 16 * cf);
#pragma unroll
        for (int rf = 0; rf < RF; ++rf)
          acc2[cf][rf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, pf[rf], acc2[cf][rf], 0, 0, 0);
      }
    }
    // epilogue: x_out = gamma (.) (acc + b2) + x   (v9's gamma-residual arithmetic)
#pragma unroll
    for (int rf = 0; rf < RF; ++rf) {
      const int m = row0 + 16 * rf + ml;
#pragma unroll
      for (int cf = 0; cf < CF; ++cf) {
        const int c = 16 * cf + 4 * gq;
        float bv[4], gv[4];
        lds_f4x2(lb2 + c, lgam + c, bv, gv);
        const uint32_t xw[4] = {xr[rf][cf].x, xr[rf][cf].y, xr[rf][cf].z, xr[rf][cf].w};
        float o[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) o[w] = fmaf(gv[w], acc2[cf][rf][w] + bv[w], __uint_as_float(xw[w]));
        const uint32_t off = m < M ? (uint32_t)(((size_t)m * C + c) * 4) : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(o[0]), __float_as_uint(o[1]),
                                                     __float_as_uint(o[2]), __float_as_uint(o[3])},
                                               rxo, off, 0, 0);
      }
    }
  }
  vm_wait<0>();  // no LDS-DMA may land after the workgroup's LDS is released
}

template <bool TRAIN>
static int launch(const uint16_t* y, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
                  const float* gamma, const float* x, float* xo, uint16_t* gh, uint16_t* a, int M, hipStream_t s) {
  if (const int rc = ensure_lds_attr(reinterpret_cast<const void*>(&mlp128_kernel<TRAIN>), LDS, s)) return rc;
  const int tiles = (M + R - 1) / R;
  const int slots = 2 * device_cus(s);
  const int grid = tiles < slots ? tiles : slots;
  mlp128_kernel<TRAIN><<<grid, THREADS, LDS, s>>>(y, w1, b1, w2, b2, gamma, x, xo, gh, a, M);
  return check_launch("sv_mlp_fwd");
}
// ---- fused backward of the same block part, C = 128: from the gradient at the block output d
// (the bf16 copy of the gradient stream), in one kernel
//     dh = (d . (W2 gamma)) (.) GELU'(h)          -> stored bf16 (the fc1 weight gradient's operand)
//     dy = bf16(dh . W1)                           -> kept on chip (the C-wide accumulator)
//     dz = LayerNorm backward of dy (bf16 z, mean, rstd, weight)  -> stored bf16;  per-wave partial sums of
//          dy x^ and dy for the LayerNorm weight / bias gradients
// -- the unfused path's fc2 data gradient (x GELU' epilogue), fc1 data gradient and LayerNorm backward: dh is not read
// back, dy never reaches HBM.  Same skeleton as the forward kernel: the weight images are the transposed operands
// (w2t = (W2 gamma)^T [512][128] in W1's layout, w1t = W1^T [128][512] in W2's), GELU'(h) is loaded a chunk ahead,
// z / mean / rstd a chunk ahead of the epilogue.  dh and bf16(dy) are bit for bit the unfused GEMMs' (same MFMA,
// operands and k order); dz and the partial sums differ from sv_layernorm_bwd only by f32 summation order.
// SV_MLPB_XLANE=3: the LayerNorm epilogue's butterflies from the cross-lane unit (common.h xlane_xor) instead of
// ds_bpermute -- opt-in A/B build; round 5 measured that form non-deterministic run to run (DESIGN "Round 6").
// Bit 1: the row sums' permlane16 / permlane32 swaps; bit 2: the weight / bias partials' DPP steps (bisection builds)
#ifndef SV_MLPB_XLANE
#define SV_MLPB_XLANE 0
#endif
// SV_MLPB_PIN=1 (default): the z / mean / rstd registers are consumed only below the epilogue's counted wait
#ifndef SV_MLPB_PIN
#define SV_MLPB_PIN 1
#endif
constexpr int MAX_BWD_WG = 512;  // the grid: min(tiles, 512) workgroups (two per CU), 4 partial rows each

__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(2, 2)))
mlpb128_kernel(const uint16_t* __restrict__ d, const uint16_t* __restrict__ w2t, const uint16_t* __restrict__ gh,
               const uint16_t* __restrict__ w1t, const uint16_t* __restrict__ z, const float* __restrict__ mean,
               const float* __restrict__ rstd, const float* __restrict__ lnw, uint16_t* __restrict__ dh,
               uint16_t* __restrict__ dz, float* __restrict__ lnpart, int M) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* llw = reinterpret_cast<float*>(smem + OFF_P);   // LayerNorm weight [C]
  float* lacc = llw + C;                                  // per-wave partials [NW][2][C]
  const int lane = threadIdx.x & 63, ml = lane & 15, gq = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tiles = (M + R - 1) / R;
  const int my_tiles = (tiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;  // >= 1 (grid <= tiles)
  for (int i = threadIdx.x; i < C; i += THREADS) llw[i] = lnw[i];
  for (int i = threadIdx.x; i < NW * 2 * C; i += THREADS) lacc[i] = 0.f;

  const auto rw1 = rsrc(w2t, (uint32_t)(H * C * 2)), rw2 = rsrc(w1t, (uint32_t)(C * H * 2));
  const auto ry = rsrc(d, (uint32_t)((size_t)M * C * 2));
  const auto rg = rsrc(gh, (uint32_t)((size_t)M * H * 2));
  const auto rdh = rsrc(dh, (uint32_t)((size_t)M * H * 2));
  const auto rz = rsrc(z, (uint32_t)((size_t)M * C * 2));
  const auto rdz = rsrc(dz, (uint32_t)((size_t)M * C * 2));
  const auto rmu = rsrc(mean, (uint32_t)((size_t)M * 4));
  const auto rrs = rsrc(rstd, (uint32_t)((size_t)M * 4));
  const int p1 = 8 * wid + (lane >> 3);
  const uint32_t v1 = (uint32_t)((perm8(p1) * C + (((lane & 7) ^ kswz(p1)) << 3)) * 2);
  const int p2 = 16 * wid + (lane >> 2);
  const uint32_t v2 = (uint32_t)((p2 * H + (((lane & 3) ^ w2swz(p2)) << 3)) * 2);
  auto issue_w1 = [&](int q) {
    const int j0 = (q % NCH) * HC;
    char* st = smem + OFF_W1 + (q & 1) * W1B;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) dma(rw1, v1, (uint32_t)((j0 * C + 64 * kb) * 2), st + kb * (HC * 128) + wid * 1024);
    SV_VMTAG("w1");
  };
  auto issue_w2 = [&](int q) {
    const int j0 = (q % NCH) * HC;
    char* st = smem + OFF_W2 + (q & 1) * W2B;
#pragma unroll
    for (int h = 0; h < 2; ++h) dma(rw2, v2, (uint32_t)((64 * h * H + j0) * 2), st + (wid + 4 * h) * 1024);
    SV_VMTAG("w2");
  };
  char* ybuf = smem + OFF_Y + wid * YB;
  auto tile_row = [&](int it) { return ((int)blockIdx.x + it * (int)gridDim.x) * R + wid * 16 * RF; };
  auto issue_y = [&](int it) {
    const int wrow = tile_row(it);
#pragma unroll
    for (int rf = 0; rf < RF; ++rf) {
      const int m = wrow + 16 * rf + ml;
      const uint32_t vy = (it < my_tiles && m < M) ? (uint32_t)((m * C + 8 * gq) * 2) : OOB;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) dma(ry, vy, (uint32_t)(64 * ks), ybuf + (rf * KS + ks) * 1024);
    }
    SV_VMTAG("y");
  };
  // GELU'(h) of chunk q (tile it = q / NCH): lane -> row, 8 consecutive hidden units, loaded a chunk ahead (two
  // chunks ahead in two alternating register sets measured slower: 444 vs 426 us at base S1)
  u32x4 ghn[RF];
  auto load_gh = [&](int q) {
    const int it = q / NCH, j0 = (q % NCH) * HC, wrow = tile_row(it);
#pragma unroll
    for (int rf = 0; rf < RF; ++rf) {
      const int m = wrow + 16 * rf + ml;
      const uint32_t off = (it < my_tiles && m < M) ? (uint32_t)(((size_t)m * H + j0 + 8 * gq) * 2) : OOB;
      ghn[rf] = __builtin_amdgcn_raw_buffer_load_b128(rg, off, 0, 0);
    }
  };
  // vector-memory instructions per wave younger than each DMA a barrier waits for (cf. mlp128_kernel): GL GELU'
  // loads and SD dh stores per chunk; per tile ZL z / mean / rstd loads, ZO dz stores
  constexpr int GL = RF, SD = RF, ZL = RF * CF + 2 * RF, ZO = RF * CF;

  issue_w1(0);
  issue_w2(0);
  issue_y(0);
  vm_wait<0>();
  load_gh(0);
  __syncthreads();
  int q = 0;
  for (int it = 0; it < my_tiles; ++it) {
    const int row0 = tile_row(it);
    SV_VMWAIT(32, "y:1");  // this tile's d fragments (issued a tile ago)
    bf16x8 yf[RF][KS];
#pragma unroll
    for (int rf = 0; rf < RF; ++rf)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) yf[rf][ks] = lds_frag(ybuf + (rf * KS + ks) * 1024 + lane * 16);
    lgkm0();
    issue_y(it + 1);
    f32x4 acc2[CF][RF];
#pragma unroll
    for (int cf = 0; cf < CF; ++cf)
#pragma unroll
      for (int rf = 0; rf < RF; ++rf) acc2[cf][rf] = f32x4{0.f, 0.f, 0.f, 0.f};
    u32x2 zr[RF][CF];
    float mu[RF], rs[RF];

    for (int ch = 0; ch < NCH; ++ch, ++q) {
#if defined(SV_MLPB_DIAG) && (SV_MLPB_DIAG & 2)
      vm_wait<0>();
#endif
      // X_q: W1(q) (here (W2 gamma)^T) landed; younger: the previous chunk's GELU' loads and dh stores, W2(q); across
      // a tile boundary also the z / mean / rstd loads, the dz stores and the d prefetch
      if (ch == 0) SV_VMWAIT(GL + SD + N2 + ZL + ZO + YP, "w1:1");
      else SV_VMWAIT(GL + SD + N2, "w1:1");
      lgkm0();
      bar();
      issue_w1(q + 1);
      u32x4 ghc[RF];
#pragma unroll
      for (int rf = 0; rf < RF; ++rf) ghc[rf] = ghn[rf];
      load_gh(q + 1);
      if (ch == NCH - 1) {  // the LayerNorm backward's operands, a chunk ahead
#pragma unroll
        for (int rf = 0; rf < RF; ++rf) {
          const int m = row0 + 16 * rf + ml;
#pragma unroll
          for (int cf = 0; cf < CF; ++cf) {
            const uint32_t off = m < M ? (uint32_t)(((size_t)m * C + 16 * cf + 4 * gq) * 2) : OOB;
            zr[rf][cf] = __builtin_amdgcn_raw_buffer_load_b64(rz, off, 0, 0);
          }
          const uint32_t mo = m < M ? (uint32_t)(m * 4) : OOB;
          mu[rf] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rmu, mo, 0, 0));
          rs[rf] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rrs, mo, 0, 0));
        }
        SV_VMTAG("zl");
      }
      const char* st1 = smem + OFF_W1 + (q & 1) * W1B;
      const int j0 = ch * HC;
      // stage 1: dA^T chunk [32 hidden (perm8)] x [32 rows] = (W2 gamma)^T . d^T, k (channels) ascending
      f32x4 acc1[2][RF];
#pragma unroll
      for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int rf = 0; rf < RF; ++rf) acc1[hf][rf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const char* img = st1 + (ks >> 1) * (HC * 128);
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
          const bf16x8 wf = frag_k(img, 16 * hf, ks & 1);
#pragma unroll
          for (int rf = 0; rf < RF; ++rf)
            acc1[hf][rf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, yf[rf][ks], acc1[hf][rf], 0, 0, 0);
        }
      }
      // dh = dA (.) GELU'(h) (the x GELU' epilogue's arithmetic), stored bf16; the packed value is stage 2's operand
      bf16x8 pf[RF];
#pragma unroll
      for (int rf = 0; rf < RF; ++rf) {
        const uint32_t wd[4] = {ghc[rf].x, ghc[rf].y, ghc[rf].z, ghc[rf].w};
        float o[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = acc1[0][rf][r] * __uint_as_float((r & 1) ? (wd[r >> 1] & 0xffff0000u) : (wd[r >> 1] << 16));
          o[4 + r] = acc1[1][rf][r] * __uint_as_float(((4 + r) & 1) ? (wd[(4 + r) >> 1] & 0xffff0000u)
                                                                      : (wd[(4 + r) >> 1] << 16));
        }
        const u32x4 pk = pack8(o);
        pf[rf] = __builtin_bit_cast(bf16x8, pk);
        const int m = row0 + 16 * rf + ml;
        const uint32_t off = m < M ? (uint32_t)(((size_t)m * H + j0 + 8 * gq) * 2) : OOB;
        __builtin_amdgcn_raw_buffer_store_b128(pk, rdh, off, 0, 0);
      }
      // Y_q: W2(q) (here W1^T) landed; younger: W1(q+1), the GELU' loads, this chunk's dh stores; in a tile's first
      // chunk also the dz stores and the d prefetch, in its last the LayerNorm operand loads
      if (ch == 0) SV_VMWAIT(ZO + YP + N1 + GL + SD, "w2:1");
      else if (ch == NCH - 1) SV_VMWAIT(N1 + GL + ZL + SD, "w2:1");
      else SV_VMWAIT(N1 + GL + SD, "w2:1");
      lgkm0();
      bar();
      issue_w2(q + 1);
      // stage 2: dy^T += W1^T[:, chunk] . dh^T, k (hidden) ascending
      const char* st2 = smem + OFF_W2 + (q & 1) * W2B;
#pragma unroll
      for (int cf = 0; cf < CF; ++cf) {
        const bf16x8 wf = frag64(st2, 16 * cf);
#pragma unroll
        for (int rf = 0; rf < RF; ++rf)
          acc2[cf][rf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, pf[rf], acc2[cf][rf], 0, 0, 0);
      }
    }
#if defined(SV_MLPB_DIAG) && (SV_MLPB_DIAG & 1)
    vm_wait<0>();
#endif
    // the z / mean / rstd loads (last chunk): younger only that chunk's dh stores and the W2 DMA.  Explicit: the
    // compiler's own wait here was short (tools/mlp_bwd_diag.py: dz / dw differed run to run at M = 524288 without it)
    SV_VMWAIT(SD + N2, "zl:1");
#if SV_MLPB_PIN
    // the operands pass through the wait: no consumer can be scheduled above it under a vmcnt of the compiler's own
    // (DESIGN "Round 6": the compiler's waits for these loads count on in-order retirement behind younger stores and
    // LDS-DMA; with the consumers hoisted that way the cross-lane build's dz / dw differed run to run)
#pragma unroll
    for (int rf = 0; rf < RF; ++rf) {
#pragma unroll
      for (int cf = 0; cf < CF; ++cf) asm volatile("" : "+v"(zr[rf][cf]));
      asm volatile("" : "+v"(mu[rf]), "+v"(rs[rf]));
    }
#endif
    float* la = lacc + wid * 2 * C;
#pragma unroll
    for (int rf = 0; rf < RF; ++rf) {
      const int m = row0 + 16 * rf + ml;
      auto dyv = [&](int cf, int w) { return __uint_as_float((uint32_t)f2bf(acc2[cf][rf][w]) << 16); };
      auto xhat = [&](int cf, int w) {
        const uint32_t zw = w < 2 ? zr[rf][cf].x : zr[rf][cf].y;
        const float zz = __uint_as_float((w & 1) ? (zw & 0xffff0000u) : (zw << 16));
        return (zz - mu[rf]) * rs[rf];
      };
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int cf = 0; cf < CF; ++cf) {
        float lw[4];
        lds_f4(llw + 16 * cf + 4 * gq, lw);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float g = dyv(cf, w) * lw[w];
          s1 += g;
          s2 += g * xhat(cf, w);
        }
      }
#if SV_MLPB_XLANE & 1
      s1 += xlane_xor<16>(s1);
      s1 += xlane_xor<32>(s1);
      s2 += xlane_xor<16>(s2);
      s2 += xlane_xor<32>(s2);
#else
      s1 += __shfl_xor(s1, 16);
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 16);
      s2 += __shfl_xor(s2, 32);
#endif
      s1 *= 1.0f / (float)C;
      s2 *= 1.0f / (float)C;
#pragma unroll
      for (int cf = 0; cf < CF; ++cf) {
        float lw[4], o[4], pw[4], pb[4];
        lds_f4(llw + 16 * cf + 4 * gq, lw);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const float dv = dyv(cf, w), xh = xhat(cf, w);
          o[w] = rs[rf] * (dv * lw[w] - s1 - xh * s2);
          {
            // the product rounded once, before the butterfly: contracted into its first add (fma), a lane would add its
            // partner's ROUNDED product to its own exact one -- the two lanes of a pair would differ
#pragma clang fp contract(off)
            pw[w] = dv * xh;
          }
          pb[w] = dv;
        }
        const uint32_t off = m < M ? (uint32_t)(((size_t)m * C + 16 * cf + 4 * gq) * 2) : OOB;
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{pack2bf(o[0], o[1]), pack2bf(o[2], o[3])}, rdz, off, 0, 0);
        // the LayerNorm weight / bias partials of these 4 channels over the 16 rows of the fragment (fixed xor order);
        // lane ml == 0 adds them into the wave's own LDS row (one writer per word: deterministic)
#pragma unroll
        for (int w = 0; w < 4; ++w)
#if SV_MLPB_XLANE & 2
        {
          pw[w] += xlane_xor<1>(pw[w]);
          pb[w] += xlane_xor<1>(pb[w]);
          pw[w] += xlane_xor<2>(pw[w]);
          pb[w] += xlane_xor<2>(pb[w]);
          pw[w] += xlane_xor<4, true>(pw[w]);  // quads uniform after xor 1 and 2
          pb[w] += xlane_xor<4, true>(pb[w]);
          pw[w] += xlane_xor<8>(pw[w]);
          pb[w] += xlane_xor<8>(pb[w]);
        }
#else
#pragma unroll
          for (int sh = 1; sh < 16; sh <<= 1) {
            pw[w] += __shfl_xor(pw[w], sh);
            pb[w] += __shfl_xor(pb[w], sh);
          }
#endif
        if (ml == 0) {
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            la[16 * cf + 4 * gq + w] += pw[w];
            la[C + 16 * cf + 4 * gq + w] += pb[w];
          }
        }
      }
    }
  }
  vm_wait<0>();
  __syncthreads();
  // the workgroup's 4 wave partials -> lnpart [2][gridDim.x * NW][C]
  const int np = (int)gridDim.x * NW;
  for (int i = threadIdx.x; i < NW * 2 * C; i += THREADS) {
    const int wv = i / (2 * C), k = (i / C) & 1, c = i % C;
    lnpart[((size_t)k * np + (size_t)blockIdx.x * NW + wv) * C + c] = lacc[i];
  }
}

static int launch_bwd(const uint16_t* d, const uint16_t* w2t, const uint16_t* gh, const uint16_t* w1t, const uint16_t* z,
                      const float* mean, const float* rstd, const float* lnw, uint16_t* dh, uint16_t* dz, float* lnpart,
                      int M, hipStream_t s) {
  if (const int rc = ensure_lds_attr(reinterpret_cast<const void*>(&mlpb128_kernel), LDS_BWD, s)) return rc;
  const int tiles = (M + R - 1) / R;
  const int grid = tiles < MAX_BWD_WG ? tiles : MAX_BWD_WG;
  mlpb128_kernel<<<grid, THREADS, LDS_BWD, s>>>(d, w2t, gh, w1t, z, mean, rstd, lnw, dh, dz, lnpart, M);
  return check_launch("sv_mlp_bwd");
}
}  // namespace c128

// ---- C = 512 (ConvNeXt-base S3: 27 blocks of 32768 rows at bs32).  A wave's C-wide fc2 accumulator and its y
// fragments grow with rows x C: at C = 512 a 16-row wave needs 128 + 64 registers, so at two waves per SIMD a wave
// holds 16 rows and every W fragment it reads from LDS feeds ONE MFMA (the LDS array at its 256 B/clk at full MFMA
// rate).  Here fc1 and fc2 split the tile differently: in fc1 each of the 8 waves computes its own 16 rows (y in
// registers, one MFMA per W1 fragment); its GELU(h) chunk (16 rows x 32 hidden, already in the MFMA operand layout)
// goes through an LDS slot of its own; in fc2 the wave pair (2 rg, 2 rg + 1) shares rows 32 rg .. + 31 and each
// takes half the 512 channels, so every W2 fragment feeds two MFMAs (32 rows) against a 16 x 2 fragment
// accumulator: 50 instead of 64 KiB of LDS reads per wave and chunk.  Chunks of 32 hidden units (W1 image [8][32][64],
// W2 image [512][32] with 64-B rows), double-buffered by group A's LDS-DMA; waves 4-7 one barrier behind (their GELU
// beside the others' MFMAs, as the general kernel).  Operands, k order and epilogue arithmetic are v9's: bit for bit
// the two-GEMM path.  MEASURED SLOWER than the two GEMMs (r10o / r10p, tools/mlp_bench.py base-S3: train 231 vs 191 us,
// eval 188 vs 160; with the GELU, the weight DMA and the barriers all compiled out still 164 us in eval against a
// 55 us MFMA floor: one W1 fragment per MFMA in fc1 and a 3-deep read pipeline at 256 VGPRs leave the LDS latency
// exposed), so the host leaves it off (convnext.py fused_mlp_c; SV_FUSED_MLP_C=128,192,256,512 turns it on).
namespace c512 {
constexpr int C = 512, H = 2048, HC = 32, NCH = H / HC, KB = C / 64, KS = C / 32, NW = 8, THREADS = 512;
constexpr int CF2 = C / 2 / 16;                 // fc2 output fragments per wave (its half of the channels)
constexpr int R = NW * 16;                      // 128 rows per tile
constexpr int W1B = KB * HC * 128;              // [8][32][64] bf16 = 32 KiB
constexpr int W2B = C * HC * 2;                 // [512][32] bf16 = 32 KiB
constexpr int OFF_W1 = 0, OFF_W2 = 2 * W1B, OFF_PB = OFF_W2 + 2 * W2B, OFF_P = OFF_PB + NW * 1024;
constexpr int LDS = OFF_P + (H + 2 * C) * 4;    // 148 KiB: one workgroup per CU
constexpr int N1 = KB, N2 = C / 64;             // DMA pieces per group-A wave per chunk: W1, W2
using c128::frag64;
using c128::w2swz;
using c128::lds_frag;
// the lane id from an asm statement the compiler cannot hoist: the per-lane offsets derived from it inside the chunk
// loop are recomputed each chunk (a few VALU) instead of held across it -- at 256 VGPRs the held ones were spilled
// and their reloads waited vmcnt(0), draining the weight DMA every chunk
__device__ __forceinline__ int lane_id() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}
__device__ __forceinline__ bf16x8 frag_k_l(const char* __restrict__ region, int base, int kh, int l) {
  const int row = base + (l & 15), ch = kh * 4 + (l >> 4);
  return *reinterpret_cast<const bf16x8*>(region + row * 128 + ((ch ^ kswz(row)) << 4));
}
__device__ __forceinline__ bf16x8 frag64_l(const char* __restrict__ region, int base, int l) {
  const int row = base + (l & 15);
  return *reinterpret_cast<const bf16x8*>(region + row * 64 + (((l >> 4) ^ w2swz(row)) << 4));
}
// LDS fragment reads software-pipelined by hand: at 256 VGPRs the compiler issues each read right before its MFMA
// (ds_read; s_waitcnt lgkmcnt(0); MFMA).  Inline-asm ds_read_b128 (the compiler inserts no wait for them) PD reads
// ahead; before a fragment's MFMAs a counted lgkmcnt wait that takes the fragment as an in/out operand, so the MFMA
// cannot be scheduled above it.  LDS reads return in order: lgkmcnt(n) = at most the n younger reads outstanding.
constexpr int PD = 4;
__device__ __forceinline__ bf16x8 ds_frag(uint32_t ad) {
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  f32x4_t u;
  asm volatile("ds_read_b128 %0, %1" : "=v"(u) : "v"(ad) : "memory");
  return __builtin_bit_cast(bf16x8, u);
}
template <int N>
__device__ __forceinline__ void lgkm_dep(bf16x8& f) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(f) : "n"(N));
}
// fragment i of an L-read sequence issued PD ahead: younger reads outstanding min(PD - 1, L - 1 - i)
__device__ __forceinline__ void wait_frag(bf16x8& f, int i, int L) {
  const int n = L - 1 - i < PD - 1 ? L - 1 - i : PD - 1;
  if (n >= 3) lgkm_dep<3>(f);
  else if (n == 2) lgkm_dep<2>(f);
  else if (n == 1) lgkm_dep<1>(f);
  else lgkm_dep<0>(f);
}
static_assert(PD == 4, "wait_frag's ladder");
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p);
}
__device__ __forceinline__ void lds_st16(char* p, u32x4 v) {  // LDS store the compiler does not see (see lds_f8)
  const uint32_t ad = (uint32_t)(size_t)(const __attribute__((address_space(3))) char*)(p);
  asm volatile("ds_write_b128 %0, %1" : : "v"(ad), "v"(v) : "memory");
}

template <bool TRAIN>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(2, 2)))
mlp512_kernel(const uint16_t* __restrict__ y, const uint16_t* __restrict__ w1, const float* __restrict__ b1,
              const uint16_t* __restrict__ w2, const float* __restrict__ b2, const float* __restrict__ gamma,
              const float* __restrict__ x, float* __restrict__ xo, uint16_t* __restrict__ gh, uint16_t* __restrict__ a,
              int M) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* lb1 = reinterpret_cast<float*>(smem + OFF_P);
  float* lb2 = lb1 + H;
  float* lgam = lb2 + C;
  const int lane = threadIdx.x & 63, ml = lane & 15, gq = lane >> 4;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = wid >> 2, wa = wid & 3, rg = wid >> 1, chh = wid & 1;
  const int tiles = (M + R - 1) / R;
  const int my_tiles = (tiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;  // >= 1 (grid <= tiles)
  const int total = my_tiles * NCH;
  for (int i = threadIdx.x; i < H; i += THREADS) lb1[i] = b1[i];
  for (int i = threadIdx.x; i < C; i += THREADS) lb2[i] = b2[i], lgam[i] = gamma[i];

  const auto rw1 = rsrc(w1, (uint32_t)(H * C * 2)), rw2 = rsrc(w2, (uint32_t)(C * H * 2));
  const auto ry = rsrc(y, (uint32_t)((size_t)M * C * 2));
  const auto rx = rsrc(x, (uint32_t)((size_t)M * C * 4));
  const auto rxo = rsrc(xo, (uint32_t)((size_t)M * C * 4));
  const auto rgh = rsrc(TRAIN ? gh : nullptr, TRAIN ? (uint32_t)((size_t)M * H * 2) : 0u);
  const auto ra = rsrc(TRAIN ? a : nullptr, TRAIN ? (uint32_t)((size_t)M * H * 2) : 0u);
  // W1 chunk: rows [j0, j0 + 32) permuted (perm8), 8 k-blocks [32][64]; A-wave wa's piece of each = rows 8 wa .. + 7
  // W2 chunk: columns [j0, j0 + 32) of the 512 channel rows; A-wave wa's pieces = rows 16 wa + 64 h .. + 15
  auto issue_w1 = [&](int q) {
    const int ln = lane_id();
    const int p1 = 8 * wa + (ln >> 3);
    const uint32_t v1 = (uint32_t)((perm8(p1) * C + (((ln & 7) ^ kswz(p1)) << 3)) * 2);
    const int j0 = (q % NCH) * HC;
    char* st = smem + OFF_W1 + (q & 1) * W1B;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) dma(rw1, v1, (uint32_t)((j0 * C + 64 * kb) * 2), st + kb * (HC * 128) + wa * 1024);
    SV_VMTAG("w1");
  };
  auto issue_w2 = [&](int q) {
    const int ln = lane_id();
    const int p2 = 16 * wa + (ln >> 2);
    const uint32_t v2 = (uint32_t)((p2 * H + (((ln & 3) ^ w2swz(p2)) << 3)) * 2);
    const int j0 = (q % NCH) * HC;
    char* st = smem + OFF_W2 + (q & 1) * W2B;
#pragma unroll
    for (int h = 0; h < N2; ++h) dma(rw2, v2, (uint32_t)((64 * h * H + j0) * 2), st + (wa + 4 * h) * 1024);
    SV_VMTAG("w2");
  };
  // P slots: this wave's GELU(h) chunk (register image) at OFF_PB + 1 KiB wid; the pair's two at 1 KiB (2 rg + rf)
  constexpr int S = TRAIN ? 2 : 0;  // the dual epilogue's stores per chunk

  if (grp == 0) {
    issue_w1(0);
    issue_w2(0);
  }
  int q = 0;
  for (int it = 0; it < my_tiles; ++it) {
    const int t0 = ((int)blockIdx.x + it * (int)gridDim.x) * R;
    const int row1 = t0 + 16 * wid;  // fc1 rows of this wave
    bf16x8 yf[KS];
    {
      const int m = row1 + ml;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const uint32_t off = m < M ? (uint32_t)((m * C + 32 * ks + 8 * gq) * 2) : OOB;
        yf[ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0));
      }
    }
    // everything in flight lands here, once per tile: y, chunk 0's weights (group A), the previous tile's x_out
    vm_wait<0>();
    if (it == 0) {
      __syncthreads();  // the per-channel vectors and chunk 0 (group A's DMA) for every wave
      if (grp == 1) bar();  // group B one barrier behind
    }
    f32x4 acc2[CF2][2];
#pragma unroll
    for (int cf = 0; cf < CF2; ++cf)
#pragma unroll
      for (int rf = 0; rf < 2; ++rf) acc2[cf][rf] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int ch = 0; ch < NCH; ++ch, ++q) {
      // X_q: W1(q) landed (A: issued after X_{q-1}; younger: chunk q-1's stores, W2(q)'s pieces)
      if (grp == 0 && ch > 0) SV_VMWAIT(S + N2, "w1:1");
      lgkm0();
      if (!(SV_MLP_DIAG & 4)) bar();
      // unconditional (past the end: a harmless re-load of chunk 0 into the free slot): every chunk issues the same
      // vector-memory instructions, which the counted waits assume.  Round 5 skipped it for q + 1 == total, which left
      // the last chunk's Y wait with fewer younger instructions than its count: W2 of a workgroup's last chunk was not
      // covered (tools/check_vmcnt.py found it)
      if (grp == 0 && !(SV_MLP_DIAG & 2)) issue_w1(q + 1);
      const int ln = lane_id();
      const char* st1 = smem + OFF_W1 + (q & 1) * W1B;
      const int j0 = ch * HC;
      // fc1: h^T chunk [32 hidden (2 fragments, perm8 rows)] x [16 rows], k ascending
      f32x4 acc1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      {
        // fragment i = (ks, hf) = (i >> 1, i & 1): frag_k(st1 + (ks >> 1) * 4 KiB, 16 hf, ks & 1); row 16 hf + (l & 15)
        // has the swizzle of row l & 15 (kswz ignores bit 4)
        const int r = ln & 15, sw = kswz(r);
        const uint32_t b1a = lds_addr(st1) + (uint32_t)(r * 128);
        const uint32_t c0 = (uint32_t)((((ln >> 4)) ^ sw) << 4), c1 = (uint32_t)(((4 + (ln >> 4)) ^ sw) << 4);
        auto rd = [&](int i) {
          return ds_frag(b1a + (uint32_t)((i >> 2) * (HC * 128) + (i & 1) * (16 * 128)) + (((i >> 1) & 1) ? c1 : c0));
        };
        bf16x8 fr[2 * KS];
#pragma unroll
        for (int i = 0; i < PD; ++i) fr[i] = rd(i);
#pragma unroll
        for (int i = 0; i < 2 * KS; ++i) {
          wait_frag(fr[i], i, 2 * KS);
          acc1[i & 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[i], yf[i >> 1], acc1[i & 1], 0, 0, 0);
          if (i + PD < 2 * KS) fr[i + PD] = rd(i + PD);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // bias + GELU pair (v9's packed form); P = bf16 GELU(h) into this wave's LDS slot (fc2's operand image).  The
      // bias is read only now: during fc1 its 8 registers deepen the fragment prefetch instead
      {
        float bia[8];
        lds_f8(lb1 + j0 + 8 * (ln >> 4), bia);
        float v[8], o[8], o2[8];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc1[0][r], v[4 + r] = acc1[1][r];
#pragma unroll
        for (int w = 0; w < 8; ++w) v[w] += bia[w];
#pragma unroll
        for (int w = 0; w < 8; w += 2) {
          const gelu_f2 hh = {v[w], v[w + 1]};
          gelu_f2 ph, de;
#if SV_MLP_DIAG & 1
          ph = (gelu_f2){1.0f, 1.0f}, de = hh;  // diagnostic: no GELU arithmetic (results wrong)
#else
          gelu_parts2(hh, ph, de);
#endif
          const gelu_f2 g = hh * ph;
          o2[w] = g.x, o2[w + 1] = g.y;
          if constexpr (TRAIN) {
            const gelu_f2 dg = __builtin_elementwise_fma(hh, de, ph);
            o[w] = dg.x, o[w + 1] = dg.y;
          }
        }
        const u32x4 pk = pack8(o2);
        lds_st16(smem + OFF_PB + wid * 1024 + ln * 16, pk);
        if constexpr (TRAIN) {
          const int m = row1 + (ln & 15);
          const uint32_t off = m < M ? (uint32_t)(((size_t)m * H + j0 + 8 * (ln >> 4)) * 2) : OOB;
          __builtin_amdgcn_raw_buffer_store_b128(pack8(o), rgh, off, 0, kGradCpol);
          __builtin_amdgcn_raw_buffer_store_b128(pk, ra, off, 0, kGradCpol);
        } else {
          (void)o;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      // Y_q: W2(q) landed (A: issued after Y_{q-1}; younger: W1(q+1)'s pieces, this chunk's stores); every wave of the
      // group wrote its P slot
      if (grp == 0) SV_VMWAIT(N1 + S, "w2:1");
      lgkm0();
      if (!(SV_MLP_DIAG & 4)) bar();
      if (grp == 0 && !(SV_MLP_DIAG & 2)) issue_w2(q + 1);
      // fc2: acc2 += W2[half, chunk] . P^T over the pair's 32 rows, k (hidden) ascending
      {
        const int ln2 = lane_id();
        bf16x8 pf[2];
        pf[0] = lds_frag(smem + OFF_PB + (2 * rg) * 1024 + ln2 * 16);
        pf[1] = lds_frag(smem + OFF_PB + (2 * rg + 1) * 1024 + ln2 * 16);
        // fragment cf: frag64(st2, 16 cf) = st2 + 1 KiB cf + the lane's offset (row l & 15: the swizzle of every
        // 16-row block is the same)
        const int r = ln2 & 15;
        const uint32_t b2a = lds_addr(smem + OFF_W2 + (q & 1) * W2B + chh * (256 * 64)) +
                             (uint32_t)(r * 64 + (((ln2 >> 4) ^ w2swz(r)) << 4));
        auto rd = [&](int cf) { return ds_frag(b2a + (uint32_t)(cf * 1024)); };
        bf16x8 fr[CF2];
#pragma unroll
        for (int i = 0; i < PD; ++i) fr[i] = rd(i);
        lgkm_dep<PD>(pf[0]);  // the two P reads were issued before the PD fragment reads
        lgkm_dep<PD>(pf[1]);
#pragma unroll
        for (int cf = 0; cf < CF2; ++cf) {
          wait_frag(fr[cf], cf, CF2);
#pragma unroll
          for (int rf = 0; rf < 2; ++rf)
            acc2[cf][rf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fr[cf], pf[rf], acc2[cf][rf], 0, 0, 0);
          if (cf + PD < CF2) fr[cf + PD] = rd(cf + PD);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // epilogue: x_out = gamma (.) (acc + b2) + x   (v9's gamma-residual arithmetic); rows 32 rg + 16 rf + (l & 15),
    // channels 256 chh + 16 cf + 4 gq .. +3; x loaded 8 fragments at a time
#pragma unroll
    for (int rf = 0; rf < 2; ++rf) {
      const int m = t0 + 32 * rg + 16 * rf + ml;
#pragma unroll
      for (int c8 = 0; c8 < CF2; c8 += 8) {
        u32x4 xr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = 256 * chh + 16 * (c8 + j) + 4 * gq;
          const uint32_t off = m < M ? (uint32_t)(((size_t)m * C + c) * 4) : OOB;
          xr[j] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
        }
        vm_wait<0>();  // explicit (a compiler wait once fell short at a fused kernel's epilogue: sv_mlp_bwd)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int c = 256 * chh + 16 * (c8 + j) + 4 * gq;
          float bv[4], gv[4];
          lds_f4x2(lb2 + c, lgam + c, bv, gv);
          const uint32_t xw[4] = {xr[j].x, xr[j].y, xr[j].z, xr[j].w};
          float o[4];
#pragma unroll
          for (int w = 0; w < 4; ++w) o[w] = fmaf(gv[w], acc2[c8 + j][rf][w] + bv[w], __uint_as_float(xw[w]));
          const uint32_t off = m < M ? (uint32_t)(((size_t)m * C + c) * 4) : OOB;
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{__float_as_uint(o[0]), __float_as_uint(o[1]),
                                                       __float_as_uint(o[2]), __float_as_uint(o[3])},
                                                 rxo, off, 0, 0);
        }
      }
    }
  }
  if (grp == 0) bar();  // the barrier group B is behind
  vm_wait<0>();  // no LDS-DMA may land after the workgroup's LDS is released
}

template <bool TRAIN>
static int launch(const uint16_t* y, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
                  const float* gamma, const float* x, float* xo, uint16_t* gh, uint16_t* a, int M, hipStream_t s) {
  if (const int rc = ensure_lds_attr(reinterpret_cast<const void*>(&mlp512_kernel<TRAIN>), LDS, s)) return rc;
  const int tiles = (M + R - 1) / R;
  const int slots = device_cus(s);
  const int grid = tiles < slots ? tiles : slots;
  mlp512_kernel<TRAIN><<<grid, THREADS, LDS, s>>>(y, w1, b1, w2, b2, gamma, x, xo, gh, a, M);
  return check_launch("sv_mlp_fwd");
}
}  // namespace c512

template <int C, bool TRAIN>
static int launch(const uint16_t* y, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
                  const float* gamma, const float* x, float* xo, uint16_t* gh, uint16_t* a, int M, hipStream_t s) {
  using K = Cfg<C>;
  if (const int rc = ensure_lds_attr(reinterpret_cast<const void*>(&mlp_fwd_kernel<C, TRAIN>), K::LDS, s)) return rc;
  const int tiles = (M + K::R - 1) / K::R;
  const int slots = K::WG_PER_CU * device_cus(s);
  const int grid = tiles < slots ? tiles : slots;
  mlp_fwd_kernel<C, TRAIN><<<grid, K::THREADS, K::LDS, s>>>(y, w1, b1, w2, b2, gamma, x, xo, gh, a, M);
  return check_launch("sv_mlp_fwd");
}

}  // namespace mlp
}  // namespace sv

namespace {
// SV_MLP128_V1=1: C = 128 on the general kernel (A/B runs)
bool getenv_flag_mlp_v1() {
  static const bool v = [] {
    const char* e = getenv("SV_MLP128_V1");
    return e && e[0] == '1';
  }();
  return v;
}
}  // namespace

extern "C" {

int sv_mlp_fwd(const uint16_t* y, const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
               const float* gamma, const float* x, float* x_out, uint16_t* gelu_grad, uint16_t* gelu_out, int64_t M,
               int32_t C, sv_stream_t stream) {
  using namespace sv;
  SV_REQUIRE(y && w1 && b1 && w2 && b2 && gamma && x && x_out, "sv_mlp_fwd: null pointer");
  SV_REQUIRE(M > 0 && M * 4 * C * 2 < 0x7fffffffLL, "sv_mlp_fwd: M out of range (the hidden tensor must be < 2 GiB)");
  SV_REQUIRE((gelu_grad == nullptr) == (gelu_out == nullptr), "sv_mlp_fwd: GELU'(h) and GELU(h) are stored together");
  SV_REQUIRE(x != x_out, "sv_mlp_fwd: x_out must not alias x");
  SV_REQUIRE(C == 128 || C == 192 || C == 256 || C == 512, "sv_mlp_fwd: C = %d not supported (128, 192, 256, 512)", C);
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  SV_REQUIRE(al(y) && al(w1) && al(w2) && al(b1) && al(b2) && al(gamma) && al(x) && al(x_out) && al(gelu_grad) &&
                 al(gelu_out),
             "sv_mlp_fwd: every pointer must be 16-B aligned");
  const hipStream_t s = (hipStream_t)stream;
  const bool tr = gelu_grad != nullptr;
  const int m = (int)M;
#define SV_MLP_CASE(CC)                                                                                           \
  case CC:                                                                                                        \
    return tr ? mlp::launch<CC, true>(y, w1, b1, w2, b2, gamma, x, x_out, gelu_grad, gelu_out, m, s)              \
              : mlp::launch<CC, false>(y, w1, b1, w2, b2, gamma, x, x_out, nullptr, nullptr, m, s);
  if (C == 128 && !getenv_flag_mlp_v1())
    return tr ? mlp::c128::launch<true>(y, w1, b1, w2, b2, gamma, x, x_out, gelu_grad, gelu_out, m, s)
              : mlp::c128::launch<false>(y, w1, b1, w2, b2, gamma, x, x_out, nullptr, nullptr, m, s);
  if (C == 512)
    return tr ? mlp::c512::launch<true>(y, w1, b1, w2, b2, gamma, x, x_out, gelu_grad, gelu_out, m, s)
              : mlp::c512::launch<false>(y, w1, b1, w2, b2, gamma, x, x_out, nullptr, nullptr, m, s);
  switch (C) {
    SV_MLP_CASE(128)
    SV_MLP_CASE(192)
    SV_MLP_CASE(256)
  }
#undef SV_MLP_CASE
  return set_error(SV_ERR_INVALID_ARG, "sv_mlp_fwd: C = %d not supported", C);
}

int sv_mlp_bwd_nparts(int64_t M, int32_t C) {
  if (C != 128 || M <= 0) return 0;
  const int64_t tiles = (M + sv::mlp::c128::R - 1) / sv::mlp::c128::R;
  return (int)((tiles < sv::mlp::c128::MAX_BWD_WG ? tiles : sv::mlp::c128::MAX_BWD_WG) * sv::mlp::c128::NW);
}

int sv_mlp_bwd(const uint16_t* d, const uint16_t* w2t, const uint16_t* gelu_grad, const uint16_t* w1t, const uint16_t* z,
               const float* mean, const float* rstd, const float* lnw, uint16_t* dh, uint16_t* dz, float* ln_part,
               int64_t M, int32_t C, sv_stream_t stream) {
  using namespace sv;
  SV_REQUIRE(d && w2t && gelu_grad && w1t && z && mean && rstd && lnw && dh && dz && ln_part, "sv_mlp_bwd: null pointer");
  SV_REQUIRE(C == 128, "sv_mlp_bwd: C = %d not supported (128)", C);
  SV_REQUIRE(M > 0 && M * 4 * C * 2 < 0x7fffffffLL, "sv_mlp_bwd: M out of range (the hidden tensor must be < 2 GiB)");
  auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  SV_REQUIRE(al(d) && al(w2t) && al(gelu_grad) && al(w1t) && al(z) && al(mean) && al(rstd) && al(lnw) && al(dh) &&
                 al(dz) && al(ln_part),
             "sv_mlp_bwd: every pointer must be 16-B aligned");
  return mlp::c128::launch_bwd(d, w2t, gelu_grad, w1t, z, mean, rstd, lnw, dh, dz, ln_part, (int)M, (hipStream_t)stream);
}

}  // extern "C"
