// Shared pieces of the MFMA GEMM kernels (gemm.hip: register-staged v1 for the f32 parity mode and
// odd shapes; gemm2.hip: LDS-DMA pipelined v2 for bf16): epilogue arguments, the fused epilogue
// math and the LDS-staged wave-tile store.
#pragma once

#include "common.h"

// statistics epilogues' column folds from the cross-lane unit (common.h xlane_xor; bitwise the ds_bpermute shuffles,
// -DSV_STATS_XLANE=0 keeps those: A/B builds)
#ifndef SV_STATS_XLANE
#define SV_STATS_XLANE SV_XLANE
#endif

namespace sv {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int EPI_LD = 64 + 4;  // f32 epilogue slab row stride (floats)

struct EpiArgs {
  int M, N;
  int epi;
  void* C; int c_dtype; int64_t ldc;
  void* C2; int c2_dtype;
  const float* bias;
  const float* gamma;
  const void* aux; int aux_dtype; int64_t ld_aux;
  int prio = 0;  // 1: the kernel's waves issue at raised priority (sv_gemm_set_priority)
  // SV_EPI_STORE_BN_BWD: the BatchNorm's batch mean / rstd and beta (gamma in `gamma`, its input in aux)
  const float* bn_mu = nullptr;
  const float* bn_rs = nullptr;
  const float* bn_be = nullptr;
  // remapped rows (the v3 kernel's stride-2 dgrad, mode 5, storing straight into dx): GEMM row m of
  // parity class `split` = (b, gy, gx) on the class's GH x GW grid -> output row
  // (b * 2GH + 2gy + py) * 2GW + 2gx + px, for the store and the epilogue operand alike; the
  // STORE_BN_BWD partial rows of class c start at row c * rm_prow
  int rm_gh = 0, rm_gw = 0, rm_prow = 0;
  uint32_t rm_gw_mul = 0, rm_gw_shift = 0, rm_ghw_mul = 0, rm_ghw_shift = 0;
};

__device__ __forceinline__ size_t remap_row(const EpiArgs& e, int m, int cls) {
  const uint32_t u = (uint32_t)m;
  const uint32_t b = (__umulhi(u, e.rm_ghw_mul) + u) >> e.rm_ghw_shift;
  const uint32_t rem = u - b * (uint32_t)(e.rm_gh * e.rm_gw);
  const uint32_t gy = (__umulhi(rem, e.rm_gw_mul) + rem) >> e.rm_gw_shift;
  const uint32_t gx = rem - gy * (uint32_t)e.rm_gw;
  const size_t y = (size_t)b * (2 * e.rm_gh) + 2 * gy + (cls >> 1);
  return y * (size_t)(2 * e.rm_gw) + 2 * gx + (cls & 1);
}

__device__ __forceinline__ float4 ld4_any(const void* p, int dt, size_t i) {
  return dt == SV_F32 ? ld4(reinterpret_cast<const float*>(p), i) : ld4(reinterpret_cast<const uint16_t*>(p), i);
}
__device__ __forceinline__ void st4_any(void* p, int dt, size_t i, float4 v) {
  if (dt == SV_F32) st4(reinterpret_cast<float*>(p), i, v);
  else st4(reinterpret_cast<uint16_t*>(p), i, v);
}

// apply the epilogue to 4 consecutive columns n..n+3 of row m
__device__ __forceinline__ void epi4(const EpiArgs& e, int m, int n, float4 v, int split) {
  if (e.epi == SV_EPI_SLAB) {
    float* C = reinterpret_cast<float*>(e.C) + (size_t)split * e.M * e.N;
    *reinterpret_cast<float4*>(C + (size_t)m * e.N + n) = v;
    return;
  }
  if (e.bias && e.epi != SV_EPI_GELU_GRAD) {
    const float4 b = *reinterpret_cast<const float4*>(e.bias + n);
    v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
  }
  const size_t ci = (size_t)m * e.ldc + n;
  if (e.epi == SV_EPI_STORE) {
    st4_any(e.C, e.c_dtype, ci, v);
  } else if (e.epi == SV_EPI_BIAS_GELU2) {
    st4_any(e.C, e.c_dtype, ci, v);
    st4_any(e.C2, e.c2_dtype, ci, make_float4(gelu_f(v.x), gelu_f(v.y), gelu_f(v.z), gelu_f(v.w)));
  } else if (e.epi == SV_EPI_BIAS_GELU) {
    st4_any(e.C, e.c_dtype, ci, make_float4(gelu_f(v.x), gelu_f(v.y), gelu_f(v.z), gelu_f(v.w)));
  } else if (e.epi == SV_EPI_BIAS_GAMMA_RES) {
    const float4 g = *reinterpret_cast<const float4*>(e.gamma + n);
    const float4 r = ld4_any(e.aux, e.aux_dtype, (size_t)m * e.ld_aux + n);
    st4_any(e.C, e.c_dtype, ci, make_float4(r.x + g.x * v.x, r.y + g.y * v.y, r.z + g.z * v.z, r.w + g.w * v.w));
  } else {  // SV_EPI_GELU_GRAD
    const float4 h = ld4_any(e.aux, e.aux_dtype, (size_t)m * e.ld_aux + n);
    st4_any(e.C, e.c_dtype, ci,
            make_float4(v.x * gelu_grad_f(h.x), v.y * gelu_grad_f(h.y), v.z * gelu_grad_f(h.z), v.w * gelu_grad_f(h.w)));
  }
}


// 8 consecutive elements <-> two float4 (bf16: one 16-B access, f32: two)
__device__ __forceinline__ void ld8_any(const void* p, int dt, size_t i, float4& a, float4& b) {
  if (dt == SV_F32) {
    const float* f = reinterpret_cast<const float*>(p) + i;
    a = *reinterpret_cast<const float4*>(f);
    b = *reinterpret_cast<const float4*>(f + 4);
  } else {
    const uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(p) + i);
    a = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                    __uint_as_float(u.y & 0xffff0000u));
    b = make_float4(__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u), __uint_as_float(u.w << 16),
                    __uint_as_float(u.w & 0xffff0000u));
  }
}
__device__ __forceinline__ void st8_any(void* p, int dt, size_t i, float4 a, float4 b) {
  if (dt == SV_F32) {
    float* f = reinterpret_cast<float*>(p) + i;
    *reinterpret_cast<float4*>(f) = a;
    *reinterpret_cast<float4*>(f + 4) = b;
  } else {
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p) + i) =
        make_uint4(pack2bf(a.x, a.y), pack2bf(a.z, a.w), pack2bf(b.x, b.y), pack2bf(b.z, b.w));
  }
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 gelu4(float4 v) { return make_float4(gelu_f(v.x), gelu_f(v.y), gelu_f(v.z), gelu_f(v.w)); }
__device__ __forceinline__ float4 fma4(float4 g, float4 v, float4 r) {
  return make_float4(fmaf(g.x, v.x, r.x), fmaf(g.y, v.y, r.y), fmaf(g.z, v.z, r.z), fmaf(g.w, v.w, r.w));
}
__device__ __forceinline__ float4 ggrad4(float4 v, float4 h) {
  return make_float4(v.x * gelu_grad_f(h.x), v.y * gelu_grad_f(h.y), v.z * gelu_grad_f(h.z), v.w * gelu_grad_f(h.w));
}
__device__ __forceinline__ float4 mul4(float4 a, float4 b) { return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
__device__ __forceinline__ void gelu_dual4(float4 v, float4& g, float4& dg) {
  gelu_and_grad(v.x, g.x, dg.x);
  gelu_and_grad(v.y, g.y, dg.y);
  gelu_and_grad(v.z, g.z, dg.z);
  gelu_and_grad(v.w, g.w, dg.w);
}

// Store one 64-row group (4 fragment rows) of a wave's accumulator; see wave_tile_epilogue.
// PRE: load the group's residual / pre-activation operands before its first slab (more loads in
// flight, 64 more VGPRs) or per slab (for kernels that must stay within 128 VGPRs).
// PRE: 1 = load the group's residual / pre-activation operands (as f32) before its first slab,
//      0 = per slab (each such load costs a `s_waitcnt vmcnt(0)` that also drains every store issued
//      before it), 2 = raw operand words one slab ahead (see fetch_raw).
// EPI >= 0: the epilogue kind is a compile-time constant (kernels specialised per epilogue carry
// only that epilogue's registers); EPI = -1: read e.epi at run time.
// AUXT: dtype of the epilogue operand when known at compile time (SV_F32 / SV_BF16), -1 = e.aux_dtype
// REMAP: output / operand rows through remap_row (e.rm_*, `split` = the parity class); not with SLAB
template <int FM, int PRE = 1, int FN = 4, int J0 = 0, int EPI = -1, int AUXT = -1, bool REMAP = false>
__device__ __forceinline__ void wave_group_epilogue(const f32x4 (&acc)[FM][FN], int i0, float* __restrict__ slab,
                                                    int mb, int nb, const EpiArgs& e_in, int split) {
  EpiArgs e = e_in;
  if constexpr (EPI >= 0) e.epi = EPI;
  if constexpr (AUXT >= 0) e.aux_dtype = AUXT;
  static_assert(!REMAP || (EPI >= 0 && EPI != SV_EPI_SLAB), "remapped rows: compile-time non-slab epilogues");
  auto orow = [&](int m) -> size_t {
    if constexpr (REMAP) return remap_row(e, m, split);
    else return (size_t)m;
  };
  const int l = threadIdx.x & 63;
  const int cu = (l & 7) * 8, r0 = l >> 3;
  const int n = nb + cu;
  const bool okn = n < e.N;  // N % 8 == 0 is enforced for bf16-output epilogues; f32 needs N % 4 only
  const bool okn4 = n + 4 < e.N;
  const bool slab_out = e.epi == SV_EPI_SLAB;
  const bool need_aux = e.epi == SV_EPI_BIAS_GAMMA_RES || e.epi == SV_EPI_GELU_GRAD || e.epi == SV_EPI_MUL_AUX;
  // SV_EPI_STORE_STATS (compile-time kernels only): per-lane column sums of the stored values
  constexpr bool kStats = EPI == SV_EPI_STORE_STATS;
  // SV_EPI_STORE_BN_BWD: a plain store, plus the backward statistics of the BatchNorm + ReLU whose output
  // gradient this is, summed column-per-lane from the staged slab (lane l owns column nb + l: one
  // parameter set and two sums per lane, so the epilogue stays within the kernel's register budget;
  // the mask and products are sv_bn_relu_bwd_stats', bit for bit, summed in another order)
  constexpr bool kBnb = EPI == SV_EPI_STORE_BN_BWD;
  const int bn_n = nb + l;
  const bool bn_ok = kBnb && bn_n < e.N;
  float bn_a = 0.f, bn_mu = 0.f, bn_rs = 0.f, bn_be = 0.f, bn_s1 = 0.f, bn_s2 = 0.f;
  if (bn_ok) {
    bn_mu = e.bn_mu[bn_n];
    bn_rs = e.bn_rs[bn_n];
    bn_a = e.gamma[bn_n] * bn_rs;
    bn_be = e.bn_be[bn_n];
  }
  float cs1[8], cs2[8];
  if constexpr (kStats) {
#pragma unroll
    for (int j = 0; j < 8; ++j) cs1[j] = cs2[j] = 0.f;
  }
  float4 b0 = make_float4(0.f, 0.f, 0.f, 0.f), b1 = b0, g0 = b0, g1 = b0;
  if (okn && e.bias && !slab_out && e.epi != SV_EPI_GELU_GRAD && e.epi != SV_EPI_MUL_AUX) {
    b0 = *reinterpret_cast<const float4*>(e.bias + n);
    if (okn4) b1 = *reinterpret_cast<const float4*>(e.bias + n + 4);
  }
  if (okn && e.epi == SV_EPI_BIAS_GAMMA_RES) {
    if (e.gamma) {
      g0 = *reinterpret_cast<const float4*>(e.gamma + n);
      if (okn4) g1 = *reinterpret_cast<const float4*>(e.gamma + n + 4);
    } else {  // gamma == NULL: C = aux + acc (in-place accumulate when aux == C)
      g0 = g1 = make_float4(1.f, 1.f, 1.f, 1.f);
    }
  }
  constexpr int NP = PRE == 1 ? 4 : 1;
  float4 xa[NP][2], xb[NP][2];
  // PRE == 2: raw operand words of slab i+1 are fetched before slab i is stored (one slab ahead,
  // 8 VGPRs bf16 / 16 f32), so the wait for them never covers the stores issued after them
  constexpr int RW = AUXT == SV_BF16 ? 1 : 2;  // raw words per 8 operands: bf16 1 x uint4, f32 2
  uint4 rcur[2][RW], rnxt[2][RW];
  auto fetch_raw = [&](int i, uint4 (&r)[2][RW]) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int m = mb + i * 16 + r0 + 8 * h;
#pragma unroll
      for (int q = 0; q < RW; ++q) r[h][q] = make_uint4(0, 0, 0, 0);
      if (need_aux && okn && m < e.M) {
        if (e.aux_dtype == SV_BF16) {
          if (okn4) r[h][0] = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(e.aux) + orow(m) * e.ld_aux + n);
          else r[h][0] = make_uint4(*reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint16_t*>(e.aux) + orow(m) * e.ld_aux + n),
                                    *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint16_t*>(e.aux) + orow(m) * e.ld_aux + n + 2), 0, 0);
        } else if constexpr (RW == 2) {
          const float* f = reinterpret_cast<const float*>(e.aux) + orow(m) * e.ld_aux + n;
          r[h][0] = *reinterpret_cast<const uint4*>(f);
          if (okn4) r[h][RW - 1] = *reinterpret_cast<const uint4*>(f + 4);
        }
      }
    }
  };
  auto unpack_raw = [&](const uint4 (&r)[2][RW], int h, float4& a, float4& b) {
    if (e.aux_dtype == SV_BF16) {
      const uint4 u = r[h][0];
      a = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                      __uint_as_float(u.y & 0xffff0000u));
      b = make_float4(__uint_as_float(u.z << 16), __uint_as_float(u.z & 0xffff0000u), __uint_as_float(u.w << 16),
                      __uint_as_float(u.w & 0xffff0000u));
    } else {
      a = make_float4(__uint_as_float(r[h][0].x), __uint_as_float(r[h][0].y), __uint_as_float(r[h][0].z),
                      __uint_as_float(r[h][0].w));
      b = make_float4(__uint_as_float(r[h][RW - 1].x), __uint_as_float(r[h][RW - 1].y),
                      __uint_as_float(r[h][RW - 1].z), __uint_as_float(r[h][RW - 1].w));
    }
  };
  if constexpr (PRE == 2) fetch_raw(0, rcur);
  auto load_aux = [&](int i, int slot) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      xa[slot][h] = xb[slot][h] = make_float4(0.f, 0.f, 0.f, 0.f);
      const int m = mb + i * 16 + r0 + 8 * h;
      if (need_aux && okn && m < e.M) {
        if (okn4) ld8_any(e.aux, e.aux_dtype, orow(m) * e.ld_aux + n, xa[slot][h], xb[slot][h]);
        else xa[slot][h] = ld4_any(e.aux, e.aux_dtype, orow(m) * e.ld_aux + n);
      }
    }
  };
  if constexpr (PRE == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) load_aux(i, i);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int si = PRE == 1 ? i : 0;
    if constexpr (PRE == 0) load_aux(i, 0);

    if constexpr (PRE == 2) {
      if (i + 1 < 4) fetch_raw(i + 1, rnxt);
#pragma unroll
      for (int h = 0; h < 2; ++h) unpack_raw(rcur, h, xa[0][h], xb[0][h]);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int q = 0; q < RW; ++q) rcur[h][q] = rnxt[h][q];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[(4 * (l >> 4) + r) * EPI_LD + j * 16 + (l & 15)] = acc[i0 + i][J0 + j][r];
    // kBnb: the BatchNorm input of this lane's column over the slab's 16 rows (loaded once the slab's
    // accumulators are in LDS, so their registers are free; waited on after the slab's stores are issued)
    float bn_y[16];
    if constexpr (kBnb) {
      const uint16_t* yp = reinterpret_cast<const uint16_t*>(e.aux);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + i * 16 + r;
        bn_y[r] = bn_ok && m < e.M ? __uint_as_float((uint32_t)yp[orow(m) * e.ld_aux + bn_n] << 16) : 0.f;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = r0 + 8 * h;
      const int m = mb + i * 16 + row;
      if (m >= e.M || !okn) continue;
      const float* sp = slab + row * EPI_LD + cu;
      float4 va = make_float4(sp[0], sp[1], sp[2], sp[3]);
      float4 vb = make_float4(sp[4], sp[5], sp[6], sp[7]);
      if (slab_out) {
        float* C = reinterpret_cast<float*>(e.C) + (size_t)split * e.M * e.N + (size_t)m * e.N + n;
        if (okn4) {
          st8_any(C, SV_F32, 0, va, vb);
        } else {
          *reinterpret_cast<float4*>(C) = va;
        }
        continue;
      }
      va = add4(va, b0);
      vb = add4(vb, b1);
      float4 oa, ob;
      if (e.epi == SV_EPI_STORE || e.epi == SV_EPI_BIAS_GELU2 || e.epi == SV_EPI_STORE_STATS || kBnb) {
        oa = va;
        ob = vb;
      } else if (e.epi == SV_EPI_BIAS_GELU_DUAL) {
        float4 ga, gb;
        gelu_dual4(va, ga, oa);
        gelu_dual4(vb, gb, ob);
        va = ga;  // C2 gets GELU, C gets GELU'
        vb = gb;
      } else if (e.epi == SV_EPI_BIAS_GELU) {
        oa = gelu4(va);
        ob = gelu4(vb);
      } else if (e.epi == SV_EPI_MUL_AUX) {
        oa = mul4(va, xa[si][h]);
        ob = mul4(vb, xb[si][h]);
      } else if (e.epi == SV_EPI_BIAS_GAMMA_RES) {
        oa = fma4(g0, va, xa[si][h]);
        ob = fma4(g1, vb, xb[si][h]);
      } else {
        oa = ggrad4(va, xa[si][h]);
        ob = ggrad4(vb, xb[si][h]);
      }
      const size_t ci = orow(m) * e.ldc + n;
      if (okn4) st8_any(e.C, e.c_dtype, ci, oa, ob);
      else st4_any(e.C, e.c_dtype, ci, oa);
      if constexpr (kStats) {  // N % 8 == 0: all 8 columns valid
        const float o8[8] = {oa.x, oa.y, oa.z, oa.w, ob.x, ob.y, ob.z, ob.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float q = e.c_dtype == SV_BF16 ? __uint_as_float((uint32_t)f2bf(o8[j]) << 16) : o8[j];
          cs1[j] += q;
          cs2[j] = fmaf(q, q, cs2[j]);
        }
      }
      if (e.epi == SV_EPI_BIAS_GELU2) {
        if (okn4) st8_any(e.C2, e.c2_dtype, ci, gelu4(va), gelu4(vb));
        else st4_any(e.C2, e.c2_dtype, ci, gelu4(va));
      } else if (e.epi == SV_EPI_BIAS_GELU_DUAL) {
        if (okn4) st8_any(e.C2, e.c2_dtype, ci, va, vb);
        else st4_any(e.C2, e.c2_dtype, ci, va);
      }
    }
    if constexpr (kBnb) {  // column bn_n of the slab, rows in order; values as stored (bf16)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mb + i * 16 + r;
        if (!bn_ok || m >= e.M) continue;
        const float q = __uint_as_float((uint32_t)f2bf(slab[r * EPI_LD + l]) << 16);
        const float g = fmaf(bn_a, bn_y[r] - bn_mu, bn_be) > 0.f ? q : 0.f;
        bn_s1 += g;
        bn_s2 = fmaf(g, (bn_y[r] - bn_mu) * bn_rs, bn_s2);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  if constexpr (kBnb) {  // the group's partial row [mb/64][2][N]: one writer per column
    if (bn_ok && mb < e.M) {
      const int prow = (mb >> 6) + (REMAP ? split * e.rm_prow : 0);
      float* P = reinterpret_cast<float*>(e.C2) + (size_t)prow * 2 * e.N + bn_n;
      P[0] = bn_s1;
      P[e.N] = bn_s2;
    }
  }
  if constexpr (kStats) {
    // lanes l, l+8, ..., l+56 hold the same 8 columns over the group's 64 rows: fold them (fixed
    // order, bit-stable), then lanes 0..7 write the group's partial row [mb/64][2][N] (one writer each)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#if SV_STATS_XLANE
      // the same partners from the cross-lane unit (exact xor 8 / 16 / 32): bitwise the shuffle form
      cs1[j] += xlane_xor<8>(cs1[j]);
      cs2[j] += xlane_xor<8>(cs2[j]);
      cs1[j] += xlane_xor<16>(cs1[j]);
      cs2[j] += xlane_xor<16>(cs2[j]);
      cs1[j] += xlane_xor<32>(cs1[j]);
      cs2[j] += xlane_xor<32>(cs2[j]);
#else
#pragma unroll
      for (int off = 8; off < 64; off <<= 1) {
        cs1[j] += __shfl_xor(cs1[j], off);
        cs2[j] += __shfl_xor(cs2[j], off);
      }
#endif
    }
    if (l < 8 && okn && mb < e.M) {  // groups wholly past M have no partial row
      float* P = reinterpret_cast<float*>(e.C2) + (size_t)(mb >> 6) * 2 * e.N + n;
      *reinterpret_cast<float4*>(P) = make_float4(cs1[0], cs1[1], cs1[2], cs1[3]);
      *reinterpret_cast<float4*>(P + 4) = make_float4(cs1[4], cs1[5], cs1[6], cs1[7]);
      *reinterpret_cast<float4*>(P + e.N) = make_float4(cs2[0], cs2[1], cs2[2], cs2[3]);
      *reinterpret_cast<float4*>(P + e.N + 4) = make_float4(cs2[4], cs2[5], cs2[6], cs2[7]);
    }
  }
}

// Store one wave's (16 FM) x 64 accumulator (acc[i][j]: 16x16 MFMA fragments, C/D map col =
// lane&15, row = 4*(lane>>4) + r), 64 rows at a time.  Each 16-row slab goes through the wave's
// private LDS region `slab` (16 x EPI_LD floats) and is re-read as 8-column units: unit
// u = lane + 64*h (h = 0,1) covers row u>>3 and columns 8*(u&7)..+7, so one wave store instruction
// writes 8 whole 128-B rows (bf16: 16 B per lane) -- full cache lines instead of 32-B fragments.
// The epilogue operands of each 64-row group (bias, gamma, residual / pre-activation) are loaded
// before its first slab.
template <int FM, int PRE = 1, int EPI = -1, int AUXT = -1, bool REMAP = false>
__device__ __forceinline__ void wave_tile_epilogue(const f32x4 (&acc)[FM][4], float* __restrict__ slab, int mb,
                                                   int nb, const EpiArgs& e, int split) {
  static_assert(FM % 4 == 0, "64-row groups");
#pragma unroll
  for (int i0 = 0; i0 < FM; i0 += 4)
    wave_group_epilogue<FM, PRE, 4, 0, EPI, AUXT, REMAP>(acc, i0, slab, mb + 16 * i0, nb, e, split);
}

// (16 FM) x (16 FN) wave tile, FN a multiple of 4: 64-column groups stored one after the other
template <int FM, int FN, int PRE = 1>
__device__ __forceinline__ void wave_tile_epilogue_wide(const f32x4 (&acc)[FM][FN], float* __restrict__ slab, int mb,
                                                        int nb, const EpiArgs& e, int split) {
  static_assert(FM % 4 == 0 && FN % 4 == 0 && FM <= 8 && FN <= 8, "64x64 groups");
  // written out (no loop): the unroller refuses a loop this large, and a rolled loop would index the
  // accumulator array dynamically and push it to scratch
  wave_group_epilogue<FM, PRE, FN, 0>(acc, 0, slab, mb, nb, e, split);
  if constexpr (FN >= 8) wave_group_epilogue<FM, PRE, FN, 4>(acc, 0, slab, mb, nb + 64, e, split);
  if constexpr (FM >= 8) {
    wave_group_epilogue<FM, PRE, FN, 0>(acc, 4, slab, mb + 64, nb, e, split);
    if constexpr (FN >= 8) wave_group_epilogue<FM, PRE, FN, 4>(acc, 4, slab, mb + 64, nb + 64, e, split);
  }
}

// Implicit-GEMM convolution geometry for the v3 kernel's gathered operands (ResNet, conv.hip):
//   CONV 1 (fprop):  A(m = (b,oy,ox), k = j*SC + c) = x[b, oy*si + tdy[j], ox*si + tdx[j], c] (0 outside),
//                    B = packed weight [Cout][T*SC] (K-major, plain);
//   CONV 2 (dgrad, stride 1): A = dy gathered the same way (SC = Cout, taps pad - kh / pad - kw),
//                    B(k = j*Cout + co, n = c) = wp[(co*Tw + twt[j])*Cs + c] (M-major rows).
// SC is a power of two >= 32, so every 32-deep k-step lies inside one tap: the tap is wave-uniform.
constexpr int CONV_MAX_TAPS = 64;
struct ConvG {
  int SH, SW, lsc;      // gather source [batch][SH][SW][1 << lsc]
  int GH, GW, si;       // output pixel grid and source step per output pixel
  uint32_t gw_mul, gw_shift, ghw_mul, ghw_shift;  // n / GW and n / (GH*GW) as multiply-shift
  int lcout, Tw, Cs;    // dgrad: B rows
  int8_t tdy[CONV_MAX_TAPS], tdx[CONV_MAX_TAPS];
  uint8_t twt[CONV_MAX_TAPS];
  uint8_t ctap0[4], ctaps[4];  // mode 5: each output parity class's run of taps in tdy/tdx/twt
  // mode 6 (fprop over 8-channel pixels, the ResNet stem): every 16-B chunk of a k-step is its own tap
  // t = k >> 3, (ty, tx) = (t / kw - pad, t % kw - pad) decoded per lane, t / kw = (t * kw_mul) >> 16
  uint32_t kw_mul;
  int kw, pad, ntaps;
};
// d = n / D for n < 2^31: (umulhi(n, mul) + n) >> shift
inline void conv_fastdiv(uint32_t D, uint32_t& mul, uint32_t& shift) {
  uint32_t l = 0;
  while ((1ull << l) < D) ++l;
  shift = l;
  mul = (uint32_t)((((1ull << l) - D) << 32) / D + 1);
}
// fprop (mode 1) / stride-1 dgrad (mode 2) through the v3 kernel; d describes the GEMM view
// (M = pixels, N = Cout or Cs, K = taps * channels), epilogue STORE or BIAS_GAMMA_RES (accumulate).
// Weight gradients, split-K slabs: mode 3 dW = dy^T gather(x) (M = Cout, N = taps * channels), mode 4
// the transposed product dW^T = gather(x)^T dy (M = taps * channels, N = Cout) for Cout < 256.
// Mode 5: the stride-2 dgrad of all four output parity classes in one launch (even H, W: every class
// has the same GH x GW grid; class c takes taps ctap0[c] .. + ctaps[c] and writes slab c, epilogue SLAB,
// or its rows straight into dx [B][2GH][2GW][N] with STORE / BIAS_GAMMA_RES (accumulate) / STORE_BN_BWD)
int launch_gemm3_conv(const sv_gemm_desc* d, const ConvG& g, int mode, hipStream_t s);

// v2 entry (gemm2.hip): returns SV_ERR_UNSUPPORTED when the shape/dtypes are outside its contract
int launch_gemm2(const sv_gemm_desc* d, hipStream_t s);
// v3 entry (gemm3.hip): same contract with K % BK == 0; cfg = "BKxSTAGES" (nullptr: 32x3)
int launch_gemm3(const sv_gemm_desc* d, hipStream_t s, const char* cfg = nullptr);
// v8 entry (gemm8.hip, 256x256 tile, 8 waves, one workgroup per CU): same contract as v3
int launch_gemm8(const sv_gemm_desc* d, hipStream_t s);
// v9 entry (gemm9.hip, persistent 256x256 BK 64 phase-interleaved, register-direct epilogue)
int launch_gemm9(const sv_gemm_desc* d, hipStream_t s);

}  // namespace sv
