// Flat-buffer optimizer step and the small reductions used by backward (gfx950).
//
// The Python host lays every parameter of the model out in ONE f32 buffer (and the gradients,
// AdamW moments and the bf16 weight shadow in buffers with identical offsets), so the reference's
// foreach clip_grad_norm_ + foreach AdamW (spine_vision/training/trainers/base.py:592-597,
// 384-390) become: one grid-stride sum-of-squares pass, one 1-block finisher producing the clip
// coefficient ON DEVICE (no host sync), and one fused AdamW pass that also refreshes the bf16
// shadow the MFMA GEMMs read.  All of them are HBM-bound streaming kernels: 16 B per lane.
#include <math.h>

#include "common.h"

namespace sv {

constexpr int kThreads = 256;

// four consecutive slab elements as floats: f32 (one 16-B load) or bf16 (one 8-B load; bf16 weight-gradient slabs)
template <typename T>
__device__ __forceinline__ float4 ld_part4(const T* p) {
  if constexpr (sizeof(T) == 4) {
    return *reinterpret_cast<const float4*>(p);
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xffff0000u));
  }
}

// out[g][i] (+)= alpha * sum_{p in group g} part[p][i].  grid = (column tiles, groups); each thread
// owns 4 consecutive columns (16-B loads) and keeps 8 independent loads in flight per round, so the
// reduction of deep split-K slabs is bandwidth- rather than latency-bound.
template <typename T>
__global__ void __launch_bounds__(kThreads) reduce_partials_kernel(const T* __restrict__ part,
                                                                    int P, int group, int64_t n,
                                                                    float* __restrict__ out,
                                                                    float alpha, int accumulate) {
  const int g = blockIdx.y;
  const int p0 = g * group;
  int p1 = p0 + group;
  if (p1 > P) p1 = P;
  float* o = out + (size_t)g * n;
  const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= n) return;
  if (i4 + 4 <= n && (n & 3) == 0) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int p = p0;
    for (; p + 8 <= p1; p += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld_part4(part + (size_t)(p + u) * n + i4);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
    }
    for (; p < p1; ++p) {
      const float4 v = ld_part4(part + (size_t)p * n + i4);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    acc.x *= alpha; acc.y *= alpha; acc.z *= alpha; acc.w *= alpha;
    float4* op = reinterpret_cast<float4*>(o + i4);
    if (accumulate) {
      const float4 q = *op;
      acc.x += q.x; acc.y += q.y; acc.z += q.z; acc.w += q.w;
    }
    *op = acc;
  } else {
    for (int64_t i = i4; i < n && i < i4 + 4; ++i) {
      float s = 0.f;
      for (int p = p0; p < p1; ++p) {
        if constexpr (sizeof(T) == 4) s += part[(size_t)p * n + i];
        else s += __uint_as_float((uint32_t)part[(size_t)p * n + i] << 16);
      }
      s *= alpha;
      o[i] = accumulate ? o[i] + s : s;
    }
  }
}

// One-launch partial reduction for up to two segments (e.g. a weight and its bias gradient):
// out_s[i] (+)= alpha * sum_p part_s[p][i].  A workgroup owns 64 columns of one segment: 16 float4
// column lanes x 16 partial groups (p = g, g+16, ...), folded through LDS in a fixed order
// (deterministic).  Works for any partial depth P in one pass: small column counts with deep P (the
// LayerNorm / depthwise / bias partials) get P-parallelism, wide slabs get column parallelism.
struct RedSeg {
  const float* part;
  int64_t n;
  float* out;
};

// Two independent column reductions in one launch: workgroup `blk` < blocks_a reduces COLS = 4 * C4
// consecutive columns of segment a over its P partial rows, the rest segment b.  256 threads =
// C4 float4 column groups x (256 / C4) partial-row groups, folded through LDS in a fixed order.  The
// launcher picks C4 so that even short outputs (LayerNorm dw/db: 2 x C columns over ~1000 partial
// rows) spread over enough workgroups.
template <int C4>
__global__ void __launch_bounds__(kThreads) reduce_pair_kernel(RedSeg a, RedSeg b, int64_t blocks_a, int P,
                                                               float alpha, int accumulate) {
  constexpr int PG = kThreads / C4;
  __shared__ float4 red[PG][C4];
  const bool sb = blockIdx.x >= blocks_a;
  const RedSeg sg = sb ? b : a;
  const int64_t blk = sb ? blockIdx.x - blocks_a : blockIdx.x;
  const int c4 = threadIdx.x % C4, pg = threadIdx.x / C4;
  const int64_t col = blk * (4 * C4) + c4 * 4;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  // 16-B loads only where every partial row starts 16-B aligned (n % 4 == 0; the host checks the base); otherwise
  // the scalar form, which adds the same partials in the same order
  if (col + 4 <= sg.n && (sg.n & 3) == 0) {
    int p = pg;
    for (; p + 3 * PG < P; p += 4 * PG) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(sg.part + (size_t)(p + PG * u) * sg.n + col);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
    }
    for (; p < P; p += PG) {
      const float4 v = *reinterpret_cast<const float4*>(sg.part + (size_t)p * sg.n + col);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  } else if (col < sg.n) {  // ragged tail (n % 4 != 0)
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    for (int p = pg; p < P; p += PG)
      for (int j = 0; j < 4 && col + j < sg.n; ++j) t[j] += sg.part[(size_t)p * sg.n + col + j];
    acc = make_float4(t[0], t[1], t[2], t[3]);
  }
  red[pg][c4] = acc;
  __syncthreads();
  // fold the PG partial groups: C4 * 16 threads each sum PG/16 groups, then 16 -> 1 in one wave
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  constexpr int F = PG >= 16 ? 16 : PG;
  if (threadIdx.x < C4 * F) {
    const int cc = threadIdx.x % C4, f = threadIdx.x / C4;
    for (int g = f; g < PG; g += F) {
      const float4 v = red[g][cc];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  __syncthreads();
  if (threadIdx.x < C4 * F) red[threadIdx.x / C4][threadIdx.x % C4] = s;
  __syncthreads();
  const int64_t c0 = blk * (4 * C4);
  if (threadIdx.x < C4) {
    float4 t = red[0][threadIdx.x];
    for (int g = 1; g < F; ++g) {
      const float4 v = red[g][threadIdx.x];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    const int64_t cl = c0 + threadIdx.x * 4;
    const float r[4] = {t.x * alpha, t.y * alpha, t.z * alpha, t.w * alpha};
    if (cl + 4 <= sg.n && ((reinterpret_cast<uintptr_t>(sg.out + cl) & 15) == 0)) {
      float4 o = make_float4(r[0], r[1], r[2], r[3]);
      if (accumulate) {
        const float4 q = *reinterpret_cast<const float4*>(sg.out + cl);
        o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
      }
      *reinterpret_cast<float4*>(sg.out + cl) = o;
    } else {
      for (int j = 0; j < 4 && cl + j < sg.n; ++j) sg.out[cl + j] = accumulate ? sg.out[cl + j] + r[j] : r[j];
    }
  }
}

// Up to SV_MAX_RED_SEGS independent partial reductions in ONE launch (a block's weight-gradient folds on the
// side stream: the fc1 wgrad slab and its bias column sums, the LayerNorm and depthwise weight / bias
// partials): segment s owns workgroups [blk0, blk0 + nblk).  A "wide" segment (a split-K slab: few partial
// rows, many columns) runs reduce_partials_kernel's body (one thread per 4 columns, the P rows in order, 8
// loads in flight); a "deep" one (many partial rows, few columns) the partial-group body of
// reduce_pair_kernel<16> (64 columns per workgroup, 16 partial-row groups folded through LDS in a fixed
// order).  Deterministic; the wide body is bitwise reduce_partials_kernel's.
struct MultiSeg {
  const float* part;
  float* out;
  int64_t n;
  int64_t blk0;
  int32_t P;
  int32_t wide;
  int32_t accumulate;
};
struct MultiSegs {
  MultiSeg s[SV_MAX_RED_SEGS];
  int32_t nseg;
};

__global__ void __launch_bounds__(kThreads) reduce_multi_kernel(MultiSegs segs, float alpha) {
  int si = 0;
  for (int k = 1; k < segs.nseg; ++k)
    if ((int64_t)blockIdx.x >= segs.s[k].blk0) si = k;
  const MultiSeg sg = segs.s[si];
  const int64_t blk = blockIdx.x - sg.blk0;
  if (sg.wide) {
    const int64_t i4 = (blk * kThreads + threadIdx.x) * 4;
    if (i4 >= sg.n) return;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int p = 0;
    for (; p + 8 <= sg.P; p += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(sg.part + (size_t)(p + u) * sg.n + i4);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
    }
    for (; p < sg.P; ++p) {
      const float4 v = *reinterpret_cast<const float4*>(sg.part + (size_t)p * sg.n + i4);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    acc.x *= alpha; acc.y *= alpha; acc.z *= alpha; acc.w *= alpha;
    float4* op = reinterpret_cast<float4*>(sg.out + i4);
    if (sg.accumulate) {
      const float4 q = *op;
      acc.x += q.x; acc.y += q.y; acc.z += q.z; acc.w += q.w;
    }
    *op = acc;
    return;
  }
  // deep segment: the body of reduce_pair_kernel<16>
  constexpr int C4 = 16, PG = kThreads / C4;
  __shared__ float4 red[PG][C4];
  const int c4 = threadIdx.x % C4, pg = threadIdx.x / C4;
  const int64_t col = blk * (4 * C4) + c4 * 4;
  const int P = sg.P;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col + 4 <= sg.n && (sg.n & 3) == 0) {  // (as reduce_pair_kernel: 16-B loads only for 16-B aligned rows)
    int p = pg;
    for (; p + 3 * PG < P; p += 4 * PG) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(sg.part + (size_t)(p + PG * u) * sg.n + col);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
    }
    for (; p < P; p += PG) {
      const float4 v = *reinterpret_cast<const float4*>(sg.part + (size_t)p * sg.n + col);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  } else if (col < sg.n) {
    float t[4] = {0.f, 0.f, 0.f, 0.f};
    for (int p = pg; p < P; p += PG)
      for (int j = 0; j < 4 && col + j < sg.n; ++j) t[j] += sg.part[(size_t)p * sg.n + col + j];
    acc = make_float4(t[0], t[1], t[2], t[3]);
  }
  red[pg][c4] = acc;
  __syncthreads();
  float4 sm = make_float4(0.f, 0.f, 0.f, 0.f);
  constexpr int F = PG >= 16 ? 16 : PG;
  if (threadIdx.x < C4 * F) {
    const int cc = threadIdx.x % C4, f = threadIdx.x / C4;
    for (int g = f; g < PG; g += F) {
      const float4 v = red[g][cc];
      sm.x += v.x; sm.y += v.y; sm.z += v.z; sm.w += v.w;
    }
  }
  __syncthreads();
  if (threadIdx.x < C4 * F) red[threadIdx.x / C4][threadIdx.x % C4] = sm;
  __syncthreads();
  if (threadIdx.x < C4) {
    float4 t = red[0][threadIdx.x];
    for (int g = 1; g < F; ++g) {
      const float4 v = red[g][threadIdx.x];
      t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
    }
    const int64_t cl = blk * (4 * C4) + threadIdx.x * 4;
    const float r[4] = {t.x * alpha, t.y * alpha, t.z * alpha, t.w * alpha};
    if (cl + 4 <= sg.n && ((reinterpret_cast<uintptr_t>(sg.out + cl) & 15) == 0)) {
      float4 o = make_float4(r[0], r[1], r[2], r[3]);
      if (sg.accumulate) {
        const float4 q = *reinterpret_cast<const float4*>(sg.out + cl);
        o.x += q.x; o.y += q.y; o.z += q.z; o.w += q.w;
      }
      *reinterpret_cast<float4*>(sg.out + cl) = o;
    } else {
      for (int j = 0; j < 4 && cl + j < sg.n; ++j) sg.out[cl + j] = sg.accumulate ? sg.out[cl + j] + r[j] : r[j];
    }
  }
}

// column sums: workgroup b sums rows [b*rpb, (b+1)*rpb) of all C columns -> part[b][C]
template <typename T>
__global__ void __launch_bounds__(kThreads) colsum_kernel(const T* __restrict__ x, int64_t rows, int C,
                                                          int64_t rpb, float* __restrict__ part) {
  const int64_t r0 = (int64_t)blockIdx.x * rpb;
  int64_t r1 = r0 + rpb;
  if (r1 > rows) r1 = rows;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int64_t r = r0; r < r1; ++r) s += ld(x, (size_t)r * C + c);
    part[(size_t)blockIdx.x * C + c] = s;
  }
}

// dW2 += gamma*G ; dgamma += rowdot(W2,G) + b2*cs ; db2 += gamma*cs.  One wave per row c.
__global__ void __launch_bounds__(kThreads) layerscale_finish_kernel(
    const float* __restrict__ G, const float* __restrict__ cs, const float* __restrict__ W2,
    const float* __restrict__ gamma, const float* __restrict__ b2, float* __restrict__ dW2,
    float* __restrict__ dgamma, float* __restrict__ db2, int C, int K4) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (c >= C) return;
  const float gc = gamma[c];
  float dot = 0.f;
  for (int k = lane; k < K4; k += 64) {
    const size_t i = (size_t)c * K4 + k;
    const float g = G[i];
    dot += W2[i] * g;
    dW2[i] += gc * g;
  }
  dot = wave_sum(dot);
  if (lane == 0) {
    dgamma[c] += dot + b2[c] * cs[c];
    db2[c] += gc * cs[c];
  }
}


// fc2 wgrad split-K reduction fused with the layer-scale finish (replaces reduce_pair + finish):
// one workgroup per row c of G = sum_p slab[p][c][:]: thread t owns the float4 column groups
// t, t + 256, ...; dW2[c] += gamma_c G[c], the row dot sum(W2[c] G[c]) and the colsum
// cs[c] = sum_p cs_part[p][c] are block sums (fixed order), so one kernel finishes dgamma / db2 too.
template <typename T>
__global__ void __launch_bounds__(kThreads) layerscale_reduce_kernel(const T* __restrict__ slab, int Ps,
                                                                     const float* __restrict__ cs_part, int P,
                                                                     const float* __restrict__ W2,
                                                                     const float* __restrict__ gamma,
                                                                     const float* __restrict__ b2,
                                                                     float* __restrict__ dW2, float* __restrict__ dgamma,
                                                                     float* __restrict__ db2, int C, int K4) {
  __shared__ float red[kThreads / 64];
  const int c = blockIdx.x;
  const int ng = K4 / 4;
  const size_t rowoff = (size_t)c * K4, pstride = (size_t)C * K4;
  const float gc = gamma[c];
  float dot = 0.f;
  for (int gi = threadIdx.x; gi < ng; gi += kThreads) {
    const size_t off = rowoff + (size_t)gi * 4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int p = 0;
    for (; p + 8 <= Ps; p += 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = ld_part4(slab + (size_t)(p + u) * pstride + off);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        acc.x += v[u].x; acc.y += v[u].y; acc.z += v[u].z; acc.w += v[u].w;
      }
    }
    for (; p < Ps; ++p) {
      const float4 v = ld_part4(slab + (size_t)p * pstride + off);
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    const float4 w = *reinterpret_cast<const float4*>(W2 + off);
    float4 o = *reinterpret_cast<const float4*>(dW2 + off);
    o.x += gc * acc.x; o.y += gc * acc.y; o.z += gc * acc.z; o.w += gc * acc.w;
    *reinterpret_cast<float4*>(dW2 + off) = o;
    dot += w.x * acc.x + w.y * acc.y + w.z * acc.z + w.w * acc.w;
  }
  float cs = 0.f;
  for (int p = threadIdx.x; p < P; p += kThreads) cs += cs_part[(size_t)p * C + c];
  dot = block_sum(dot, red);
  cs = block_sum(cs, red);
  if (threadIdx.x == 0) {
    dgamma[c] += dot + b2[c] * cs;
    db2[c] += gc * cs;
  }
}

constexpr int kSqBlocks = 1024;

__global__ void __launch_bounds__(kThreads) sqnorm_kernel(const float* __restrict__ g, int64_t n,
                                                          float* __restrict__ part) {
  __shared__ float red[kThreads / 64];
  float s = 0.f;
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 v = reinterpret_cast<const float4*>(g)[i];
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) s += g[i] * g[i];
  s = block_sum(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void __launch_bounds__(kThreads) clip_coef_kernel(const float* __restrict__ part, int P,
                                                             float max_norm, float* __restrict__ out) {
  __shared__ float red[kThreads / 64];
  // fixed-order (deterministic) sum of the per-block partials
  float s = 0.f;
  for (int p = threadIdx.x; p < P; p += blockDim.x) s += part[p];
  s = block_sum(s, red);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s);
    float coef = max_norm / (norm + 1e-6f);
    coef = coef < 1.0f ? coef : 1.0f;
    out[0] = norm;
    out[1] = coef;
  }
}

__global__ void __launch_bounds__(kThreads) adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v,
                                                         uint16_t* __restrict__ pb, int64_t n, float lr,
                                                         float b1, float b2, float eps, float wd,
                                                         float bc1, float bc2_sqrt,
                                                         const float* __restrict__ gscale,
                                                         const float* __restrict__ hyper) {
  const float sc = gscale ? *gscale : 1.0f;
  if (hyper) {  // graph replay: [lr, bc1, sqrt(bc2)] of this step from device memory
    lr = hyper[0];
    bc1 = hyper[1];
    bc2_sqrt = hyper[2];
  }
  const float step_size = lr / bc1;
  const float decay = 1.0f - lr * wd;
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    float* pa = &pp.x; const float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = ga[k] * sc;
      float pk = pa[k] * decay;
      ma[k] = b1 * ma[k] + (1.0f - b1) * gk;
      va[k] = b2 * va[k] + (1.0f - b2) * gk * gk;
      const float denom = sqrtf(va[k]) / bc2_sqrt + eps;
      pa[k] = pk - step_size * (ma[k] / denom);
    }
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (pb) reinterpret_cast<uint2*>(pb)[i] = make_uint2(pack2bf(pp.x, pp.y), pack2bf(pp.z, pp.w));
  }
  for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gk = g[i] * sc;
    const float pk = p[i] * decay;
    m[i] = b1 * m[i] + (1.0f - b1) * gk;
    v[i] = b2 * v[i] + (1.0f - b2) * gk * gk;
    p[i] = pk - step_size * (m[i] / (sqrtf(v[i]) / bc2_sqrt + eps));
    if (pb) pb[i] = f2bf(p[i]);
  }
}

// out[r][k] = bf16(W[r][k] * scale[r])   (the layer-scale gamma folded into fc2's weight for dgrad)
__global__ void __launch_bounds__(kThreads) scale_rows_bf16_kernel(const float* __restrict__ W,
                                                                   const float* __restrict__ scale,
                                                                   uint16_t* __restrict__ out, int rows, int cols) {
  const int64_t n = (int64_t)rows * cols;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = f2bf(W[i] * scale[i / cols]);
}

// out[c][r] = bf16(W[r][c] * (scale ? scale[r] : 1)): the transposed bf16 operand images of the fused MLP backward
// (W2 gamma and W1); 32 x 32 tiles through LDS so both the reads and the writes are row-contiguous
__global__ void __launch_bounds__(256) transpose_scale_bf16_kernel(const float* __restrict__ W,
                                                                   const float* __restrict__ scale,
                                                                   uint16_t* __restrict__ out, int rows, int cols) {
  __shared__ float t[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, c = c0 + tx;
    t[k][tx] = (r < rows && c < cols) ? W[(size_t)r * cols + c] * (scale ? scale[r] : 1.0f) : 0.f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, r = r0 + tx;
    if (c < cols && r < rows) out[(size_t)c * rows + r] = f2bf(t[tx][k]);
  }
}

__global__ void __launch_bounds__(kThreads) cast_bf16_kernel(const float* __restrict__ x,
                                                             uint16_t* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = f2bf(x[i]);
}

static int stream_grid(int64_t n, int per_thread) {
  const int64_t g = (n / per_thread + kThreads - 1) / kThreads;
  return (int)(g < 2048 ? (g < 1 ? 1 : g) : 2048);
}

}  // namespace sv

using namespace sv;

extern "C" {

int sv_reduce_partials_pair(const float* part_a, int64_t n_a, float* out_a, const float* part_b, int64_t n_b,
                            float* out_b, int32_t P, float alpha, int32_t accumulate, sv_stream_t stream) {
  SV_REQUIRE(part_a && out_a && P >= 1 && n_a >= 0, "sv_reduce_partials_pair: bad args");
  SV_REQUIRE(!n_b || (part_b && out_b), "sv_reduce_partials_pair: bad second segment");
  if (n_a % 4 == 0) SV_REQUIRE((((uintptr_t)part_a) & 15) == 0, "sv_reduce_partials_pair: part_a must be 16-B aligned");
  if (n_b % 4 == 0 && n_b) SV_REQUIRE((((uintptr_t)part_b) & 15) == 0, "sv_reduce_partials_pair: part_b must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  if (P <= 64 && n_a >= 65536 && n_a % 4 == 0 && (((uintptr_t)out_a) & 15) == 0) {
    // a wide split-K slab (weight gradient): one thread per 4 columns summing the P slices in order
    // with 8 loads in flight (the partial-row groups of the kernel below would each issue ONE load
    // per thread before the LDS fold: latency-bound at ~1 TB/s); the narrow b segment follows
    const int64_t t4 = n_a / 4;
    reduce_partials_kernel<float><<<dim3((unsigned)((t4 + kThreads - 1) / kThreads), 1), kThreads, 0, s>>>(part_a, P, P, n_a,
                                                                                                   out_a, alpha, accumulate);
    const int rc = check_launch("sv_reduce_partials_pair");
    if (rc != SV_OK || !n_b) return rc;
    part_a = part_b, n_a = n_b, out_a = out_b;
    part_b = nullptr, n_b = 0, out_b = nullptr;
  }
  RedSeg a{part_a, n_a, out_a}, b{part_b, n_b, out_b};
  // widest column block that still gives >= 512 workgroups (or 4 columns per workgroup); with few
  // partial rows (split-K slabs: P = 2..8) up to 256 columns, so that no partial-row group idles
  int cols = P <= 4 ? 256 : (P <= 8 ? 128 : 64);
  while (cols > 4 && (n_a + cols - 1) / cols + (n_b + cols - 1) / cols < 512) cols >>= 1;
  const int64_t ba = (n_a + cols - 1) / cols, bb = (n_b + cols - 1) / cols;
  if (ba + bb == 0) return SV_OK;
  switch (cols) {
    case 256: reduce_pair_kernel<64><<<(unsigned)(ba + bb), kThreads, 0, s>>>(a, b, ba, P, alpha, accumulate); break;
    case 128: reduce_pair_kernel<32><<<(unsigned)(ba + bb), kThreads, 0, s>>>(a, b, ba, P, alpha, accumulate); break;
    case 64: reduce_pair_kernel<16><<<(unsigned)(ba + bb), kThreads, 0, s>>>(a, b, ba, P, alpha, accumulate); break;
    case 32: reduce_pair_kernel<8><<<(unsigned)(ba + bb), kThreads, 0, s>>>(a, b, ba, P, alpha, accumulate); break;
    case 16: reduce_pair_kernel<4><<<(unsigned)(ba + bb), kThreads, 0, s>>>(a, b, ba, P, alpha, accumulate); break;
    case 8: reduce_pair_kernel<2><<<(unsigned)(ba + bb), kThreads, 0, s>>>(a, b, ba, P, alpha, accumulate); break;
    default: reduce_pair_kernel<1><<<(unsigned)(ba + bb), kThreads, 0, s>>>(a, b, ba, P, alpha, accumulate); break;
  }
  return check_launch("sv_reduce_partials_pair");
}

int sv_reduce_partials_multi(const sv_red_seg* segs, int32_t nseg, float alpha, sv_stream_t stream) {
  SV_REQUIRE(segs && nseg >= 1 && nseg <= SV_MAX_RED_SEGS, "sv_reduce_partials_multi: 1..%d segments", SV_MAX_RED_SEGS);
  MultiSegs m{};
  int64_t blocks = 0;
  int k = 0;
  for (int i = 0; i < nseg; ++i) {
    const sv_red_seg& g = segs[i];
    SV_REQUIRE(g.part && g.out && g.P >= 1 && g.n >= 0, "sv_reduce_partials_multi: bad segment %d", i);
    if (g.n == 0) continue;
    // the wide body needs whole 16-B column groups; sv_reduce_partials_pair's choice of body
    const bool wide = g.P <= 64 && g.n >= 65536 && g.n % 4 == 0 && (((uintptr_t)g.out) & 15) == 0;
    // the 16-B bodies (wide; deep with n % 4 == 0) read every partial row from a 16-B aligned start
    if (g.n % 4 == 0) SV_REQUIRE((((uintptr_t)g.part) & 15) == 0, "sv_reduce_partials_multi: partials must be 16-B aligned");
    const int64_t nb = wide ? (g.n / 4 + kThreads - 1) / kThreads : (g.n + 63) / 64;
    m.s[k] = MultiSeg{g.part, g.out, g.n, blocks, g.P, wide ? 1 : 0, g.accumulate ? 1 : 0};
    blocks += nb;
    ++k;
  }
  m.nseg = k;
  if (k == 0) return SV_OK;
  SV_REQUIRE(blocks < (1ll << 31), "sv_reduce_partials_multi: too many workgroups");
  reduce_multi_kernel<<<(unsigned)blocks, kThreads, 0, (hipStream_t)stream>>>(m, alpha);
  return check_launch("sv_reduce_partials_multi");
}

int sv_reduce_partials(const float* part, int32_t P, int32_t group, int64_t n, float* out, float alpha,
                       int32_t accumulate, sv_stream_t stream) {
  SV_REQUIRE(part && out && P >= 1, "sv_reduce_partials: bad args");
  if (group <= 0 || group > P) group = P;
  if (n <= 0) return SV_OK;
  const int64_t threads = (n + 3) / 4;
  const dim3 grid((unsigned)((threads + kThreads - 1) / kThreads), (unsigned)((P + group - 1) / group));
  if ((n & 3) == 0)
    SV_REQUIRE((((uintptr_t)part | (uintptr_t)out) & 15) == 0, "sv_reduce_partials: buffers must be 16-B aligned");
  reduce_partials_kernel<float><<<grid, kThreads, 0, (hipStream_t)stream>>>(part, P, group, n, out, alpha, accumulate);
  return check_launch("sv_reduce_partials");
}

int sv_reduce_partials_bf16(const uint16_t* part, int32_t P, int64_t n, float* out, float alpha, int32_t accumulate,
                            sv_stream_t stream) {
  SV_REQUIRE(part && out && P >= 1, "sv_reduce_partials_bf16: bad args");
  if (n <= 0) return SV_OK;
  if ((n & 3) == 0)
    SV_REQUIRE(((uintptr_t)part & 7) == 0 && ((uintptr_t)out & 15) == 0,
               "sv_reduce_partials_bf16: part must be 8-B and out 16-B aligned");
  const int64_t threads = (n + 3) / 4;
  const dim3 grid((unsigned)((threads + kThreads - 1) / kThreads), 1);
  reduce_partials_kernel<uint16_t><<<grid, kThreads, 0, (hipStream_t)stream>>>(part, P, P, n, out, alpha, accumulate);
  return check_launch("sv_reduce_partials_bf16");
}

static int64_t colsum_rpb(int64_t rows) {
  int64_t rpb = (rows + 511) / 512;
  return rpb < 1 ? 1 : rpb;
}

int sv_colsum_nparts(int64_t rows, int32_t C) {
  (void)C;
  const int64_t rpb = colsum_rpb(rows);
  return (int)((rows + rpb - 1) / rpb);
}

int sv_colsum(const void* x, int32_t x_dtype, int64_t rows, int32_t C, float* part, sv_stream_t stream) {
  SV_REQUIRE(x && part && C > 0, "sv_colsum: bad args");
  if (rows <= 0) return SV_OK;
  const int64_t rpb = colsum_rpb(rows);
  const int grid = sv_colsum_nparts(rows, C);
  if (x_dtype == SV_F32)
    colsum_kernel<float><<<grid, kThreads, 0, (hipStream_t)stream>>>((const float*)x, rows, C, rpb, part);
  else if (x_dtype == SV_BF16)
    colsum_kernel<uint16_t><<<grid, kThreads, 0, (hipStream_t)stream>>>((const uint16_t*)x, rows, C, rpb, part);
  else
    return set_error(SV_ERR_INVALID_ARG, "sv_colsum: bad dtype");
  return check_launch("sv_colsum");
}

int sv_layerscale_wgrad_finish(const float* G, const float* cs, const float* W2, const float* gamma,
                               const float* b2, float* dW2, float* dgamma, float* db2, int32_t C,
                               int32_t K4, sv_stream_t stream) {
  SV_REQUIRE(G && cs && W2 && gamma && b2 && dW2 && dgamma && db2, "sv_layerscale_wgrad_finish: null");
  if (C <= 0) return SV_OK;
  layerscale_finish_kernel<<<ceil_div(C, kThreads / 64), kThreads, 0, (hipStream_t)stream>>>(
      G, cs, W2, gamma, b2, dW2, dgamma, db2, C, K4);
  return check_launch("sv_layerscale_wgrad_finish");
}

int sv_layerscale_wgrad_reduce_ws(int32_t C, int32_t K4) {
  (void)C;
  (void)K4;
  return 0;  // no workspace: one workgroup per row finishes everything
}

int sv_layerscale_wgrad_reduce(const float* slab, const float* cs_part, int32_t P, const float* W2,
                               const float* gamma, const float* b2, float* dW2, float* dgamma, float* db2,
                               float* ws, int32_t C, int32_t K4, sv_stream_t stream) {
  (void)ws;
  SV_REQUIRE(slab && cs_part && W2 && gamma && b2 && dW2 && dgamma && db2 && P >= 1,
             "sv_layerscale_wgrad_reduce: bad arguments");
  SV_REQUIRE(K4 % 4 == 0 && C > 0, "sv_layerscale_wgrad_reduce: K4=%d must be a multiple of 4", K4);
  SV_REQUIRE((((uintptr_t)slab | (uintptr_t)W2 | (uintptr_t)dW2) & 15) == 0,
             "sv_layerscale_wgrad_reduce: buffers must be 16-B aligned");
  layerscale_reduce_kernel<float><<<C, kThreads, 0, (hipStream_t)stream>>>(slab, P, cs_part, P, W2, gamma, b2, dW2,
                                                                          dgamma, db2, C, K4);
  return check_launch("sv_layerscale_wgrad_reduce");
}

int sv_layerscale_wgrad_reduce_bf16(const uint16_t* slab, const float* cs_part, int32_t P, const float* W2,
                                    const float* gamma, const float* b2, float* dW2, float* dgamma, float* db2, int32_t C,
                                    int32_t K4, sv_stream_t stream) {
  SV_REQUIRE(slab && cs_part && W2 && gamma && b2 && dW2 && dgamma && db2 && P >= 1,
             "sv_layerscale_wgrad_reduce_bf16: bad arguments");
  SV_REQUIRE(K4 % 4 == 0 && C > 0, "sv_layerscale_wgrad_reduce_bf16: K4=%d must be a multiple of 4", K4);
  SV_REQUIRE(((uintptr_t)slab & 7) == 0 && (((uintptr_t)W2 | (uintptr_t)dW2) & 15) == 0,
             "sv_layerscale_wgrad_reduce_bf16: slab 8-B, W2 / dW2 16-B aligned");
  layerscale_reduce_kernel<uint16_t><<<C, kThreads, 0, (hipStream_t)stream>>>(slab, P, cs_part, P, W2, gamma, b2, dW2,
                                                                             dgamma, db2, C, K4);
  return check_launch("sv_layerscale_wgrad_reduce_bf16");
}

int sv_layerscale_wgrad_fold_finish(const float* G, const float* cs_part, int32_t P, const float* W2, const float* gamma,
                                    const float* b2, float* dW2, float* dgamma, float* db2, int32_t C, int32_t K4,
                                    sv_stream_t stream) {
  SV_REQUIRE(G && cs_part && W2 && gamma && b2 && dW2 && dgamma && db2 && P >= 1,
             "sv_layerscale_wgrad_fold_finish: bad arguments");
  SV_REQUIRE(K4 % 4 == 0 && C > 0, "sv_layerscale_wgrad_fold_finish: K4=%d must be a multiple of 4", K4);
  SV_REQUIRE((((uintptr_t)G | (uintptr_t)W2 | (uintptr_t)dW2) & 15) == 0,
             "sv_layerscale_wgrad_fold_finish: buffers must be 16-B aligned");
  layerscale_reduce_kernel<float><<<C, kThreads, 0, (hipStream_t)stream>>>(G, 1, cs_part, P, W2, gamma, b2, dW2, dgamma,
                                                                          db2, C, K4);
  return check_launch("sv_layerscale_wgrad_fold_finish");
}

int sv_sqnorm_nparts(int64_t n) {
  const int g = stream_grid(n, 4);
  return g < kSqBlocks ? g : kSqBlocks;
}

int sv_sqnorm_partial(const float* g, int64_t n, float* part, sv_stream_t stream) {
  SV_REQUIRE(g && part, "sv_sqnorm_partial: null");
  SV_REQUIRE(((uintptr_t)g & 15) == 0, "sv_sqnorm_partial: buffer must be 16-byte aligned");
  sqnorm_kernel<<<sv_sqnorm_nparts(n), kThreads, 0, (hipStream_t)stream>>>(g, n, part);
  return check_launch("sv_sqnorm_partial");
}

int sv_clip_coef(const float* part, int32_t nparts, float max_norm, float* out, sv_stream_t stream) {
  SV_REQUIRE(part && out && nparts >= 1, "sv_clip_coef: bad args");
  clip_coef_kernel<<<1, kThreads, 0, (hipStream_t)stream>>>(part, nparts, max_norm, out);
  return check_launch("sv_clip_coef");
}

int sv_adamw_flat(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n,
                  float lr, float beta1, float beta2, float eps, float weight_decay, int32_t step,
                  const float* grad_scale, sv_stream_t stream) {
  SV_REQUIRE(p && g && m && v && step >= 1, "sv_adamw_flat: bad args");
  SV_REQUIRE((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0 &&
                 (((uintptr_t)p_bf16) & 7) == 0,
             "sv_adamw_flat: buffers must be 16-byte aligned");
  if (n <= 0) return SV_OK;
  // bias corrections in double on the host, as torch computes them in Python floats
  const float bc1 = (float)(1.0 - pow((double)beta1, (double)step));
  const float bc2 = (float)(1.0 - pow((double)beta2, (double)step));
  adamw_kernel<<<stream_grid(n, 4), kThreads, 0, (hipStream_t)stream>>>(
      p, g, m, v, p_bf16, n, lr, beta1, beta2, eps, weight_decay, bc1, sqrtf(bc2), grad_scale, nullptr);
  return check_launch("sv_adamw_flat");
}

int sv_adamw_flat_dev(float* p, const float* g, float* m, float* v, uint16_t* p_bf16, int64_t n, float beta1,
                      float beta2, float eps, float weight_decay, const float* hyper, const float* grad_scale,
                      sv_stream_t stream) {
  SV_REQUIRE(p && g && m && v && hyper, "sv_adamw_flat_dev: bad args");
  SV_REQUIRE((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0 &&
                 (((uintptr_t)p_bf16) & 7) == 0,
             "sv_adamw_flat_dev: buffers must be 16-byte aligned");
  if (n <= 0) return SV_OK;
  adamw_kernel<<<stream_grid(n, 4), kThreads, 0, (hipStream_t)stream>>>(
      p, g, m, v, p_bf16, n, 0.f, beta1, beta2, eps, weight_decay, 1.f, 1.f, grad_scale, hyper);
  return check_launch("sv_adamw_flat_dev");
}

int sv_scale_rows_bf16(const float* W, const float* scale, uint16_t* out, int32_t rows, int32_t cols,
                       sv_stream_t stream) {
  SV_REQUIRE(W && scale && out && rows > 0 && cols > 0, "sv_scale_rows_bf16: bad args");
  scale_rows_bf16_kernel<<<stream_grid((int64_t)rows * cols, 1), kThreads, 0, (hipStream_t)stream>>>(W, scale, out,
                                                                                                      rows, cols);
  return check_launch("sv_scale_rows_bf16");
}

int sv_transpose_scale_bf16(const float* W, const float* scale, uint16_t* out, int32_t rows, int32_t cols,
                            sv_stream_t stream) {
  SV_REQUIRE(W && out && rows > 0 && cols > 0, "sv_transpose_scale_bf16: bad args");
  const dim3 grid((unsigned)((cols + 31) / 32), (unsigned)((rows + 31) / 32));
  transpose_scale_bf16_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(W, scale, out, rows, cols);
  return check_launch("sv_transpose_scale_bf16");
}

int sv_cast_f32_bf16(const float* x, uint16_t* y, int64_t n, sv_stream_t stream) {
  SV_REQUIRE(x && y, "sv_cast_f32_bf16: null");
  if (n <= 0) return SV_OK;
  cast_bf16_kernel<<<stream_grid(n, 1), kThreads, 0, (hipStream_t)stream>>>(x, y, n);
  return check_launch("sv_cast_f32_bf16");
}

}  // extern "C"
