// BatchNorm2d (train-mode batch statistics), ReLU, MaxPool2d(3,2,1) and global average pooling for
// the ResNet-18/50 classification backbone (gfx950), NHWC.
//
// Replaces timm ResNet's nn.BatchNorm2d / nn.ReLU / nn.MaxPool2d / SelectAdaptivePool2d
// (timm/models/resnet.py, built at spine_vision/training/models/backbone.py:166) and their autograd
// backward.  All kernels are HBM-bound streaming passes: one thread owns 4 consecutive channels
// (16-B f32 / 8-B bf16 accesses), channel statistics are reduced per block into deterministic
// partials [nparts][2][C] and finished by a 16-wave fold per 32 channels (no atomics, bit-stable).
// Batch statistics use shifted sums (shift = the channel's value in row 0) so mean^2 >> var does
// not cancel catastrophically in f32.
#include <math.h>
#include <stdlib.h>

#include "common.h"

namespace sv {
namespace bn {

constexpr int kThreads = 256;

template <typename T>
__device__ __forceinline__ float4 ld4t(const void* p, size_t i) {
  return ld4(reinterpret_cast<const T*>(p), i);
}
__device__ __forceinline__ float4 ld4d(const void* p, int dt, size_t i) {
  return dt == SV_F32 ? ld4t<float>(p, i) : ld4t<uint16_t>(p, i);
}
__device__ __forceinline__ void st4d(void* p, int dt, size_t i, float4 v) {
  if (dt == SV_F32) st4(reinterpret_cast<float*>(p), i, v);
  else st4(reinterpret_cast<uint16_t*>(p), i, v);
}
__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
// channel of flat element e: 32-bit division where the tensor fits (64-bit division is a long software sequence
// on the GPU and these passes run it once per element group); `n` = the tensor's element count
__device__ __forceinline__ int chan_of(size_t e, int C, int64_t n) {
  return n <= 0xffffffffll ? (int)((uint32_t)e % (uint32_t)C) : (int)(e % (size_t)C);
}
__device__ __forceinline__ float4 ld4f(const float* p, int c) { return *reinterpret_cast<const float4*>(p + c); }

// V consecutive channels per thread: 8 (one 16-B bf16 access, two 16-B f32 accesses) when C % 8 == 0,
// else 4.  Per-channel parameters are read as float4s from L1/L2.
template <int V>
__device__ __forceinline__ void ldv(const void* p, int dt, size_t i, float (&o)[V]) {
  if constexpr (V == 8) {
    if (dt == SV_F32) {
      const float* f = reinterpret_cast<const float*>(p) + i;
      const float4 a = *reinterpret_cast<const float4*>(f), b = *reinterpret_cast<const float4*>(f + 4);
      o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
    } else {
      const uint4 u = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(p) + i);
      const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[2 * k] = __uint_as_float(w[k] << 16);
        o[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
      }
    }
  } else {
    const float4 a = ld4d(p, dt, i);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
  }
}
template <int V>
__device__ __forceinline__ void stv(void* p, int dt, size_t i, const float (&v)[V]) {
  if constexpr (V == 8) {
    if (dt == SV_F32) {
      float* f = reinterpret_cast<float*>(p) + i;
      *reinterpret_cast<float4*>(f) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(f + 4) = make_float4(v[4], v[5], v[6], v[7]);
    } else {
      *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(p) + i) =
          make_uint4(pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7]));
    }
  } else {
    st4d(p, dt, i, make_float4(v[0], v[1], v[2], v[3]));
  }
}
// the elementwise forms every pass shares (so the one-launch small-row kernels at the end of this file give
// the multi-launch path's bits): the affine pre-activation and the train-mode data gradient, every fused
// multiply-add written out -- hipcc contracts a*b+c by context (a product hoisted out of a loop or shared by two
// expressions stays unfused), which would let two kernels computing the same formula round differently
__device__ __forceinline__ float bn_pre(float g, float rs, float v, float mu, float b) { return fmaf(g * rs, v - mu, b); }
__device__ __forceinline__ float bn_dx(float ga, float rs, float g, float sg, float v, float mu, float sgx, float inv_n) {
  const float a1 = fmaf(-sg, inv_n, g);                 // g - sum g / n
  const float xs = ((v - mu) * rs) * sgx;               // xhat * sum g xhat
  return (ga * rs) * fmaf(-xs, inv_n, a1);              // gamma rstd (g - sum g / n - xhat sum g xhat / n)
}

template <int V>
__device__ __forceinline__ void ldp(const float* p, int c, float (&o)[V]) {
#pragma unroll
  for (int k = 0; k < V; k += 4) {
    const float4 a = *reinterpret_cast<const float4*>(p + c + k);
    o[k] = a.x; o[k + 1] = a.y; o[k + 2] = a.z; o[k + 3] = a.w;
  }
}

static int vec_for(int C) { return (C % 8 == 0 && ((C / 8) <= kThreads || (C / 8) % kThreads == 0)) ? 8 : 4; }

// Block layout for per-channel reductions: tpr threads cover one row (V channels each), rp rows in
// parallel; grid.x = channel slices of V*tpr channels, grid.y = row parts.
struct RedGeo {
  int vec, tpr, rp, cslices;
};
static RedGeo red_geo(int C) {
  RedGeo g;
  g.vec = vec_for(C);
  const int cg = C / g.vec;
  g.tpr = cg < kThreads ? cg : kThreads;
  g.rp = kThreads / g.tpr;
  g.cslices = cg / g.tpr;
  return g;
}

static int nparts_for(int64_t rows, int C) {
  const RedGeo g = red_geo(C);
  int64_t p = rows / (8 * g.rp);  // >= 8 rows per thread
  const int64_t cap = 1024 / g.cslices;
  if (p > cap) p = cap;
  if (p < 1) p = 1;
  return (int)p;
}

// block-level reduce of two V-vectors per thread over the rp row-groups; writes part[p][0|1][c..c+V-1]
template <int V>
__device__ __forceinline__ void reduce_write(float (&s1)[V], float (&s2)[V], int tpr, int rp, int c, int C, float* part) {
  __shared__ float red[2][V][kThreads];
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    red[0][k][t] = s1[k];
    red[1][k][t] = s2[k];
  }
  __syncthreads();
  if (t < tpr) {
    for (int r = 1; r < rp; ++r)
#pragma unroll
      for (int k = 0; k < V; ++k) {
        s1[k] += red[0][k][r * tpr + t];
        s2[k] += red[1][k][r * tpr + t];
      }
    float* o = part + (size_t)blockIdx.y * 2 * C;
#pragma unroll
    for (int k = 0; k < V; k += 4) {
      *reinterpret_cast<float4*>(o + c + k) = make_float4(s1[k], s1[k + 1], s1[k + 2], s1[k + 3]);
      *reinterpret_cast<float4*>(o + C + c + k) = make_float4(s2[k], s2[k + 1], s2[k + 2], s2[k + 3]);
    }
  }
}

// forward statistics: shifted sums S1 = sum (y - y0), S2 = sum (y - y0)^2
template <int V>
__global__ void __launch_bounds__(kThreads) stats_kernel(const void* __restrict__ y, int ydt, int64_t rows, int C,
                                                         int tpr, int rp, int64_t rpp, float* __restrict__ part) {
  const int t = threadIdx.x;
  const int c = (blockIdx.x * tpr + t % tpr) * V;
  const int rsub = t / tpr;
  float k[V], s1[V], s2[V];
  ldv<V>(y, ydt, (size_t)c, k);
#pragma unroll
  for (int q = 0; q < V; ++q) s1[q] = s2[q] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.y * rpp;
  int64_t r1 = r0 + rpp;
  if (r1 > rows) r1 = rows;
  for (int64_t r = r0 + rsub; r < r1; r += rp) {
    float v[V];
    ldv<V>(y, ydt, (size_t)r * C + c, v);
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const float dv = v[q] - k[q];
      s1[q] += dv;
      s2[q] = fmaf(dv, dv, s2[q]);
    }
  }
  reduce_write<V>(s1, s2, tpr, rp, c, C, part);
}

// 4-B stores / loads that bypass L1 and write through L2 (sc1): the hand-off of values between workgroups of one
// launch (the fold kernels below), MI355X_MICROARCH.md's inter-workgroup table row 1
__device__ __forceinline__ void st_sc1(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum of the per-block partials [P][2][C] for kFinCh = 32 channels per workgroup.  Lane l of wave w
// reads channels 4 (l & 7) .. +3 of its slice (one 16-B load per sum; 8 lanes cover a 128-B row
// segment) from partials j, j + 128, j + 256, .. with j = 8 w + (l >> 3): 128 partial streams per
// workgroup, each lane with 4 partials (8 loads) in flight.  Wave 0 then folds the 128 stream sums in a
// fixed order through LDS (lanes 0-31: S1, lanes 32-63: S2), so the result is bit-stable.  Round 2's
// version (64 channels per workgroup, lane = channel, one 4-B load per lane and sum) kept a quarter of
// the bytes in flight on half the workgroups: 7-8 us per finish at P = 512-2048.
constexpr int kFinWaves = 16, kFinCh = 32, kFinStreams = kFinWaves * 64 / (kFinCh / 4);
// Partials are folded in chunks of kFoldQ parts: each chunk as above (128 streams, then the streams in order), the
// chunk sums then added in chunk order.  One chunk up to 1024 parts (every backward statistics pass, and the
// one-launch small kernels, whose order is the single-chunk one); the forward's GEMM-epilogue partials of the
// stem and layer 1 (one per 64 rows: 2048-8192) take 2-8 chunks, which the fold kernels below hand to as many
// workgroups.
constexpr int kFoldQ = 1024, kFoldMaxS = 16;
__host__ __device__ __forceinline__ int fold_chunks(int P) { return (P + kFoldQ - 1) / kFoldQ; }

// The 128 stream sums of parts [p0, p1) for channels 32 cg .. +31, folded in stream order by wave 0: lane l of
// wave 0 returns sum (l >> 5) (0: of g or y, 1: of the second quantity) of channel 32 cg + (l & 31); other waves 0.
// Every thread of the 1024-thread workgroup calls it (two barriers; the LDS is free again on return).
__device__ __forceinline__ float fold_chunk(const float* __restrict__ part, int p0, int p1, int C, int cg) {
  __shared__ float red[2][kFinStreams][kFinCh];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane & 7, j = w * 8 + (lane >> 3);
  const int c = cg * kFinCh + 4 * q;
  float4 a1[4], a2[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) a1[u] = a2[u] = f4(0.f);
  if (c < C) {  // C % 4 == 0: a 4-channel group is wholly in or out
    int p = p0 + j;
    // 8 partials (16 loads) in flight per lane, then 4, then 1: accumulator u still takes parts p + u S, p + (u + 4) S,
    // .. in ascending order, so the sums are those of the 4-part loop (one HBM round trip per 8 parts, not per 4:
    // the finishes of 2048 partials measured 14 us, four round trips)
    for (; p + 7 * kFinStreams < p1; p += 8 * kFinStreams) {
      float4 x1[8], x2[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float* r = part + (size_t)(p + u * kFinStreams) * 2 * C + c;
        x1[u] = ld4f(r, 0);
        x2[u] = ld4f(r + C, 0);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float4& b1 = a1[u & 3];
        float4& b2 = a2[u & 3];
        b1.x += x1[u].x; b1.y += x1[u].y; b1.z += x1[u].z; b1.w += x1[u].w;
        b2.x += x2[u].x; b2.y += x2[u].y; b2.z += x2[u].z; b2.w += x2[u].w;
      }
    }
    for (; p + 3 * kFinStreams < p1; p += 4 * kFinStreams) {
      float4 x1[4], x2[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* r = part + (size_t)(p + u * kFinStreams) * 2 * C + c;
        x1[u] = ld4f(r, 0);
        x2[u] = ld4f(r + C, 0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a1[u].x += x1[u].x; a1[u].y += x1[u].y; a1[u].z += x1[u].z; a1[u].w += x1[u].w;
        a2[u].x += x2[u].x; a2[u].y += x2[u].y; a2[u].z += x2[u].z; a2[u].w += x2[u].w;
      }
    }
    for (; p < p1; p += kFinStreams) {
      const float* r = part + (size_t)p * 2 * C + c;
      const float4 x1 = ld4f(r, 0), x2 = ld4f(r + C, 0);
      a1[0].x += x1.x; a1[0].y += x1.y; a1[0].z += x1.z; a1[0].w += x1.w;
      a2[0].x += x2.x; a2[0].y += x2.y; a2[0].z += x2.z; a2[0].w += x2.w;
    }
  }
  const float4 t1 = make_float4((a1[0].x + a1[1].x) + (a1[2].x + a1[3].x), (a1[0].y + a1[1].y) + (a1[2].y + a1[3].y),
                                (a1[0].z + a1[1].z) + (a1[2].z + a1[3].z), (a1[0].w + a1[1].w) + (a1[2].w + a1[3].w));
  const float4 t2 = make_float4((a2[0].x + a2[1].x) + (a2[2].x + a2[3].x), (a2[0].y + a2[1].y) + (a2[2].y + a2[3].y),
                                (a2[0].z + a2[1].z) + (a2[2].z + a2[3].z), (a2[0].w + a2[1].w) + (a2[2].w + a2[3].w));
  *reinterpret_cast<float4*>(&red[0][j][4 * q]) = t1;
  *reinterpret_cast<float4*>(&red[1][j][4 * q]) = t2;
  __syncthreads();
  float s = 0.f;
  if (w == 0) {
    const int which = lane >> 5, ch = lane & 31;
#pragma unroll 16
    for (int i = 0; i < kFinStreams; ++i) s += red[which][i][ch];
  }
  __syncthreads();
  return s;
}

// Sum of the per-block partials [P][2][C] for kFinCh = 32 channels per workgroup.  Lane l of wave w
// reads channels 4 (l & 7) .. +3 of its slice (one 16-B load per sum; 8 lanes cover a 128-B row
// segment) from partials j, j + 128, j + 256, .. with j = 8 w + (l >> 3): 128 partial streams per
// workgroup, each lane with 4 partials (8 loads) in flight.  Wave 0 then folds the 128 stream sums in a
// fixed order through LDS (lanes 0-31: S1, lanes 32-63: S2), so the result is bit-stable; chunks of kFoldQ parts
// in chunk order.  Round 2's version (64 channels per workgroup, lane = channel, one 4-B load per lane and sum)
// kept a quarter of the bytes in flight on half the workgroups: 7-8 us per finish at P = 512-2048.
// Split form (gridDim.y = the chunk count, cnt / ws given): workgroup (x, y) folds chunk y of channel group x, stores
// its 64 sums write-through (sc1) and adds one to cnt[x] once that wave's stores are complete; the workgroup whose
// add returns S - 1 reads the S chunk sums (sc1 loads), adds them in chunk order -- the sequential form's bits -- and
// re-arms cnt[x] (MICROARCH inter-workgroup table row 1: the last adder told by its add's return value).
__device__ __forceinline__ bool fold_partials(const float* __restrict__ part, int P, int C, float& s1, float& s2,
                                              int& c_out, int* cnt = nullptr, float* ws = nullptr) {
  const int S = fold_chunks(P);
  float tot = 0.f;
  if (gridDim.y == 1) {
    for (int k = 0; k < S; ++k) {
      const int p0 = k * kFoldQ, p1 = p0 + kFoldQ < P ? p0 + kFoldQ : P;
      const float v = fold_chunk(part, p0, p1, C, blockIdx.x);
      tot = k == 0 ? v : tot + v;
    }
    if (threadIdx.x >= 64) return false;
  } else {
    const int k = blockIdx.y, p0 = k * kFoldQ, p1 = p0 + kFoldQ < P ? p0 + kFoldQ : P;
    const float v = fold_chunk(part, p0, p1, C, blockIdx.x);
    if (threadIdx.x >= 64) return false;
    const int lane = threadIdx.x;
    float* slot = ws + (size_t)blockIdx.x * S * 64;
    st_sc1(slot + k * 64 + lane, v);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int old = 0;
    // acq_rel: the add releases this workgroup's chunk sums and acquires the others' for the last adder, so
    // the hand-off is ordered by the memory model, not only by the sc1 encoding and the wait above
    if (lane == 0) old = __hip_atomic_fetch_add(cnt + blockIdx.x, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (__shfl(old, 0) != S - 1) return false;
    tot = ld_sc1(slot + lane);
    for (int q = 1; q < S; ++q) tot += ld_sc1(slot + q * 64 + lane);
    if (lane == 0) __hip_atomic_store(cnt + blockIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const int lane = threadIdx.x, which = lane >> 5, ch = lane & 31;
  const float other = __shfl_xor(tot, 32);
  c_out = blockIdx.x * kFinCh + ch;
  if (which != 0 || c_out >= C) return false;
  s1 = tot;
  s2 = other;
  return true;
}

// batch statistics of channel c from its (shifted by k) sums; running statistics updated torch's way.  SC1: mean /
// rstd stored write-through for other workgroups of the same launch
template <bool SC1 = false>
__device__ __forceinline__ float bn_finish_channel(float s1, float s2, float k, int64_t rows, float eps, float momentum,
                                                   int c, float* mean, float* rstd, float* rmean, float* rvar) {
  const float n = (float)rows;
  const float m1 = s1 / n;
  const float var = fmaxf(fmaf(-m1, m1, s2 / n), 0.f);
  const float mu = k + m1;
  const float r = 1.0f / sqrtf(var + eps);
  if constexpr (SC1) {
    st_sc1(mean + c, mu);
    st_sc1(rstd + c, r);
  } else {
    mean[c] = mu;
    rstd[c] = r;
  }
  if (rmean) rmean[c] = fmaf(momentum, mu, (1.f - momentum) * rmean[c]);
  if (rvar) rvar[c] = fmaf(momentum, rows > 1 ? (var * n) / (n - 1.f) : var, (1.f - momentum) * rvar[c]);
  return r;
}

__global__ void __launch_bounds__(64 * kFinWaves) stats_finish_kernel(
    const void* __restrict__ y, int ydt, const float* __restrict__ part, int P, int64_t rows, int C, float eps,
    float momentum, float* __restrict__ mean, float* __restrict__ rstd, float* __restrict__ rmean,
    float* __restrict__ rvar, int64_t* __restrict__ nbt, int* cnt, float* ws) {
  if (nbt && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) nbt[0] += 1;
  float s1, s2;
  int c;
  if (!fold_partials(part, P, C, s1, s2, c, cnt, ws)) return;
  // shift k: row 0 of y (sv_bn_stats partials); y == NULL: unshifted partials (SV_EPI_STORE_STATS)
  const float k = y == nullptr ? 0.f
                  : ydt == SV_F32 ? reinterpret_cast<const float*>(y)[c] : bf2f(reinterpret_cast<const uint16_t*>(y)[c]);
  bn_finish_channel(s1, s2, k, rows, eps, momentum, c, mean, rstd, rmean, rvar);
}

__global__ void eval_params_kernel(const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                   float* __restrict__ mean, float* __restrict__ rstd, int C) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  rstd[c] = 1.0f / sqrtf(rv[c] + eps);
}

struct ActArgs {
  const void* y; int ydt;
  const float *mean, *rstd, *gamma, *beta;
  const void* res; int rdt;
  const float *rmean, *rrstd, *rgamma, *rbeta;
  int relu;
  void* out; int odt;
  int64_t rows; int C;
};

// FIXC: the grid's stride is a multiple of C (host: grid * kThreads * V % C == 0), so each thread's V channels are the
// same at every grid-stride step and their parameters are loaded once, not per element group (8 of the 10 loads of
// an iteration were those L1 / L2 reads); the arithmetic is the same
template <int V, bool FIXC = false>
__global__ void __launch_bounds__(kThreads) act_kernel(const ActArgs a) {
  const int64_t nv = a.rows * a.C / V;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  auto body = [&](size_t e, const float (&mu)[V], const float (&rs)[V], const float (&g)[V], const float (&b)[V],
                  const float (&rm)[V], const float (&rr)[V], const float (&rg)[V], const float (&rb)[V]) {
    float v[V], o[V];
    ldv<V>(a.y, a.ydt, e, v);
#pragma unroll
    for (int q = 0; q < V; ++q) o[q] = bn_pre(g[q], rs[q], v[q], mu[q], b[q]);
    if (a.res) {
      float r[V];
      ldv<V>(a.res, a.rdt, e, r);
      if (a.rmean) {
#pragma unroll
        for (int q = 0; q < V; ++q) r[q] = bn_pre(rg[q], rr[q], r[q], rm[q], rb[q]);
      }
#pragma unroll
      for (int q = 0; q < V; ++q) o[q] += r[q];
    }
    if (a.relu) {
#pragma unroll
      for (int q = 0; q < V; ++q) o[q] = fmaxf(o[q], 0.f);
    }
    stv<V>(a.out, a.odt, e, o);
  };
  auto params = [&](int c, float (&mu)[V], float (&rs)[V], float (&g)[V], float (&b)[V], float (&rm)[V],
                    float (&rr)[V], float (&rg)[V], float (&rb)[V]) {
    ldp<V>(a.mean, c, mu);
    ldp<V>(a.rstd, c, rs);
    ldp<V>(a.gamma, c, g);
    ldp<V>(a.beta, c, b);
    if (a.rmean) {
      ldp<V>(a.rmean, c, rm);
      ldp<V>(a.rrstd, c, rr);
      ldp<V>(a.rgamma, c, rg);
      ldp<V>(a.rbeta, c, rb);
    }
  };
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (FIXC) {
    if (i >= nv) return;
    float mu[V], rs[V], g[V], b[V], rm[V], rr[V], rg[V], rb[V];
    params(chan_of((size_t)i * V, a.C, a.rows * a.C), mu, rs, g, b, rm, rr, rg, rb);
    for (; i < nv; i += stride) body((size_t)i * V, mu, rs, g, b, rm, rr, rg, rb);
  } else {
    for (; i < nv; i += stride) {
      const size_t e = (size_t)i * V;
      float mu[V], rs[V], g[V], b[V], rm[V], rr[V], rg[V], rb[V];
      params(chan_of(e, a.C, a.rows * a.C), mu, rs, g, b, rm, rr, rg, rb);
      body(e, mu, rs, g, b, rm, rr, rg, rb);
    }
  }
}

__device__ __forceinline__ float4 masked(float4 g, const void* act, int adt, size_t e) {
  if (act) {
    const float4 m = ld4d(act, adt, e);
    g.x = m.x > 0.f ? g.x : 0.f;
    g.y = m.y > 0.f ? g.y : 0.f;
    g.z = m.z > 0.f ? g.z : 0.f;
    g.w = m.w > 0.f ? g.w : 0.f;
  }
  return g;
}

__host__ __device__ __forceinline__ int pool_out(int n) { return (n + 2 - 3) / 2 + 1; }

// The max-pool 3x3/2 (pad 1) backward as a gather, for BatchNorm passes that read the pooled layer's
// input gradient without materialising it: channels c .. c+V-1 of input pixel e / C, the sum of the
// output gradients d [B][OH][OW][C] (f32) whose argmax tap (idx) is this pixel, windows taken in the
// order of maxpool_bwd_kernel (oy, then ox, ascending) so the values are bit for bit its output.
struct PoolSrc {
  const void* d;
  const uint8_t* idx;
  int H, W;
  int ddt;  // d's dtype (SV_F32 = 0 when omitted)
};

template <int V>
__device__ __forceinline__ void pool_grad(const PoolSrc& p, int C, size_t e, float (&g)[V]) {
  const int OH = pool_out(p.H), OW = pool_out(p.W);
  // pixel coordinates in 32-bit arithmetic (the host guarantees B*H*W*C < 2^31): 64-bit division is a long
  // software sequence on the GPU, and this runs once per element group in both BatchNorm passes
  const uint32_t ee = (uint32_t)e, uC = (uint32_t)C;
  const int c = (int)(ee % uC);
  const uint32_t pix = ee / uC, rowi = pix / (uint32_t)p.W;
  const int ix = (int)(pix - rowi * (uint32_t)p.W);
  const uint32_t bq = rowi / (uint32_t)p.H;
  const int iy = (int)(rowi - bq * (uint32_t)p.H);
  const int64_t b = (int64_t)bq;
#pragma unroll
  for (int q = 0; q < V; ++q) g[q] = 0.f;
  const int oy0 = iy / 2, oy1 = (iy + 1) / 2;
  const int ox0 = ix / 2, ox1 = (ix + 1) / 2;
  for (int oy = oy0; oy <= oy1 && oy < OH; ++oy) {
    const int kh = iy - (2 * oy - 1);
    if (kh < 0 || kh > 2) continue;
    for (int ox = ox0; ox <= ox1 && ox < OW; ++ox) {
      const int kw = ix - (2 * ox - 1);
      if (kw < 0 || kw > 2) continue;
      const size_t o = (size_t)((b * OH + oy) * OW + ox) * C + c;
      const int tap = kh * 3 + kw;
      uint32_t ib[V / 4];
#pragma unroll
      for (int k = 0; k < V / 4; ++k) ib[k] = *reinterpret_cast<const uint32_t*>(p.idx + o + 4 * k);
      float dv[V];
      ldv<V>(p.d, p.ddt, o, dv);
#pragma unroll
      for (int q = 0; q < V; ++q)
        if ((int)((ib[q >> 2] >> (8 * (q & 3))) & 0xffu) == tap) g[q] += dv[q];
    }
  }
}

// g = dout * mask: mask = (act > 0), or (RELU_Y) recomputed from y as act_kernel computes the
// pre-activation -- fmaf(gamma rstd, y - mean, beta) > 0 -- so the activation is not read again.
// POOL: dout is the max-pool backward of `pool` (pool_grad), gathered in place of a load.
// ga / be: the BatchNorm's gamma / beta at c .. c+V-1 when the caller has them in registers (RELU_Y), else loaded here
template <int V, bool RELU_Y, bool POOL = false>
__device__ __forceinline__ void grad_masked(const void* dout, int ddt, const void* act, int adt, size_t e,
                                            const float (&v)[V], const float (&mu)[V], const float (&rs)[V],
                                            const float* gamma, const float* beta, int c, float (&g)[V],
                                            const PoolSrc* pool = nullptr, int C = 0, const float* ga_pre = nullptr,
                                            const float* be_pre = nullptr) {
  if constexpr (POOL) pool_grad<V>(*pool, C, e, g);
  else ldv<V>(dout, ddt, e, g);
  if constexpr (RELU_Y) {
    float ga[V], be[V];
    if (ga_pre) {
#pragma unroll
      for (int q = 0; q < V; ++q) ga[q] = ga_pre[q], be[q] = be_pre[q];
    } else {
      ldp<V>(gamma, c, ga);
      ldp<V>(beta, c, be);
    }
#pragma unroll
    for (int q = 0; q < V; ++q) g[q] = bn_pre(ga[q], rs[q], v[q], mu[q], be[q]) > 0.f ? g[q] : 0.f;
  } else {
    if (act) {
      float m[V];
      ldv<V>(act, adt, e, m);
#pragma unroll
      for (int q = 0; q < V; ++q) g[q] = m[q] > 0.f ? g[q] : 0.f;
    }
  }
}

// backward statistics: sum g and sum g * xhat
template <int V, bool RELU_Y, bool POOL = false>
// (dout is not __restrict__: sv_bn_bwd_stats_mask passes it as gout too and writes g back over it)
__global__ void __launch_bounds__(kThreads) bwd_stats_kernel(const void* dout, int ddt,
                                                             const void* __restrict__ act, int adt,
                                                             const void* __restrict__ y, int ydt,
                                                             const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, int64_t rows, int C,
                                                             int tpr, int rp, int64_t rpp, float* __restrict__ part,
                                                             void* gout, const PoolSrc pool) {
  // gout (act-mask form): g = dout * (act > 0) written back over dout (its dtype: the ResNet gradient stream is
  // bf16 in the bf16 model) by the thread that read it, so the apply pass and the block's shortcut read the masked
  // gradient without a separate copy
  const int t = threadIdx.x;
  const int c = (blockIdx.x * tpr + t % tpr) * V;
  const int rsub = t / tpr;
  float mu[V], rs[V], s1[V], s2[V], ga[V], be[V];
  ldp<V>(mean, c, mu);
  ldp<V>(rstd, c, rs);
  if constexpr (RELU_Y) {  // once per thread: gout's stores may alias them, so the compiler would reload per row
    ldp<V>(gamma, c, ga);
    ldp<V>(beta, c, be);
  }
#pragma unroll
  for (int q = 0; q < V; ++q) s1[q] = s2[q] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.y * rpp;
  int64_t r1 = r0 + rpp;
  if (r1 > rows) r1 = rows;
  int64_t r = r0 + rsub;
  // two rows per iteration: both rows' loads are issued before either is accumulated (the thread's
  // rows are still summed in ascending order, so the partials are bit-identical to the one-row loop)
  for (; r + rp < r1; r += 2 * rp) {
    const size_t e0 = (size_t)r * C + c, e1 = e0 + (size_t)rp * C;
    float v0[V], g0[V], v1[V], g1[V];
    ldv<V>(y, ydt, e0, v0);
    ldv<V>(y, ydt, e1, v1);
    grad_masked<V, RELU_Y, POOL>(dout, ddt, act, adt, e0, v0, mu, rs, gamma, beta, c, g0, &pool, C,
                                 RELU_Y ? ga : nullptr, RELU_Y ? be : nullptr);
    grad_masked<V, RELU_Y, POOL>(dout, ddt, act, adt, e1, v1, mu, rs, gamma, beta, c, g1, &pool, C,
                                 RELU_Y ? ga : nullptr, RELU_Y ? be : nullptr);
    if (gout) {
      stv<V>(gout, ddt, e0, g0);
      stv<V>(gout, ddt, e1, g1);
    }
#pragma unroll
    for (int q = 0; q < V; ++q) {
      s1[q] += g0[q];
      s2[q] = fmaf(g0[q], (v0[q] - mu[q]) * rs[q], s2[q]);
      s1[q] += g1[q];
      s2[q] = fmaf(g1[q], (v1[q] - mu[q]) * rs[q], s2[q]);
    }
  }
  for (; r < r1; r += rp) {
    const size_t e = (size_t)r * C + c;
    float v[V], g[V];
    ldv<V>(y, ydt, e, v);
    grad_masked<V, RELU_Y, POOL>(dout, ddt, act, adt, e, v, mu, rs, gamma, beta, c, g, &pool, C,
                                 RELU_Y ? ga : nullptr, RELU_Y ? be : nullptr);
    if (gout) stv<V>(gout, ddt, e, g);
#pragma unroll
    for (int q = 0; q < V; ++q) {
      s1[q] += g[q];
      s2[q] = fmaf(g[q], (v[q] - mu[q]) * rs[q], s2[q]);
    }
  }
  reduce_write<V>(s1, s2, tpr, rp, c, C, part);
}

__global__ void __launch_bounds__(64 * kFinWaves) bwd_finish_kernel(const float* __restrict__ part, int P, int C,
                                                                     float* __restrict__ sums,
                                                                     float* __restrict__ dgamma,
                                                                     float* __restrict__ dbeta, int* cnt,
                                                                     float* ws) {
  float s1, s2;
  int c;
  if (!fold_partials(part, P, C, s1, s2, c, cnt, ws)) return;
  sums[c] = s1;
  sums[C + c] = s2;
  if (dgamma) dgamma[c] += s2;
  if (dbeta) dbeta[c] += s1;
}

// A residual block with a projection shortcut: its output gradient d feeds two BatchNorms (the main path's
// last, y, and the shortcut's, y2) through the same ReLU mask.  One pass: g = d * (act > 0) written over d,
// the main BN's sums (g, g * xhat) and the shortcut BN's g * xhat2 (its sum of g is the same), in the order of
// bwd_stats_kernel (bit for bit its partials for either BatchNorm), reading d once instead of twice.
template <int V>
__global__ void __launch_bounds__(kThreads) bwd_stats_dual_kernel(void* __restrict__ dout, int ddt, const void* __restrict__ act,
                                                                  int adt, const void* __restrict__ y, int ydt,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ rstd,
                                                                  const void* __restrict__ y2, int y2dt,
                                                                  const float* __restrict__ mean2,
                                                                  const float* __restrict__ rstd2, int64_t rows, int C,
                                                                  int tpr, int rp, int64_t rpp, float* __restrict__ part,
                                                                  float* __restrict__ part2) {
  const int t = threadIdx.x;
  const int c = (blockIdx.x * tpr + t % tpr) * V;
  const int rsub = t / tpr;
  float mu[V], rs[V], mu2[V], rs2[V], s1[V], s2[V], s3[V];
  ldp<V>(mean, c, mu);
  ldp<V>(rstd, c, rs);
  ldp<V>(mean2, c, mu2);
  ldp<V>(rstd2, c, rs2);
#pragma unroll
  for (int q = 0; q < V; ++q) s1[q] = s2[q] = s3[q] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.y * rpp;
  int64_t r1 = r0 + rpp;
  if (r1 > rows) r1 = rows;
  int64_t r = r0 + rsub;
  for (; r + rp < r1; r += 2 * rp) {
    const size_t e0 = (size_t)r * C + c, e1 = e0 + (size_t)rp * C;
    float v0[V], g0[V], v1[V], g1[V], w0[V], w1[V];
    ldv<V>(y, ydt, e0, v0);
    ldv<V>(y, ydt, e1, v1);
    ldv<V>(y2, y2dt, e0, w0);
    ldv<V>(y2, y2dt, e1, w1);
    grad_masked<V, false>(dout, ddt, act, adt, e0, v0, mu, rs, nullptr, nullptr, c, g0);
    grad_masked<V, false>(dout, ddt, act, adt, e1, v1, mu, rs, nullptr, nullptr, c, g1);
    stv<V>(dout, ddt, e0, g0);
    stv<V>(dout, ddt, e1, g1);
#pragma unroll
    for (int q = 0; q < V; ++q) {
      s1[q] += g0[q];
      s2[q] = fmaf(g0[q], (v0[q] - mu[q]) * rs[q], s2[q]);
      s3[q] = fmaf(g0[q], (w0[q] - mu2[q]) * rs2[q], s3[q]);
      s1[q] += g1[q];
      s2[q] = fmaf(g1[q], (v1[q] - mu[q]) * rs[q], s2[q]);
      s3[q] = fmaf(g1[q], (w1[q] - mu2[q]) * rs2[q], s3[q]);
    }
  }
  for (; r < r1; r += rp) {
    const size_t e = (size_t)r * C + c;
    float v[V], g[V], w[V];
    ldv<V>(y, ydt, e, v);
    ldv<V>(y2, y2dt, e, w);
    grad_masked<V, false>(dout, ddt, act, adt, e, v, mu, rs, nullptr, nullptr, c, g);
    stv<V>(dout, ddt, e, g);
#pragma unroll
    for (int q = 0; q < V; ++q) {
      s1[q] += g[q];
      s2[q] = fmaf(g[q], (v[q] - mu[q]) * rs[q], s2[q]);
      s3[q] = fmaf(g[q], (w[q] - mu2[q]) * rs2[q], s3[q]);
    }
  }
  float s1b[V];
#pragma unroll
  for (int q = 0; q < V; ++q) s1b[q] = s1[q];
  reduce_write<V>(s1, s2, tpr, rp, c, C, part);
  __syncthreads();  // reduce_write's LDS is reused
  reduce_write<V>(s1b, s3, tpr, rp, c, C, part2);
}

struct BwdArgs {
  const void* dout; int ddt;
  const void* act; int adt;
  const void* y; int ydt;
  const float *mean, *rstd, *gamma, *beta, *sums;
  void* dx; int xdt;
  float* gmask;
  int64_t rows; int C;
  PoolSrc pool;  // POOL instantiations: dout is the max-pool backward of pool.d (gathered)
};

template <int V, bool RELU_Y, bool POOL = false, bool FIXC = false>
__global__ void __launch_bounds__(kThreads) bwd_apply_kernel(const BwdArgs a) {
  const int64_t nv = a.rows * a.C / V;
  const float inv_n = 1.0f / (float)a.rows;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (FIXC) {  // see act_kernel: the channel's parameters once per thread; the same arithmetic
    if (i >= nv) return;
    const int c = chan_of((size_t)i * V, a.C, a.rows * a.C);
    float mu[V], rs[V], ga[V], be[V], sg[V], sgx[V];
    ldp<V>(a.mean, c, mu);
    ldp<V>(a.rstd, c, rs);
    ldp<V>(a.gamma, c, ga);
    if constexpr (RELU_Y) ldp<V>(a.beta, c, be);
    ldp<V>(a.sums, c, sg);
    ldp<V>(a.sums + a.C, c, sgx);
    for (; i < nv; i += stride) {
      const size_t e = (size_t)i * V;
      float v[V], g[V], o[V];
      ldv<V>(a.y, a.ydt, e, v);
      if constexpr (POOL) pool_grad<V>(a.pool, a.C, e, g);
      else ldv<V>(a.dout, a.ddt, e, g);
      if constexpr (RELU_Y) {
#pragma unroll
        for (int q = 0; q < V; ++q) g[q] = bn_pre(ga[q], rs[q], v[q], mu[q], be[q]) > 0.f ? g[q] : 0.f;
      } else if (a.act) {
        float m[V];
        ldv<V>(a.act, a.adt, e, m);
#pragma unroll
        for (int q = 0; q < V; ++q) g[q] = m[q] > 0.f ? g[q] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < V; ++q)
        o[q] = bn_dx(ga[q], rs[q], g[q], sg[q], v[q], mu[q], sgx[q], inv_n);
      stv<V>(a.dx, a.xdt, e, o);
      if (a.gmask) stv<V>(a.gmask, SV_F32, e, g);
    }
    return;
  }
  for (; i < nv; i += stride) {
    const size_t e = (size_t)i * V;
    const int c = chan_of(e, a.C, a.rows * a.C);
    float v[V], mu[V], rs[V], ga[V], sg[V], sgx[V], g[V], o[V];
    ldv<V>(a.y, a.ydt, e, v);
    ldp<V>(a.mean, c, mu);
    ldp<V>(a.rstd, c, rs);
    grad_masked<V, RELU_Y, POOL>(a.dout, a.ddt, a.act, a.adt, e, v, mu, rs, a.gamma, a.beta, c, g, &a.pool, a.C);
    ldp<V>(a.gamma, c, ga);
    ldp<V>(a.sums, c, sg);
    ldp<V>(a.sums + a.C, c, sgx);
#pragma unroll
    for (int q = 0; q < V; ++q)
      o[q] = bn_dx(ga[q], rs[q], g[q], sg[q], v[q], mu[q], sgx[q], inv_n);
    stv<V>(a.dx, a.xdt, e, o);
    if (a.gmask) stv<V>(a.gmask, SV_F32, e, g);
  }
}

// both BatchNorms' data gradients from the shared masked gradient g (bwd_apply_kernel's formula for each)
struct BwdDualArgs {
  const void* g; int gdt;
  const void* y; int ydt;
  const float *mean, *rstd, *gamma, *sums;
  const void* y2; int y2dt;
  const float *mean2, *rstd2, *gamma2, *sums2;
  void* dx; void* dx2; int xdt;
  int64_t rows; int C;
};

template <int V>
__global__ void __launch_bounds__(kThreads) bwd_apply_dual_kernel(const BwdDualArgs a) {
  const int64_t nv = a.rows * a.C / V;
  const float inv_n = 1.0f / (float)a.rows;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    const size_t e = (size_t)i * V;
    const int c = chan_of(e, a.C, a.rows * a.C);
    float g[V], v[V], w[V], o[V], o2[V], mu[V], rs[V], ga[V], sg[V], sgx[V];
    ldv<V>(a.g, a.gdt, e, g);
    ldv<V>(a.y, a.ydt, e, v);
    ldv<V>(a.y2, a.y2dt, e, w);
    ldp<V>(a.mean, c, mu);
    ldp<V>(a.rstd, c, rs);
    ldp<V>(a.gamma, c, ga);
    ldp<V>(a.sums, c, sg);
    ldp<V>(a.sums + a.C, c, sgx);
#pragma unroll
    for (int q = 0; q < V; ++q)
      o[q] = bn_dx(ga[q], rs[q], g[q], sg[q], v[q], mu[q], sgx[q], inv_n);
    ldp<V>(a.mean2, c, mu);
    ldp<V>(a.rstd2, c, rs);
    ldp<V>(a.gamma2, c, ga);
    ldp<V>(a.sums2, c, sg);
    ldp<V>(a.sums2 + a.C, c, sgx);
#pragma unroll
    for (int q = 0; q < V; ++q)
      o2[q] = bn_dx(ga[q], rs[q], g[q], sg[q], w[q], mu[q], sgx[q], inv_n);
    stv<V>(a.dx, a.xdt, e, o);
    stv<V>(a.dx2, a.xdt, e, o2);
  }
}

__global__ void __launch_bounds__(kThreads) relu_mask_kernel(const void* __restrict__ dout, int ddt,
                                                             const void* __restrict__ act, int adt, float* __restrict__ g,
                                                             int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const size_t e = (size_t)i * 4;
    *reinterpret_cast<float4*>(g + e) = masked(ld4d(dout, ddt, e), act, adt, e);
  }
}

// ---- pooling -------------------------------------------------------------------------------------

__global__ void __launch_bounds__(kThreads) maxpool_fwd_kernel(const void* __restrict__ x, int xdt, void* __restrict__ y,
                                                               uint8_t* __restrict__ idx, int B, int H, int W, int C) {
  const int OH = pool_out(H), OW = pool_out(W);
  const int64_t n4 = (int64_t)B * OH * OW * C / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 4;
    int c, ox, oy;
    int64_t b;
    if (n4 * 4 <= 0xffffffffll) {  // 32-bit index arithmetic (see chan_of)
      const uint32_t ee = (uint32_t)e, pix = ee / (uint32_t)C, r = pix / (uint32_t)OW, bq = r / (uint32_t)OH;
      c = (int)(ee - pix * (uint32_t)C);
      ox = (int)(pix - r * (uint32_t)OW);
      oy = (int)(r - bq * (uint32_t)OH);
      b = bq;
    } else {
      const int64_t pix = e / C;
      c = (int)(e % C);
      ox = (int)(pix % OW);
      oy = (int)((pix / OW) % OH);
      b = pix / ((int64_t)OW * OH);
    }
    float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int arg[4] = {-1, -1, -1, -1};
    for (int kh = 0; kh < 3; ++kh) {
      const int iy = 2 * oy - 1 + kh;
      if ((unsigned)iy >= (unsigned)H) continue;
      for (int kw = 0; kw < 3; ++kw) {
        const int ix = 2 * ox - 1 + kw;
        if ((unsigned)ix >= (unsigned)W) continue;
        const float4 v = ld4d(x, xdt, (size_t)((b * H + iy) * W + ix) * C + c);
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (arg[u] < 0 || vv[u] > best[u] || vv[u] != vv[u]) {
            best[u] = vv[u];
            arg[u] = kh * 3 + kw;
          }
      }
    }
    st4d(y, xdt, (size_t)e, make_float4(best[0], best[1], best[2], best[3]));
    *reinterpret_cast<uchar4*>(idx + e) = make_uchar4((uint8_t)arg[0], (uint8_t)arg[1], (uint8_t)arg[2], (uint8_t)arg[3]);
  }
}

__global__ void __launch_bounds__(kThreads) maxpool_bwd_kernel(const void* __restrict__ dout, int ddt,
                                                               const uint8_t* __restrict__ idx, void* __restrict__ dx,
                                                               int xdt, int B, int H, int W, int C) {
  const int OH = pool_out(H), OW = pool_out(W);
  const int64_t n4 = (int64_t)B * H * W * C / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 4;
    const int c = (int)(e % C);
    const int64_t pix = e / C;
    const int ix = (int)(pix % W), iy = (int)((pix / W) % H);
    const int64_t b = pix / ((int64_t)W * H);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    // windows oy with 2 oy - 1 <= iy <= 2 oy + 1
    const int oy0 = iy / 2, oy1 = (iy + 1) / 2;
    const int ox0 = ix / 2, ox1 = (ix + 1) / 2;
    for (int oy = oy0; oy <= oy1 && oy < OH; ++oy) {
      const int kh = iy - (2 * oy - 1);
      if (kh < 0 || kh > 2) continue;
      for (int ox = ox0; ox <= ox1 && ox < OW; ++ox) {
        const int kw = ix - (2 * ox - 1);
        if (kw < 0 || kw > 2) continue;
        const size_t o = (size_t)((b * OH + oy) * OW + ox) * C + c;
        const uchar4 a = *reinterpret_cast<const uchar4*>(idx + o);
        const float4 g = ld4d(dout, ddt, o);
        const int tap = kh * 3 + kw;
        if (a.x == tap) acc[0] += g.x;
        if (a.y == tap) acc[1] += g.y;
        if (a.z == tap) acc[2] += g.z;
        if (a.w == tap) acc[3] += g.w;
      }
    }
    st4d(dx, xdt, (size_t)e, make_float4(acc[0], acc[1], acc[2], acc[3]));
  }
}

__global__ void __launch_bounds__(kThreads) avgpool_fwd_kernel(const void* __restrict__ x, int xdt, float* __restrict__ feat,
                                                               int B, int HW, int C) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over B*C/4
  if (i >= (int64_t)B * C / 4) return;
  const int c = (int)((i * 4) % C);
  const int64_t b = i * 4 / C;
  float4 s = f4(0.f);
  for (int p = 0; p < HW; ++p) {
    const float4 v = ld4d(x, xdt, (size_t)((b * HW + p) * C + c));
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const float inv = 1.0f / (float)HW;
  *reinterpret_cast<float4*>(feat + b * C + c) = make_float4(s.x * inv, s.y * inv, s.z * inv, s.w * inv);
}

__global__ void __launch_bounds__(kThreads) avgpool_bwd_kernel(const float* __restrict__ dfeat, void* __restrict__ dx,
                                                               int xdt, int B, int HW, int C) {
  const int64_t n4 = (int64_t)B * HW * C / 4;
  const float inv = 1.0f / (float)HW;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 4;
    const int c = (int)(e % C);
    const int64_t b = e / ((int64_t)HW * C);
    const float4 g = *reinterpret_cast<const float4*>(dfeat + b * C + c);
    st4d(dx, xdt, (size_t)e, make_float4(g.x * inv, g.y * inv, g.z * inv, g.w * inv));
  }
}


// ---- one launch per BatchNorm for small row counts (ResNet layers 3-4 at 256 px: rows <= 8192) ------------
// Every BatchNorm backward above is three launches (statistics partials, their fold, the apply) and every
// train-mode forward two (the fold of the conv epilogue's partials, the activation).  At layers 3-4 each of
// those kernels costs 4-7 us of launch and fill whatever its bytes.  Here ONE workgroup
// of 1024 threads owns 8 channels over ALL rows, so the statistics need no other workgroup and the pass that
// uses them follows in the same launch.  The arithmetic is the multi-launch path's, in its order:
//   * thread t is "cell" (p, rsub) of bwd_stats_kernel's geometry (nparts_for: P parts of rpp rows, rp row
//     groups per part): it sums rows p*rpp + rsub, + rp, .. in ascending order, as that kernel's thread does;
//   * the rp cells of a part are added in rsub order (reduce_write), and the P part sums are folded in
//     fold_partials' order (128 streams of 4 accumulators, then the streams in order);
// so sums, gamma / beta gradients, data gradients (and the forward's mean, rstd, running statistics and
// activation) are bit for bit the multi-launch results (tests/test_bn_small_gpu.py).  Channel slices are dealt
// XCD-contiguously (blocks b and b + 8 share an XCD under round-robin placement and get neighbouring slices),
// so the 8 slices of one 128-B bf16 line read it through one L2.
constexpr int kSmallThreads = 1024, kSmallStreams = 128;

__device__ __forceinline__ int small_slice(int G) {
  const int b = blockIdx.x;
  return (G & 7) == 0 ? (b & 7) * (G >> 3) + (b >> 3) : b;
}

// fold_partials' order for channel c + q of one sum: stream j (0..127) over parts j, j + 128, ..; -> stream sum
template <typename F>
__device__ __forceinline__ float stream_fold(F&& part_at, int j, int P) {
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  int p = j;
  for (; p + 3 * kSmallStreams < P; p += 4 * kSmallStreams) {
    float x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = part_at(p + u * kSmallStreams);
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += x[u];
  }
  for (; p < P; p += kSmallStreams) a[0] += part_at(p);
  return (a[0] + a[1]) + (a[2] + a[3]);
}

struct SmallBwdArgs {
  void* dout; int ddt;             // MODE 0 / 2: overwritten with g = dout * (act > 0) (in its dtype)
  const void* act; int adt;
  const void* y; int ydt;
  const float *mean, *rstd, *gamma, *beta;  // beta: MODE 1 (the BN's own ReLU, recomputed from y)
  const void* y2; int y2dt;                 // MODE 2: the projection shortcut's BatchNorm
  const float *mean2, *rstd2, *gamma2;
  const float* part; int npart;             // GIVEN: the statistics partials [npart][2][C] its producer summed
  void* dx; void* dx2; int xdt;
  float *dgamma, *dbeta, *dgamma2, *dbeta2;
  int batch_stats;
  int rows, C, P, rp, rpp;                  // nparts_for geometry
};

// MODE 0: act-mask form in place (sv_bn_bwd_stats_mask + finish + apply); 1: ReLU recomputed from y
// (sv_bn_relu_bwd_stats + finish + apply; GIVEN: the statistics pass skipped, `part` folded); 2: dual
// (sv_bn_bwd_stats_mask_dual + two finishes + sv_bn_bwd_apply_dual)
template <int MODE, bool GIVEN>
__global__ void __launch_bounds__(kSmallThreads) bwd_small_kernel(const SmallBwdArgs a) {
  constexpr int NS = MODE == 2 ? 3 : 2;
  __shared__ float cell[GIVEN ? 1 : kSmallThreads][NS][8];
  __shared__ float fold[NS][kSmallStreams][8];
  __shared__ float tot[NS][8];
  const int t = threadIdx.x;
  const int c = small_slice(a.C >> 3) * 8;
  float mu[8], rs[8], be[8], mu2[8], rs2[8];
  ldp<8>(a.mean, c, mu);
  ldp<8>(a.rstd, c, rs);
  if constexpr (MODE == 1) ldp<8>(a.beta, c, be);
  if constexpr (MODE == 2) {
    ldp<8>(a.mean2, c, mu2);
    ldp<8>(a.rstd2, c, rs2);
  }
  const int cells = a.P * a.rp;
  const int p = t / a.rp, rsub = t - p * a.rp;
  const int r0 = p * a.rpp + rsub;
  const int r1 = min((p + 1) * a.rpp, a.rows);
  float ga[8];
  ldp<8>(a.gamma, c, ga);
  if constexpr (!GIVEN) {
    float s1[8], s2[8], s3[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) s1[q] = s2[q] = s3[q] = 0.f;
    if (t < cells) {
      for (int r = r0; r < r1; r += a.rp) {
        const size_t e = (size_t)r * a.C + c;
        float v[8], g[8];
        ldv<8>(a.y, a.ydt, e, v);
        ldv<8>(a.dout, a.ddt, e, g);
        if constexpr (MODE == 1) {
#pragma unroll
          for (int q = 0; q < 8; ++q) g[q] = bn_pre(ga[q], rs[q], v[q], mu[q], be[q]) > 0.f ? g[q] : 0.f;
        } else {
          float m[8];
          ldv<8>(a.act, a.adt, e, m);
#pragma unroll
          for (int q = 0; q < 8; ++q) g[q] = m[q] > 0.f ? g[q] : 0.f;
          stv<8>(a.dout, a.ddt, e, g);
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          s1[q] += g[q];
          s2[q] = fmaf(g[q], (v[q] - mu[q]) * rs[q], s2[q]);
        }
        if constexpr (MODE == 2) {
          float w[8];
          ldv<8>(a.y2, a.y2dt, e, w);
#pragma unroll
          for (int q = 0; q < 8; ++q) s3[q] = fmaf(g[q], (w[q] - mu2[q]) * rs2[q], s3[q]);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      cell[t][0][q] = s1[q];
      cell[t][1][q] = s2[q];
      if constexpr (MODE == 2) cell[t][2][q] = s3[q];
    }
    __syncthreads();
    // part sums in reduce_write's order, written over the part's first cell (its own)
    for (int i = t; i < a.P * 8; i += kSmallThreads) {
      const int pp = i >> 3, q = i & 7;
#pragma unroll
      for (int k = 0; k < NS; ++k) {
        float acc = cell[pp * a.rp][k][q];
        for (int r = 1; r < a.rp; ++r) acc += cell[pp * a.rp + r][k][q];
        cell[pp * a.rp][k][q] = acc;
      }
    }
    __syncthreads();
  }
  {
    const int j = t >> 3, q = t & 7;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      if constexpr (GIVEN)
        fold[k][j][q] = stream_fold([&](int pp) { return a.part[(size_t)pp * 2 * a.C + (size_t)k * a.C + c + q]; }, j,
                                    a.npart);
      else
        fold[k][j][q] = stream_fold([&](int pp) { return cell[pp * a.rp][k][q]; }, j, a.P);
    }
  }
  __syncthreads();
  if (t < NS * 8) {
    const int k = t >> 3, q = t & 7;
    float sum = 0.f;
    for (int i = 0; i < kSmallStreams; ++i) sum += fold[k][i][q];
    tot[k][q] = sum;
    if (k == 0) {
      if (a.dbeta) a.dbeta[c + q] += sum;
      if (MODE == 2 && a.dbeta2) a.dbeta2[c + q] += sum;
    } else if (k == 1) {
      if (a.dgamma) a.dgamma[c + q] += sum;
    } else {
      if (a.dgamma2) a.dgamma2[c + q] += sum;
    }
  }
  __syncthreads();
  float sg[8], sgx[8], sgx2[8], ga2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    sg[q] = a.batch_stats ? tot[0][q] : 0.f;
    sgx[q] = a.batch_stats ? tot[1][q] : 0.f;
    sgx2[q] = (MODE == 2 && a.batch_stats) ? tot[NS - 1][q] : 0.f;
  }
  if constexpr (MODE == 2) ldp<8>(a.gamma2, c, ga2);
  const float inv_n = 1.0f / (float)a.rows;
  // the apply over this thread's own cell rows (MODE 0 / 2 read back the g they wrote)
  if (t < cells) {
    for (int r = r0; r < r1; r += a.rp) {
      const size_t e = (size_t)r * a.C + c;
      float v[8], g[8], o[8];
      ldv<8>(a.y, a.ydt, e, v);
      if constexpr (MODE == 1) {
        ldv<8>(a.dout, a.ddt, e, g);
#pragma unroll
        for (int q = 0; q < 8; ++q) g[q] = bn_pre(ga[q], rs[q], v[q], mu[q], be[q]) > 0.f ? g[q] : 0.f;
      } else {
        ldv<8>(a.dout, a.ddt, e, g);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = bn_dx(ga[q], rs[q], g[q], sg[q], v[q], mu[q], sgx[q], inv_n);
      stv<8>(a.dx, a.xdt, e, o);
      if constexpr (MODE == 2) {
        float w[8], o2[8];
        ldv<8>(a.y2, a.y2dt, e, w);
#pragma unroll
        for (int q = 0; q < 8; ++q) o2[q] = bn_dx(ga2[q], rs2[q], g[q], sg[q], w[q], mu2[q], sgx2[q], inv_n);
        stv<8>(a.dx2, a.xdt, e, o2);
      }
    }
  }
}

// The train-mode forward from the conv epilogue's UNSHIFTED partials [P][2][C]: fold (sv_bn_stats_finish with
// y == NULL, same order), mean / rstd / running statistics, then out = act(BN(y) + res) as act_kernel computes it,
// res = the identity shortcut or (RBN) the projection shortcut's BN from its own partials.
struct SmallActArgs {
  const void* y; int ydt;
  const float* part; int P; float eps, momentum;
  const float *gamma, *beta;
  float *mean, *rstd, *rmean, *rvar; int64_t* nbt;
  const void* res; int rdt;
  const float* rpart; int rP; float reps, rmomentum;
  const float *rgamma, *rbeta;
  float *rmean_o, *rrstd_o, *rrmean, *rrvar; int64_t* rnbt;
  int relu; void* out; int odt;
  int rows, C;
};

template <bool RES, bool RBN>
__global__ void __launch_bounds__(kSmallThreads) act_small_kernel(const SmallActArgs a) {
  constexpr int NB = RBN ? 2 : 1;
  __shared__ float fold[NB][2][kSmallStreams][8];
  __shared__ float stat[NB][2][8];
  const int t = threadIdx.x;
  const int c = small_slice(a.C >> 3) * 8;
  if (blockIdx.x == 0 && t == 0) {
    if (a.nbt) a.nbt[0] += 1;
    if (RBN && a.rnbt) a.rnbt[0] += 1;
  }
  {
    const int j = t >> 3, q = t & 7;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const float* part = nb ? a.rpart : a.part;
      const int P = nb ? a.rP : a.P;
#pragma unroll
      for (int k = 0; k < 2; ++k)
        fold[nb][k][j][q] = stream_fold([&](int pp) { return part[(size_t)pp * 2 * a.C + (size_t)k * a.C + c + q]; }, j, P);
    }
  }
  __syncthreads();
  if (t < NB * 8) {
    const int nb = t >> 3, q = t & 7;
    float s1 = 0.f, s2 = 0.f;
    for (int i = 0; i < kSmallStreams; ++i) s1 += fold[nb][0][i][q];
    for (int i = 0; i < kSmallStreams; ++i) s2 += fold[nb][1][i][q];
    if (nb == 0)
      bn_finish_channel(s1, s2, 0.f, a.rows, a.eps, a.momentum, c + q, a.mean, a.rstd, a.rmean, a.rvar);
    else
      bn_finish_channel(s1, s2, 0.f, a.rows, a.reps, a.rmomentum, c + q, a.rmean_o, a.rrstd_o, a.rrmean, a.rrvar);
    stat[nb][0][q] = nb ? a.rmean_o[c + q] : a.mean[c + q];
    stat[nb][1][q] = nb ? a.rrstd_o[c + q] : a.rstd[c + q];
  }
  __syncthreads();
  float mu[8], rs[8], g[8], b[8], rm[8], rr[8], rg[8], rb[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    mu[q] = stat[0][0][q];
    rs[q] = stat[0][1][q];
    rm[q] = stat[NB - 1][0][q];
    rr[q] = stat[NB - 1][1][q];
  }
  ldp<8>(a.gamma, c, g);
  ldp<8>(a.beta, c, b);
  if constexpr (RBN) {
    ldp<8>(a.rgamma, c, rg);
    ldp<8>(a.rbeta, c, rb);
  }
  for (int r = t; r < a.rows; r += kSmallThreads) {
    const size_t e = (size_t)r * a.C + c;
    float v[8], o[8];
    ldv<8>(a.y, a.ydt, e, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = bn_pre(g[q], rs[q], v[q], mu[q], b[q]);
    if constexpr (RES) {
      float x[8];
      ldv<8>(a.res, a.rdt, e, x);
      if constexpr (RBN) {
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = bn_pre(rg[q], rr[q], x[q], rm[q], rb[q]);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] += x[q];
    }
    if (a.relu) {
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = fmaxf(o[q], 0.f);
    }
    stv<8>(a.out, a.odt, e, o);
  }
}

// ---- the statistics fold inside the pass that consumes it ---------------------------------------------------
// Every BatchNorm above is a statistics producer (the conv GEMM epilogue, or bwd_stats), a fold launch
// (stats_finish / bwd_finish) and the apply pass.  At bs32 the 106 folds of a ResNet-50 step are 4.5-43 us each,
// mostly launch and one-CU latency: skipping them (SV_DIAG_SKIP=bn_fin) measured 7.88 -> 7.05 ms/step (r11c).  Here
// the apply pass folds the partials itself.  Its first workgroups to start (tickets from an agent-scope counter, so
// the folding workgroups are always resident ones -- no wait on an unscheduled workgroup, whatever the dispatch
// order) each fold one chunk of one 32-channel group exactly as fold_partials does (same code, same order: the
// results are bit for bit the separate fold's); with several chunks the last to arrive adds the chunk sums in chunk
// order.  The finished mean / rstd (forward) or correction sums (backward) are stored write-through (sc1), one
// counter add per channel group after that wave's stores complete; every workgroup polls the counter (one lane,
// sc1), then reads them with sc1 loads -- MI355X_MICROARCH.md's inter-workgroup table, row 1.  The last workgroup
// past the poll re-arms the counters for the next launch on the stream (ctl is per stream).
constexpr int kFoldThreads = 1024, kFoldMaxC = 2048, kFoldMaxGrid = 2048;
constexpr int kFoldSlot = 16;                   // ctl: [0] tickets, [1] channel groups finished, [2] exits,
                                                // [3] poll timeout flag, [16 + job * ncg + cg] chunk arrivals
constexpr int kFoldWsSums = 2 * 2 * kFoldMaxC;  // ws: backward correction sums [job][2][C], then the chunk sums
                                                // [job][cg][chunk][64] (lane l: sum l >> 5 of channel l & 31)
struct FoldJob {
  const float* part;
  float *mean, *rstd, *rmean, *rvar;  // forward: batch statistics (mean / rstd handed off), running statistics
  int64_t* nbt;
  float eps, momentum;
  float *dgamma, *dbeta;              // backward (the sums go to ws)
};
struct FoldCtl {
  int* ctl;
  float* ws;
  FoldJob job[2];
  int njobs, P, S, ncg, C, stats;     // stats = 0: eval-mode backward (zero correction sums)
  int64_t rows;
  int diag;                           // SV_FOLD_DIAG (timing only, results wrong): 1 = no tickets, poll or re-arm
};

template <bool BWD>
__device__ __forceinline__ void fold_phase(const FoldCtl& f) {
  __shared__ int s_ticket;
  int* const ctl = f.ctl;
  if (threadIdx.x == 0)
    s_ticket = f.diag & 1 ? (int)blockIdx.x : __hip_atomic_fetch_add(ctl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const int t = s_ticket, per_job = f.ncg * f.S;
  if (t < f.njobs * per_job) {  // workgroup-uniform: this workgroup folds chunk s of channel group cg of job
    const int job = t >= per_job ? 1 : 0, r = t - job * per_job, cg = r / f.S, s = r - cg * f.S;
    const FoldJob J = job ? f.job[1] : f.job[0];
    const int p0 = s * kFoldQ, p1 = p0 + kFoldQ < f.P ? p0 + kFoldQ : f.P;
    float v = fold_chunk(J.part, p0, p1, f.C, cg);
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      bool fin = true;
      if (f.S > 1) {
        float* slot = f.ws + kFoldWsSums + (size_t)(job * f.ncg + cg) * f.S * 64;
        st_sc1(slot + s * 64 + lane, v);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        int old = 0;
        if (lane == 0)
          old = __hip_atomic_fetch_add(ctl + kFoldSlot + job * f.ncg + cg, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        fin = __shfl(old, 0) == f.S - 1;
        if (fin) {  // every chunk of this channel group has landed: their sums in chunk order
          float tot = ld_sc1(slot + lane);
          for (int k = 1; k < f.S; ++k) tot += ld_sc1(slot + k * 64 + lane);
          v = tot;
          if (lane == 0) __hip_atomic_store(ctl + kFoldSlot + job * f.ncg + cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (fin) {
        const float other = __shfl_xor(v, 32);
        const int c = cg * kFinCh + lane;
        if (lane < 32 && c < f.C) {
          if constexpr (BWD) {
            float* sums = f.ws + (size_t)job * 2 * f.C;
            st_sc1(sums + c, v);
            st_sc1(sums + f.C + c, other);
            if (J.dgamma) J.dgamma[c] += other;
            if (J.dbeta) J.dbeta[c] += v;
          } else {
            bn_finish_channel<true>(v, other, 0.f, f.rows, J.eps, J.momentum, c, J.mean, J.rstd, J.rmean, J.rvar);
            if (c == 0 && J.nbt) J.nbt[0] += 1;
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(ctl + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (threadIdx.x == 0 && !(f.diag & 1)) {
    const int target = f.njobs * f.ncg;
    int n = 0;
    while (__hip_atomic_load(ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++n > (1 << 24)) {  // never expected: flag it (tests read ctl[3]) rather than hang the queue
        __hip_atomic_store(ctl + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    // past the poll: the last workgroup here re-arms the launch's counters (every ticket is taken by then)
    if (__hip_atomic_fetch_add(ctl + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
      __hip_atomic_store(ctl, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctl + 2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
}

// 8 per-channel values handed off by the fold (sc1 loads)
__device__ __forceinline__ void ldp_sc1(const float* p, int c, float (&o)[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = ld_sc1(p + c + k);
}

// act_kernel with the forward fold (mean / rstd of a.y, and with RBN of the projection shortcut, from their GEMM
// epilogue partials).  Each thread's 8 channels are the same every grid-stride step (host: grid * 8192 % C == 0),
// so the statistics are read once.
template <bool RES, bool RBN>
__global__ void __launch_bounds__(kFoldThreads) act_fold_kernel(const ActArgs a, const FoldCtl f) {
  fold_phase<false>(f);
  const int64_t nv = a.rows * a.C / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nv) return;
  const int c = chan_of((size_t)i * 8, a.C, a.rows * a.C);
  float mu[8], rs[8], g[8], b[8], rm[8], rr[8], rg[8], rb[8];
  ldp_sc1(a.mean, c, mu);
  ldp_sc1(a.rstd, c, rs);
  ldp<8>(a.gamma, c, g);
  ldp<8>(a.beta, c, b);
  if constexpr (RBN) {
    ldp_sc1(a.rmean, c, rm);
    ldp_sc1(a.rrstd, c, rr);
    ldp<8>(a.rgamma, c, rg);
    ldp<8>(a.rbeta, c, rb);
  }
  for (; i < nv; i += stride) {
    const size_t e = (size_t)i * 8;
    float v[8], o[8];
    ldv<8>(a.y, a.ydt, e, v);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = bn_pre(g[q], rs[q], v[q], mu[q], b[q]);
    if constexpr (RES) {
      float r[8];
      ldv<8>(a.res, a.rdt, e, r);
      if constexpr (RBN) {
#pragma unroll
        for (int q = 0; q < 8; ++q) r[q] = bn_pre(rg[q], rr[q], r[q], rm[q], rb[q]);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] += r[q];
    }
    if (a.relu) {
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = fmaxf(o[q], 0.f);
    }
    stv<8>(a.out, a.odt, e, o);
  }
}

// bwd_apply_kernel with the backward fold (the correction sums from bwd_stats' or the dgrad epilogue's partials)
template <bool RELU_Y, bool POOL>
__global__ void __launch_bounds__(kFoldThreads) bwd_apply_fold_kernel(const BwdArgs a, const FoldCtl f) {
  fold_phase<true>(f);
  const int64_t nv = a.rows * a.C / 8;
  const float inv_n = 1.0f / (float)a.rows;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nv) return;
  const int c = chan_of((size_t)i * 8, a.C, a.rows * a.C);
  float mu[8], rs[8], ga[8], sg[8], sgx[8];
  ldp<8>(a.mean, c, mu);
  ldp<8>(a.rstd, c, rs);
  ldp<8>(a.gamma, c, ga);
  if (f.stats) {
    ldp_sc1(f.ws, c, sg);
    ldp_sc1(f.ws + a.C, c, sgx);
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) sg[q] = sgx[q] = 0.f;
  }
  for (; i < nv; i += stride) {
    const size_t e = (size_t)i * 8;
    float v[8], g[8], o[8];
    ldv<8>(a.y, a.ydt, e, v);
    grad_masked<8, RELU_Y, POOL>(a.dout, a.ddt, a.act, a.adt, e, v, mu, rs, a.gamma, a.beta, c, g, &a.pool, a.C);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = bn_dx(ga[q], rs[q], g[q], sg[q], v[q], mu[q], sgx[q], inv_n);
    stv<8>(a.dx, a.xdt, e, o);
  }
}

// bwd_apply_dual_kernel with both BatchNorms' folds (jobs 0 and 1)
__global__ void __launch_bounds__(kFoldThreads) bwd_apply_dual_fold_kernel(const BwdDualArgs a, const FoldCtl f) {
  fold_phase<true>(f);
  const int64_t nv = a.rows * a.C / 8;
  const float inv_n = 1.0f / (float)a.rows;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nv) return;
  const int c = chan_of((size_t)i * 8, a.C, a.rows * a.C);
  float mu[8], rs[8], ga[8], sg[8], sgx[8], mu2[8], rs2[8], ga2[8], sg2[8], sgx2[8];
  ldp<8>(a.mean, c, mu);
  ldp<8>(a.rstd, c, rs);
  ldp<8>(a.gamma, c, ga);
  ldp<8>(a.mean2, c, mu2);
  ldp<8>(a.rstd2, c, rs2);
  ldp<8>(a.gamma2, c, ga2);
  if (f.stats) {
    ldp_sc1(f.ws, c, sg);
    ldp_sc1(f.ws + a.C, c, sgx);
    ldp_sc1(f.ws + 2 * a.C, c, sg2);
    ldp_sc1(f.ws + 3 * a.C, c, sgx2);
  } else {
#pragma unroll
    for (int q = 0; q < 8; ++q) sg[q] = sgx[q] = sg2[q] = sgx2[q] = 0.f;
  }
  for (; i < nv; i += stride) {
    const size_t e = (size_t)i * 8;
    float g[8], v[8], w[8], o[8], o2[8];
    ldv<8>(a.g, a.gdt, e, g);
    ldv<8>(a.y, a.ydt, e, v);
    ldv<8>(a.y2, a.y2dt, e, w);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      o[q] = bn_dx(ga[q], rs[q], g[q], sg[q], v[q], mu[q], sgx[q], inv_n);
      o2[q] = bn_dx(ga2[q], rs2[q], g[q], sg2[q], w[q], mu2[q], sgx2[q], inv_n);
    }
    stv<8>(a.dx, a.xdt, e, o);
    stv<8>(a.dx2, a.xdt, e, o2);
  }
}

// launch geometry of the fold kernels: -> grid, 0 when (rows, C, P) is not theirs
// chunk workgroups per channel group of a separate fold launch: one per kFoldQ partials given a workspace (ctl, ws
// of SV_BN_FOLD_*), else 1 (the workgroup folds the chunks in turn: same bits)
static int fin_split(int P, int C, const int* ctl, const float* ws) {
  static const bool on = !getenv("SV_FIN_SPLIT") || atoi(getenv("SV_FIN_SPLIT")) != 0;
  const int S = fold_chunks(P);
  return (on && ctl && ws && S > 1 && S <= kFoldMaxS && C <= kFoldMaxC) ? S : 1;
}
static int fold_diag() {
  static const int d = getenv("SV_FOLD_DIAG") ? atoi(getenv("SV_FOLD_DIAG")) : 0;
  return d;
}
static int fold_grid(int64_t rows, int C, int P) {
  static const int cap = getenv("SV_FOLD_MAX_GRID") ? atoi(getenv("SV_FOLD_MAX_GRID")) : kFoldMaxGrid;
  if (C < 32 || C > kFoldMaxC || (C & (C - 1)) || rows <= 0 || P <= 0 || fold_chunks(P) > kFoldMaxS) return 0;
  const int64_t nv = rows * C / 8;
  int64_t g = (nv + kFoldThreads - 1) / kFoldThreads;
  if (g > cap) g = cap;
  const int64_t units = 2 * (C / kFinCh) * fold_chunks(P);
  if (g < units) g = units;
  return (g * kFoldThreads * 8) % C == 0 ? (int)g : 0;
}

// the hoisted-parameter kernels' condition: a thread's channel is the same at every grid-stride step (SV_BN_FIXC=0: off)
static bool fixc_ok(int grid, int V, int C) {
  static const bool on = !getenv("SV_BN_FIXC") || atoi(getenv("SV_BN_FIXC")) != 0;
  return on && ((int64_t)grid * kThreads * V) % C == 0;
}
static int grid_for(int64_t n4) {
  int64_t b = (n4 + kThreads - 1) / kThreads;
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}
static bool dt_ok(int dt) { return dt == SV_F32 || dt == SV_BF16; }

}  // namespace bn
}  // namespace sv

using namespace sv;
using namespace sv::bn;

#define BN_REQUIRE_C(C, who) SV_REQUIRE((C) >= 4 && (C) % 4 == 0 && (((C) / 4) <= kThreads || ((C) / 4) % kThreads == 0), \
                                         "%s: C=%d must be a multiple of 4 (and of 1024 above 1024)", who, (int)(C))

extern "C" int sv_bn_nparts(int64_t rows, int32_t C) {
  if (rows <= 0 || C < 4 || C % 4) return 1;
  return nparts_for(rows, C);
}

extern "C" int sv_bn_stats(const void* y, int32_t y_dtype, int64_t rows, int32_t C, float* part, sv_stream_t stream) {
  BN_REQUIRE_C(C, "sv_bn_stats");
  SV_REQUIRE(y && part && rows > 0 && dt_ok(y_dtype), "sv_bn_stats: bad arguments");
  const RedGeo g = red_geo(C);
  const int P = nparts_for(rows, C);
  const int64_t rpp = (rows + P - 1) / P;
  if (g.vec == 8)
    stats_kernel<8><<<dim3(g.cslices, P), kThreads, 0, (hipStream_t)stream>>>(y, y_dtype, rows, C, g.tpr, g.rp, rpp, part);
  else
    stats_kernel<4><<<dim3(g.cslices, P), kThreads, 0, (hipStream_t)stream>>>(y, y_dtype, rows, C, g.tpr, g.rp, rpp, part);
  return check_launch("sv_bn_stats");
}

extern "C" int sv_bn_stats_finish(const void* y, int32_t y_dtype, const float* part, int32_t nparts, int64_t rows,
                                  int32_t C, float eps, float momentum, float* mean, float* rstd, float* running_mean,
                                  float* running_var, int64_t* num_batches_tracked, int32_t* ctl, float* ws,
                                  sv_stream_t stream) {
  SV_REQUIRE(part && mean && rstd && nparts > 0 && rows > 0 && C > 0 && C % 4 == 0 && dt_ok(y_dtype),
             "sv_bn_stats_finish: bad arguments");
  const int S = fin_split(nparts, C, ctl, ws);
  stats_finish_kernel<<<dim3((C + kFinCh - 1) / kFinCh, S), 64 * kFinWaves, 0, (hipStream_t)stream>>>(
      y, y_dtype, part, nparts, rows, C, eps, momentum, mean, rstd, running_mean, running_var, num_batches_tracked,
      ctl ? ctl + kFoldSlot : nullptr, ws);
  return check_launch("sv_bn_stats_finish");
}

extern "C" int sv_bn_eval_params(const float* running_mean, const float* running_var, float eps, float* mean,
                                 float* rstd, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(running_mean && running_var && mean && rstd && C > 0, "sv_bn_eval_params: bad arguments");
  eval_params_kernel<<<(C + 255) / 256, 256, 0, (hipStream_t)stream>>>(running_mean, running_var, eps, mean, rstd, C);
  return check_launch("sv_bn_eval_params");
}

extern "C" int sv_bn_act_fwd(const void* y, int32_t y_dtype, const float* mean, const float* rstd, const float* gamma,
                             const float* beta, const void* res, int32_t res_dtype, const float* res_mean,
                             const float* res_rstd, const float* res_gamma, const float* res_beta, int32_t relu,
                             void* out, int32_t out_dtype, int64_t rows, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(C % 4 == 0 && C > 0 && rows > 0, "sv_bn_act_fwd: C must be a multiple of 4");
  SV_REQUIRE(y && mean && rstd && gamma && beta && out && dt_ok(y_dtype) && dt_ok(out_dtype),
             "sv_bn_act_fwd: bad arguments");
  SV_REQUIRE(!res || dt_ok(res_dtype), "sv_bn_act_fwd: bad residual dtype");
  SV_REQUIRE(!res_mean || (res && res_rstd && res_gamma && res_beta), "sv_bn_act_fwd: incomplete residual BN");
  ActArgs a{y, y_dtype, mean, rstd, gamma, beta, res, res_dtype, res_mean, res_rstd, res_gamma, res_beta,
            relu, out, out_dtype, rows, C};
  hipStream_t st = (hipStream_t)stream;
  const int V = vec_for(C), grid = grid_for(rows * C / V);
  const bool fixc = fixc_ok(grid, V, C);
  if (V == 8) {
    if (fixc) act_kernel<8, true><<<grid, kThreads, 0, st>>>(a);
    else act_kernel<8><<<grid, kThreads, 0, st>>>(a);
  } else {
    if (fixc) act_kernel<4, true><<<grid, kThreads, 0, st>>>(a);
    else act_kernel<4><<<grid, kThreads, 0, st>>>(a);
  }
  return check_launch("sv_bn_act_fwd");
}

static int bwd_stats_launch(const void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype, const void* y,
                            int32_t y_dtype, const float* mean, const float* rstd, const float* gamma,
                            const float* beta, int64_t rows, int32_t C, float* part, sv_stream_t stream,
                            void* gout = nullptr, const PoolSrc* pool = nullptr) {
  const RedGeo g = red_geo(C);
  const int P = nparts_for(rows, C);
  const int64_t rpp = (rows + P - 1) / P;
  const dim3 grid(g.cslices, P);
  hipStream_t st = (hipStream_t)stream;
  const PoolSrc ps = pool ? *pool : PoolSrc{nullptr, nullptr, 0, 0, SV_F32};
#define BWDS(VV, RY)                                                                                              \
  bwd_stats_kernel<VV, RY><<<grid, kThreads, 0, st>>>(dout, dout_dtype, act, act_dtype, y, y_dtype, mean, rstd, gamma, \
                                                      beta, rows, C, g.tpr, g.rp, rpp, part, gout, ps)
  if (pool) {  // the stem's BatchNorm (its own ReLU) reading the max-pool backward
    if (g.vec == 8)
      bwd_stats_kernel<8, true, true><<<grid, kThreads, 0, st>>>(nullptr, SV_F32, nullptr, SV_F32, y, y_dtype, mean, rstd,
                                                                 gamma, beta, rows, C, g.tpr, g.rp, rpp, part, nullptr, ps);
    else
      bwd_stats_kernel<4, true, true><<<grid, kThreads, 0, st>>>(nullptr, SV_F32, nullptr, SV_F32, y, y_dtype, mean, rstd,
                                                                 gamma, beta, rows, C, g.tpr, g.rp, rpp, part, nullptr, ps);
  } else if (beta) {
    if (g.vec == 8) BWDS(8, true); else BWDS(4, true);
  } else {
    if (g.vec == 8) BWDS(8, false); else BWDS(4, false);
  }
#undef BWDS
  return check_launch("sv_bn_bwd_stats");
}

extern "C" int sv_bn_bwd_stats(const void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype, const void* y,
                               int32_t y_dtype, const float* mean, const float* rstd, int64_t rows, int32_t C,
                               float* part, sv_stream_t stream) {
  BN_REQUIRE_C(C, "sv_bn_bwd_stats");
  SV_REQUIRE(dout && y && mean && rstd && part && rows > 0 && dt_ok(dout_dtype) && dt_ok(y_dtype) &&
                 (!act || dt_ok(act_dtype)),
             "sv_bn_bwd_stats: bad arguments");
  return bwd_stats_launch(dout, dout_dtype, act, act_dtype, y, y_dtype, mean, rstd, nullptr, nullptr, rows, C, part,
                          stream);
}

extern "C" int sv_bn_bwd_stats_mask(void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype, const void* y,
                                    int32_t y_dtype, const float* mean, const float* rstd, int64_t rows, int32_t C,
                                    float* part, sv_stream_t stream) {
  BN_REQUIRE_C(C, "sv_bn_bwd_stats_mask");
  SV_REQUIRE(dout && act && y && mean && rstd && part && rows > 0 && dt_ok(dout_dtype) && dt_ok(act_dtype) &&
                 dt_ok(y_dtype),
             "sv_bn_bwd_stats_mask: bad arguments");
  return bwd_stats_launch(dout, dout_dtype, act, act_dtype, y, y_dtype, mean, rstd, nullptr, nullptr, rows, C, part,
                          stream, dout);
}

extern "C" int sv_bn_relu_bwd_stats(const void* dout, int32_t dout_dtype, const void* y, int32_t y_dtype,
                                    const float* mean, const float* rstd, const float* gamma, const float* beta,
                                    int64_t rows, int32_t C, float* part, sv_stream_t stream) {
  BN_REQUIRE_C(C, "sv_bn_relu_bwd_stats");
  SV_REQUIRE(dout && y && mean && rstd && gamma && beta && part && rows > 0 && dt_ok(dout_dtype) && dt_ok(y_dtype),
             "sv_bn_relu_bwd_stats: bad arguments");
  return bwd_stats_launch(dout, dout_dtype, nullptr, SV_F32, y, y_dtype, mean, rstd, gamma, beta, rows, C, part,
                          stream);
}

extern "C" int sv_bn_bwd_finish(const float* part, int32_t nparts, int32_t C, float* sums, float* dgamma, float* dbeta,
                                int32_t* ctl, float* ws, sv_stream_t stream) {
  SV_REQUIRE(part && sums && nparts > 0 && C > 0 && C % 4 == 0, "sv_bn_bwd_finish: bad arguments");
  const int S = fin_split(nparts, C, ctl, ws);
  bwd_finish_kernel<<<dim3((C + kFinCh - 1) / kFinCh, S), 64 * kFinWaves, 0, (hipStream_t)stream>>>(
      part, nparts, C, sums, dgamma, dbeta, ctl ? ctl + kFoldSlot : nullptr, ws);
  return check_launch("sv_bn_bwd_finish");
}

static int bwd_apply_launch(const BwdArgs& a, sv_stream_t stream) {
  hipStream_t st = (hipStream_t)stream;
  const bool v8 = vec_for(a.C) == 8;
  const int grid = grid_for(a.rows * a.C / (v8 ? 8 : 4));
  const bool fixc = fixc_ok(grid, v8 ? 8 : 4, a.C);
#define BWDA(VV, RY, PL)                                                                              \
  (fixc ? (bwd_apply_kernel<VV, RY, PL, true><<<grid, kThreads, 0, st>>>(a), 0)                    \
        : (bwd_apply_kernel<VV, RY, PL><<<grid, kThreads, 0, st>>>(a), 0))
  if (a.pool.d) {
    if (v8) BWDA(8, true, true);
    else BWDA(4, true, true);
  } else if (a.beta) {
    if (v8) BWDA(8, true, false);
    else BWDA(4, true, false);
  } else {
    if (v8) BWDA(8, false, false);
    else BWDA(4, false, false);
  }
#undef BWDA
  return check_launch("sv_bn_bwd_apply");
}

extern "C" int sv_bn_bwd_apply(const void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype, const void* y,
                               int32_t y_dtype, const float* mean, const float* rstd, const float* gamma,
                               const float* sums, void* dx, int32_t dx_dtype, float* gmask, int64_t rows, int32_t C,
                               sv_stream_t stream) {
  SV_REQUIRE(C % 4 == 0 && C > 0 && rows > 0, "sv_bn_bwd_apply: C must be a multiple of 4");
  SV_REQUIRE(dout && y && mean && rstd && gamma && sums && dx && dt_ok(dout_dtype) && dt_ok(y_dtype) &&
                 dt_ok(dx_dtype) && (!act || dt_ok(act_dtype)),
             "sv_bn_bwd_apply: bad arguments");
  BwdArgs a{dout, dout_dtype, act, act_dtype, y, y_dtype, mean, rstd, gamma, nullptr, sums, dx, dx_dtype, gmask,
            rows, C};
  return bwd_apply_launch(a, stream);
}

extern "C" int sv_bn_relu_bwd_apply(const void* dout, int32_t dout_dtype, const void* y, int32_t y_dtype,
                                    const float* mean, const float* rstd, const float* gamma, const float* beta,
                                    const float* sums, void* dx, int32_t dx_dtype, int64_t rows, int32_t C,
                                    sv_stream_t stream) {
  SV_REQUIRE(C % 4 == 0 && C > 0 && rows > 0, "sv_bn_relu_bwd_apply: C must be a multiple of 4");
  SV_REQUIRE(dout && y && mean && rstd && gamma && beta && sums && dx && dt_ok(dout_dtype) && dt_ok(y_dtype) &&
                 dt_ok(dx_dtype),
             "sv_bn_relu_bwd_apply: bad arguments");
  BwdArgs a{dout, dout_dtype, nullptr, SV_F32, y, y_dtype, mean, rstd, gamma, beta, sums, dx, dx_dtype, nullptr,
            rows, C};
  return bwd_apply_launch(a, stream);
}

// The stem: BatchNorm (+ its own ReLU) backward whose incoming gradient is the max-pool 3x3/2 backward of
// dpool [B][OH][OW][C] (f32 or bf16: the gradient stream's dtype) through idx, gathered inside both passes instead of
// materialised
static bool pool_args_ok(const void* dpool, int dpool_dtype, const uint8_t* idx, int B, int H, int W, int C) {
  return dpool && dt_ok(dpool_dtype) && idx && B > 0 && H > 0 && W > 0 && C % 4 == 0 && C > 0 && ((uintptr_t)dpool & 15) == 0 &&
         ((uintptr_t)idx & 3) == 0 && (int64_t)B * H * W * C < (1ll << 31);  // pool_grad's 32-bit indexing
}

extern "C" int sv_bn_relu_bwd_stats_pool(const void* dpool, int32_t dpool_dtype, const uint8_t* idx, int32_t B,
                                         int32_t H, int32_t W, const void* y, int32_t y_dtype, const float* mean,
                                         const float* rstd, const float* gamma, const float* beta, int32_t C,
                                         float* part, sv_stream_t stream) {
  BN_REQUIRE_C(C, "sv_bn_relu_bwd_stats_pool");
  SV_REQUIRE(pool_args_ok(dpool, dpool_dtype, idx, B, H, W, C) && y && mean && rstd && gamma && beta && part &&
                 dt_ok(y_dtype),
             "sv_bn_relu_bwd_stats_pool: bad arguments");
  const PoolSrc ps{dpool, idx, H, W, dpool_dtype};
  return bwd_stats_launch(nullptr, SV_F32, nullptr, SV_F32, y, y_dtype, mean, rstd, gamma, beta, (int64_t)B * H * W, C,
                          part, stream, nullptr, &ps);
}

extern "C" int sv_bn_relu_bwd_apply_pool(const void* dpool, int32_t dpool_dtype, const uint8_t* idx, int32_t B,
                                         int32_t H, int32_t W, const void* y, int32_t y_dtype, const float* mean,
                                         const float* rstd, const float* gamma, const float* beta, const float* sums,
                                         void* dx, int32_t dx_dtype, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(pool_args_ok(dpool, dpool_dtype, idx, B, H, W, C) && y && mean && rstd && gamma && beta && sums && dx &&
                 dt_ok(y_dtype) && dt_ok(dx_dtype),
             "sv_bn_relu_bwd_apply_pool: bad arguments");
  BwdArgs a{nullptr, SV_F32, nullptr, SV_F32, y, y_dtype, mean, rstd, gamma, beta, sums, dx, dx_dtype, nullptr,
            (int64_t)B * H * W, C, PoolSrc{dpool, idx, H, W, dpool_dtype}};
  return bwd_apply_launch(a, stream);
}

extern "C" int sv_relu_mask(const void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype, float* g,
                            int64_t n, sv_stream_t stream) {
  SV_REQUIRE(dout && act && g && n >= 0 && n % 4 == 0 && dt_ok(dout_dtype) && dt_ok(act_dtype),
             "sv_relu_mask: bad arguments");
  if (n == 0) return SV_OK;
  relu_mask_kernel<<<grid_for(n / 4), kThreads, 0, (hipStream_t)stream>>>(dout, dout_dtype, act, act_dtype, g, n / 4);
  return check_launch("sv_relu_mask");
}

extern "C" int sv_maxpool3s2_fwd(const void* x, int32_t x_dtype, void* y, uint8_t* idx, int32_t B, int32_t H, int32_t W,
                                 int32_t C, sv_stream_t stream) {
  SV_REQUIRE(x && y && idx && B > 0 && H > 0 && W > 0 && C % 4 == 0 && C > 0 && dt_ok(x_dtype),
             "sv_maxpool3s2_fwd: bad arguments");
  const int64_t n4 = (int64_t)B * pool_out(H) * pool_out(W) * C / 4;
  maxpool_fwd_kernel<<<grid_for(n4), kThreads, 0, (hipStream_t)stream>>>(x, x_dtype, y, idx, B, H, W, C);
  return check_launch("sv_maxpool3s2_fwd");
}

extern "C" int sv_maxpool3s2_bwd(const void* dout, int32_t dout_dtype, const uint8_t* idx, void* dx, int32_t dx_dtype,
                                 int32_t B, int32_t H, int32_t W, int32_t C, sv_stream_t stream) {
  SV_REQUIRE(dout && idx && dx && B > 0 && H > 0 && W > 0 && C % 4 == 0 && C > 0 && dt_ok(dout_dtype) &&
                 dt_ok(dx_dtype),
             "sv_maxpool3s2_bwd: bad arguments");
  maxpool_bwd_kernel<<<grid_for((int64_t)B * H * W * C / 4), kThreads, 0, (hipStream_t)stream>>>(
      dout, dout_dtype, idx, dx, dx_dtype, B, H, W, C);
  return check_launch("sv_maxpool3s2_bwd");
}

extern "C" int sv_avgpool_fwd(const void* x, int32_t x_dtype, float* feat, int32_t B, int32_t HW, int32_t C,
                              sv_stream_t stream) {
  SV_REQUIRE(x && feat && B > 0 && HW > 0 && C % 4 == 0 && C > 0 && dt_ok(x_dtype), "sv_avgpool_fwd: bad arguments");
  const int64_t n = (int64_t)B * C / 4;
  avgpool_fwd_kernel<<<(int)((n + kThreads - 1) / kThreads), kThreads, 0, (hipStream_t)stream>>>(x, x_dtype, feat, B,
                                                                                                 HW, C);
  return check_launch("sv_avgpool_fwd");
}

extern "C" int sv_avgpool_bwd(const float* dfeat, void* dx, int32_t dx_dtype, int32_t B, int32_t HW, int32_t C,
                              sv_stream_t stream) {
  SV_REQUIRE(dfeat && dx && B > 0 && HW > 0 && C % 4 == 0 && C > 0 && dt_ok(dx_dtype), "sv_avgpool_bwd: bad arguments");
  avgpool_bwd_kernel<<<grid_for((int64_t)B * HW * C / 4), kThreads, 0, (hipStream_t)stream>>>(dfeat, dx, dx_dtype, B, HW,
                                                                                             C);
  return check_launch("sv_avgpool_bwd");
}

extern "C" int sv_bn_bwd_stats_mask_dual(void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype,
                                         const void* y, int32_t y_dtype, const float* mean, const float* rstd,
                                         const void* y2, int32_t y2_dtype, const float* mean2, const float* rstd2,
                                         int64_t rows, int32_t C, float* part, float* part2, sv_stream_t stream) {
  BN_REQUIRE_C(C, "sv_bn_bwd_stats_mask_dual");
  SV_REQUIRE(dout && act && y && mean && rstd && y2 && mean2 && rstd2 && part && part2 && rows > 0 && dt_ok(dout_dtype) &&
                 dt_ok(act_dtype) && dt_ok(y_dtype) && dt_ok(y2_dtype),
             "sv_bn_bwd_stats_mask_dual: bad arguments");
  const RedGeo g = red_geo(C);
  const int P = nparts_for(rows, C);
  const int64_t rpp = (rows + P - 1) / P;
  const dim3 grid(g.cslices, P);
  hipStream_t st = (hipStream_t)stream;
  if (g.vec == 8)
    bwd_stats_dual_kernel<8><<<grid, kThreads, 0, st>>>(dout, dout_dtype, act, act_dtype, y, y_dtype, mean, rstd, y2, y2_dtype, mean2,
                                                        rstd2, rows, C, g.tpr, g.rp, rpp, part, part2);
  else
    bwd_stats_dual_kernel<4><<<grid, kThreads, 0, st>>>(dout, dout_dtype, act, act_dtype, y, y_dtype, mean, rstd, y2, y2_dtype, mean2,
                                                        rstd2, rows, C, g.tpr, g.rp, rpp, part, part2);
  return check_launch("sv_bn_bwd_stats_mask_dual");
}

extern "C" int sv_bn_bwd_apply_dual(const void* g, int32_t g_dtype, const void* y, int32_t y_dtype, const float* mean,
                                    const float* rstd, const float* gamma, const float* sums, const void* y2,
                                    int32_t y2_dtype, const float* mean2, const float* rstd2, const float* gamma2,
                                    const float* sums2, void* dx, void* dx2, int32_t dx_dtype, int64_t rows, int32_t C,
                                    sv_stream_t stream) {
  SV_REQUIRE(C % 4 == 0 && C > 0 && rows > 0, "sv_bn_bwd_apply_dual: C must be a multiple of 4");
  SV_REQUIRE(g && y && mean && rstd && gamma && sums && y2 && mean2 && rstd2 && gamma2 && sums2 && dx && dx2 &&
                 dt_ok(g_dtype) && dt_ok(y_dtype) && dt_ok(y2_dtype) && dt_ok(dx_dtype),
             "sv_bn_bwd_apply_dual: bad arguments");
  BwdDualArgs a{g, g_dtype, y, y_dtype, mean, rstd, gamma, sums, y2, y2_dtype, mean2, rstd2, gamma2, sums2, dx, dx2, dx_dtype,
                rows, C};
  hipStream_t st = (hipStream_t)stream;
  if (vec_for(C) == 8)
    bwd_apply_dual_kernel<8><<<grid_for(rows * C / 8), kThreads, 0, st>>>(a);
  else
    bwd_apply_dual_kernel<4><<<grid_for(rows * C / 4), kThreads, 0, st>>>(a);
  return check_launch("sv_bn_bwd_apply_dual");
}

// ---- one-launch small-row BatchNorm (see bwd_small_kernel) --------------------------------------------------
static bool small_geo(int64_t rows, int32_t C, RedGeo& g, int& P, int& rpp) {
  if (rows <= 0 || rows > SV_BN_SMALL_MAX_ROWS || C < 8 || C % 8) return false;
  g = red_geo(C);
  if (g.vec != 8) return false;
  P = nparts_for(rows, C);
  rpp = (int)((rows + P - 1) / P);
  return (int64_t)P * g.rp <= kSmallThreads;
}
static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

extern "C" int sv_bn_small_ok(int64_t rows, int32_t C) {
  RedGeo g;
  int P, rpp;
  return small_geo(rows, C, g, P, rpp) ? 1 : 0;
}

extern "C" int sv_bn_bwd_small(int32_t mode, void* dout, int32_t dout_dtype, const void* act, int32_t act_dtype,
                               const void* y, int32_t y_dtype, const float* mean, const float* rstd, const float* gamma,
                               const float* beta, const void* y2, int32_t y2_dtype, const float* mean2,
                               const float* rstd2, const float* gamma2, const float* part, int32_t nparts, void* dx,
                               void* dx2, int32_t dx_dtype, float* dgamma, float* dbeta, float* dgamma2, float* dbeta2,
                               int32_t batch_stats, int64_t rows, int32_t C, sv_stream_t stream) {
  RedGeo g;
  int P, rpp;
  SV_REQUIRE(small_geo(rows, C, g, P, rpp), "sv_bn_bwd_small: rows=%lld C=%d outside the one-launch geometry",
             (long long)rows, (int)C);
  SV_REQUIRE(mode >= SV_BN_SMALL_MASK && mode <= SV_BN_SMALL_DUAL, "sv_bn_bwd_small: bad mode %d", (int)mode);
  SV_REQUIRE(dout && y && mean && rstd && gamma && dx && dt_ok(dout_dtype) && dt_ok(y_dtype) && dt_ok(dx_dtype) &&
                 al16(dout) && al16(y) && al16(dx) && al16(mean) && al16(rstd) && al16(gamma),
             "sv_bn_bwd_small: bad arguments");
  SV_REQUIRE(mode == SV_BN_SMALL_RELU || (act && dt_ok(act_dtype) && al16(act) && !part),
             "sv_bn_bwd_small: the mask modes need act and no given partials");
  SV_REQUIRE(mode != SV_BN_SMALL_RELU || (beta && al16(beta)), "sv_bn_bwd_small: the ReLU mode needs beta");
  SV_REQUIRE(mode != SV_BN_SMALL_DUAL || (y2 && mean2 && rstd2 && gamma2 && dx2 && dt_ok(y2_dtype) && al16(y2) &&
                                          al16(dx2) && al16(mean2) && al16(rstd2) && al16(gamma2)),
             "sv_bn_bwd_small: the dual mode needs y2, mean2, rstd2, gamma2 and dx2");
  SV_REQUIRE(!part || (nparts > 0 && al16(part)), "sv_bn_bwd_small: bad partials");
  SmallBwdArgs a{dout, dout_dtype, act, act_dtype, y, y_dtype, mean, rstd, gamma, beta, y2, y2_dtype, mean2, rstd2,
                 gamma2, part, nparts, dx, dx2, dx_dtype, dgamma, dbeta, dgamma2, dbeta2, batch_stats ? 1 : 0,
                 (int)rows, C, P, g.rp, rpp};
  hipStream_t st = (hipStream_t)stream;
  const int grid = C / 8;
  if (mode == SV_BN_SMALL_MASK) bwd_small_kernel<0, false><<<grid, kSmallThreads, 0, st>>>(a);
  else if (mode == SV_BN_SMALL_DUAL) bwd_small_kernel<2, false><<<grid, kSmallThreads, 0, st>>>(a);
  else if (part) bwd_small_kernel<1, true><<<grid, kSmallThreads, 0, st>>>(a);
  else bwd_small_kernel<1, false><<<grid, kSmallThreads, 0, st>>>(a);
  return check_launch("sv_bn_bwd_small");
}

extern "C" int sv_bn_act_small(const void* y, int32_t y_dtype, const float* part, int32_t nparts, float eps,
                               float momentum, const float* gamma, const float* beta, float* mean, float* rstd,
                               float* running_mean, float* running_var, int64_t* num_batches_tracked, const void* res,
                               int32_t res_dtype, const float* res_part, int32_t res_nparts, float res_eps,
                               float res_momentum, const float* res_gamma, const float* res_beta, float* res_mean,
                               float* res_rstd, float* res_running_mean, float* res_running_var,
                               int64_t* res_num_batches_tracked, int32_t relu, void* out, int32_t out_dtype,
                               int64_t rows, int32_t C, sv_stream_t stream) {
  RedGeo g;
  int P, rpp;
  SV_REQUIRE(small_geo(rows, C, g, P, rpp), "sv_bn_act_small: rows=%lld C=%d outside the one-launch geometry",
             (long long)rows, (int)C);
  SV_REQUIRE(y && part && nparts > 0 && gamma && beta && mean && rstd && out && dt_ok(y_dtype) && dt_ok(out_dtype) &&
                 al16(y) && al16(part) && al16(gamma) && al16(beta) && al16(out),
             "sv_bn_act_small: bad arguments");
  SV_REQUIRE(!res || (dt_ok(res_dtype) && al16(res)), "sv_bn_act_small: bad residual");
  SV_REQUIRE(!res_part || (res && res_nparts > 0 && al16(res_part) && res_gamma && res_beta && res_mean && res_rstd &&
                           al16(res_gamma) && al16(res_beta)),
             "sv_bn_act_small: incomplete residual BatchNorm");
  SmallActArgs a{y, y_dtype, part, nparts, eps, momentum, gamma, beta, mean, rstd, running_mean, running_var,
                 num_batches_tracked, res, res_dtype, res_part, res_nparts, res_eps, res_momentum, res_gamma, res_beta,
                 res_mean, res_rstd, res_running_mean, res_running_var, res_num_batches_tracked, relu ? 1 : 0, out,
                 out_dtype, (int)rows, C};
  hipStream_t st = (hipStream_t)stream;
  const int grid = C / 8;
  if (res_part) act_small_kernel<true, true><<<grid, kSmallThreads, 0, st>>>(a);
  else if (res) act_small_kernel<true, false><<<grid, kSmallThreads, 0, st>>>(a);
  else act_small_kernel<false, false><<<grid, kSmallThreads, 0, st>>>(a);
  return check_launch("sv_bn_act_small");
}

// ---- fold kernels (the statistics fold inside the consuming pass) -------------------------------------------
extern "C" int sv_bn_fold_ok(int64_t rows, int32_t C, int32_t nparts) { return fold_grid(rows, C, nparts) > 0 ? 1 : 0; }

extern "C" int sv_bn_act_fold(const void* y, int32_t y_dtype, const float* part, int32_t nparts, float eps,
                              float momentum, const float* gamma, const float* beta, float* mean, float* rstd,
                              float* running_mean, float* running_var, int64_t* num_batches_tracked, const void* res,
                              int32_t res_dtype, const float* res_part, int32_t res_nparts, float res_eps,
                              float res_momentum, const float* res_gamma, const float* res_beta, float* res_mean,
                              float* res_rstd, float* res_running_mean, float* res_running_var,
                              int64_t* res_num_batches_tracked, int32_t relu, void* out, int32_t out_dtype,
                              int64_t rows, int32_t C, int32_t* ctl, float* ws, sv_stream_t stream) {
  const int grid = fold_grid(rows, C, nparts);
  SV_REQUIRE(grid > 0, "sv_bn_act_fold: rows=%lld C=%d nparts=%d outside the fold kernels' geometry (sv_bn_fold_ok)",
             (long long)rows, (int)C, (int)nparts);
  SV_REQUIRE(y && part && gamma && beta && mean && rstd && out && ctl && ws && dt_ok(y_dtype) && dt_ok(out_dtype) &&
                 al16(y) && al16(part) && al16(gamma) && al16(beta) && al16(out),
             "sv_bn_act_fold: bad arguments");
  SV_REQUIRE(nparts == (rows + 63) / 64, "sv_bn_act_fold: nparts=%d is not the conv epilogue's ceil(rows / 64)",
             (int)nparts);
  SV_REQUIRE(!res || (dt_ok(res_dtype) && al16(res)), "sv_bn_act_fold: bad residual");
  SV_REQUIRE(!res_part || (res && res_nparts == nparts && al16(res_part) && res_gamma && res_beta && res_mean &&
                           res_rstd && al16(res_gamma) && al16(res_beta)),
             "sv_bn_act_fold: incomplete residual BatchNorm (its partials must match the main ones)");
  ActArgs a{y, y_dtype, mean, rstd, gamma, beta, res, res_dtype, res_mean, res_rstd, res_gamma, res_beta,
            relu ? 1 : 0, out, out_dtype, rows, C};
  FoldCtl f{};
  f.ctl = ctl;
  f.ws = ws;
  f.job[0] = FoldJob{part, mean, rstd, running_mean, running_var, num_batches_tracked, eps, momentum, nullptr, nullptr};
  f.job[1] = FoldJob{res_part, res_mean, res_rstd, res_running_mean, res_running_var, res_num_batches_tracked, res_eps,
                     res_momentum, nullptr, nullptr};
  f.njobs = res_part ? 2 : 1;
  f.P = nparts;
  f.S = fold_chunks(nparts);
  f.ncg = C / kFinCh;
  f.C = C;
  f.stats = 1;
  f.rows = rows;
  f.diag = fold_diag();
  hipStream_t st = (hipStream_t)stream;
  if (res_part) act_fold_kernel<true, true><<<grid, kFoldThreads, 0, st>>>(a, f);
  else if (res) act_fold_kernel<true, false><<<grid, kFoldThreads, 0, st>>>(a, f);
  else act_fold_kernel<false, false><<<grid, kFoldThreads, 0, st>>>(a, f);
  return check_launch("sv_bn_act_fold");
}

extern "C" int sv_bn_bwd_apply_fold(int32_t mode, const void* dout, int32_t dout_dtype, const uint8_t* pool_idx,
                                    int32_t pool_H, int32_t pool_W, const void* y, int32_t y_dtype, const float* mean,
                                    const float* rstd, const float* gamma, const float* beta, const void* y2,
                                    int32_t y2_dtype, const float* mean2, const float* rstd2, const float* gamma2,
                                    const float* part, const float* part2, int32_t nparts, void* dx, void* dx2,
                                    int32_t dx_dtype, float* dgamma, float* dbeta, float* dgamma2, float* dbeta2,
                                    int32_t batch_stats, int64_t rows, int32_t C, int32_t* ctl, float* ws,
                                    sv_stream_t stream) {
  const int grid = fold_grid(rows, C, nparts);
  SV_REQUIRE(grid > 0, "sv_bn_bwd_apply_fold: rows=%lld C=%d nparts=%d outside the fold kernels' geometry",
             (long long)rows, (int)C, (int)nparts);
  SV_REQUIRE(mode >= SV_BN_SMALL_MASK && mode <= SV_BN_SMALL_DUAL, "sv_bn_bwd_apply_fold: bad mode %d", (int)mode);
  SV_REQUIRE(dout && y && mean && rstd && gamma && part && dx && ctl && ws && dt_ok(dout_dtype) && dt_ok(y_dtype) &&
                 dt_ok(dx_dtype) && al16(dout) && al16(y) && al16(mean) && al16(rstd) && al16(gamma) && al16(part) &&
                 al16(dx),
             "sv_bn_bwd_apply_fold: bad arguments");
  SV_REQUIRE(mode != SV_BN_SMALL_RELU || (beta && al16(beta)), "sv_bn_bwd_apply_fold: the ReLU mode needs beta");
  SV_REQUIRE(!pool_idx || (mode == SV_BN_SMALL_RELU && pool_H > 0 && pool_W > 0 && rows % ((int64_t)pool_H * pool_W) == 0 &&
                           rows * C < (1ll << 31)),
             "sv_bn_bwd_apply_fold: the pooled form is the ReLU mode over rows = B * H * W (< 2^31 elements)");
  SV_REQUIRE(mode != SV_BN_SMALL_DUAL || (y2 && dt_ok(y2_dtype) && al16(y2) && mean2 && rstd2 && gamma2 && part2 &&
                                          dx2 && al16(mean2) && al16(rstd2) && al16(gamma2) && al16(part2) && al16(dx2)),
             "sv_bn_bwd_apply_fold: the dual mode needs y2, mean2, rstd2, gamma2, part2 and dx2");
  FoldCtl f{};
  f.ctl = ctl;
  f.ws = ws;
  f.job[0] = FoldJob{part, nullptr, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, dgamma, dbeta};
  f.job[1] = FoldJob{part2, nullptr, nullptr, nullptr, nullptr, nullptr, 0.f, 0.f, dgamma2, dbeta2};
  f.njobs = mode == SV_BN_SMALL_DUAL ? 2 : 1;
  f.P = nparts;
  f.S = fold_chunks(nparts);
  f.ncg = C / kFinCh;
  f.C = C;
  f.stats = batch_stats ? 1 : 0;
  f.rows = rows;
  f.diag = fold_diag();
  hipStream_t st = (hipStream_t)stream;
  if (mode == SV_BN_SMALL_DUAL) {
    BwdDualArgs a{dout, dout_dtype, y, y_dtype, mean, rstd, gamma, nullptr, y2, y2_dtype, mean2, rstd2, gamma2,
                  nullptr, dx, dx2, dx_dtype, rows, C};
    bwd_apply_dual_fold_kernel<<<grid, kFoldThreads, 0, st>>>(a, f);
    return check_launch("sv_bn_bwd_apply_fold");
  }
  const PoolSrc ps = pool_idx ? PoolSrc{dout, pool_idx, pool_H, pool_W, dout_dtype} : PoolSrc{nullptr, nullptr, 0, 0, SV_F32};
  BwdArgs a{dout, dout_dtype, nullptr, SV_F32, y, y_dtype, mean, rstd, gamma, beta, nullptr, dx, dx_dtype, nullptr,
            rows, C, ps};
  if (mode == SV_BN_SMALL_MASK) bwd_apply_fold_kernel<false, false><<<grid, kFoldThreads, 0, st>>>(a, f);
  else if (pool_idx) bwd_apply_fold_kernel<true, true><<<grid, kFoldThreads, 0, st>>>(a, f);
  else bwd_apply_fold_kernel<true, false><<<grid, kFoldThreads, 0, st>>>(a, f);
  return check_launch("sv_bn_bwd_apply_fold");
}
