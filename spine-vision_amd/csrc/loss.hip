// The classification trainer's multi-task loss in one launch (gfx950).
//
// Replaces Classifier.get_loss over the fused head's logits (spine_vision/training/models/generic.py: the
// per-task loss_fn(pred, format_target(target)) weighted sum; core/tasks.py create_loss_functions:
// nn.CrossEntropyLoss(label_smoothing) for multiclass / ordinal tasks, nn.BCEWithLogitsLoss for binary /
// multilabel ones, mean reduction) and its autograd backward.  At bs32 the torch form is ~60 launches of a few
// microseconds each for a [32 x 10] logits tensor; here ONE workgroup computes every task's loss and d(loss)/d(logits)
// in the same pass (the backward then only scales dlogits by the incoming gradient).
//   CE (label smoothing e, C classes, targets int64, ignore_index -100): per row with a valid target
//       loss_i = -sum_c q_c log p_c,  q = (1 - e) onehot(y) + e / C,  dl_c = (p_c - q_c) / N_valid
//   BCE (targets f32, ncls columns): per element  max(x, 0) - x t + log1p(exp(-|x|)),  dl = (sigmoid(x) - t) / (B ncls)
// A CE target outside [0, C) that is not -100 makes the loss and that row's d(loss)/d(logits) NaN (torch stops with a
// device-side assert; a silently dropped one-hot term would train on a wrong loss).
// Sums run in a fixed order (each thread its rows in ascending order, a butterfly per wave, the 4 waves in order):
// deterministic.
#include <math.h>

#include "common.h"

namespace sv {
namespace loss {

constexpr int kThreads = 256, kMaxTasks = 8;

struct Task {
  int kind;       // SV_HEAD_CE / SV_HEAD_BCE
  int offset;     // first logits column of the task
  int ncls;
  float weight;
  float smoothing;
  const void* target;
  int tdt;        // BCE target dtype (SV_F32 / SV_BF16); CE targets are int64
};
struct Tasks {
  Task t[kMaxTasks];
  int n;
};

// sum over the workgroup of one value per thread: a butterfly within each wave, then the 4 wave sums in order (fixed
// order: deterministic); every thread gets the total
__device__ __forceinline__ float block_sum(float v, float* __restrict__ wsum) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();  // wsum may still be read from the previous call
  if ((threadIdx.x & 63) == 0) wsum[w] = v;
  __syncthreads();
  return (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
}

__global__ void __launch_bounds__(kThreads) head_loss_kernel(const float* __restrict__ logits, int B, int K, const Tasks ts,
                                                             float* __restrict__ loss, float* __restrict__ dlogits) {
  static_assert(kThreads == 256, "block_sum: 4 waves");
  __shared__ float wsum[4];
  __shared__ float scale[kMaxTasks];
  const int tid = threadIdx.x;
  // pass 1: the number of rows each task averages over (CE: valid targets; BCE: every element)
  for (int k = 0; k < ts.n; ++k) {
    const Task& t = ts.t[k];
    float c;
    if (t.kind == SV_HEAD_CE) {
      float cnt = 0.f;
      for (int i = tid; i < B; i += kThreads) cnt += reinterpret_cast<const int64_t*>(t.target)[i] != -100 ? 1.f : 0.f;
      c = block_sum(cnt, wsum);
    } else {
      c = (float)B * (float)t.ncls;
    }
    if (tid == 0) scale[k] = c > 0.f ? 1.0f / c : 0.f;  // torch: a mean over no elements is NaN; here 0
  }
  __syncthreads();
  // pass 2: per-row losses and the gradient, the latter already divided by the count and weighted
  float part[kMaxTasks];
  float nbad = 0.f;  // CE targets outside [0, ncls) that are not ignore_index
#pragma unroll
  for (int k = 0; k < kMaxTasks; ++k) part[k] = 0.f;
  for (int i = tid; i < B; i += kThreads) {
    const float* x = logits + (size_t)i * K;
    float* dx = dlogits + (size_t)i * K;
#pragma unroll
    for (int k = 0; k < kMaxTasks; ++k) {
      if (k >= ts.n) break;
      const Task& t = ts.t[k];
      const float ws = t.weight * scale[k];
      if (t.kind == SV_HEAD_CE) {
        const int64_t y = reinterpret_cast<const int64_t*>(t.target)[i];
        if (y == -100) {
          for (int c = 0; c < t.ncls; ++c) dx[t.offset + c] = 0.f;
          continue;
        }
        if (y < 0 || y >= t.ncls) {  // torch raises a device-side assert here: poison the row and the loss instead
          for (int c = 0; c < t.ncls; ++c) dx[t.offset + c] = NAN;
          nbad += 1.f;
          continue;
        }
        float mx = -INFINITY;
        for (int c = 0; c < t.ncls; ++c) mx = fmaxf(mx, x[t.offset + c]);
        float se = 0.f;
        for (int c = 0; c < t.ncls; ++c) se += expf(x[t.offset + c] - mx);
        const float lse = mx + logf(se);
        const float e = t.smoothing, off = e / (float)t.ncls;
        float nll = 0.f, smooth = 0.f;
        for (int c = 0; c < t.ncls; ++c) {
          const float lp = x[t.offset + c] - lse;
          smooth -= lp;
          const float q = (c == (int)y ? 1.f - e : 0.f) + off;
          if (c == (int)y) nll = -lp;
          dx[t.offset + c] = (expf(lp) - q) * ws;
        }
        part[k] += (1.f - e) * nll + e * (smooth / (float)t.ncls);
      } else {
        for (int c = 0; c < t.ncls; ++c) {
          const float v = x[t.offset + c];
          const size_t ti = (size_t)i * t.ncls + c;
          const float tg = t.tdt == SV_F32 ? reinterpret_cast<const float*>(t.target)[ti]
                                           : __uint_as_float((uint32_t)reinterpret_cast<const uint16_t*>(t.target)[ti] << 16);
          part[k] += fmaxf(v, 0.f) - v * tg + log1pf(expf(-fabsf(v)));
          dx[t.offset + c] = (1.f / (1.f + expf(-v)) - tg) * ws;
        }
      }
    }
  }
  float total = 0.f;
  for (int k = 0; k < ts.n; ++k) {
    float pk = 0.f;
#pragma unroll
    for (int q = 0; q < kMaxTasks; ++q) pk = q == k ? part[q] : pk;  // constant-indexed: part stays in registers
    total += ts.t[k].weight * (block_sum(pk, wsum) * scale[k]);
  }
  nbad = block_sum(nbad, wsum);
  if (tid == 0) loss[0] = nbad > 0.f ? NAN : total;
}

}  // namespace loss
}  // namespace sv

using namespace sv;

extern "C" int sv_head_loss(const float* logits, int32_t B, int32_t K, const sv_head_task* tasks, int32_t ntasks,
                            float* loss, float* dlogits, sv_stream_t stream) {
  SV_REQUIRE(logits && tasks && loss && dlogits && B > 0 && K > 0 && ntasks >= 1 && ntasks <= loss::kMaxTasks,
             "sv_head_loss: bad arguments (1..%d tasks)", loss::kMaxTasks);
  loss::Tasks ts{};
  ts.n = ntasks;
  for (int k = 0; k < ntasks; ++k) {
    const sv_head_task& h = tasks[k];
    SV_REQUIRE(h.kind == SV_HEAD_CE || h.kind == SV_HEAD_BCE, "sv_head_loss: task %d: bad kind %d", k, (int)h.kind);
    SV_REQUIRE(h.target && h.ncls >= 1 && h.offset >= 0 && h.offset + h.ncls <= K,
               "sv_head_loss: task %d: columns [%d, %d) outside the %d logits", k, (int)h.offset,
               (int)(h.offset + h.ncls), (int)K);
    SV_REQUIRE(h.kind != SV_HEAD_BCE || h.target_dtype == SV_F32 || h.target_dtype == SV_BF16,
               "sv_head_loss: task %d: BCE targets f32 or bf16", k);
    ts.t[k] = loss::Task{h.kind, h.offset, h.ncls, h.weight, h.label_smoothing, h.target, h.target_dtype};
  }
  loss::head_loss_kernel<<<1, loss::kThreads, 0, (hipStream_t)stream>>>(logits, B, K, ts, loss, dlogits);
  return check_launch("sv_head_loss");
}
