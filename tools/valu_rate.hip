// VALU multiply-add throughput microbenchmark (diagnostic, not on the product path): 1 / 2 / 4 / 8 waves per SIMD,
// 16 independent accumulators per lane, a long unrolled chain of
//   v_fma_f32 (1 MAC / lane), v_pk_fma_f32 (2), v_dot2_f32_bf16 (2, bf16 inputs, f32 accumulate)
// -> MACs per cycle per SIMD from the wall time (hipEvent) and the in-kernel clock (s_memtime / s_memrealtime of
// workgroup 0): the VALU multiply-add rate the depthwise kernels (49 f32 FMA per element) are measured against.
//
//   hipcc --offload-arch=gfx950 -O3 -o valu_rate tools/valu_rate.hip && ./valu_rate
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
constexpr int ITERS = 4096, ACC = 16;

__device__ unsigned long long g_clk[2];  // s_memtime / s_memrealtime deltas of workgroup 0 (the loop's clock)

template <int KIND>
__global__ void __launch_bounds__(256) rate_kernel(float* out, float seed) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const float s = seed + threadIdx.x * 1e-7f;
  float a[ACC];
  f2 p[ACC];
#pragma unroll
  for (int i = 0; i < ACC; ++i) a[i] = s * i, p[i] = f2{s, s * i};
  const f2 x = {s * 0.5f, s * 0.25f};
  const bf2 xb = {(__bf16)(s * 0.5f), (__bf16)(s * 0.25f)}, yb = {(__bf16)0.75f, (__bf16)1.25f};
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) {
      if constexpr (KIND == 0) a[i] = fmaf(a[i], 0.999f, s);
      else if constexpr (KIND == 1) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(p[i]) : "v"(x), "v"(x));
      else a[i] = __builtin_amdgcn_fdot2_f32_bf16(xb, yb, a[i], false);
    }
  }
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < ACC; ++i) r += a[i] + p[i].x + p[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    g_clk[0] = __builtin_amdgcn_s_memtime() - t0;
    g_clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
}

template <int KIND>
static double run(float* out, int wgs_per_cu) {
  const int grid = 256 * wgs_per_cu;  // 256 threads = one wave per SIMD per workgroup
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  rate_kernel<KIND><<<grid, 256>>>(out, 1.0f);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) rate_kernel<KIND><<<grid, 256>>>(out, 1.0f);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double macs_per_lane = (double)ITERS * ACC * (KIND == 0 ? 1 : 2);
  const double waves = (double)grid * 4 * 5;
  const double macs = macs_per_lane * 64 * waves;
  unsigned long long clk[2];
  (void)hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof(clk));
  const double ghz = clk[1] ? (double)clk[0] / (double)clk[1] * 0.1 : 2.4;  // s_memrealtime ticks at 100 MHz
  printf("  [kind %d, %d wave(s)/SIMD: in-kernel clock %.3f GHz] ", KIND, wgs_per_cu, ghz);
  return macs / (ms * 1e-3) / (1024.0 * ghz * 1e9);  // MACs per cycle per SIMD at the measured clock
}

int main() {
  float* out;
  if (hipMalloc(&out, 256 * 8 * 256 * sizeof(float))) return 1;  // the largest grid: 2048 x 256 threads
  const char* names[3] = {"v_fma_f32", "v_pk_fma_f32", "v_dot2_f32_bf16"};
  for (int w = 1; w <= 8; w *= 2) {
    const double r[3] = {run<0>(out, w), run<1>(out, w), run<2>(out, w)};
    for (int k = 0; k < 3; ++k)
      printf("\n%-16s %d wave(s)/SIMD: %6.2f MAC/cycle/SIMD", names[k], w, r[k]);
    printf("\n");
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
