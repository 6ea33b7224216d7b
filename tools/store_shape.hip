// Store / load access-shape microbenchmark for the v9 GEMM epilogue (diagnostic, not on the product path).
//
// A persistent grid of 256 workgroups x 512 threads walks the 256x256 tiles of a [32768 x 2048] bf16
// matrix (128 MiB, fc1's output at S3) the way gemm9 does (8 waves, 128 x 64 per wave) and moves each
// wave's 16 KiB with one of two shapes per 16-B-per-lane buffer instruction:
//   shape 0 (v9 today): 16 rows x 64 B   (row = 16 i + (l & 15), columns 32 c + 8 (l >> 4))
//   shape 1:             8 rows x 128 B  (row = 16 i + 8 h + (l >> 3), columns 8 (l & 7))
// Modes: 0/1 store one output, 2/3 store two outputs (the GELU dual epilogue), 4/5 load (bf16 operand).
//
// Then the per-CU store rate: the same bytes stored by 256 / 128 / 64 / 32 workgroups.
//
//   hipcc --offload-arch=gfx950 -O3 -o store_shape tools/store_shape.hip && ./store_shape
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int M = 32768, N = 2048, BM = 256, BN = 256;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int MODE>
__global__ void __launch_bounds__(512) shape_kernel(uint16_t* out, uint16_t* out2, const uint16_t* in, float* sink) {
  const int l = threadIdx.x & 63, wid = threadIdx.x >> 6, wm = wid >> 2, wn = wid & 3;
  const int tilesN = N / BN, total = (M / BM) * tilesN;
  const auto r0 = rsrc(out, (uint32_t)M * N * 2), r1 = rsrc(out2, (uint32_t)M * N * 2), ri = rsrc(in, (uint32_t)M * N * 2);
  constexpr int SHAPE = MODE & 1;
  u32x4 v = {(uint32_t)l, (uint32_t)wid, (uint32_t)blockIdx.x, 7u};
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (int t = blockIdx.x; t < total; t += gridDim.x) {
    const int m_w = (t / tilesN) * BM + wm * 128, n_w = (t % tilesN) * BN + wn * 64;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        int row, col;
        if (SHAPE == 0) row = m_w + 16 * i + (l & 15), col = n_w + 32 * c + 8 * (l >> 4);
        else row = m_w + 16 * i + 8 * c + (l >> 3), col = n_w + 8 * (l & 7);
        const uint32_t off = (uint32_t)(row * N + col) * 2;
        if (MODE < 4) {
          __builtin_amdgcn_raw_buffer_store_b128(v, r0, off, 0, 0);
          if (MODE >= 2) __builtin_amdgcn_raw_buffer_store_b128(v, r1, off, 0, 0);
        } else {
          acc += __builtin_amdgcn_raw_buffer_load_b128(ri, off, 0, 0);
        }
      }
    v.w += 1u;
  }
  if (MODE >= 4 && acc.x == 0x12345678u) sink[threadIdx.x] = (float)acc.y;
}

static int g_grid = 256;
template <int MODE>
static float run(uint16_t* a, uint16_t* b, uint16_t* c, float* s, int iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) shape_kernel<MODE><<<g_grid, 512>>>(a, b, c, s);
  hipEventRecord(e0);
  for (int i = 0; i < iters; ++i) shape_kernel<MODE><<<g_grid, 512>>>(a, b, c, s);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / iters;
}

int main() {
  uint16_t *a, *b, *c;
  float* s;
  const size_t bytes = (size_t)M * N * 2;
  if (hipMalloc(&a, bytes) || hipMalloc(&b, bytes) || hipMalloc(&c, bytes) || hipMalloc(&s, 4096)) return 1;
  hipMemset(c, 1, bytes);
  const char* names[6] = {"store 1 out, 16 rows x 64 B", "store 1 out,  8 rows x 128 B", "store 2 out, 16 rows x 64 B",
                          "store 2 out,  8 rows x 128 B", "load,        16 rows x 64 B", "load,         8 rows x 128 B"};
  for (int rep = 0; rep < 2; ++rep) {
    g_grid = 256;
    float us[6] = {run<0>(a, b, c, s, 20), run<1>(a, b, c, s, 20), run<2>(a, b, c, s, 20),
                   run<3>(a, b, c, s, 20), run<4>(a, b, c, s, 20), run<5>(a, b, c, s, 20)};
    for (int m = 0; m < 6; ++m) {
      const double mb = (double)bytes * (m == 2 || m == 3 ? 2 : 1) / 1e6;
      printf("%-30s %8.1f us  %7.1f GB/s\n", names[m], us[m], mb / us[m] * 1e3);
    }
  }
  // per-CU store rate: the same bytes from fewer workgroups (one per CU)
  for (int gsz : {256, 128, 64, 32}) {
    g_grid = gsz;
    const float us = run<1>(a, b, c, s, 10);
    printf("store 1 out, 8 x 128 B, %3d workgroups %8.1f us  %7.1f GB/s  %6.1f GB/s per workgroup\n", gsz, us,
           (double)bytes / us / 1e3, (double)bytes / us / 1e3 / gsz);
  }
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
