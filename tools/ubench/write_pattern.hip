// Write-pattern microbenchmark for the Winograd U preparation: the same
// 268 MB (64 planes x 1024 rows x 1024 items x 4 B) written (a) item-major
// (one thread per item writes its 64 planes, 4 MB apart: prep_weights_kernel's
// pattern), (b) plane-major (consecutive threads, consecutive addresses),
// (c) item-major with a plane-row group of 8 per block pass.
// hipcc --offload-arch=gfx950 -O3 write_pattern.hip -o write_pattern
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NP = 64, ROWS = 1024, COLS = 1024;

__global__ void __launch_bounds__(256) item_major(float* __restrict__ U, float v) {
  const long long item = (long long)blockIdx.x * 256 + threadIdx.x;  // n * COLS + k
  const size_t plane = (size_t)ROWS * COLS;
#pragma unroll
  for (int p = 0; p < NP; ++p) U[p * plane + item] = v + p;
}

__global__ void __launch_bounds__(256) plane_major(float* __restrict__ U, float v) {
  const size_t i = (size_t)blockIdx.x * 256 * 4 + threadIdx.x * 4;
  *(float4*)&U[i] = make_float4(v, v, v, v);
}

// one block: 8 planes of a 2048-item run (8 items per thread, 4 B each, as
// 2 x 16 B), i.e. 8 KB contiguous per plane per block
__global__ void __launch_bounds__(256) item_run8(float* __restrict__ U, float v) {
  const size_t plane = (size_t)ROWS * COLS;
  const int runs = ROWS * COLS / 2048;
  const int run = blockIdx.x % runs, pg = blockIdx.x / runs;
  const size_t base = (size_t)run * 2048 + threadIdx.x * 8;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    float* o = U + (size_t)(pg * 8 + q) * plane + base;
    *(float4*)o = make_float4(v, v, v, v);
    *(float4*)(o + 4) = make_float4(v, v, v, v);
  }
}

// item-major, 8 items per thread (16-B x 2 per plane): a thread's 64 planes
__global__ void __launch_bounds__(256) item_major8(float* __restrict__ U, float v) {
  const size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  const size_t plane = (size_t)ROWS * COLS;
#pragma unroll 8
  for (int p = 0; p < NP; ++p) {
    float* o = U + p * plane + base;
    *(float4*)o = make_float4(v + p, v, v, v);
    *(float4*)(o + 4) = make_float4(v, v, v, v);
  }
}

int main() {
  const size_t n = (size_t)NP * ROWS * COLS;
  float* U;
  if (hipMalloc(&U, n * 4) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < 20; ++i) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double us = ms * 1e3 / 20;
    printf("%-12s %8.1f us  %6.2f TB/s\n", name, us, n * 4 / us / 1e6);
  };
  run("item_major", [&] { hipLaunchKernelGGL(item_major, dim3(ROWS * COLS / 256), dim3(256), 0, 0, U, 1.f); });
  run("plane_major", [&] { hipLaunchKernelGGL(plane_major, dim3(n / 1024), dim3(256), 0, 0, U, 1.f); });
  run("item_run8", [&] { hipLaunchKernelGGL(item_run8, dim3(ROWS * COLS / 2048 * 8), dim3(256), 0, 0, U, 1.f); });
  run("item_major8", [&] { hipLaunchKernelGGL(item_major8, dim3(ROWS * COLS / 2048), dim3(256), 0, 0, U, 1.f); });
  hipFree(U);
  return 0;
}
