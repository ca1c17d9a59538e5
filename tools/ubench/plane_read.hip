// Read-pattern microbenchmark for the Winograd output transform: each thread
// reads its (tile, 4-channel group) value in 64 planes (16 B each) and writes
// one 16-B sum. (a) planes PLANE bytes apart ([p][t][N] layout, the
// transform's), (b) the same bytes with the 64 values of a (tile, group)
// adjacent ([t][p][N] layout), (c) as (a) with 8 planes per load batch.
// hipcc --offload-arch=gfx950 -O3 plane_read.hip -o plane_read
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int NP = 64, T = 968 * 4, N = 512;  // conv7-like: 3872 tiles x 512 channels
typedef float f4 __attribute__((ext_vector_type(4)));

template <bool TP>
__global__ void __launch_bounds__(256) rd(const float* __restrict__ M, float* __restrict__ out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;  // (t, c4)
  if (i >= (long long)T * (N / 4)) return;
  const int c = (int)(i % (N / 4)) * 4;
  const long long t = i / (N / 4);
  f4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const size_t off = TP ? ((size_t)t * NP + p) * N + c : ((size_t)p * T + t) * N + c;
    s += *(const f4*)(M + off) * (float)(p + 1);
  }
  *(f4*)(out + (size_t)t * N + c) = s;
}

// one channel per thread (the F(6x6) transforms' width), 4-B loads
__global__ void __launch_bounds__(256) rd1(const float* __restrict__ M, float* __restrict__ out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;  // (t, c)
  if (i >= (long long)T * N) return;
  const int c = (int)(i % N);
  const long long t = i / N;
  float s = 0.f;
#pragma unroll
  for (int p = 0; p < NP; ++p) s += M[((size_t)p * T + t) * N + c] * (float)(p + 1);
  out[(size_t)t * N + c] = s;
}
// two channels per thread, 8-B loads
__global__ void __launch_bounds__(256) rd2(const float* __restrict__ M, float* __restrict__ out) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)T * (N / 2)) return;
  const int c = (int)(i % (N / 2)) * 2;
  const long long t = i / (N / 2);
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 s = {0.f, 0.f};
#pragma unroll
  for (int p = 0; p < NP; ++p) s += *(const f2*)(M + ((size_t)p * T + t) * N + c) * (float)(p + 1);
  *(f2*)(out + (size_t)t * N + c) = s;
}

int main() {
  const size_t n = (size_t)NP * T * N;
  float *M, *out;
  if (hipMalloc(&M, n * 4) != hipSuccess || hipMalloc(&out, (size_t)T * N * 4) != hipSuccess) return 1;
  hipMemset(M, 0, n * 4);
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
    printf("%-14s %8.1f us  %6.2f TB/s (read %zu MB)\n", name, us, (n + (size_t)T * N) * 4 / us / 1e6,
           n * 4 >> 20);
  };
  const int g = (int)(((long long)T * (N / 4) + 255) / 256);
  run("planes [p][t]", [&] { hipLaunchKernelGGL(rd<false>, dim3(g), dim3(256), 0, 0, M, out); });
  run("1 ch / thread", [&] { hipLaunchKernelGGL(rd1, dim3((T * N + 255) / 256), dim3(256), 0, 0, M, out); });
  run("2 ch / thread", [&] { hipLaunchKernelGGL(rd2, dim3((T * N / 2 + 255) / 256), dim3(256), 0, 0, M, out); });
  run("planes [t][p]", [&] { hipLaunchKernelGGL(rd<true>, dim3(g), dim3(256), 0, 0, M, out); });
  return 0;
}
