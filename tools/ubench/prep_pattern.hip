// The U preparation's load + store pattern (conv6: cin = cout = 1024, F(6x6),
// 64 planes of 4-B words), with a trivial transform: (a) unflipped reads
// w[(n*cin + k)*9 + t], (b) flipped reads w[(k*cin + n)*9 + 8 - t] (item
// (n, k) = thread, k fastest), (c) flipped through an LDS transpose of a
// 32 x 32 (n, k) tile's filters, read coalesced along n.
// hipcc --offload-arch=gfx950 -O3 prep_pattern.hip -o prep_pattern
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int C = 1024, NP = 64;

__device__ __forceinline__ void emit(float (&g)[9], float* __restrict__ U, size_t item) {
  const size_t plane = (size_t)C * C;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const float v = g[p % 9] * (1.f + p) + g[(p + 3) % 9];
    U[p * plane + item] = v;
  }
}

template <bool FLIP>
__global__ void __launch_bounds__(256) direct(const float* __restrict__ w, float* __restrict__ U) {
  const size_t item = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int k = item % C, n = item / C;
  float g[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
    g[t] = FLIP ? w[((size_t)k * C + n) * 9 + 8 - t] : w[((size_t)n * C + k) * 9 + t];
  emit(g, U, item);
}

// R items per thread (item = block * 256 R + r * 256 + lane): SEQ loads each
// item's filter after the previous item's stores (the stores share vmcnt with
// the loads on CDNA, so that wait also drains them); otherwise all R filters
// are loaded first
template <int R, bool SEQ>
__global__ void __launch_bounds__(256) multi(const float* __restrict__ w, float* __restrict__ U) {
  const size_t base = (size_t)blockIdx.x * 256 * R + threadIdx.x;
  if constexpr (SEQ) {
    for (int r = 0; r < R; ++r) {
      const size_t item = base + r * 256;
      const int k = item % C, n = item / C;
      float g[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) g[t] = w[((size_t)n * C + k) * 9 + t];
      emit(g, U, item);
    }
  } else {
    float g[R][9];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const size_t item = base + r * 256;
      const int k = item % C, n = item / C;
#pragma unroll
      for (int t = 0; t < 9; ++t) g[r][t] = w[((size_t)n * C + k) * 9 + t];
    }
#pragma unroll
    for (int r = 0; r < R; ++r) emit(g[r], U, base + r * 256);
  }
}

// block: 32 n x 32 k = 1024 items, 4 per thread; the tile's filters
// (32 k rows x 32 n x 9 floats, contiguous 1152 B per k row) staged in LDS
__global__ void __launch_bounds__(256) flip_lds(const float* __restrict__ w, float* __restrict__ U) {
  __shared__ float s[32][32 * 9 + 1];
  const int tn = blockIdx.x % (C / 32), tk = blockIdx.x / (C / 32);
  const int n0 = tn * 32, k0 = tk * 32;
  for (int i = threadIdx.x; i < 32 * 32 * 9; i += 256) {
    const int kr = i / (32 * 9), o = i % (32 * 9);
    s[kr][o] = w[((size_t)(k0 + kr) * C + n0) * 9 + o];
  }
  __syncthreads();
  for (int r = 0; r < 4; ++r) {
    const int li = r * 256 + threadIdx.x, kk = li & 31, nn = li >> 5;
    float g[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t] = s[kk][nn * 9 + 8 - t];
    emit(g, U, (size_t)(n0 + nn) * C + k0 + kk);
  }
}

int main() {
  float *w, *U;
  if (hipMalloc(&w, (size_t)C * C * 9 * 4) != hipSuccess) return 1;
  if (hipMalloc(&U, (size_t)NP * C * C * 4) != hipSuccess) return 1;
  hipMemset(w, 0, (size_t)C * C * 9 * 4);
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
    printf("%-10s %8.1f us  %6.2f TB/s of U\n", name, us, (double)NP * C * C * 4 / us / 1e6);
  };
  run("unflipped", [&] { hipLaunchKernelGGL(direct<false>, dim3(C * C / 256), dim3(256), 0, 0, w, U); });
  run("flipped", [&] { hipLaunchKernelGGL(direct<true>, dim3(C * C / 256), dim3(256), 0, 0, w, U); });
  run("seq2", [&] { hipLaunchKernelGGL((multi<2, true>), dim3(C * C / 512), dim3(256), 0, 0, w, U); });
  run("pre2", [&] { hipLaunchKernelGGL((multi<2, false>), dim3(C * C / 512), dim3(256), 0, 0, w, U); });
  run("pre4", [&] { hipLaunchKernelGGL((multi<4, false>), dim3(C * C / 1024), dim3(256), 0, 0, w, U); });
  run("flip_lds", [&] { hipLaunchKernelGGL(flip_lds, dim3(C * C / 1024), dim3(256), 0, 0, w, U); });
  return 0;
}
