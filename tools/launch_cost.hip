// Host cost of a kernel launch by argument-block size (tools, not shipped):
// back-to-back launches of an empty kernel taking a by-value struct of
// 16 B / 256 B / 1 KiB / 2 KiB, host time per launch over 2000 launches and
// device time per launch (events).  The collective kernels pass ~1 KiB
// argument blocks (FoldArgs / CopyArgs); this says what that costs per call.
//   hipcc --offload-arch=gfx950 -O2 tools/launch_cost.hip -o tools/launch_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

template <int B>
struct Args {
  unsigned w[B / 4];
};

template <int B>
__global__ void k_empty(Args<B> a, unsigned* sink) {
  if (a.w[0] == 0xdeadbeefu && threadIdx.x == 0) sink[0] = a.w[B / 4 - 1];
}

template <int B>
void run(unsigned* sink, hipStream_t s, int grid) {
  Args<B> a{};
  for (int i = 0; i < B / 4; ++i) a.w[i] = i;
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty<B>, dim3(grid), dim3(256), 0, s, a, sink);
  hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int n = 2000;
  auto t0 = std::chrono::steady_clock::now();
  hipEventRecord(e0, s);
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty<B>, dim3(grid), dim3(256), 0, s, a, sink);
  hipEventRecord(e1, s);
  auto t1 = std::chrono::steady_clock::now();
  hipStreamSynchronize(s);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double host_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
  printf("{\"arg_bytes\": %d, \"grid\": %d, \"host_us_per_launch\": %.3f, \"stream_us_per_launch\": %.3f}\n", B, grid,
         host_us, ms * 1e3 / n);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
}

int main() {
  unsigned* sink;
  hipMalloc(&sink, 64);
  hipStream_t s;
  hipStreamCreate(&s);
  for (int grid : {1, 256, 1024}) {
    run<16>(sink, s, grid);
    run<256>(sink, s, grid);
    run<1024>(sink, s, grid);
    run<2048>(sink, s, grid);
  }
  hipFree(sink);
  return 0;
}
