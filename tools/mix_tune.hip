// Where config 2's read/write mix loses time (tools, not shipped): the
// 8-read : 1-write stream runs at ~6.35 TB/s on MI355X while reading the
// same 8 inputs alone reaches ~7.1 TB/s and a 1:1 copy ~7.0 TB/s
// (profiles/r06k_kernel_stats.csv, r05zd).  This times, interleaved in one
// process (median of rounds), the mix-probe access pattern (copy.hip
// mix_probe_kernel: U = 4 vectors per thread of every input, XOR, the fold's
// write-through store) for:
//   * k-read : 1-write streams, k = 1, 2, 4, 8 (how the rate falls with the
//     share of writes);
//   * the 8:1 stream written in place of input 0 / input 7 (the store hits a
//     row the same thread just read) instead of a separate output;
//   * read-only streams of 1 and 8 inputs.
//   hipcc --offload-arch=gfx950 -O3 tools/mix_tune.hip -o tools/mix_tune
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct P {
  const u32x4* in[8];
  u32x4* out;  // null: read only
  long long nv;
  u32x4* sink;
};

template <int K, bool STORE>
__global__ __launch_bounds__(256) void mix(P a) {
  constexpr int U = 4;
  const long long base = (long long)blockIdx.x * (U * 256) + threadIdx.x;
  u32x4 x[U][K];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int k = 0; k < K; ++k) x[u][k] = __builtin_nontemporal_load(a.in[k] + base + u * 256);
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    u32x4 r = x[u][0];
#pragma unroll
    for (int k = 1; k < K; ++k) r ^= x[u][k];
    if constexpr (STORE) {
      __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.out + (base - threadIdx.x), 0, U * 256 * 16,
                                                                    0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(r, rs, (int)(threadIdx.x + u * 256) * 16, 0, 16);
    } else {
      acc ^= r;
    }
  }
  if (!STORE && acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) a.sink[threadIdx.x] = acc;
}

// the same 8 : 1 stream with the inputs read one after another inside each
// thread (G inputs at a time, a vmcnt(0) wait between groups): the blocks of
// one dispatch wave start together, so across the GPU only G input streams
// (+ the output) are active at once instead of 8
template <int G>
__global__ __launch_bounds__(256) void mix_seq(P a) {
  constexpr int U = 4;
  const long long base = (long long)blockIdx.x * (U * 256) + threadIdx.x;
  u32x4 acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = u32x4{0, 0, 0, 0};
#pragma unroll
  for (int k0 = 0; k0 < 8; k0 += G) {
    u32x4 x[U][G];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < G; ++k) x[u][k] = __builtin_nontemporal_load(a.in[k0 + k] + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < G; ++k) acc[u] ^= x[u][k];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.out + (base - threadIdx.x), 0, U * 256 * 16,
                                                                  0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(acc[u], rs, (int)(threadIdx.x + u * 256) * 16, 0, 16);
  }
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 7;
  const long long S = 256ll << 20;
  void* in[8];
  for (int k = 0; k < 8; ++k) {
    CK(hipMalloc(&in[k], S));
    CK(hipMemset(in[k], 0x11 * (k + 1), S));
  }
  void *out, *sink;
  CK(hipMalloc(&out, S));
  CK(hipMalloc(&sink, 4096));
  P p;
  for (int k = 0; k < 8; ++k) p.in[k] = (const u32x4*)in[k];
  p.out = (u32x4*)out;
  p.nv = S / 16;
  p.sink = (u32x4*)sink;
  P p0 = p, p7 = p;
  p0.out = (u32x4*)in[0];
  p7.out = (u32x4*)in[7];
  const dim3 G((unsigned)(p.nv / 1024)), B(256);
  struct V {
    std::string name;
    double bytes;
    std::function<void()> go;
  };
  std::vector<V> vs = {
      {"8R:1W separate out", 9.0 * S, [&] { hipLaunchKernelGGL((mix<8, true>), G, B, 0, 0, p); }},
      {"8R:1W in place of input 0", 9.0 * S, [&] { hipLaunchKernelGGL((mix<8, true>), G, B, 0, 0, p0); }},
      {"8R:1W in place of input 7", 9.0 * S, [&] { hipLaunchKernelGGL((mix<8, true>), G, B, 0, 0, p7); }},
      {"4R:1W separate out", 5.0 * S, [&] { hipLaunchKernelGGL((mix<4, true>), G, B, 0, 0, p); }},
      {"2R:1W separate out", 3.0 * S, [&] { hipLaunchKernelGGL((mix<2, true>), G, B, 0, 0, p); }},
      {"1R:1W copy", 2.0 * S, [&] { hipLaunchKernelGGL((mix<1, true>), G, B, 0, 0, p); }},
      {"8R:1W inputs one at a time", 9.0 * S, [&] { hipLaunchKernelGGL((mix_seq<1>), G, B, 0, 0, p); }},
      {"8R:1W inputs two at a time", 9.0 * S, [&] { hipLaunchKernelGGL((mix_seq<2>), G, B, 0, 0, p); }},
      {"8R:1W inputs four at a time", 9.0 * S, [&] { hipLaunchKernelGGL((mix_seq<4>), G, B, 0, 0, p); }},
      {"8R read only", 8.0 * S, [&] { hipLaunchKernelGGL((mix<8, false>), G, B, 0, 0, p); }},
      {"1R read only", 1.0 * S, [&] { hipLaunchKernelGGL((mix<1, false>), G, B, 0, 0, p); }},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int IT = 10;
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < R; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      vs[v].go();
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < IT; ++i) vs[v].go();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / IT);
    }
  CK(hipGetLastError());
  printf("{\"what\": \"tools/mix_tune.hip, 256 MiB streams, median of %d rounds x %d launches\", \"variants\": {", R,
         IT);
  for (size_t v = 0; v < vs.size(); ++v) {
    auto m = ms[v];
    std::sort(m.begin(), m.end());
    printf("%s\"%s\": {\"us\": %.1f, \"GBps\": %.1f}", v ? ", " : "", vs[v].name.c_str(), m[R / 2] * 1e3,
           vs[v].bytes / (m[R / 2] * 1e-3) / 1e9);
  }
  printf("}}\n");
  return 0;
}
