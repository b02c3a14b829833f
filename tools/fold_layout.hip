// Access-layout experiment for the config-2 local fold (8 x 256 MiB f32 SUM
// -> 1, the product's pairwise tree) on MI355X: which assignment of vectors
// to lanes / waves / blocks, which load/store cache policy and which load
// order get closest to the read-only stream.  Tooling only (not linked into
// libmpigx); build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off.
//
//   LAYOUT 0  block-interleaved: vector (b*U + u)*256 + t   (the product)
//   LAYOUT 1  wave-contiguous:   vector b*U*256 + w*U*64 + u*64 + lane
//             (each wave streams U KiB contiguous of every input and output)
//   ORDER  0  loads u-major (all inputs of vector u, then u+1)
//          1  loads input-major (U consecutive KiB of input k, then k+1)
//   LAUX / SAUX  buffer-instruction cache bits (gfx950: 1 sc0, 2 nt, 16 sc1)
//   PERSIST  0 one pass over the grid; G > 0: G blocks loop over the chunks
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct P8 {
  const void* in[8];
  void* out;
  long long nv;  // 16-B vectors per buffer
  unsigned bytes;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}

template <int LAYOUT, int U, int ORDER, int LAUX, int SAUX>
__device__ __forceinline__ void chunk(const P8& a, long long c) {
  const int t = threadIdx.x, w = t >> 6, lane = t & 63;
  unsigned idx[U];
#pragma unroll
  for (int u = 0; u < U; ++u)
    idx[u] = (unsigned)(LAYOUT == 0 ? (c * U + u) * 256 + t : c * U * 256 + w * U * 64 + u * 64 + lane);
  f32x4 v[U][8];
  if constexpr (ORDER == 0) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k)
        v[u][k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc(a.in[k], a.bytes), idx[u] * 16, 0, LAUX));
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int u = 0; u < U; ++u)
        v[u][k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc(a.in[k], a.bytes), idx[u] * 16, 0, LAUX));
  }
  const __amdgpu_buffer_rsrc_t o = rsrc(a.out, a.bytes);
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const f32x4 r = ((v[u][0] + v[u][1]) + (v[u][2] + v[u][3])) + ((v[u][4] + v[u][5]) + (v[u][6] + v[u][7]));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, r), o, idx[u] * 16, 0, SAUX);
  }
}

template <int LAYOUT, int U, int ORDER, int LAUX, int SAUX, int PERSIST>
__global__ __launch_bounds__(256) void fold8(P8 a) {
  const long long nc = a.nv / (U * 256);
  if constexpr (PERSIST == 0) {
    chunk<LAYOUT, U, ORDER, LAUX, SAUX>(a, blockIdx.x);
  } else {
    // XCD-aware: block b runs on XCD b % 8; give each XCD a contiguous range
    const unsigned b = blockIdx.x, per = gridDim.x / 8;
    const unsigned lb = (b % 8) * per + b / 8;
    const long long cper = (nc + gridDim.x - 1) / gridDim.x;
    const long long c0 = (long long)lb * cper, c1 = c0 + cper < nc ? c0 + cper : nc;
    for (long long c = c0; c < c1; ++c) chunk<LAYOUT, U, ORDER, LAUX, SAUX>(a, c);
  }
}

__global__ __launch_bounds__(256) void read8(P8 a) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 8; ++k) acc += __builtin_nontemporal_load((const f32x4*)a.in[k] + i);
  if (acc[0] == 123.456f) ((f32x4*)a.out)[i] = acc;
}

template <int LAYOUT, int U, int ORDER, int LAUX, int SAUX, int PERSIST = 0>
hipError_t go(const P8& p) {
  const unsigned g = PERSIST ? PERSIST : (unsigned)(p.nv / (U * 256));
  hipLaunchKernelGGL((fold8<LAYOUT, U, ORDER, LAUX, SAUX, PERSIST>), dim3(g), dim3(256), 0, 0, p);
  return hipGetLastError();
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 7;
  const long long S = 256ll << 20;
  void* in[8];
  for (int k = 0; k < 8; ++k) {
    CK(hipMalloc(&in[k], S));
    std::vector<float> h(S / 4);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u + k * 40503u) % 1000003) * 1e-3f - 500.f;
    CK(hipMemcpy(in[k], h.data(), S, hipMemcpyHostToDevice));
  }
  void *out, *ref;
  CK(hipMalloc(&out, S));
  CK(hipMalloc(&ref, S));
  P8 p;
  for (int k = 0; k < 8; ++k) p.in[k] = in[k];
  p.out = out;
  p.nv = S / 16;
  p.bytes = (unsigned)S;
  P8 pr = p;
  pr.out = ref;

  struct V {
    std::string name;
    double bytes;
    std::function<hipError_t()> f;
  };
  const double B9 = 9.0 * S;
  std::vector<V> vs = {
      {"L0 U4 o0 nt sc1 (product)", B9, [&] { return go<0, 4, 0, 2, 16>(p); }},
      {"L1 U4 o0 nt sc1", B9, [&] { return go<1, 4, 0, 2, 16>(p); }},
      {"L1 U4 o1 nt sc1", B9, [&] { return go<1, 4, 1, 2, 16>(p); }},
      {"L1 U2 o1 nt sc1", B9, [&] { return go<1, 2, 1, 2, 16>(p); }},
      {"L1 U4 o1 plain sc1", B9, [&] { return go<1, 4, 1, 0, 16>(p); }},
      {"L1 U4 o1 nt plain", B9, [&] { return go<1, 4, 1, 2, 0>(p); }},
      {"L1 U4 o1 nt nt", B9, [&] { return go<1, 4, 1, 2, 2>(p); }},
      {"L1 U4 o1 sc1 sc1", B9, [&] { return go<1, 4, 1, 16, 16>(p); }},
      {"L0 U4 o1 nt sc1", B9, [&] { return go<0, 4, 1, 2, 16>(p); }},
      {"L0 U4 o0 plain sc1", B9, [&] { return go<0, 4, 0, 0, 16>(p); }},
      {"L1 U4 o1 nt sc1 P2048", B9, [&] { return go<1, 4, 1, 2, 16, 2048>(p); }},
      {"L1 U4 o1 nt sc1 P4096", B9, [&] { return go<1, 4, 1, 2, 16, 4096>(p); }},
      {"L1 U2 o1 nt sc1 P4096", B9, [&] { return go<1, 2, 1, 2, 16, 4096>(p); }},
      {"read 8 streams", 8.0 * S, [&] {
         hipLaunchKernelGGL(read8, dim3((unsigned)(p.nv / 256)), dim3(256), 0, 0, p);
         return hipGetLastError();
       }},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int IT = 10;
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < R; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      CK(vs[v].f());
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < IT; ++i) CK(vs[v].f());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / IT);
    }
  printf("{\"what\": \"tools/fold_layout.hip, 8 x 256 MiB f32 SUM, median of %d rounds x %d launches\", \"variants\": {", R, IT);
  for (size_t v = 0; v < vs.size(); ++v) {
    auto m = ms[v];
    std::sort(m.begin(), m.end());
    printf("%s\"%s\": {\"us\": %.1f, \"GBps\": %.1f, \"min_us\": %.1f}", v ? ", " : "", vs[v].name.c_str(), m[R / 2] * 1e3,
           vs[v].bytes / (m[R / 2] * 1e-3) / 1e9, m[0] * 1e3);
  }
  printf("}");
  // every fold variant writes the same bits as the product layout
  CK((go<0, 4, 0, 2, 16>(pr)));
  std::vector<unsigned> h1(S / 4), h2(S / 4);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(h1.data(), ref, S, hipMemcpyDeviceToHost));
  bool ok = true;
  for (size_t v = 0; v + 1 < vs.size(); ++v) {
    CK(hipMemset(out, 0, S));
    CK(vs[v].f());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h2.data(), out, S, hipMemcpyDeviceToHost));
    if (memcmp(h1.data(), h2.data(), S)) {
      ok = false;
      printf(", \"mismatch\": \"%s\"", vs[v].name.c_str());
    }
  }
  printf(", \"bit_identical\": %s}\n", ok ? "true" : "false");
  return 0;
}
