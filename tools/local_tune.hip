// Microbenchmark: variants of the config-2 streaming fold (8 x 256 MiB f32
// SUM -> 1), timed interleaved in one process (cdna_hip_programming.md §5.4
// rule 24).  Tooling only; the product kernel is csrc/kernels.hpp.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

struct P { const f32x4* in[8]; f32x4* out; long long nv; };

template <bool NT> __device__ __forceinline__ f32x4 L(const f32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}
template <bool NT> __device__ __forceinline__ void S(f32x4* p, f32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}
template <int U, bool NTL, bool NTS>
__global__ void fold8(P a) {
  const long long nt = (long long)gridDim.x * blockDim.x;
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * nt < a.nv; i += U * nt) {
    f32x4 v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[u][k] = L<NTL>(a.in[k] + i + u * nt);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      f32x4 r = ((v[u][0] + v[u][1]) + (v[u][2] + v[u][3])) + ((v[u][4] + v[u][5]) + (v[u][6] + v[u][7]));
      S<NTS>(a.out + i + u * nt, r);
    }
  }
  for (; i < a.nv; i += nt) {
    f32x4 r = ((L<NTL>(a.in[0] + i) + L<NTL>(a.in[1] + i)) + (L<NTL>(a.in[2] + i) + L<NTL>(a.in[3] + i))) +
              ((L<NTL>(a.in[4] + i) + L<NTL>(a.in[5] + i)) + (L<NTL>(a.in[6] + i) + L<NTL>(a.in[7] + i)));
    S<NTS>(a.out + i, r);
  }
}
// block-contiguous variant: block b owns a contiguous span; threads stride inside
template <int U>
__global__ void fold8_span(P a, long long span) {
  long long lo = (long long)blockIdx.x * span, hi = lo + span < a.nv ? lo + span : a.nv;
  for (long long i = lo + threadIdx.x; i < hi; i += U * blockDim.x) {
    f32x4 v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[u][k] = (i + u * blockDim.x < hi) ? __builtin_nontemporal_load(a.in[k] + i + u * blockDim.x) : f32x4{0,0,0,0};
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * blockDim.x < hi) {
        f32x4 r = ((v[u][0] + v[u][1]) + (v[u][2] + v[u][3])) + ((v[u][4] + v[u][5]) + (v[u][6] + v[u][7]));
        __builtin_nontemporal_store(r, a.out + i + u * blockDim.x);
      }
  }
}
template <int U, bool NTS>
__global__ void fold8_once(P a) {
  const long long base = ((long long)blockIdx.x * U) * blockDim.x + threadIdx.x;
  f32x4 v[U][8];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + (long long)u * blockDim.x;
    if (i < a.nv) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[u][k] = __builtin_nontemporal_load(a.in[k] + i);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = base + (long long)u * blockDim.x;
    if (i < a.nv) {
      f32x4 r = ((v[u][0] + v[u][1]) + (v[u][2] + v[u][3])) + ((v[u][4] + v[u][5]) + (v[u][6] + v[u][7]));
      S<NTS>(a.out + i, r);
    }
  }
}
// wave-contiguous: each wave owns W*1 KiB contiguous of every input (lane l
// loads l, l+64, ... inside the wave's span)
template <int W, bool NTS>
__global__ void fold8_wave(P a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  const long long base = ((long long)blockIdx.x * wpb + wave) * (64 * W) + lane;
  f32x4 v[W][8];
#pragma unroll
  for (int u = 0; u < W; ++u) {
    const long long i = base + 64 * u;
    if (i < a.nv) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[u][k] = __builtin_nontemporal_load(a.in[k] + i);
    }
  }
#pragma unroll
  for (int u = 0; u < W; ++u) {
    const long long i = base + 64 * u;
    if (i < a.nv) {
      f32x4 r = ((v[u][0] + v[u][1]) + (v[u][2] + v[u][3])) + ((v[u][4] + v[u][5]) + (v[u][6] + v[u][7]));
      S<NTS>(a.out + i, r);
    }
  }
}
__global__ void copyk(const f32x4* s, f32x4* d, long long nv) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (long long)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), d + i);
}
__global__ void readk(const f32x4* s, f32x4* d, long long nv) {
  f32x4 acc = {0, 0, 0, 0};
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += (long long)gridDim.x * blockDim.x)
    acc += __builtin_nontemporal_load(s + i);
  if (acc[0] == 123.456f) d[0] = acc;
}

struct V { const char* name; int grid, block, kind; long long span; };

int main() {
  const long long count = 64ll << 20, nv = count / 4;
  const size_t S = count * 4;
  P a;
  std::vector<void*> bufs;
  for (int k = 0; k < 8; ++k) { void* p; CK(hipMalloc(&p, S)); CK(hipMemset(p, 0x3c, S)); a.in[k] = (const f32x4*)p; }
  void* o; CK(hipMalloc(&o, S)); a.out = (f32x4*)o; a.nv = nv;
  P b = a;  // inputs staggered inside one allocation
  void* slab; CK(hipMalloc(&slab, 8 * S + 8 * 69632)); CK(hipMemset(slab, 0x3c, 8 * S + 8 * 69632));
  for (int k = 0; k < 8; ++k) b.in[k] = (const f32x4*)((char*)slab + k * (S + 69632));
  void* big; CK(hipMalloc(&big, 8 * S));  // 2 GiB single buffer for copy/read peaks
  CK(hipMemset(big, 0, 8 * S));
  std::vector<V> vs = {
      {"wave W1 b256 plainS", 65536, 256, 20}, {"wave W2 b256 plainS", 32768, 256, 21},
      {"wave W4 b256 plainS", 16384, 256, 22}, {"wave W2 b64 plainS", 131072, 64, 21},
      {"wave W1 b64 plainS", 262144, 64, 20}, {"wave W4 b128 plainS", 16384*2, 128, 22},
      {"once U1 b256 NTS", 65536, 256, 10}, {"once U1 b256 staggered", 65536, 256, 14}, {"once U1 b256 plainS", 65536, 256, 11},
      {"once U2 b256 NTS", 32768, 256, 12}, {"once U4 b256 NTS", 16384, 256, 13},
      {"once U1 b512 NTS", 32768, 512, 10}, {"once U1 b1024 NTS", 16384, 1024, 10},
      {"once U2 b512 NTS", 16384, 512, 12}, {"once U1 b128 NTS", 131072, 128, 10},
      {"U1 NT g4096 b256", 4096, 256, 0}, {"U2 NT g4096 b256", 4096, 256, 1}, {"U4 NT g2048 b256", 2048, 256, 2},
      {"U1 plain g4096", 4096, 256, 3}, {"U1 NTload plainstore g4096", 4096, 256, 4},
      {"U1 NT g1792 b256", 1792, 256, 0}, {"U1 NT g16384 b256", 16384, 256, 0}, {"U1 NT g65536 b256 (1 iter)", 65536, 256, 0},
      {"U2 NT g1024 b512", 1024, 512, 1}, {"U2 NT g2048 b512", 2048, 512, 1}, {"U1 NT g2048 b1024", 2048, 1024, 0},
      {"U2 NT g8192 b256", 8192, 256, 1},
      {"span U2 g2048 b256", 2048, 256, 5}, {"span U4 g1024 b256", 1024, 256, 6}, {"span U2 g4096 b256", 4096, 256, 5},
      {"copy 256MiB", 4096, 256, 7}, {"copy 1GiB", 4096, 256, 8}, {"read 2GiB", 4096, 256, 9},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int R = 7, IT = 10;
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < R; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      auto launch = [&]() {
        const V& x = vs[v];
        switch (x.kind) {
          case 0: hipLaunchKernelGGL((fold8<1, true, true>), x.grid, x.block, 0, 0, a); break;
          case 1: hipLaunchKernelGGL((fold8<2, true, true>), x.grid, x.block, 0, 0, a); break;
          case 2: hipLaunchKernelGGL((fold8<4, true, true>), x.grid, x.block, 0, 0, a); break;
          case 3: hipLaunchKernelGGL((fold8<1, false, false>), x.grid, x.block, 0, 0, a); break;
          case 4: hipLaunchKernelGGL((fold8<1, true, false>), x.grid, x.block, 0, 0, a); break;
          case 5: hipLaunchKernelGGL((fold8_span<2>), x.grid, x.block, 0, 0, a, (nv + x.grid - 1) / x.grid); break;
          case 6: hipLaunchKernelGGL((fold8_span<4>), x.grid, x.block, 0, 0, a, (nv + x.grid - 1) / x.grid); break;
          case 7: hipLaunchKernelGGL(copyk, x.grid, x.block, 0, 0, a.in[0], a.out, nv); break;
          case 8: hipLaunchKernelGGL(copyk, x.grid, x.block, 0, 0, (const f32x4*)big, (f32x4*)big + 4 * nv, 4 * nv); break;
          case 9: hipLaunchKernelGGL(readk, x.grid, x.block, 0, 0, (const f32x4*)big, a.out, 8 * nv); break;
          case 10: hipLaunchKernelGGL((fold8_once<1, true>), x.grid, x.block, 0, 0, a); break;
          case 20: hipLaunchKernelGGL((fold8_wave<1, false>), x.grid, x.block, 0, 0, a); break;
          case 21: hipLaunchKernelGGL((fold8_wave<2, false>), x.grid, x.block, 0, 0, a); break;
          case 22: hipLaunchKernelGGL((fold8_wave<4, false>), x.grid, x.block, 0, 0, a); break;
          case 14: hipLaunchKernelGGL((fold8_once<1, true>), x.grid, x.block, 0, 0, b); break;
          case 11: hipLaunchKernelGGL((fold8_once<1, false>), x.grid, x.block, 0, 0, a); break;
          case 12: hipLaunchKernelGGL((fold8_once<2, true>), x.grid, x.block, 0, 0, a); break;
          case 13: hipLaunchKernelGGL((fold8_once<4, true>), x.grid, x.block, 0, 0, a); break;
        }
      };
      launch();
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < IT; ++i) launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t; CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / IT);
    }
  for (size_t v = 0; v < vs.size(); ++v) {
    auto m = ms[v];
    std::sort(m.begin(), m.end());
    double bytes = vs[v].kind == 7 ? 2.0 * S : vs[v].kind == 8 ? 8.0 * S : vs[v].kind == 9 ? 8.0 * S : 9.0 * S;
    printf("%-30s median %8.1f us  %7.1f GB/s  (min %7.1f us)\n", vs[v].name, m[R / 2] * 1e3, bytes / (m[R / 2] * 1e-3) / 1e9, m[0] * 1e3);
  }
  return 0;
}
