// Microbenchmark of the config-2 local fold (8 x 256 MiB -> 1) on MI355X:
// the product kernel (csrc/kernels.hpp fold_local_kernel) at several
// vectors-per-thread U, against simple reference streams (one-pass fold with
// plain / nt stores, XCD-remapped block order, read-only and copy streams),
// timed interleaved in one process (median of rounds).  Also checks the
// gfx950 f32 -> bf16 conversion (v_cvt_pk_bf16_f32) against the software
// RNE definition (device.hpp f2bf) on all 2^32 f32 bit patterns.
// Tooling only; build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../mpi.jl_amd/csrc/kernels.hpp"

using namespace mpigx;
#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));   \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
struct P8 {
  const f32x4* in[8];
  f32x4* out;
  long long nv;
};

template <bool NTS, bool XCD>
__global__ __launch_bounds__(256) void ref_once(P8 a) {
  unsigned b = blockIdx.x;
  if constexpr (XCD) {  // blocks b, b+8, ... (one XCD) take a contiguous range
    const unsigned G = gridDim.x, per = G / 8;
    if (b < per * 8) b = (b % 8) * per + b / 8;
  }
  const long long i = (long long)b * 256 + threadIdx.x;
  if (i >= a.nv) return;
  f32x4 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(a.in[k] + i);
  const f32x4 r = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
  if constexpr (NTS) __builtin_nontemporal_store(r, a.out + i);
  else a.out[i] = r;
}
__global__ __launch_bounds__(256) void read8(P8 a) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.nv) return;
  f32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 8; ++k) acc += __builtin_nontemporal_load(a.in[k] + i);
  if (acc[0] == 123.456f) a.out[i] = acc;
}
__global__ __launch_bounds__(256) void copy1(const f32x4* s, f32x4* d, long long nv) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < nv) d[i] = __builtin_nontemporal_load(s + i);
}
// placement / store-policy experiments on the 8 -> 1 f32 SUM stream (U = 4
// vectors per thread, the product's pairwise tree):
//   SP = 0 plain stores, 1 nt stores, 2 sc1 (write-through) stores
//   SHIFT: the result of vector i is written to out[(i + SHIFT) mod nv] —
//   same bytes, but the write stream no longer shares the reads' offsets
template <int SP, long long SHIFT>
__global__ __launch_bounds__(256) void exp4(P8 a) {
  const long long base = (long long)blockIdx.x * 1024 + threadIdx.x;
  f32x4 v[4][8];
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int k = 0; k < 8; ++k) v[u][k] = __builtin_nontemporal_load(a.in[k] + base + u * 256);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const f32x4 r = ((v[u][0] + v[u][1]) + (v[u][2] + v[u][3])) + ((v[u][4] + v[u][5]) + (v[u][6] + v[u][7]));
    long long j = base + u * 256 + SHIFT;
    if (j >= a.nv) j -= a.nv;
    f32x4* q = a.out + j;
    if constexpr (SP == 0) *q = r;
    else if constexpr (SP == 1) __builtin_nontemporal_store(r, q);
    else if constexpr (SP == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(q), "v"(r) : "memory");
    else if constexpr (SP == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(q), "v"(r) : "memory");
    else if constexpr (SP == 4) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" : : "v"(q), "v"(r) : "memory");
    else if constexpr (SP == 5) asm volatile("global_store_dwordx4 %0, %1, off sc0" : : "v"(q), "v"(r) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" : : "v"(q), "v"(r) : "memory");
  }
}

// write bursts: each thread folds T consecutive tiles (U = 4 vectors each)
// and keeps the results in registers, then stores all 4T of them together —
// the write stream reaches HBM in bursts of T tiles per wave instead of one
// store group after every 32 loads (fewer read/write turnarounds, if that is
// what costs the fold its gap to the read-only stream)
template <int T>
__global__ __launch_bounds__(256) void expb(P8 a) {
  f32x4 res[T][4];
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const long long base = ((long long)blockIdx.x * T + t) * 1024 + threadIdx.x;
    f32x4 v[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[u][k] = __builtin_nontemporal_load(a.in[k] + base + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      res[t][u] = ((v[u][0] + v[u][1]) + (v[u][2] + v[u][3])) + ((v[u][4] + v[u][5]) + (v[u][6] + v[u][7]));
  }
#pragma unroll
  for (int t = 0; t < T; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x4* q = a.out + ((long long)blockIdx.x * T + t) * 1024 + threadIdx.x + u * 256;
      asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(q), "v"(res[t][u]) : "memory");
    }
}

// exhaustive f32 -> bf16: hardware pair conversion vs the software RNE; each
// thread checks 16 pairs, one atomic per block (bounded even if all differ)
__global__ __launch_bounds__(256) void cvt_check(unsigned long long base, unsigned long long* bad, unsigned* first) {
  __shared__ unsigned s_cnt, s_first;
  if (threadIdx.x == 0) { s_cnt = 0; s_first = 0xffffffffu; }
  __syncthreads();
  unsigned cnt = 0, fst = 0xffffffffu;
  for (int k = 0; k < 16; ++k) {
    const unsigned long long i = base + ((unsigned long long)blockIdx.x * 16 + k) * 256 + threadIdx.x;
    const uint32_t u0 = (uint32_t)(2 * i), u1 = (uint32_t)(2 * i + 1);
    const uint32_t hw = f32x2_to_bf16x2(f32x2_t{__uint_as_float(u0), __uint_as_float(u1)});
    const uint32_t sw = (uint32_t)f2bf(__uint_as_float(u0)).u | ((uint32_t)f2bf(__uint_as_float(u1)).u << 16);
    if (hw != sw) {
      ++cnt;
      const unsigned f = (hw & 0xffffu) != (sw & 0xffffu) ? u0 : u1;
      fst = f < fst ? f : fst;
    }
  }
  if (cnt) { atomicAdd(&s_cnt, cnt); atomicMin(&s_first, fst); }
  __syncthreads();
  if (threadIdx.x == 0 && s_cnt) { atomicAdd(bad, (unsigned long long)s_cnt); atomicMin(first, s_first); }
}

template <class OP, class T, int U, int SHAPE = SH_FULL>
hipError_t launch_prod(const FoldArgs& a) {
  const int W = VecW<T>::v;
  const long long nv = a.count / W;
  const long long g = (nv + 256ll * U - 1) / (256ll * U);
  hipLaunchKernelGGL((fold_local_kernel<OP, T, 8, S_TREE, SHAPE, U>), dim3((unsigned)g), dim3(256), 0, 0, a);
  return hipGetLastError();
}

FoldArgs make_args(void* const* in, void* out, long long count, int es) {
  FoldArgs a;
  memset(&a, 0, sizeof a);
  a.mode = M_LOCAL;
  a.esize = es;
  a.count = count;
  a.recv = out;
  a.ntree = 8;
  a.rem = 0;
  a.owner_mode = 1;
  a.pof2_log = 3;
  a.blk_len = count / 8;
  a.blk_inv = 1.0 / (double)a.blk_len;
  for (int k = 0; k < 8; ++k) a.src[k] = in[k];
  return a;
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? atoi(argv[1]) : 7;
  const long long S = 256ll << 20;  // bytes per buffer
  void* outb;
  CK(hipMalloc(&outb, S));  // allocated before the inputs
  void* in[8];
  for (int k = 0; k < 8; ++k) {
    CK(hipMalloc(&in[k], S));
    CK(hipMemset(in[k], 0x3c + k, S));
  }
  void *out, *out2;
  CK(hipMalloc(&out, S));
  CK(hipMalloc(&out2, S));
  // staggered slab: the 8 inputs inside one allocation, 69632 B apart past 256 MiB
  const long long stag = 69632;
  char* slab;
  CK(hipMalloc((void**)&slab, 8 * (S + stag)));
  CK(hipMemset(slab, 0x3c, 8 * (S + stag)));
  void* sin[8];
  for (int k = 0; k < 8; ++k) sin[k] = slab + k * (S + stag);

  const long long cf = S / 4, cb = S / 2;
  FoldArgs af = make_args(in, out, cf, 4), ab = make_args(in, out, cb, 2), as = make_args(sin, out, cf, 4);
  P8 p;
  for (int k = 0; k < 8; ++k) p.in[k] = (const f32x4*)in[k];
  p.out = (f32x4*)out2;
  p.nv = S / 16;
  const unsigned G1 = (unsigned)(p.nv / 256);

  struct V {
    std::string name;
    double bytes;
    std::function<hipError_t()> go;
  };
  const double B9 = 9.0 * S;
  // output placements: out allocated after the inputs (out2 / out), an
  // output allocated BEFORE them (outb), an output 68 KiB into its allocation
  char* outo_raw;
  CK(hipMalloc((void**)&outo_raw, S + stag));
  void* outo = outo_raw + stag;
  FoldArgs ab4 = make_args(in, outb, cf, 4), ao4 = make_args(in, outo, cf, 4);
  P8 pb = p, po = p, pa = p;
  pb.out = (f32x4*)outb;
  po.out = (f32x4*)outo;
  pa.out = (f32x4*)out;
  const unsigned G4 = (unsigned)(p.nv / 1024);
  std::vector<V> vs = {
      {"prod f32 SUM U4 out-after", B9, [&] { return launch_prod<OpSum, float, 4>(af); }},
      {"prod f32 SUM U4 out-before", B9, [&] { return launch_prod<OpSum, float, 4>(ab4); }},
      {"prod f32 SUM U4 out+68K", B9, [&] { return launch_prod<OpSum, float, 4>(ao4); }},
      {"prod f32 SUM U4 stag inputs", B9, [&] { return launch_prod<OpSum, float, 4>(as); }},
      {"exp plain shift0", B9, [&] { hipLaunchKernelGGL((exp4<0, 0>), dim3(G4), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"exp nt shift0", B9, [&] { hipLaunchKernelGGL((exp4<1, 0>), dim3(G4), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"exp sc1 shift0", B9, [&] { hipLaunchKernelGGL((exp4<2, 0>), dim3(G4), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"exp sc0sc1", B9, [&] { hipLaunchKernelGGL((exp4<3, 0>), dim3(G4), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"exp sc1nt", B9, [&] { hipLaunchKernelGGL((exp4<4, 0>), dim3(G4), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"exp sc0", B9, [&] { hipLaunchKernelGGL((exp4<5, 0>), dim3(G4), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"exp sc0sc1nt", B9, [&] { hipLaunchKernelGGL((exp4<6, 0>), dim3(G4), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"burst T2", B9, [&] { hipLaunchKernelGGL((expb<2>), dim3(G4 / 2), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"burst T4", B9, [&] { hipLaunchKernelGGL((expb<4>), dim3(G4 / 4), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"burst T8", B9, [&] { hipLaunchKernelGGL((expb<8>), dim3(G4 / 8), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"exp plain shift16M", B9, [&] { hipLaunchKernelGGL((exp4<0, (1 << 20)>), dim3(G4), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"exp plain shift68K", B9, [&] { hipLaunchKernelGGL((exp4<0, 4352>), dim3(G4), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"exp sc1 shift16M", B9, [&] { hipLaunchKernelGGL((exp4<2, (1 << 20)>), dim3(G4), dim3(256), 0, 0, pa); return hipGetLastError(); }},
      {"exp plain shift0 out-before", B9, [&] { hipLaunchKernelGGL((exp4<0, 0>), dim3(G4), dim3(256), 0, 0, pb); return hipGetLastError(); }},
      {"exp plain shift0 out+68K", B9, [&] { hipLaunchKernelGGL((exp4<0, 0>), dim3(G4), dim3(256), 0, 0, po); return hipGetLastError(); }},
      {"read 8 streams", 8.0 * S, [&] { hipLaunchKernelGGL(read8, dim3(G1), dim3(256), 0, 0, p); return hipGetLastError(); }},
      {"copy 256MiB", 2.0 * S, [&] { hipLaunchKernelGGL(copy1, dim3(G1), dim3(256), 0, 0, (const f32x4*)in[0], (f32x4*)out2, p.nv); return hipGetLastError(); }},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int IT = 10;
  std::vector<std::vector<float>> ms(vs.size());
  for (int r = 0; r < R; ++r)
    for (size_t v = 0; v < vs.size(); ++v) {
      CK(vs[v].go());
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < IT; ++i) CK(vs[v].go());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[v].push_back(t / IT);
    }
  printf("{\"what\": \"tools/fold_tune.hip, 8 x 256 MiB, median of %d rounds x %d launches\", \"variants\": {", R, IT);
  for (size_t v = 0; v < vs.size(); ++v) {
    auto m = ms[v];
    std::sort(m.begin(), m.end());
    printf("%s\"%s\": {\"us\": %.1f, \"GBps\": %.1f, \"min_us\": %.1f}", v ? ", " : "", vs[v].name.c_str(),
           m[R / 2] * 1e3, vs[v].bytes / (m[R / 2] * 1e-3) / 1e9, m[0] * 1e3);
  }
  printf("}");
  // parity: product U1/U2/U4 f32 SUM identical; reference stream == product (SUM tree of 8)
  std::vector<uint32_t> h1(1 << 20), h2(1 << 20);
  auto same = [&](void* a, void* b) -> bool {
    for (long long off = 0; off < S; off += 4ll << 20) {
      if (hipMemcpy(h1.data(), (char*)a + off, 4 << 20, hipMemcpyDeviceToHost) != hipSuccess) return false;
      if (hipMemcpy(h2.data(), (char*)b + off, 4 << 20, hipMemcpyDeviceToHost) != hipSuccess) return false;
      if (memcmp(h1.data(), h2.data(), 4 << 20)) return false;
    }
    return true;
  };
  { hipError_t e_ = launch_prod<OpSum, float, 1>(af); CK(e_); }
  hipLaunchKernelGGL((ref_once<false, false>), dim3(G1), dim3(256), 0, 0, p);
  CK(hipDeviceSynchronize());
  bool ok = same(out, out2);
  { FoldArgs t_ = make_args(in, out2, cf, 4); hipError_t e_ = launch_prod<OpSum, float, 2>(t_); CK(e_); }
  CK(hipDeviceSynchronize());
  ok &= same(out, out2);
  { hipError_t e_ = launch_prod<OpMax, bf16, 1>(ab); CK(e_); }
  { FoldArgs t_ = make_args(in, out2, cb, 2); hipError_t e_ = launch_prod<OpMax, bf16, 2>(t_); CK(e_); }
  CK(hipDeviceSynchronize());
  ok &= same(out, out2);
  { FoldArgs t_ = make_args(in, out2, cf, 4); hipError_t e_ = launch_prod<OpSum, float, 4>(t_); CK(e_); }
  { hipError_t e_ = launch_prod<OpSum, float, 1, SH_POW2>(af); CK(e_); }
  CK(hipDeviceSynchronize());
  ok &= same(out, out2);
  printf(", \"U_variants_bit_identical\": %s", ok ? "true" : "false");
  if (argc > 2) { printf("}\n"); return 0; }
  // exhaustive conversion check
  unsigned long long* bad;
  unsigned* first;
  CK(hipMalloc(&bad, 8));
  CK(hipMalloc(&first, 4));
  CK(hipMemset(bad, 0, 8));
  CK(hipMemset(first, 0xff, 4));
  const unsigned long long pairs = 1ull << 31, per = 1ull << 28;
  for (unsigned long long b0 = 0; b0 < pairs; b0 += per)
    hipLaunchKernelGGL(cvt_check, dim3((unsigned)(per / (256 * 16))), dim3(256), 0, 0, b0, bad, first);
  CK(hipDeviceSynchronize());
  unsigned long long nbad = 0;
  unsigned f = 0;
  CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost));
  printf(", \"bf16_hw_vs_sw_mismatches\": %llu, \"first_mismatch_f32_bits\": \"0x%08x\"}\n", nbad, nbad ? f : 0u);
  return 0;
}
