// device.hpp — CDNA4 device code shared by all kernel translation units:
// element types, the built-in MPI.Op set as functors, 16-byte vector access,
// the fold schedules, block-level copies and the cross-rank block barrier.
//
// Op semantics restate MPICH 3.3.2's MPIR op loops (the arithmetic MPI.jl
// delegates to libmpi, src/operators.jl:22-45): inout = OP(inout, in) with
// MAX = inout > in ? inout : in, MIN = inout < in ? inout : in, logical ops
// giving 0/1 in the element type, two's-complement wrap, complex PROD without
// FMA contraction (build with -ffp-contract=off; the _rn intrinsics below make
// it explicit).  oracle/mpich_model.py is the CPU statement they are checked
// against.
#pragma once
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace mpigx {

// ---------------------------------------------------------------------------
// element types
// ---------------------------------------------------------------------------
struct c64 { float re, im; };
struct c128 { double re, im; };
struct bf16 { uint16_t u; };

template <int R> struct RepType;
template <> struct RepType<R_I8> { using T = int8_t; };
template <> struct RepType<R_U8> { using T = uint8_t; };
template <> struct RepType<R_I16> { using T = int16_t; };
template <> struct RepType<R_U16> { using T = uint16_t; };
template <> struct RepType<R_I32> { using T = int32_t; };
template <> struct RepType<R_U32> { using T = uint32_t; };
template <> struct RepType<R_I64> { using T = int64_t; };
template <> struct RepType<R_U64> { using T = uint64_t; };
template <> struct RepType<R_F32> { using T = float; };
template <> struct RepType<R_F64> { using T = double; };
template <> struct RepType<R_C64> { using T = c64; };
template <> struct RepType<R_C128> { using T = c128; };
template <> struct RepType<R_BF16> { using T = bf16; };

template <class T> struct is_int { static constexpr bool v = false; };
#define MPIGX_ISINT_(TY) template <> struct is_int<TY> { static constexpr bool v = true; };
MPIGX_ISINT_(int8_t) MPIGX_ISINT_(uint8_t) MPIGX_ISINT_(int16_t) MPIGX_ISINT_(uint16_t)
MPIGX_ISINT_(int32_t) MPIGX_ISINT_(uint32_t) MPIGX_ISINT_(int64_t) MPIGX_ISINT_(uint64_t)
#undef MPIGX_ISINT_
template <class T> struct is_cplx { static constexpr bool v = false; };
template <> struct is_cplx<c64> { static constexpr bool v = true; };
template <> struct is_cplx<c128> { static constexpr bool v = true; };
template <class T> struct is_real_fp { static constexpr bool v = false; };
template <> struct is_real_fp<float> { static constexpr bool v = true; };
template <> struct is_real_fp<double> { static constexpr bool v = true; };
template <> struct is_real_fp<bf16> { static constexpr bool v = true; };

template <class T> struct unsigned_of { using U = T; };
template <> struct unsigned_of<int8_t> { using U = uint8_t; };
template <> struct unsigned_of<int16_t> { using U = uint16_t; };
template <> struct unsigned_of<int32_t> { using U = uint32_t; };
template <> struct unsigned_of<int64_t> { using U = uint64_t; };

__device__ __forceinline__ float bf2f(bf16 x) { return __uint_as_float(((uint32_t)x.u) << 16); }
// RNE fp32 -> bf16; NaN -> quiet NaN with the same sign/top payload
// (oracle/mpich_model.py f32_to_bf16).
__device__ __forceinline__ bf16 f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  bf16 r;
  if ((u & 0x7fffffffu) > 0x7f800000u) r.u = (uint16_t)((u >> 16) | 0x0040u);
  else r.u = (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
  return r;
}

// ---------------------------------------------------------------------------
// ops: apply(inout, in) -> new inout
// ---------------------------------------------------------------------------
template <class T> __device__ __forceinline__ T add_(T a, T b) {
  if constexpr (is_int<T>::v) {
    using U = typename unsigned_of<T>::U;
    return (T)(U)((U)a + (U)b);
  } else {
    return a + b;
  }
}
template <class T> __device__ __forceinline__ T mul_(T a, T b) {
  if constexpr (is_int<T>::v) {
    using U = typename unsigned_of<T>::U;
    if constexpr (sizeof(T) < 4) return (T)(U)((uint32_t)(U)a * (uint32_t)(U)b);
    else return (T)(U)((U)a * (U)b);
  } else {
    return a * b;
  }
}
template <class T> __device__ __forceinline__ bool nz_(T a) {
  if constexpr (is_int<T>::v) return a != 0;
  else return a != (T)0;
}

struct OpSum {
  static constexpr int code = O_SUM;
  template <class T> __device__ __forceinline__ static T apply(T a, T b) {
    if constexpr (std::is_same<T, float>::value) return __fadd_rn(a, b);
    else if constexpr (std::is_same<T, double>::value) return __dadd_rn(a, b);
    else if constexpr (std::is_same<T, bf16>::value) return f2bf(__fadd_rn(bf2f(a), bf2f(b)));
    else if constexpr (std::is_same<T, c64>::value) return c64{__fadd_rn(a.re, b.re), __fadd_rn(a.im, b.im)};
    else if constexpr (std::is_same<T, c128>::value) return c128{__dadd_rn(a.re, b.re), __dadd_rn(a.im, b.im)};
    else return add_(a, b);
  }
};
struct OpProd {
  static constexpr int code = O_PROD;
  template <class T> __device__ __forceinline__ static T apply(T a, T b) {
    if constexpr (std::is_same<T, float>::value) return __fmul_rn(a, b);
    else if constexpr (std::is_same<T, double>::value) return __dmul_rn(a, b);
    else if constexpr (std::is_same<T, bf16>::value) return f2bf(__fmul_rn(bf2f(a), bf2f(b)));
    else if constexpr (std::is_same<T, c64>::value)
      return c64{__fsub_rn(__fmul_rn(a.re, b.re), __fmul_rn(a.im, b.im)),
                 __fadd_rn(__fmul_rn(a.re, b.im), __fmul_rn(a.im, b.re))};
    else if constexpr (std::is_same<T, c128>::value)
      return c128{__dsub_rn(__dmul_rn(a.re, b.re), __dmul_rn(a.im, b.im)),
                  __dadd_rn(__dmul_rn(a.re, b.im), __dmul_rn(a.im, b.re))};
    else return mul_(a, b);
  }
};
struct OpMax {
  static constexpr int code = O_MAX;
  template <class T> __device__ __forceinline__ static T apply(T a, T b) {
    if constexpr (std::is_same<T, bf16>::value) return bf2f(a) > bf2f(b) ? a : b;
    else return a > b ? a : b;
  }
};
struct OpMin {
  static constexpr int code = O_MIN;
  template <class T> __device__ __forceinline__ static T apply(T a, T b) {
    if constexpr (std::is_same<T, bf16>::value) return bf2f(a) < bf2f(b) ? a : b;
    else return a < b ? a : b;
  }
};
template <class T> __device__ __forceinline__ T from_bool(bool v) {
  if constexpr (std::is_same<T, bf16>::value) return bf16{(uint16_t)(v ? 0x3f80u : 0u)};
  else return (T)(v ? 1 : 0);
}
template <class T> __device__ __forceinline__ bool truth(T a) {
  if constexpr (std::is_same<T, bf16>::value) return bf2f(a) != 0.0f;
  else return nz_(a);
}
struct OpLand {
  static constexpr int code = O_LAND;
  template <class T> __device__ __forceinline__ static T apply(T a, T b) { return from_bool<T>(truth(a) && truth(b)); }
};
struct OpLor {
  static constexpr int code = O_LOR;
  template <class T> __device__ __forceinline__ static T apply(T a, T b) { return from_bool<T>(truth(a) || truth(b)); }
};
struct OpLxor {
  static constexpr int code = O_LXOR;
  template <class T> __device__ __forceinline__ static T apply(T a, T b) { return from_bool<T>(truth(a) != truth(b)); }
};
struct OpBand {
  static constexpr int code = O_BAND;
  template <class T> __device__ __forceinline__ static T apply(T a, T b) { return (T)(a & b); }
};
struct OpBor {
  static constexpr int code = O_BOR;
  template <class T> __device__ __forceinline__ static T apply(T a, T b) { return (T)(a | b); }
};
struct OpBxor {
  static constexpr int code = O_BXOR;
  template <class T> __device__ __forceinline__ static T apply(T a, T b) { return (T)(a ^ b); }
};

// MIN/MAX on floating types are the only (op, type) pairs whose bits depend
// on which operand is inout (NaN, +0/-0 ties); everything else is symmetric.
template <class OP, class T> struct role_sensitive {
  static constexpr bool v = is_real_fp<T>::v && (OP::code == O_MIN || OP::code == O_MAX);
};

// 16-byte register vector for the streaming paths
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#ifndef MPIGX_NT
#define MPIGX_NT 1  // non-temporal hints on streamed (read-once) loads
#endif
#ifndef MPIGX_NT_STORE
#define MPIGX_NT_STORE 0  // fold outputs: plain stores measured >= nt (tools/local_tune.hip)
#endif
__device__ __forceinline__ u32x4 ld16(const void* p) {
#if MPIGX_NT
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
#else
  return *reinterpret_cast<const u32x4*>(p);
#endif
}
__device__ __forceinline__ void st16(void* p, u32x4 v) {
#if MPIGX_NT_STORE
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
#else
  *reinterpret_cast<u32x4*>(p) = v;
#endif
}

// ---------------------------------------------------------------------------
// vector access: W elements of T at p (W*sizeof(T) == 16 when vectorised)
// ---------------------------------------------------------------------------
template <class T> struct VecW { static constexpr int v = sizeof(T) >= 16 ? 1 : 16 / (int)sizeof(T); };

template <class T, int W>
__device__ __forceinline__ void ld(T (&d)[W], const T* p) {
  if constexpr (W * sizeof(T) == 16) {
    *reinterpret_cast<u32x4*>(d) = ld16(p);
  } else {
#pragma unroll
    for (int w = 0; w < W; ++w) d[w] = p[w];
  }
}
template <class T, int W>
__device__ __forceinline__ void st(T* p, const T (&d)[W]) {
  if constexpr (W * sizeof(T) == 16) {
    st16(p, *reinterpret_cast<const u32x4*>(d));
  } else {
#pragma unroll
    for (int w = 0; w < W; ++w) p[w] = d[w];
  }
}

// ---------------------------------------------------------------------------
// fold of the leaves at element e (W consecutive elements)
//   TREE  : pre-step (leaf s < rem: src[s] = OP(src[s], src2[s])), then the
//           pairwise tree over ntree leaves truncated binomially, with the
//           inout operand of each node chosen by the owner rule.
//   LINEAR: ((x0 op x1) op x2) ... over ntree leaves.
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned bitrev(unsigned j, int L) {
  return L == 0 ? 0u : (__builtin_bitreverse32(j) >> (32 - L));
}

template <class OP, class T, int NMAX, int SCHED, int W>
__device__ __forceinline__ void fold_at(const FoldArgs& A, const T* const* src, const T* const* src2,
                                        long long e, T (&res)[W]) {
  T v[NMAX][W];
#pragma unroll
  for (int s = 0; s < NMAX; ++s)
    if (s < A.ntree) ld<T, W>(v[s], src[s] + e);
  if constexpr (SCHED == S_LINEAR) {
#pragma unroll
    for (int s = 1; s < NMAX; ++s)
      if (s < A.ntree) {
#pragma unroll
        for (int w = 0; w < W; ++w) v[0][w] = OP::apply(v[0][w], v[s][w]);
      }
  } else {
    if (A.rem > 0) {
#pragma unroll
      for (int s = 0; s < NMAX / 2; ++s)
        if (s < A.rem) {
          T u[W];
          ld<T, W>(u, src2[s] + e);
#pragma unroll
          for (int w = 0; w < W; ++w) v[s][w] = OP::apply(v[s][w], u[w]);
        }
    }
    unsigned own[W];
#pragma unroll
    for (int w = 0; w < W; ++w) own[w] = 0;
    if constexpr (role_sensitive<OP, T>::v) {
      if (A.owner_mode) {
        // Rabenseifner block of each element: one 64-bit division per vector,
        // then step across the (rare) block boundaries inside the vector
        const unsigned pof2 = 1u << A.pof2_log;
        const unsigned long long g0 = (unsigned long long)(A.gbase + e), bl = (unsigned long long)A.blk_len;
        // no data-dependent loop here: a `while` inside the unrolled w loop
        // kept it rolled and pushed v[][] to scratch (840 B/lane, f32 MAX
        // at 0.67 TB/s).  bl >= W crosses at most one boundary per vector.
        const unsigned long long j0 = g0 / bl, next = (j0 + 1) * bl;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const unsigned long long j = bl >= (unsigned long long)W ? j0 + (g0 + w >= next ? 1ull : 0ull)
                                                                  : (g0 + w) / bl;
          own[w] = bitrev((unsigned)(j > pof2 - 1 ? pof2 - 1 : j), A.pof2_log);
        }
      }
    }
#pragma unroll
    for (int m = 1; m < NMAX; m <<= 1) {
#pragma unroll
      for (int s = 0; s + m < NMAX; s += 2 * m) {
        if (s + m < A.ntree) {
#pragma unroll
          for (int w = 0; w < W; ++w) {
            if constexpr (role_sensitive<OP, T>::v) {
              // operands are swapped by value: a select between the two
              // array slots became a select of addresses and moved v[][]
              // to scratch (840 B/lane)
              const T lo = v[s][w], hi = v[s + m][w];
              const T r0 = OP::apply(lo, hi), r1 = OP::apply(hi, lo);
              v[s][w] = (own[w] & (unsigned)m) ? r1 : r0;
            } else {
              v[s][w] = OP::apply(v[s][w], v[s + m][w]);
            }
          }
        }
      }
    }
  }
#pragma unroll
  for (int w = 0; w < W; ++w) res[w] = v[0][w];
}

// Fold [lo, hi) (element indices into the sources) into out1 (and out2 if
// non-null), the whole block cooperating.  lo is a multiple of the vector
// width; `vec` says whether every pointer involved is 16-byte aligned.
template <class OP, class T, int NMAX, int SCHED>
__device__ __forceinline__ void fold_range(const FoldArgs& A, const T* const* src, const T* const* src2,
                                           long long lo, long long hi, T* out1, T* out2, bool vec,
                                           long long tid, long long nthr) {
  constexpr int W = VecW<T>::v;
  if (vec) {
    const long long nv = (hi - lo) / W;
    for (long long i = tid; i < nv; i += nthr) {
      const long long e = lo + i * W;
      T r[W];
      fold_at<OP, T, NMAX, SCHED, W>(A, src, src2, e, r);
      st<T, W>(out1 + e, r);
      if (out2) st<T, W>(out2 + e, r);
    }
    lo += nv * W;
  }
  for (long long e = lo + tid; e < hi; e += nthr) {
    T r[1];
    fold_at<OP, T, NMAX, SCHED, 1>(A, src, src2, e, r);
    out1[e] = r[0];
    if (out2) out2[e] = r[0];
  }
}

// ---------------------------------------------------------------------------
// block-cooperative byte copy (alignment-peeling, 16-B vectors when possible)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void block_copy(char* dst, const char* src, long long bytes) {
  if (bytes <= 0 || dst == src) return;
  const int tid = threadIdx.x, nt = blockDim.x;
  const uintptr_t da = (uintptr_t)dst, sa = (uintptr_t)src;
  if (((da ^ sa) & 15) == 0) {
    long long head = (long long)((16 - (da & 15)) & 15);
    if (head > bytes) head = bytes;
    for (long long i = tid; i < head; i += nt) dst[i] = src[i];
    const long long nv = (bytes - head) / 16;
    const u32x4* s4 = reinterpret_cast<const u32x4*>(src + head);
    u32x4* d4 = reinterpret_cast<u32x4*>(dst + head);
    long long i = tid;
    for (; i + 3 * nt < nv; i += 4 * nt) {  // 4 loads in flight per thread
      const u32x4 a = ld16(s4 + i), b = ld16(s4 + i + nt);
      const u32x4 c = ld16(s4 + i + 2 * nt), d = ld16(s4 + i + 3 * nt);
      st16(d4 + i, a);
      st16(d4 + i + nt, b);
      st16(d4 + i + 2 * nt, c);
      st16(d4 + i + 3 * nt, d);
    }
    for (; i < nv; i += nt) st16(d4 + i, ld16(s4 + i));
    for (long long j = head + nv * 16 + tid; j < bytes; j += nt) dst[j] = src[j];
  } else if (((da ^ sa) & 3) == 0) {
    long long head = (long long)((4 - (da & 3)) & 3);
    if (head > bytes) head = bytes;
    for (long long i = tid; i < head; i += nt) dst[i] = src[i];
    const long long nv = (bytes - head) / 4;
    const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src + head);
    uint32_t* d4 = reinterpret_cast<uint32_t*>(dst + head);
    for (long long i = tid; i < nv; i += nt) d4[i] = s4[i];
    for (long long j = head + nv * 4 + tid; j < bytes; j += nt) dst[j] = src[j];
  } else {
    for (long long i = tid; i < bytes; i += nt) dst[i] = src[i];
  }
}

// ---------------------------------------------------------------------------
// block-cooperative copy of up to NMAX (dst, src, len) pairs with the pairs
// INTERLEAVED per thread: every iteration issues one 16-B load per pair
// before storing, so when the sources are different peers every xGMI link
// carries traffic at all times (a peer-by-peer loop would drive one link at
// a time across the whole grid).  Falls back to per-pair block_copy when a
// pair is not 16-B aligned.
// ---------------------------------------------------------------------------
template <int NMAX>
__device__ __forceinline__ void block_gather(char* const (&dst)[NMAX], const char* const (&src)[NMAX],
                                             const long long (&len)[NMAX], int m) {
  bool vec = true;
  long long nvmax = 0;
#pragma unroll
  for (int p = 0; p < NMAX; ++p)
    if (p < m) {
      vec &= ((((uintptr_t)dst[p]) | ((uintptr_t)src[p])) & 15) == 0;
      const long long nv = len[p] / 16;
      nvmax = nv > nvmax ? nv : nvmax;
    }
  if (!vec) {
#pragma unroll
    for (int p = 0; p < NMAX; ++p)
      if (p < m) block_copy(dst[p], src[p], len[p]);
    return;
  }
  const long long tid = threadIdx.x, nt = blockDim.x;
  for (long long i = tid; i < nvmax; i += nt) {
    u32x4 v[NMAX];
#pragma unroll
    for (int p = 0; p < NMAX; ++p)
      if (p < m && i < len[p] / 16) v[p] = ld16(src[p] + 16 * i);
#pragma unroll
    for (int p = 0; p < NMAX; ++p)
      if (p < m && i < len[p] / 16) st16(dst[p] + 16 * i, v[p]);
  }
#pragma unroll
  for (int p = 0; p < NMAX; ++p)
    if (p < m)
      for (long long j = (len[p] / 16) * 16 + tid; j < len[p]; j += nt) dst[p][j] = src[p][j];
}

// ---------------------------------------------------------------------------
// Pull kernels launched after a HOST-side hand-off (p2p / RMA: the producer's
// kernel finished and the host saw it) read peer memory mapped through IPC.
// Kernel boundaries order local memory, but this CU's L1 / this XCD's L2 may
// still hold lines of the peer allocation from an earlier pull of the same
// bytes, so every block drops them first (system-scope acquire, one lane,
// then the block barrier) and publishes its own stores at system scope at
// the end (a peer may pull them next).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void pull_acquire(int on) {
  if (!on) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
}
__device__ __forceinline__ void pull_release(int on) {
  if (!on) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
}

// ---------------------------------------------------------------------------
// cross-rank barrier of block `blockIdx.x` on every rank, at epoch `ep`.
// Producer side: every wave drains its stores, block barrier, one wave issues
// a SYSTEM-scope release (writes this XCD's L2 back so peers reading our HBM
// over xGMI see it), then one lane per peer stores `ep` into that peer's
// signal slot [block][my rank].  Consumer side: lane p polls my slot
// [block][p] (relaxed, system scope, uncached memory) until >= ep, then a
// system-scope acquire invalidates this CU's L1 and the stale non-coherent
// L2 lines before any wave reads peer data (MI355X_MICROARCH.md
// "inter-workgroup visibility"; cdna_hip_programming.md Guideline 16, at
// system instead of agent scope because the peers are other GPUs).
// Epochs are monotone per communicator, so slots never need resetting.
// Returns false (and sets *err) if a peer did not arrive within the timeout.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool rank_barrier(const PeerView& pv, uint64_t ep) {
  __shared__ int s_fail;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bool ok = true;
    if (lane < pv.n) {
      uint64_t* peer_slot = pv.sig[lane] + (size_t)blockIdx.x * kMaxRanks + pv.rank;
      __hip_atomic_store(peer_slot, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      uint64_t* mine = pv.sig[pv.rank] + (size_t)blockIdx.x * kMaxRanks + lane;
      const uint64_t t0 = wall_clock64();
      while (__hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < ep) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > pv.timeout_ticks) {
          ok = false;
          break;
        }
      }
    }
    const bool all_ok = __all(ok);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (lane == 0) {
      s_fail = all_ok ? 0 : 1;
      if (!all_ok) __hip_atomic_store(pv.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();
  return s_fail == 0;
}

}  // namespace mpigx
