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

// ---------------------------------------------------------------------------
// bf16 pairs: two bf16 in one dword, the ops on both at once.  The same
// definition as OpSum/OpProd/OpMax/OpMin::apply on bf16 (fp32 compute, RNE to
// bf16 after the op, NaN kept quiet with its sign and top payload), in fewer
// instructions: one v_pk_add_f32 / v_pk_mul_f32 and one v_cvt_pk_bf16_f32 per
// pair instead of 2 x (add + software RNE + repack); MIN/MAX select whole
// dwords and merge the halves with one bitfield insert.  gfx950's
// v_cvt_pk_bf16_f32 rounds to nearest even and turns a NaN into
// (bits >> 16) | 0x40 — the software f2bf above (MPIGX_HW_BF16=0 builds that
// instead; tests/test_local_gpu.py checks random bit patterns against the oracle).
// ---------------------------------------------------------------------------
#ifndef MPIGX_HW_BF16
#define MPIGX_HW_BF16 1
#endif
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2_t bf16x2_to_f32x2(uint32_t a) {
  return f32x2_t{__uint_as_float(a << 16), __uint_as_float(a & 0xffff0000u)};
}
__device__ __forceinline__ uint32_t f32x2_to_bf16x2(f32x2_t f) {
#if MPIGX_HW_BF16
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f, bf16x2_t));
#else
  return (uint32_t)f2bf(f.x).u | ((uint32_t)f2bf(f.y).u << 16);
#endif
}

template <class OP>
__device__ __forceinline__ uint32_t bf16x2_apply(uint32_t a, uint32_t b) {  // a = inout, b = in
  if constexpr (OP::code == O_SUM) {
    return f32x2_to_bf16x2(bf16x2_to_f32x2(a) + bf16x2_to_f32x2(b));
  } else if constexpr (OP::code == O_PROD) {
    return f32x2_to_bf16x2(bf16x2_to_f32x2(a) * bf16x2_to_f32x2(b));
  } else if constexpr (OP::code == O_MAX || OP::code == O_MIN) {
    const f32x2_t fa = bf16x2_to_f32x2(a), fb = bf16x2_to_f32x2(b);
    const bool lo = OP::code == O_MAX ? fa.x > fb.x : fa.x < fb.x;
    const bool hi = OP::code == O_MAX ? fa.y > fb.y : fa.y < fb.y;
    return ((lo ? a : b) & 0xffffu) | ((hi ? a : b) & 0xffff0000u);
  } else {
    bf16 x0{(uint16_t)a}, x1{(uint16_t)(a >> 16)}, y0{(uint16_t)b}, y1{(uint16_t)(b >> 16)};
    return (uint32_t)OP::apply(x0, y0).u | ((uint32_t)OP::apply(x1, y1).u << 16);
  }
}

// 16-byte register vector for the streaming paths
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#ifndef MPIGX_NT
#define MPIGX_NT 1  // non-temporal hints on streamed (read-once) loads
#endif
#ifndef MPIGX_NT_STORE
#define MPIGX_NT_STORE 0  // fold outputs: plain stores measured >= nt (tools/local_tune.hip)
#endif
// Every streamed operand is HBM (ours or a peer's, IPC-mapped): accessed
// through GLOBAL address-space pointers.  Through generic pointers the
// compiler emits FLAT loads/stores, which count against lgkmcnt as well as
// vmcnt and may alias LDS; in the kernels that stage their argument block
// in LDS (fold/ar_zc/copy/scan) every re-read of a source pointer from LDS
// then waited for all outstanding loads (s_waitcnt vmcnt(0) lgkmcnt(0)
// between the loads of one thread: ~1 load in flight whatever the unroll).
#define MPIGX_GPTR(T, p) ((__attribute__((address_space(1))) T*)(p))
__device__ __forceinline__ u32x4 ld16(const void* p) {
#if MPIGX_NT
  return __builtin_nontemporal_load(MPIGX_GPTR(const u32x4, p));
#else
  return *MPIGX_GPTR(const u32x4, p);
#endif
}
__device__ __forceinline__ void st16(void* p, u32x4 v) {
#if MPIGX_NT_STORE
  __builtin_nontemporal_store(v, MPIGX_GPTR(u32x4, p));
#else
  *MPIGX_GPTR(u32x4, p) = v;
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

// Register vector of W elements of T for the fold / scan arithmetic.  bf16
// vectors live as packed dword pairs — the form a 16-B load delivers and the
// pair ops (bf16x2_apply) consume — so no 16-bit element ever occupies a
// register of its own (an array of bf16 structs was split into eight 16-bit
// values per vector: twice the VGPRs plus unpack / repack instructions).
template <class T, int W>
struct Vec {
  static constexpr bool packed = std::is_same<T, bf16>::value && W % 2 == 0;
  using S = typename std::conditional<packed, uint32_t, T>::type;
  static constexpr int N = packed ? W / 2 : W;
  S x[N];
  __device__ __forceinline__ T at(int w) const {
    if constexpr (packed) return bf16{(uint16_t)(x[w / 2] >> (16 * (w & 1)))};
    else return x[w];
  }
};

template <class T, int W>
__device__ __forceinline__ void ldv(Vec<T, W>& d, const T* p) {
  if constexpr (W * sizeof(T) == 16) {
    *reinterpret_cast<u32x4*>(d.x) = ld16(p);
  } else {
    static_assert(!Vec<T, W>::packed, "packed vectors are 16 B");
#pragma unroll
    for (int w = 0; w < W; ++w) d.x[w] = p[w];
  }
}
template <class T, int W>
__device__ __forceinline__ void stv(T* p, const Vec<T, W>& d) {
  if constexpr (W * sizeof(T) == 16) {
    st16(p, *reinterpret_cast<const u32x4*>(d.x));
  } else {
#pragma unroll
    for (int w = 0; w < W; ++w) p[w] = d.x[w];
  }
}

// Write-through (sc1) 16-B stores: the line leaves the XCD's L2 with the
// store instead of staying dirty there until an eviction interleaves its
// write-back with the read streams.  Config-2 fold output only (nobody reads
// it back soon): 8 x 256 MiB f32 SUM 387 -> 380 us on the same box
// (tools/fold_tune.hip, profiles/r02_fold_tune_placement.json; nt stores
// 400 us).  A buffer store with cache bits (aux 16 = sc1), so the compiler
// owns the data-register hazard an inline-asm store would leave open; the
// descriptor is built per block span from wave-uniform values.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t span_rsrc(void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
}
template <class T, int W>
__device__ __forceinline__ void stv_wt(__amdgpu_buffer_rsrc_t r, int byte_off, const Vec<T, W>& d) {
  static_assert(W * sizeof(T) == 16, "16-B vectors only");
  __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(d.x), r, byte_off, 0, 16);
}

// d = OP(a, b) element-wise, a = inout (d may alias a or b)
template <class OP, class T, int W>
__device__ __forceinline__ void vapply(Vec<T, W>& d, const Vec<T, W>& a, const Vec<T, W>& b) {
  using V = Vec<T, W>;
  typename V::S t[V::N];
  if constexpr (V::packed) {
#pragma unroll
    for (int i = 0; i < V::N; ++i) t[i] = bf16x2_apply<OP>(a.x[i], b.x[i]);
  } else {
#pragma unroll
    for (int i = 0; i < V::N; ++i) t[i] = OP::apply(a.x[i], b.x[i]);
  }
#pragma unroll
  for (int i = 0; i < V::N; ++i) d.x[i] = t[i];
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

// The leaves of W consecutive elements, loaded before any arithmetic so a
// thread's loads (and with U > 1 several vectors' loads) are all in flight
// together.  SHAPE (common.hpp): SH_PRE — pre-step partners possible (n not a
// power of two; they exist only for s < rem <= NMAX/2); SH_POW2 — none;
// SH_FULL — none and ntree == NMAX, so no leaf load or tree node carries a
// runtime guard (the 8-buffer headline shape).
template <class T, int NMAX, int SHAPE, int W>
struct Leaves {
  Vec<T, W> v[NMAX];
  Vec<T, W> u[SHAPE == SH_PRE ? NMAX / 2 : 1];
};

template <int NMAX, int SHAPE>
__device__ __forceinline__ int ntree_of(const FoldArgs& A) {
  return SHAPE == SH_FULL ? NMAX : A.ntree;
}

template <class T, int NMAX, int SCHED, int SHAPE, int W>
__device__ __forceinline__ void load_leaves(const FoldArgs& A, const T* const* src, const T* const* src2,
                                            long long e, Leaves<T, NMAX, SHAPE, W>& L) {
  const int nt = ntree_of<NMAX, SHAPE>(A);
#pragma unroll
  for (int s = 0; s < NMAX; ++s)
    if (s < nt) ldv<T, W>(L.v[s], src[s] + e);
  if constexpr (SHAPE == SH_PRE && SCHED == S_TREE) {
#pragma unroll
    for (int s = 0; s < NMAX / 2; ++s)
      if (s < A.rem) ldv<T, W>(L.u[s], src2[s] + e);
  }
}

// Pairwise tree over the leaves with MPICH's operand roles.  At level m the
// node (s, s+m) takes as inout the subtree holding the element's owner
// newrank (Rabenseifner: block j is finished on newrank bitrev(j); binomial:
// the lower subtree, i.e. owner 0).  The owner is the same for all W
// elements (fold_leaves guarantees it) and a compile-time constant here, so
// every node is ONE op with fixed roles — no evaluation of both orders and no
// selects; fold_tree_own dispatches the runtime owner (wave-uniform except at
// the pof2-1 block boundaries) to the NMAX instantiations.
template <class OP, class T, int NMAX, int W, int OWN>
__device__ __forceinline__ void fold_tree(int ntree, Vec<T, W> (&v)[NMAX]) {
  if constexpr (Vec<T, W>::packed && OWN > 0) {
    // every owner instantiation starts by widening the same packed leaves;
    // hoisted above fold_tree_own's dispatch, the widened copies of all
    // leaves stay live at once (twice the VGPRs of the packed ones)
#pragma unroll
    for (int s = 0; s < NMAX; ++s)
#pragma unroll
      for (int i = 0; i < Vec<T, W>::N; ++i) asm volatile("" : "+v"(v[s].x[i]));
  }
#pragma unroll
  for (int m = 1; m < NMAX; m <<= 1) {
#pragma unroll
    for (int s = 0; s + m < NMAX; s += 2 * m) {
      if (s + m < ntree) {
        if ((OWN & m) != 0) vapply<OP, T, W>(v[s], v[s + m], v[s]);
        else vapply<OP, T, W>(v[s], v[s], v[s + m]);
      }
    }
  }
}

// Rabenseifner block of element g: j = min(pof2-1, g / blk_len) from a double
// reciprocal plus a one-step correction (no 64-bit division per vector).
__device__ __forceinline__ unsigned owner_block(const FoldArgs& A, unsigned long long g) {
  const unsigned long long bl = (unsigned long long)A.blk_len;
  unsigned long long j = (unsigned long long)((double)g * A.blk_inv);
  if (j * bl > g) --j;
  else if ((j + 1) * bl <= g) ++j;
  const unsigned long long top = (1ull << A.pof2_log) - 1;
  return (unsigned)(j > top ? top : j);
}

template <class OP, class T, int NMAX, int W, int K>
__device__ __forceinline__ void fold_tree_own(int own, int ntree, Vec<T, W> (&v)[NMAX]) {
  if constexpr (K < NMAX) {
    if (own == K) fold_tree<OP, T, NMAX, W, K>(ntree, v);
    else fold_tree_own<OP, T, NMAX, W, K + 1>(own, ntree, v);
  }
}

// Fold the loaded leaves of the W elements starting at e into res.  Returns
// false, leaving res unset, when the W elements straddle a Rabenseifner block
// boundary with role-sensitive operands (at most pof2-1 vectors per call):
// the caller then folds those elements one at a time (fold_elems), so the
// W-wide code only ever runs with one owner per vector.
template <class OP, class T, int NMAX, int SCHED, int SHAPE, int W>
__device__ __forceinline__ bool fold_leaves(const FoldArgs& A, long long e, Leaves<T, NMAX, SHAPE, W>& L,
                                            Vec<T, W>& res) {
  auto& v = L.v;
  const int nt = ntree_of<NMAX, SHAPE>(A);
  if constexpr (SCHED == S_LINEAR) {
#pragma unroll
    for (int s = 1; s < NMAX; ++s)
      if (s < nt) vapply<OP, T, W>(v[0], v[0], v[s]);
  } else {
    if constexpr (SHAPE == SH_PRE) {
#pragma unroll
      for (int s = 0; s < NMAX / 2; ++s)
        if (s < A.rem) vapply<OP, T, W>(v[s], v[s], L.u[s]);  // inout = even rank 2s (MPICH Reduce pre-step)
    }
    if constexpr (!role_sensitive<OP, T>::v) {
      fold_tree<OP, T, NMAX, W, 0>(nt, v);
    } else {
      if (!A.owner_mode) {
        fold_tree<OP, T, NMAX, W, 0>(nt, v);
      } else {
        const unsigned long long g0 = (unsigned long long)(A.gbase + e);
        const unsigned j0 = owner_block(A, g0);
        const unsigned top = (1u << A.pof2_log) - 1;
        const bool uniform = W == 1 || j0 == top ||
                             g0 + (W - 1) < (unsigned long long)(j0 + 1) * (unsigned long long)A.blk_len;
        if (!uniform) return false;
        fold_tree_own<OP, T, NMAX, W, 0>((int)bitrev(j0, A.pof2_log), nt, v);
      }
    }
  }
  res = v[0];
  return true;
}

template <class OP, class T, int NMAX, int SCHED, int SHAPE, int W>
__device__ __forceinline__ bool fold_at(const FoldArgs& A, const T* const* src, const T* const* src2,
                                        long long e, Vec<T, W>& res) {
  Leaves<T, NMAX, SHAPE, W> L;
  load_leaves<T, NMAX, SCHED, SHAPE, W>(A, src, src2, e, L);
  return fold_leaves<OP, T, NMAX, SCHED, SHAPE, W>(A, e, L, res);
}

// Elements [e, e+k) one at a time into out1 (and out2): the straddling
// vectors of fold_leaves and ragged tails.  Not unrolled: one copy of the
// scalar fold.
template <class OP, class T, int NMAX, int SCHED, int SHAPE>
__device__ __forceinline__ void fold_elems(const FoldArgs& A, const T* const* src, const T* const* src2, long long e,
                                        int k, T* out1, T* out2) {
#pragma unroll 1
  for (int w = 0; w < k; ++w) {
    Vec<T, 1> r;
    fold_at<OP, T, NMAX, SCHED, SHAPE, 1>(A, src, src2, e + w, r);
    out1[e + w] = r.x[0];
    if (out2) out2[e + w] = r.x[0];
  }
}

// Fold [lo, hi) (element indices into the sources) into out1 (and out2 if
// non-null), the whole block cooperating.  lo is a multiple of the vector
// width; `vec` says whether every pointer involved is 16-byte aligned.
template <class OP, class T, int NMAX, int SCHED, int SHAPE, int U>
__device__ __forceinline__ void fold_span(const FoldArgs& A, const T* const* src, const T* const* src2, long long lo,
                                          long long hi, T* out, T* out2);
// U > 1 (block-cooperative callers): the aligned range goes through fold_span
// (U vectors' leaves in flight per thread)
template <class OP, class T, int NMAX, int SCHED, int SHAPE, int U = 1>
__device__ __forceinline__ void fold_range(const FoldArgs& A, const T* const* src, const T* const* src2,
                                           long long lo, long long hi, T* out1, T* out2, bool vec,
                                           long long tid, long long nthr) {
  constexpr int W = VecW<T>::v;
  if constexpr (U > 1) {
    if (vec) {
      fold_span<OP, T, NMAX, SCHED, SHAPE, U>(A, src, src2, lo, hi, out1, out2);
      return;
    }
  }
  if (vec) {
    const long long nv = (hi - lo) / W;
    for (long long i = tid; i < nv; i += nthr) {
      const long long e = lo + i * W;
      Vec<T, W> r;
      if (fold_at<OP, T, NMAX, SCHED, SHAPE, W>(A, src, src2, e, r)) {
        stv<T, W>(out1 + e, r);
        if (out2) stv<T, W>(out2 + e, r);
      } else {
        fold_elems<OP, T, NMAX, SCHED, SHAPE>(A, src, src2, e, W, out1, out2);
      }
    }
    lo += nv * W;
  }
  for (long long e = lo + tid; e < hi; e += nthr) fold_elems<OP, T, NMAX, SCHED, SHAPE>(A, src, src2, e, 1, out1, out2);
}

// A pointer every lane of the wave holds the same value of, read from LDS
// (the kernels stage their argument blocks there): the compiler cannot prove
// it uniform and keeps a 64-bit address per lane per use (and waterfall
// loops around buffer descriptors); readfirstlane puts it in SGPRs.
template <class P>
__device__ __forceinline__ P* wave_uniform(P* p) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  return (P*)(uintptr_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32)) << 32) |
                         (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a));
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

// block_gather with UG 16-B vectors per pair per iteration: UG * m loads in
// flight per thread before any store (ar_zc_kernel / copy_kernel size UG so
// that a thread keeps ~16 loads outstanding at any rank count; with one peer
// the plain block_gather keeps ONE).  The loads carry no guard at all — a
// lane past the end of a shorter pair re-reads that pair's last vector, an
// empty pair re-reads another pair's — and only the stores are guarded: any
// branch between the loads (per-lane range guards, or even a wave-uniform
// "pair p < m" test) made the compiler wait for the outstanding loads at the
// join (vmcnt(0)), one or two loads in flight.  So the pair count is a
// template parameter: block_gather_u dispatches m to block_gather_k<m>.
// Unaligned pairs fall back to block_gather.
template <int K, int UG, int MP>
__device__ __forceinline__ void block_gather_k(char* const (&dst)[MP], const char* const (&src)[MP],
                                               const long long (&len)[MP]) {
  const long long tid = threadIdx.x, nt = blockDim.x;
  long long nvmax = 0;
  int any = -1;
#pragma unroll
  for (int p = 0; p < K; ++p) {
    const long long nv = len[p] / 16;
    nvmax = nv > nvmax ? nv : nvmax;
    if (nv > 0 && any < 0) any = p;
  }
  if (any < 0) return;
  const char* s_any = src[0];
  long long l_any = 0;
#pragma unroll
  for (int p = 0; p < K; ++p)
    if (p == any) {
      s_any = src[p];
      l_any = len[p] / 16 - 1;
    }
  const char* s[K];
  long long last[K];
#pragma unroll
  for (int p = 0; p < K; ++p) {
    const bool own = len[p] >= 16;
    s[p] = own ? src[p] : s_any;
    last[p] = own ? len[p] / 16 - 1 : l_any;
  }
  for (long long i = tid; i < nvmax; i += UG * nt) {
    u32x4 v[K][UG];
#pragma unroll
    for (int p = 0; p < K; ++p)
#pragma unroll
      for (int u = 0; u < UG; ++u) {
        const long long k = i + u * nt;
        v[p][u] = ld16(s[p] + 16 * (k < last[p] ? k : last[p]));
      }
#pragma unroll
    for (int p = 0; p < K; ++p)
#pragma unroll
      for (int u = 0; u < UG; ++u) {
        const long long k = i + u * nt;
        if (k < len[p] / 16) st16(dst[p] + 16 * k, v[p][u]);
      }
  }
}

template <int MP, int UG>
__device__ __forceinline__ void block_gather_u(char* const (&dst)[MP], const char* const (&src)[MP],
                                               const long long (&len)[MP], int m) {
  bool vec = true;
#pragma unroll
  for (int p = 0; p < MP; ++p)
    if (p < m) vec &= ((((uintptr_t)dst[p]) | ((uintptr_t)src[p])) & 15) == 0;
  if (!vec) {
    block_gather<MP>(dst, src, len, m);
    return;
  }
  switch (m) {  // wave-uniform
#define MPIGX_GK(K) \
  case K:           \
    if constexpr (K <= MP) block_gather_k<K, UG, MP>(dst, src, len); \
    break;
    MPIGX_GK(1) MPIGX_GK(2) MPIGX_GK(3) MPIGX_GK(4) MPIGX_GK(5) MPIGX_GK(6) MPIGX_GK(7) MPIGX_GK(8)
    MPIGX_GK(9) MPIGX_GK(10) MPIGX_GK(11) MPIGX_GK(12) MPIGX_GK(13) MPIGX_GK(14) MPIGX_GK(15) MPIGX_GK(16)
#undef MPIGX_GK
    default: break;
  }
  const long long tid = threadIdx.x, nt = blockDim.x;
#pragma unroll
  for (int p = 0; p < MP; ++p)
    if (p < m)
      for (long long j = (len[p] / 16) * 16 + tid; j < len[p]; j += nt) dst[p][j] = src[p][j];
}

// Fold [lo, hi) into out with U vectors per thread per iteration: all
// U * (ntree + rem) leaf loads of a thread are issued before any arithmetic
// (fold_range keeps one vector's leaves in flight).  lo is a multiple of the
// vector width and every pointer is 16-B aligned (the caller checked).
template <class OP, class T, int NMAX, int SCHED, int SHAPE, int U>
__device__ __forceinline__ void fold_span(const FoldArgs& A, const T* const* src, const T* const* src2, long long lo,
                                          long long hi, T* out, T* out2) {
  constexpr int W = VecW<T>::v;
  const long long tid = threadIdx.x, nt = blockDim.x;
  const long long nv = (hi - lo) / W;
  long long v0 = tid;
  for (; v0 + (long long)(U - 1) * nt < nv; v0 += U * nt) {
    Leaves<T, NMAX, SHAPE, W> L[U];
#pragma unroll
    for (int u = 0; u < U; ++u) load_leaves<T, NMAX, SCHED, SHAPE, W>(A, src, src2, lo + (v0 + u * nt) * W, L[u]);
    unsigned strad = 0;  // vectors straddling a Rabenseifner block boundary
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long e = lo + (v0 + u * nt) * W;
      Vec<T, W> r;
      if (fold_leaves<OP, T, NMAX, SCHED, SHAPE, W>(A, e, L[u], r)) {
        stv<T, W>(out + e, r);
        if (out2) stv<T, W>(out2 + e, r);
      } else {
        strad |= 1u << u;
      }
    }
#pragma unroll 1
    for (int u = 0; u < U; ++u)
      if ((strad >> u) & 1u) fold_elems<OP, T, NMAX, SCHED, SHAPE>(A, src, src2, lo + (v0 + u * nt) * W, W, out, out2);
  }
  for (; v0 < nv; v0 += nt) {
    const long long e = lo + v0 * W;
    Vec<T, W> r;
    if (fold_at<OP, T, NMAX, SCHED, SHAPE, W>(A, src, src2, e, r)) {
      stv<T, W>(out + e, r);
      if (out2) stv<T, W>(out2 + e, r);
    } else {
      fold_elems<OP, T, NMAX, SCHED, SHAPE>(A, src, src2, e, W, out, out2);
    }
  }
  for (long long e = lo + nv * W + tid; e < hi; e += nt) fold_elems<OP, T, NMAX, SCHED, SHAPE>(A, src, src2, e, 1, out, out2);
}

// fold_span with every folded vector stored into m outputs (outs[0..m-1]:
// my recvbuf, then the peers' — the pull-push two-shot, kernels.hpp
// ar_zc_kernel AG_PUSH; the root's recvbuf alone for Reduce).  The store
// guards are wave-uniform and follow the loads.
// Each element is read (all its leaves) and then written by ONE thread, so
// in-place buffers (sendbuf == recvbuf on some rank) are safe: no other
// thread of any rank touches that element.  `vec` false (a pointer not 16-B
// aligned): scalar folds throughout.
template <class OP, class T, int NMAX, int SCHED, int SHAPE, int U>
__device__ __forceinline__ void fold_span_scatter(const FoldArgs& A, const T* const* src, const T* const* src2,
                                                  long long lo, long long hi, T* const (&outs)[NMAX], int m,
                                                  bool vec) {
  constexpr int W = VecW<T>::v;
  const long long tid = threadIdx.x, nt = blockDim.x;
  auto put1 = [&](long long e) {  // scalar fold of element e into every output
    Vec<T, 1> r;
    fold_at<OP, T, NMAX, SCHED, SHAPE, 1>(A, src, src2, e, r);
#pragma unroll
    for (int p = 0; p < NMAX; ++p)
      if (p < m) outs[p][e] = r.x[0];
  };
  if (!vec) {
    for (long long e = lo + tid; e < hi; e += nt) put1(e);
    return;
  }
  const long long nv = (hi - lo) / W;
  long long v0 = tid;
  for (; v0 + (long long)(U - 1) * nt < nv; v0 += U * nt) {
    Leaves<T, NMAX, SHAPE, W> L[U];
#pragma unroll
    for (int u = 0; u < U; ++u) load_leaves<T, NMAX, SCHED, SHAPE, W>(A, src, src2, lo + (v0 + u * nt) * W, L[u]);
    unsigned strad = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long e = lo + (v0 + u * nt) * W;
      Vec<T, W> r;
      if (fold_leaves<OP, T, NMAX, SCHED, SHAPE, W>(A, e, L[u], r)) {
#pragma unroll
        for (int p = 0; p < NMAX; ++p)
          if (p < m) stv<T, W>(outs[p] + e, r);
      } else {
        strad |= 1u << u;
      }
    }
#pragma unroll 1
    for (int u = 0; u < U; ++u)
      if ((strad >> u) & 1u)
        for (int w = 0; w < W; ++w) put1(lo + (v0 + u * nt) * W + w);
  }
  for (; v0 < nv; v0 += nt) {
    const long long e = lo + v0 * W;
    Vec<T, W> r;
    if (fold_at<OP, T, NMAX, SCHED, SHAPE, W>(A, src, src2, e, r)) {
#pragma unroll
      for (int p = 0; p < NMAX; ++p)
        if (p < m) stv<T, W>(outs[p] + e, r);
    } else {
      for (int w = 0; w < W; ++w) put1(e + w);
    }
  }
  for (long long e = lo + nv * W + tid; e < hi; e += nt) put1(e);
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
// over xGMI see it), then one lane per peer stores its signal word into that
// peer's slot [block][my rank].  Consumer side: lane p polls my slot
// [block][p] (relaxed, system scope, uncached memory) until it reaches `ep`,
// then a system-scope acquire invalidates this CU's L1 and the stale
// non-coherent L2 lines before any wave reads peer data (MI355X_MICROARCH.md
// "inter-workgroup visibility"; cdna_hip_programming.md Guideline 16, at
// system instead of agent scope because the peers are other GPUs).
//
// Signal word = ep << 25 | abort << 24 | key (24 bits).  Epochs are monotone
// per communicator, so slots never need resetting.  `abort` (optional, the
// block's running flag, identical in every thread) is published and ORed with
// every peer's: once any rank aborts a launch every later barrier of it
// carries the bit, so all ranks of all blocks learn it by the barrier after.
// check_key: a peer whose word for THIS epoch carries another key aborts the
// launch (zero-copy views, mpigx.cpp zc_run: every rank must use the buffer
// mappings agreed in the same exchange).  A peer already past this epoch has
// itself compared our word for it, so a mismatch is never missed.
// Returns false (and sets *err) if a peer did not arrive within the timeout.
// ---------------------------------------------------------------------------
constexpr int kSigShift = 25;
// Error word values (PeerView.err; host: mpigx.cpp finish): a peer did not
// arrive in time (MPI_ERR_OTHER), or the protocol itself was violated — a
// signal word beyond what any peer can have stored yet, a kernel
// precondition that does not hold (MPI_ERR_INTERN).
constexpr unsigned kErrTimeout = 1u, kErrProtocol = 2u;

// Write-back of this XCD's L2 after stores into a PEER's signal array or LL
// area, before the writer spins.  Those arrays are uncached in their owner's
// mapping, but the owner's allocation flags do not carry over to an IPC import
// (the peer's mapping is ordinary device memory), so a flag store can stay a
// dirty line in the writer's L2 for as long as nothing writes that L2 back —
// and a spinning writer issues no more fences.  Seen on the 1-GPU box (ranks
// sharing the device): one rank saw none of its peers' entry words for 20 s
// while every peer had passed the same barrier on its words
// (tools/scan_repro.py, per-block phase stamps).  On distinct GPUs the line
// would wait in the writer GPU's L2 the same way.  A LL sender's kernel
// usually ended (end-of-kernel write-back) soon after its stores, which hid it
// there; the LL two-shot polls between its two pushes.
__device__ __forceinline__ void flush_remote_stores() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, ""); }

// One pause of a poll loop on a flag / LL line.  Only s_sleep: the polled
// words are read with system-scope loads of memory that is uncached in my own
// mapping (or, between ranks of one device, ordinary memory the hardware
// keeps coherent), so no cache maintenance is needed to see a peer's store,
// and the acquire comes once, after the loop.  Round 3 invalidated the L2
// every 16th pause (buffer_inv sc0 sc1: the whole L2 of the XCD); with 8 ranks
// on one GPU, spinning blocks then invalidated every XCD's L2 every few
// hundred cycles while their peers ran ordinary kernels: a 64 Mi-element
// torch compare took 5.7 s instead of milliseconds, a device synchronize
// waited a minute, and the stalls looked like lost signal words (r04k).
__device__ __forceinline__ void spin_pause(unsigned& k) {
  if (k < 64) __builtin_amdgcn_s_sleep(1);  // first ~4 us: tight
  else __builtin_amdgcn_s_sleep(4);
  ++k;
}

// When a poll loop gives up (PeerView.cancel): only when its host stores the
// cancel word — every launch, blocking or stream-ordered, carries it
// (mpigx.cpp make_view): a blocking call's host stores it from finish(), a
// stream-ordered launch's from the process-wide watcher (watch_peers).  The
// word is read once per kCancelPoll of waiting (a PCIe read of a host-pinned
// word), so a late peer is waited for as long as its host says it is coming.
// A zero timeout (a failed host gate) gives up at once; a view without a
// cancel word (none is built today) would fall back to timeout_ticks.
constexpr uint64_t kCancelPoll = 100000;  // 1 ms of the 100 MHz wall clock
__device__ __forceinline__ bool spin_expired(const PeerView& pv, uint64_t t0, uint64_t& next) {
  const uint64_t el = wall_clock64() - t0;
  if (!pv.cancel || pv.timeout_ticks == 0) return el > pv.timeout_ticks;
  if (el < next) return false;
  next = el + kCancelPoll;
  return __hip_atomic_load(pv.cancel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

// Kernel entry of every collective kernel: block 0 tells the host which
// launch its GPU has reached (PeerView.started, one posted PCIe write), then
// the phase stamp.
__device__ __forceinline__ void kernel_started(const PeerView& pv) {
  if (pv.started && blockIdx.x == 0 && threadIdx.x == 0) {
    __hip_atomic_store(pv.started, pv.kseq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  }
}

// Phase timestamp k of this block (mpigx_comm_set_stamps, diagnostic): one
// lane stores the 100 MHz device wall clock; a scalar branch when off.
__device__ __forceinline__ void stamp(const PeerView& pv, int k) {
  if (pv.stamps && threadIdx.x == 0) pv.stamps[(size_t)blockIdx.x * 8 + k] = wall_clock64();
}

// A zero the compiler cannot see through (an `atomicrmw or 0` is folded into
// a plain load otherwise).
__device__ __forceinline__ uint64_t opaque_zero() {
  uint64_t z = 0;
  asm volatile("" : "+v"(z));
  return z;
}
// Signal word into a peer's slot, then written back out of this XCD's L2
// (flush_remote_stores); a poll of my own slot.
__device__ __forceinline__ void sig_put(uint64_t* slot, uint64_t word) {
  __hip_atomic_store(slot, word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  flush_remote_stores();
}
__device__ __forceinline__ uint64_t sig_get(const uint64_t* slot) {
  return __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ bool rank_barrier(const PeerView& pv, uint64_t ep, int* abort = nullptr,
                                             unsigned key = 0, bool check_key = false, bool fences = true,
                                             bool strict = true) {
  __shared__ int s_fail, s_abort;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int ab_in = abort ? *abort : 0;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (fences) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bool ok = true, ab = false, bad = false;
    if (lane < pv.n) {
      const uint64_t word = (ep << kSigShift) | ((uint64_t)(ab_in ? 1 : 0) << 24) | (uint64_t)(key & 0xffffffu);
      uint64_t* peer_slot = pv.sig[lane] + sig_index(blockIdx.x, pv.rank);
      sig_put(peer_slot, word);
      uint64_t* mine = sig_in(pv, lane) + sig_index(blockIdx.x, lane);
      const uint64_t t0 = wall_clock64();
      uint64_t v, next = kCancelPoll;
      unsigned k = 0;
      while (((v = sig_get(mine)) >> kSigShift) < ep) {
        spin_pause(k);
        if (spin_expired(pv, t0, next)) {
          ok = false;
          if (pv.stamps) {  // diagnostic: the epoch awaited and the word last seen from that peer
            pv.stamps[(size_t)blockIdx.x * 8 + 6] = ep;
            pv.stamps[(size_t)blockIdx.x * 8 + 7] = (v >> kSigShift) | ((uint64_t)lane << 56);
            pv.stamps[(size_t)blockIdx.x * 8 + 2] = wall_clock64();  // when this block gave up
            // the same slot read three other ways: RMW, non-temporal, after an acquire
            pv.stamps[(size_t)blockIdx.x * 8 + 3] =
                __hip_atomic_fetch_add(mine, opaque_zero(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >> kSigShift;
            pv.stamps[(size_t)blockIdx.x * 8 + 4] = __builtin_nontemporal_load(mine) >> kSigShift;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            pv.stamps[(size_t)blockIdx.x * 8 + 5] =
                __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >> kSigShift;
          }
          break;
        }
      }
      // A peer can be at most one barrier ahead of me (it cannot pass this
      // one before my word for it arrived): a word beyond ep + 1 means the
      // ranks' epochs diverged — fail loudly instead of passing on it.  Not
      // at the ring's entry (strict = false): a left neighbour runs its ring
      // steps as soon as ITS left one signals, and its step signals share
      // my slot for it (kernels.hpp ring_body).
      if (strict && ok && (v >> kSigShift) > ep + 1) {
        ok = false;
        bad = true;
      }
      ab = ok && (((v >> 24) & 1u) || (check_key && (v >> kSigShift) == ep && (v & 0xffffffu) != (key & 0xffffffu)));
    }
    const bool all_ok = __all(ok);
    const bool any_ab = __any(ab);
    const bool any_bad = __any(bad);
    if (fences) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (lane == 0) {
      s_fail = all_ok ? 0 : 1;
      s_abort = (ab_in || any_ab) ? 1 : 0;
      if (!all_ok)
        __hip_atomic_store(pv.err, any_bad ? kErrProtocol : kErrTimeout, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();
  if (abort) *abort = s_abort;
  return s_fail == 0;
}

// The LAST barrier of a pull-only launch means only "no peer reads my memory
// any more": nothing is published across it (every byte this rank wrote is
// its own, read by no peer after this point, and the next launch's entry
// barrier releases again), so it needs no system-scope release (L2
// write-back) or acquire (L2 invalidate) — only every wave's loads retired
// (s_waitcnt vmcnt(0) + block barrier) before the flag store.  Not for a
// launch whose peers STORE into this rank's memory (push two-shot).
__device__ __forceinline__ bool rank_barrier_exit(const PeerView& pv, uint64_t ep, int* abort = nullptr) {
  return rank_barrier(pv, ep, abort, 0, false, false);
}

// Whole-launch barrier across ranks (the dynamic pull-push two-shot,
// kernels.hpp ar_zc_kernel): every block of this rank counts itself on a
// device counter after a system-scope release of its stores; the block that
// completes the count (`last`) stores the rank's word into row kMaxBlocks of
// every rank's signal array (slot [kMaxBlocks][my rank], after one more
// release), and every block then waits until all n ranks' words reached
// `ep` (acquire).  Counter values are monotone per communicator: base =
// pv.fbase, this launch's blocks take base .. base + grid - 1.  The abort bit
// travels as in rank_barrier (identical in every block of a launch).
__device__ __forceinline__ bool rank_barrier_grid(const PeerView& pv, uint64_t ep, int* abort) {
  __shared__ int s_fail, s_abort, s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int ab_in = *abort;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // this block's stores, peers' memory included
    const unsigned long long prev =
        __hip_atomic_fetch_add(pv.dcount + 2, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == pv.fbase + gridDim.x - 1;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const size_t row = kMaxBlocks;  // the whole-launch row after the per-block ones
    if (s_last) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    bool ok = true, ab = false;
    if (lane < pv.n) {
      if (s_last) {
        const uint64_t word = (ep << kSigShift) | ((uint64_t)(ab_in ? 1 : 0) << 24);
        __hip_atomic_store(pv.sig[lane] + sig_index(row, pv.rank), word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        flush_remote_stores();
      }
      const uint64_t* mine = sig_in(pv, lane) + sig_index(row, lane);
      const uint64_t t0 = wall_clock64();
      uint64_t v, next = kCancelPoll;
      unsigned k = 0;
      while (((v = __hip_atomic_load(mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) >> kSigShift) < ep) {
        spin_pause(k);
        if (spin_expired(pv, t0, next)) {
          ok = false;
          break;
        }
      }
      ab = ok && ((v >> 24) & 1u);
    }
    const bool all_ok = __all(ok);
    const bool any_ab = __any(ab);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (lane == 0) {
      s_fail = all_ok ? 0 : 1;
      s_abort = (ab_in || any_ab) ? 1 : 0;
      if (!all_ok) __hip_atomic_store(pv.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
  __syncthreads();
  *abort = s_abort;
  return s_fail == 0;
}

// Zero-copy launches (mpigx.cpp zc_run): entry barrier with the view key and
// this rank's own verdict (pv.zc_bad: no agreed mapping / a failed import).
// The launch's abort state (identical in every block of every rank) reaches
// the host in the completion word itself (kernels.hpp signal_done): ONE store
// carries both "done" and "aborted", so every rank's host reads the same
// verdict — a separate flag word raced the completion store over PCIe.
//
// Before the barrier (round 5): the argument block must be
// the one the host sealed for THIS launch — its checksum (args_fault) and,
// for blocking launches, its completion base: at entry the device counter
// holds every earlier launch's blocks and at most this launch's own, so a
// stale block (an older launch's arguments) shows.  A zero-copy kernel
// dereferences the peers' mapped buffers straight from this block; round 3
// saw an aperture violation (an address past the legal range, not a missing
// mapping) in the pull-push Scan on 5 of 8 ranks at once.  A block that fails
// touches no pointer of it (the barrier's too): it records kErrProtocol and
// leaves; its host breaks the communicator and says so in the shm block, and
// every peer's host then cancels its own wait (mpigx.cpp finish), so all
// ranks fail the call instead of one rank faulting the GPU.
// Returns 0 when the block is intact, 1 = checksum mismatch, 2 = stale
// (another launch's completion base).  By value, not through an out pointer:
// a pointer to the caller's local would put that local on a stack, i.e. give
// every collective kernel a private segment (tests/test_kernel_resources_cpu.py).
__device__ __noinline__ unsigned args_fault(const PeerView& pv) {
  __shared__ unsigned s_sum, s_why;
  if (threadIdx.x == 0) s_sum = 0;
  __syncthreads();
  const unsigned nw = pv.args_words;
  if (nw) {
    constexpr unsigned kSumWord = (unsigned)(offsetof(PeerView, args_sum) / 4);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&pv);
    unsigned part = 0;
    for (unsigned i = threadIdx.x; i < nw; i += blockDim.x) part += args_mix(i == kSumWord ? 0u : w[i], i);
    atomicAdd(&s_sum, part);  // LDS atomic
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned why = (nw == 0 || s_sum == pv.args_sum) ? 0u : 1u;
    if (!why && pv.done) {
      const unsigned long long c = __hip_atomic_load(pv.dcount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (c < pv.dbase || c >= pv.dbase + gridDim.x) why = 2u;
    }
    s_why = why;
  }
  __syncthreads();
  return s_why;
}

__device__ __forceinline__ bool zc_enter(const PeerView& pv, uint64_t ep, int* abort, bool strict = true) {
  const unsigned why = args_fault(pv);
  if (why) {
    if (threadIdx.x == 0) {
      __hip_atomic_store(pv.err, kErrProtocol, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (pv.stamps) pv.stamps[(size_t)blockIdx.x * 8 + 6] = 0xA765000000000000ull | why;
    }
    *abort = 1;
    return false;
  }
  *abort = pv.zc_bad;
  return rank_barrier(pv, ep, abort, pv.zc_key, true, true, strict);
}

// LL lines of byte messages (common.hpp kLLLine; ll_exchange below):
// message bytes [8i, 8i+8) of `src` (zero-padded past `bytes`)
__device__ __forceinline__ uint64_t ll_pack8(const char* src, long long i, long long bytes) {
  const long long o = 8 * i;
  if ((((uintptr_t)src) & 7) == 0 && o + 8 <= bytes) return *reinterpret_cast<const uint64_t*>(src + o);
  uint64_t d = 0;
  for (int k = 0; k < 8; ++k)
    if (o + k < bytes) d |= (uint64_t)(uint8_t)src[o + k] << (8 * k);
  return d;
}
__device__ __forceinline__ void ll_put(char* area, long long i, uint64_t d, unsigned flag) {
  uint64_t* q = reinterpret_cast<uint64_t*>(area + kLLLine * i);
  const uint64_t fw = (uint64_t)flag << 32;
  __hip_atomic_store(q, (d & 0xffffffffull) | fw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(q + 1, (d >> 32) | fw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// waits for line i of a sender's area to carry `flag`; false when the wait
// gives up (spin_expired; t0 = the start of the caller's wait, `next` its
// deadline for the next cancel-word read, kept across the caller's lines so
// the host-pinned word is read at most once per kCancelPoll, not at the first
// miss of every line once the wait has passed 1 ms)
__device__ __forceinline__ bool ll_get(const PeerView& pv, const char* area, long long i, unsigned flag, uint64_t t0,
                                       uint64_t& next, uint64_t* d) {
  const uint64_t* q = reinterpret_cast<const uint64_t*>(area + kLLLine * i);
  unsigned k = 0;
  for (;;) {
    const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((unsigned)(a >> 32) == flag && (unsigned)(b >> 32) == flag) {
      *d = (a & 0xffffffffull) | (b << 32);
      return true;
    }
    if (spin_expired(pv, t0, next)) return false;
    spin_pause(k);
  }
}
// bytes [8i, 8i+8) ∩ [0, bytes) of dst <- d
__device__ __forceinline__ void ll_store8(char* dst, long long i, long long bytes, uint64_t d) {
  const long long o = 8 * i;
  if ((((uintptr_t)dst) & 7) == 0 && o + 8 <= bytes) {
    *reinterpret_cast<uint64_t*>(dst + o) = d;
    return;
  }
  for (int k = 0; k < 8 && o + k < bytes; ++k) dst[o + k] = (char)(d >> (8 * k));
}

// ---------------------------------------------------------------------------
// LL exchange (M_AR_LL, common.hpp kLLLine) of lines [l0, l1) of a `bytes`-byte
// message, the block cooperating.  Line i carries message bytes [8i, 8i+8).
//   push: my line i -> every peer's area at push[p] + 16 i (two 64-bit
//         system-scope stores into uncached HBM; over xGMI for other GPUs);
//         my own bytes -> my unpack slot r
//   poll: sender q's line i at in + q*stride + 16 i until both halves carry
//         `flag`, payload -> unpack slot q (my arena, ordinary stores)
// Every peer's lines land in MY memory, so the only cross-GPU latency is one
// posted write: no release fence, no signal word, no acquire.  Area reuse:
// the launch alternates parities; a sender can only reach the next launch of
// the same parity after it received my lines of the launch in between, which
// I push only after this launch has finished reading (stream order).
// Returns false (and sets *pv.err) if a sender does not arrive in time.
// ---------------------------------------------------------------------------
__device__ __noinline__ bool ll_exchange(const PeerView& pv, char* const* push, const char* in, long long stride,
                                         unsigned flag, const char* send, long long bytes, long long l0, long long l1,
                                         char* unp, long long ustride, int n, int r, unsigned* err) {
  __shared__ int s_ok;
  const long long tid = threadIdx.x, nt = blockDim.x;
  const bool al8 = (((uintptr_t)send) & 7) == 0;
  const uint64_t fw = (uint64_t)flag << 32;
  if (tid == 0) s_ok = 1;
  for (long long i = l0 + tid; i < l1; i += nt) {
    const long long o = 8 * i;
    uint64_t d = 0;
    if (al8 && o + 8 <= bytes) {
      d = *reinterpret_cast<const uint64_t*>(send + o);
    } else {
      for (int k = 0; k < 8; ++k)
        if (o + k < bytes) d |= (uint64_t)(uint8_t)send[o + k] << (8 * k);
    }
    const uint64_t h0 = (d & 0xffffffffull) | fw, h1 = (d >> 32) | fw;
    for (int p = 0; p < n; ++p) {
      if (p == r) continue;
      uint64_t* q = reinterpret_cast<uint64_t*>(push[p] + kLLLine * i);
      __hip_atomic_store(q, h0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(q + 1, h1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    *reinterpret_cast<uint64_t*>(unp + r * ustride + o) = d;
  }
  flush_remote_stores();
  bool ok = true;
  const uint64_t t0 = wall_clock64();
  uint64_t next = kCancelPoll;  // one cancel-word read per kCancelPoll of waiting (ll_get)
  for (long long i = l0 + tid; i < l1 && ok; i += nt) {
    for (int p = 0; p < n && ok; ++p) {
      if (p == r) continue;
      const uint64_t* q = reinterpret_cast<const uint64_t*>(ll_from(pv, in, p, stride) + kLLLine * i);
      uint64_t a, b;
      unsigned k = 0;
      for (;;) {
        a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if ((unsigned)(a >> 32) == flag && (unsigned)(b >> 32) == flag) break;
        if (spin_expired(pv, t0, next)) {
          ok = false;
          break;
        }
        spin_pause(k);
      }
      if (ok) *reinterpret_cast<uint64_t*>(unp + p * ustride + 8 * i) = (a & 0xffffffffull) | (b << 32);
    }
  }
  __syncthreads();
  if (!ok) {
    s_ok = 0;
    __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();  // the unpacked bytes are visible to the whole block
  return s_ok != 0;
}

}  // namespace mpigx
