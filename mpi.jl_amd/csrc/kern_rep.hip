// kern_rep.hip — instantiates the fold / ring / scan / accumulate kernels of
// ONE element representation and exposes launchers.  Compiled once per
// (Rep, part) (see Makefile):
//   -DMPIGX_REP=<Rep> -DMPIGX_REP_NAME=<name> -DMPIGX_PART=<0..6>
// Parts 0-5 each instantiate the kernels of a few ops (the role-sensitive
// MIN / MAX trees of the packed bf16 type alone take minutes to compile, so
// one translation unit per rep serialised the build); part 6 holds MPI_REPLACE
// / MPI_NO_OP (accumulate only) and the per-rep dispatchers launch.hpp
// declares, which call the other parts through per-op entry points.
// Only the (op, type) pairs MPICH accepts are instantiated (op x type matrix:
// tests/golden/op_type_matrix.json); the host rejects the rest with
// MPI_ERR_OP before launching.
#include "kernels.hpp"
#include "launch.hpp"

#ifndef MPIGX_REP
#error "compile with -DMPIGX_REP=<Rep> -DMPIGX_REP_NAME=<name> -DMPIGX_PART=<part>"
#endif
#ifndef MPIGX_PART
#error "compile with -DMPIGX_PART=<0..6>"
#endif
#define MPIGX_CAT2(a, b) a##b
#define MPIGX_CAT(a, b) MPIGX_CAT2(a, b)
#define MPIGX_CAT4(a, b, c, d) MPIGX_CAT(MPIGX_CAT(a, b), MPIGX_CAT(c, d))

// per-op entry points of this rep: launch_<kind>_<name>_o<op code>
#define MPIGX_FOLD_FN(K) MPIGX_CAT4(launch_fold_, MPIGX_REP_NAME, _o, K)
#define MPIGX_RING_FN(K) MPIGX_CAT4(launch_ring_, MPIGX_REP_NAME, _o, K)
#define MPIGX_SCAN_FN(K) MPIGX_CAT4(launch_scan_, MPIGX_REP_NAME, _o, K)
#define MPIGX_ACC_FN(K) MPIGX_CAT4(launch_acc_, MPIGX_REP_NAME, _o, K)

namespace mpigx {
namespace {
using T = RepType<MPIGX_REP>::T;
constexpr bool kInt = is_int<T>::v;
constexpr bool kCplx = is_cplx<T>::v;

// the op x type matrix (collectives); accumulate adds REPLACE / NO_OP
constexpr bool valid_op(int op) {
  return op == O_SUM || op == O_PROD || (!kCplx && op >= O_MIN && op <= O_LXOR) ||
         (kInt && op >= O_BAND && op <= O_BXOR);
}

template <int K> struct OpOf;
template <> struct OpOf<O_SUM> { using type = OpSum; };
template <> struct OpOf<O_PROD> { using type = OpProd; };
template <> struct OpOf<O_MIN> { using type = OpMin; };
template <> struct OpOf<O_MAX> { using type = OpMax; };
template <> struct OpOf<O_LAND> { using type = OpLand; };
template <> struct OpOf<O_LOR> { using type = OpLor; };
template <> struct OpOf<O_LXOR> { using type = OpLxor; };
template <> struct OpOf<O_BAND> { using type = OpBand; };
template <> struct OpOf<O_BOR> { using type = OpBor; };
template <> struct OpOf<O_BXOR> { using type = OpBxor; };
template <> struct OpOf<O_REPLACE> { using type = OpReplace; };
template <> struct OpOf<O_NOOP> { using type = OpNoop; };

// SH_FULL local fold at the U the host chose (local_u: UF at large sizes,
// halved for small inputs)
template <class OP, int SCHED, int UF>
void local_full(int lu, dim3 grid, hipStream_t s, const FoldArgs& a) {
  if constexpr (UF >= 4) {
    if (lu >= 4) {
      hipLaunchKernelGGL((fold_local_kernel<OP, T, 8, SCHED, SH_FULL, 4>), grid, dim3(kThreads), 0, s, a);
      return;
    }
    if (lu == 2) {
      hipLaunchKernelGGL((fold_local_kernel<OP, T, 8, SCHED, SH_FULL, 2>), grid, dim3(kThreads), 0, s, a);
      return;
    }
  }
  hipLaunchKernelGGL((fold_local_kernel<OP, T, 8, SCHED, SH_FULL, 1>), grid, dim3(kThreads), 0, s, a);
}

template <class OP>
hipError_t fold_op(int nmax, int sched, dim3 grid, hipStream_t s, const FoldArgs& a) {
  if (a.mode == M_LOCAL) {
    // shape and vectors per thread: fold_shape / local_u (common.hpp), the
    // rule the host sized the grid with (a.lu); the kernel is correct for any
    // grid, U only sets how much of the range one pass covers
    constexpr int UF = local_u_max(MPIGX_REP, OP::code, SH_FULL);
    const int shape = fold_shape(sched, nmax, a.ntree, a.rem);
    if (sched == S_LINEAR) {
      if (nmax > 8)
        hipLaunchKernelGGL((fold_local_kernel<OP, T, 16, S_LINEAR, SH_POW2, 1>), grid, dim3(kThreads), 0, s, a);
      else if (shape == SH_FULL)
        local_full<OP, S_LINEAR, UF>(a.lu, grid, s, a);
      else
        hipLaunchKernelGGL((fold_local_kernel<OP, T, 8, S_LINEAR, SH_POW2, 1>), grid, dim3(kThreads), 0, s, a);
    } else if (nmax <= 8) {
      if (shape == SH_FULL)
        local_full<OP, S_TREE, UF>(a.lu, grid, s, a);
      else if (shape == SH_POW2)
        hipLaunchKernelGGL((fold_local_kernel<OP, T, 8, S_TREE, SH_POW2, 1>), grid, dim3(kThreads), 0, s, a);
      else
        hipLaunchKernelGGL((fold_local_kernel<OP, T, 8, S_TREE, SH_PRE, 1>), grid, dim3(kThreads), 0, s, a);
    } else {
      if (shape == SH_PRE)
        hipLaunchKernelGGL((fold_local_kernel<OP, T, 16, S_TREE, SH_PRE, 1>), grid, dim3(kThreads), 0, s, a);
      else
        hipLaunchKernelGGL((fold_local_kernel<OP, T, 16, S_TREE, SH_POW2, 1>), grid, dim3(kThreads), 0, s, a);
    }
  } else if (sched == S_LINEAR && nmax <= 8) {
    hipLaunchKernelGGL((fold_kernel<OP, T, 8, S_LINEAR>), grid, dim3(kThreads), 0, s, a);
  } else if (sched == S_LINEAR) {
    hipLaunchKernelGGL((fold_kernel<OP, T, 16, S_LINEAR>), grid, dim3(kThreads), 0, s, a);
  } else if (nmax <= 8) {
    hipLaunchKernelGGL((fold_kernel<OP, T, 8, S_TREE>), grid, dim3(kThreads), 0, s, a);
  } else {
    hipLaunchKernelGGL((fold_kernel<OP, T, 16, S_TREE>), grid, dim3(kThreads), 0, s, a);
  }
  return hipGetLastError();
}

// ar_zc_kernel instantiations (kernels.hpp): NMAX = n rounded up to a power
// of two, U = 16 / NMAX vectors per thread scaled by the registers one vector
// takes (zc_u, kernels.hpp: 8- and 16-bit elements hold one element per
// VGPR); SH_FULL when every one of the NMAX leaves is present with no
// pre-step, else SH_PRE.  nmax/shape come from arzc_shape (launch.hpp).
template <class OP, int AG>
hipError_t arzc_ag(int nmax, int shape, dim3 grid, hipStream_t s, const FoldArgs& a) {
  if (nmax == 2)
    hipLaunchKernelGGL((ar_zc_kernel<OP, T, 2, SH_FULL, zc_u<T>(8), AG>), grid, dim3(kThreads), 0, s, a);
  else if (nmax == 4 && shape == SH_FULL)
    hipLaunchKernelGGL((ar_zc_kernel<OP, T, 4, SH_FULL, zc_u<T>(4), AG>), grid, dim3(kThreads), 0, s, a);
  else if (nmax == 4)
    hipLaunchKernelGGL((ar_zc_kernel<OP, T, 4, SH_PRE, zc_u<T>(4), AG>), grid, dim3(kThreads), 0, s, a);
  else if (shape == SH_FULL)
    hipLaunchKernelGGL((ar_zc_kernel<OP, T, 8, SH_FULL, zc_u<T>(2), AG>), grid, dim3(kThreads), 0, s, a);
  else
    hipLaunchKernelGGL((ar_zc_kernel<OP, T, 8, SH_PRE, zc_u<T>(2), AG>), grid, dim3(kThreads), 0, s, a);
  return hipGetLastError();
}
// ag: AG_PULL (pull two-shot) or AG_PUSH (pull reduce-scatter + push allgather)
template <class OP>
hipError_t arzc_op(int nmax, int shape, int ag, dim3 grid, hipStream_t s, const FoldArgs& a) {
  return ag == AG_PUSH ? arzc_ag<OP, AG_PUSH>(nmax, shape, grid, s, a) : arzc_ag<OP, AG_PULL>(nmax, shape, grid, s, a);
}

// Resident 256-thread blocks per CU of ONE kernel that spins on its peers
// (the host caps that launch's grid with it, mpigx.cpp kernel_cap).
//   kind 0 fold_kernel (a = nmax, b = sched), 1 ar_zc_kernel (a = nmax,
//   b = shape), 2 ring_kernel, 3 scan_kernel, 4 ar_zc_kernel AG_PUSH
template <class K>
int occ1(K k) {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, kThreads, 0) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return nb;
}
template <class OP, int AG>
int occ_arzc(int a, int b) {
  if (a == 2) return occ1(ar_zc_kernel<OP, T, 2, SH_FULL, zc_u<T>(8), AG>);
  if (a == 4) return b == SH_FULL ? occ1(ar_zc_kernel<OP, T, 4, SH_FULL, zc_u<T>(4), AG>)
                                  : occ1(ar_zc_kernel<OP, T, 4, SH_PRE, zc_u<T>(4), AG>);
  return b == SH_FULL ? occ1(ar_zc_kernel<OP, T, 8, SH_FULL, zc_u<T>(2), AG>)
                      : occ1(ar_zc_kernel<OP, T, 8, SH_PRE, zc_u<T>(2), AG>);
}
template <class OP>
int occ_op(int kind, int a, int b) {
  switch (kind) {
    case 0:
      if (a <= 8) return b == S_LINEAR ? occ1(fold_kernel<OP, T, 8, S_LINEAR>) : occ1(fold_kernel<OP, T, 8, S_TREE>);
      return b == S_LINEAR ? occ1(fold_kernel<OP, T, 16, S_LINEAR>) : occ1(fold_kernel<OP, T, 16, S_TREE>);
    case 1: return occ_arzc<OP, AG_PULL>(a, b);
    case 4: return occ_arzc<OP, AG_PUSH>(a, b);
    case 2: return occ1(ring_kernel<OP, T>);
    default: return occ1(scan_kernel<OP, T>);
  }
}
}  // namespace

// Per-op entry points: declared for every op code here (the dispatchers of
// part 6 reference only the valid ones), defined by the part that owns the op.
#define MPIGX_ARZC_FN(K) MPIGX_CAT4(launch_arzc_, MPIGX_REP_NAME, _o, K)
#define MPIGX_OCC_FN(K) MPIGX_CAT4(occupancy_, MPIGX_REP_NAME, _o, K)
#define MPIGX_DECL_OP(K)                                                                               \
  hipError_t MPIGX_ARZC_FN(K)(int nmax, int shape, int ag, dim3 grid, hipStream_t s, const FoldArgs& a);      \
  int MPIGX_OCC_FN(K)(int kind, int a, int b);                                                         \
  hipError_t MPIGX_FOLD_FN(K)(int nmax, int sched, dim3 grid, hipStream_t s, const FoldArgs& a);      \
  hipError_t MPIGX_RING_FN(K)(dim3 grid, hipStream_t s, const RingArgs& a);                            \
  hipError_t MPIGX_SCAN_FN(K)(dim3 grid, hipStream_t s, const ScanArgs& a);                            \
  hipError_t MPIGX_ACC_FN(K)(dim3 grid, hipStream_t s, const AccArgs& a);
MPIGX_DECL_OP(0) MPIGX_DECL_OP(1) MPIGX_DECL_OP(2) MPIGX_DECL_OP(3) MPIGX_DECL_OP(4) MPIGX_DECL_OP(5)
MPIGX_DECL_OP(6) MPIGX_DECL_OP(7) MPIGX_DECL_OP(8) MPIGX_DECL_OP(9) MPIGX_DECL_OP(16) MPIGX_DECL_OP(17)
#undef MPIGX_DECL_OP

// Definitions for op code K (a collective op: all four kernel families).
#define MPIGX_DEF_OP(K)                                                                                \
  hipError_t MPIGX_FOLD_FN(K)(int nmax, int sched, dim3 grid, hipStream_t s, const FoldArgs& a) {     \
    if constexpr (valid_op(K)) return fold_op<OpOf<K>::type>(nmax, sched, grid, s, a);                 \
    return hipErrorInvalidValue;                                                                       \
  }                                                                                                    \
  hipError_t MPIGX_ARZC_FN(K)(int nmax, int shape, int ag, dim3 grid, hipStream_t s, const FoldArgs& a) { \
    if constexpr (valid_op(K)) return arzc_op<OpOf<K>::type>(nmax, shape, ag, grid, s, a);             \
    return hipErrorInvalidValue;                                                                       \
  }                                                                                                    \
  int MPIGX_OCC_FN(K)(int kind, int a, int b) {                                                        \
    if constexpr (valid_op(K)) return occ_op<OpOf<K>::type>(kind, a, b);                               \
    return 0;                                                                                          \
  }                                                                                                    \
  hipError_t MPIGX_RING_FN(K)(dim3 grid, hipStream_t s, const RingArgs& a) {                           \
    if constexpr (valid_op(K)) {                                                                       \
      hipLaunchKernelGGL((ring_kernel<OpOf<K>::type, T>), grid, dim3(kThreads), 0, s, a);              \
      return hipGetLastError();                                                                        \
    }                                                                                                  \
    return hipErrorInvalidValue;                                                                       \
  }                                                                                                    \
  hipError_t MPIGX_SCAN_FN(K)(dim3 grid, hipStream_t s, const ScanArgs& a) {                           \
    if constexpr (valid_op(K)) {                                                                       \
      hipLaunchKernelGGL((scan_kernel<OpOf<K>::type, T>), grid, dim3(kThreads), 0, s, a);              \
      return hipGetLastError();                                                                        \
    }                                                                                                  \
    return hipErrorInvalidValue;                                                                       \
  }                                                                                                    \
  hipError_t MPIGX_ACC_FN(K)(dim3 grid, hipStream_t s, const AccArgs& a) {                             \
    if constexpr (valid_op(K)) {                                                                       \
      hipLaunchKernelGGL((acc_kernel<OpOf<K>::type, T>), grid, dim3(kThreads), 0, s, a);               \
      return hipGetLastError();                                                                        \
    }                                                                                                  \
    return hipErrorInvalidValue;                                                                       \
  }

#if MPIGX_PART == 0
MPIGX_DEF_OP(0)
#elif MPIGX_PART == 1
MPIGX_DEF_OP(1)
#elif MPIGX_PART == 2
MPIGX_DEF_OP(2)
#elif MPIGX_PART == 3
MPIGX_DEF_OP(3)
#elif MPIGX_PART == 4
MPIGX_DEF_OP(4) MPIGX_DEF_OP(5) MPIGX_DEF_OP(6)
#elif MPIGX_PART == 5
MPIGX_DEF_OP(7) MPIGX_DEF_OP(8) MPIGX_DEF_OP(9)
#elif MPIGX_PART == 6
// RMA-only ops: accumulate kernels, any type
hipError_t MPIGX_ACC_FN(16)(dim3 grid, hipStream_t s, const AccArgs& a) {
  hipLaunchKernelGGL((acc_kernel<OpReplace, T>), grid, dim3(kThreads), 0, s, a);
  return hipGetLastError();
}
hipError_t MPIGX_ACC_FN(17)(dim3 grid, hipStream_t s, const AccArgs& a) {
  hipLaunchKernelGGL((acc_kernel<OpNoop, T>), grid, dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

// The per-rep dispatchers (launch.hpp).  Each valid op goes to its part's
// entry point; invalid pairs never get here (host validation) and would
// return hipErrorInvalidValue.
#define MPIGX_SWITCH(FN, ...)                                        \
  switch (op) {                                                      \
    case O_SUM: return FN(0)(__VA_ARGS__);                           \
    case O_PROD: return FN(1)(__VA_ARGS__);                          \
    default: break;                                                  \
  }                                                                  \
  if constexpr (!kCplx) {                                            \
    switch (op) {                                                    \
      case O_MIN: return FN(2)(__VA_ARGS__);                         \
      case O_MAX: return FN(3)(__VA_ARGS__);                         \
      case O_LAND: return FN(4)(__VA_ARGS__);                        \
      case O_LOR: return FN(5)(__VA_ARGS__);                         \
      case O_LXOR: return FN(6)(__VA_ARGS__);                        \
      default: break;                                                \
    }                                                                \
  }                                                                  \
  if constexpr (kInt) {                                              \
    switch (op) {                                                    \
      case O_BAND: return FN(7)(__VA_ARGS__);                        \
      case O_BOR: return FN(8)(__VA_ARGS__);                         \
      case O_BXOR: return FN(9)(__VA_ARGS__);                        \
      default: break;                                                \
    }                                                                \
  }                                                                  \
  return hipErrorInvalidValue;

hipError_t MPIGX_CAT(launch_fold_, MPIGX_REP_NAME)(int op, int nmax, int sched, dim3 grid, hipStream_t s,
                                                  const FoldArgs& a) {
  MPIGX_SWITCH(MPIGX_FOLD_FN, nmax, sched, grid, s, a)
}
hipError_t MPIGX_CAT(launch_arzc_, MPIGX_REP_NAME)(int op, int nmax, int shape, int ag, dim3 grid, hipStream_t s,
                                                  const FoldArgs& a) {
  MPIGX_SWITCH(MPIGX_ARZC_FN, nmax, shape, ag, grid, s, a)
}
int MPIGX_CAT(occupancy_, MPIGX_REP_NAME)(int op, int kind, int a, int b) {
  switch (op) {
    case O_SUM: return MPIGX_OCC_FN(0)(kind, a, b);
    case O_PROD: return MPIGX_OCC_FN(1)(kind, a, b);
    case O_MIN: return MPIGX_OCC_FN(2)(kind, a, b);
    case O_MAX: return MPIGX_OCC_FN(3)(kind, a, b);
    case O_LAND: return MPIGX_OCC_FN(4)(kind, a, b);
    case O_LOR: return MPIGX_OCC_FN(5)(kind, a, b);
    case O_LXOR: return MPIGX_OCC_FN(6)(kind, a, b);
    case O_BAND: return MPIGX_OCC_FN(7)(kind, a, b);
    case O_BOR: return MPIGX_OCC_FN(8)(kind, a, b);
    case O_BXOR: return MPIGX_OCC_FN(9)(kind, a, b);
    default: return 0;
  }
}
hipError_t MPIGX_CAT(launch_ring_, MPIGX_REP_NAME)(int op, dim3 grid, hipStream_t s, const RingArgs& a) {
  MPIGX_SWITCH(MPIGX_RING_FN, grid, s, a)
}
hipError_t MPIGX_CAT(launch_scan_, MPIGX_REP_NAME)(int op, dim3 grid, hipStream_t s, const ScanArgs& a) {
  MPIGX_SWITCH(MPIGX_SCAN_FN, grid, s, a)
}
// RMA accumulate: the collective op set plus REPLACE / NO_OP (any type).
hipError_t MPIGX_CAT(launch_acc_, MPIGX_REP_NAME)(int op, dim3 grid, hipStream_t s, const AccArgs& a) {
  if (op == O_REPLACE) return MPIGX_ACC_FN(16)(grid, s, a);
  if (op == O_NOOP) return MPIGX_ACC_FN(17)(grid, s, a);
  MPIGX_SWITCH(MPIGX_ACC_FN, grid, s, a)
}
#undef MPIGX_SWITCH
#else
#error "MPIGX_PART must be 0..6"
#endif

}  // namespace mpigx
