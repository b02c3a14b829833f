// kern_rep.hip — instantiates the fold and scan kernels for ONE element
// representation (compiled once per Rep; see Makefile) and exposes launchers.
// Only the (op, type) pairs MPICH accepts are instantiated (op x type matrix:
// tests/golden/op_type_matrix.json); the host rejects the rest with
// MPI_ERR_OP before launching.
#include "kernels.hpp"
#include "launch.hpp"

#ifndef MPIGX_REP
#error "compile with -DMPIGX_REP=<Rep> -DMPIGX_REP_NAME=<name>"
#endif
#define MPIGX_CAT2(a, b) a##b
#define MPIGX_CAT(a, b) MPIGX_CAT2(a, b)

namespace mpigx {
namespace {
using T = RepType<MPIGX_REP>::T;
constexpr bool kInt = is_int<T>::v;
constexpr bool kCplx = is_cplx<T>::v;

template <class OP>
hipError_t fold_op(int nmax, int sched, dim3 grid, hipStream_t s, const FoldArgs& a) {
  if (a.mode == M_LOCAL) {
    // shape and vectors per thread: fold_shape / local_u (common.hpp), the
    // rule the host sized the grid with
    constexpr int UF = local_u(MPIGX_REP, OP::code, SH_FULL);
    const int shape = fold_shape(sched, nmax, a.ntree, a.rem);
    if (sched == S_LINEAR) {
      if (nmax > 8)
        hipLaunchKernelGGL((fold_local_kernel<OP, T, 16, S_LINEAR, SH_POW2, 1>), grid, dim3(kThreads), 0, s, a);
      else if (shape == SH_FULL)
        hipLaunchKernelGGL((fold_local_kernel<OP, T, 8, S_LINEAR, SH_FULL, UF>), grid, dim3(kThreads), 0, s, a);
      else
        hipLaunchKernelGGL((fold_local_kernel<OP, T, 8, S_LINEAR, SH_POW2, 1>), grid, dim3(kThreads), 0, s, a);
    } else if (nmax <= 8) {
      if (shape == SH_FULL)
        hipLaunchKernelGGL((fold_local_kernel<OP, T, 8, S_TREE, SH_FULL, UF>), grid, dim3(kThreads), 0, s, a);
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
template <class OP>
hipError_t ring_op(dim3 grid, hipStream_t s, const RingArgs& a) {
  hipLaunchKernelGGL((ring_kernel<OP, T>), grid, dim3(kThreads), 0, s, a);
  return hipGetLastError();
}
template <class OP>
hipError_t scan_op(dim3 grid, hipStream_t s, const ScanArgs& a) {
  hipLaunchKernelGGL((scan_kernel<OP, T>), grid, dim3(kThreads), 0, s, a);
  return hipGetLastError();
}
template <class OP>
hipError_t acc_op(dim3 grid, hipStream_t s, const AccArgs& a) {
  hipLaunchKernelGGL((acc_kernel<OP, T>), grid, dim3(kThreads), 0, s, a);
  return hipGetLastError();
}
}  // namespace

hipError_t MPIGX_CAT(launch_fold_, MPIGX_REP_NAME)(int op, int nmax, int sched, dim3 grid, hipStream_t s,
                                                  const FoldArgs& a) {
  switch (op) {
    case O_SUM: return fold_op<OpSum>(nmax, sched, grid, s, a);
    case O_PROD: return fold_op<OpProd>(nmax, sched, grid, s, a);
    default: break;
  }
  if constexpr (!kCplx) {
    switch (op) {
      case O_MIN: return fold_op<OpMin>(nmax, sched, grid, s, a);
      case O_MAX: return fold_op<OpMax>(nmax, sched, grid, s, a);
      case O_LAND: return fold_op<OpLand>(nmax, sched, grid, s, a);
      case O_LOR: return fold_op<OpLor>(nmax, sched, grid, s, a);
      case O_LXOR: return fold_op<OpLxor>(nmax, sched, grid, s, a);
      default: break;
    }
  }
  if constexpr (kInt) {
    switch (op) {
      case O_BAND: return fold_op<OpBand>(nmax, sched, grid, s, a);
      case O_BOR: return fold_op<OpBor>(nmax, sched, grid, s, a);
      case O_BXOR: return fold_op<OpBxor>(nmax, sched, grid, s, a);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}

hipError_t MPIGX_CAT(launch_ring_, MPIGX_REP_NAME)(int op, dim3 grid, hipStream_t s, const RingArgs& a) {
  switch (op) {
    case O_SUM: return ring_op<OpSum>(grid, s, a);
    case O_PROD: return ring_op<OpProd>(grid, s, a);
    default: break;
  }
  if constexpr (!kCplx) {
    switch (op) {
      case O_MIN: return ring_op<OpMin>(grid, s, a);
      case O_MAX: return ring_op<OpMax>(grid, s, a);
      case O_LAND: return ring_op<OpLand>(grid, s, a);
      case O_LOR: return ring_op<OpLor>(grid, s, a);
      case O_LXOR: return ring_op<OpLxor>(grid, s, a);
      default: break;
    }
  }
  if constexpr (kInt) {
    switch (op) {
      case O_BAND: return ring_op<OpBand>(grid, s, a);
      case O_BOR: return ring_op<OpBor>(grid, s, a);
      case O_BXOR: return ring_op<OpBxor>(grid, s, a);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}

hipError_t MPIGX_CAT(launch_scan_, MPIGX_REP_NAME)(int op, dim3 grid, hipStream_t s, const ScanArgs& a) {
  switch (op) {
    case O_SUM: return scan_op<OpSum>(grid, s, a);
    case O_PROD: return scan_op<OpProd>(grid, s, a);
    default: break;
  }
  if constexpr (!kCplx) {
    switch (op) {
      case O_MIN: return scan_op<OpMin>(grid, s, a);
      case O_MAX: return scan_op<OpMax>(grid, s, a);
      case O_LAND: return scan_op<OpLand>(grid, s, a);
      case O_LOR: return scan_op<OpLor>(grid, s, a);
      case O_LXOR: return scan_op<OpLxor>(grid, s, a);
      default: break;
    }
  }
  if constexpr (kInt) {
    switch (op) {
      case O_BAND: return scan_op<OpBand>(grid, s, a);
      case O_BOR: return scan_op<OpBor>(grid, s, a);
      case O_BXOR: return scan_op<OpBxor>(grid, s, a);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}

// RMA accumulate: the collective op set plus REPLACE / NO_OP (any type).
hipError_t MPIGX_CAT(launch_acc_, MPIGX_REP_NAME)(int op, dim3 grid, hipStream_t s, const AccArgs& a) {
  switch (op) {
    case O_REPLACE: return acc_op<OpReplace>(grid, s, a);
    case O_NOOP: return acc_op<OpNoop>(grid, s, a);
    case O_SUM: return acc_op<OpSum>(grid, s, a);
    case O_PROD: return acc_op<OpProd>(grid, s, a);
    default: break;
  }
  if constexpr (!kCplx) {
    switch (op) {
      case O_MIN: return acc_op<OpMin>(grid, s, a);
      case O_MAX: return acc_op<OpMax>(grid, s, a);
      case O_LAND: return acc_op<OpLand>(grid, s, a);
      case O_LOR: return acc_op<OpLor>(grid, s, a);
      case O_LXOR: return acc_op<OpLxor>(grid, s, a);
      default: break;
    }
  }
  if constexpr (kInt) {
    switch (op) {
      case O_BAND: return acc_op<OpBand>(grid, s, a);
      case O_BOR: return acc_op<OpBor>(grid, s, a);
      case O_BXOR: return acc_op<OpBxor>(grid, s, a);
      default: break;
    }
  }
  return hipErrorInvalidValue;
}

}  // namespace mpigx
