// launch.hpp — host-side entry points into the per-representation kernel
// translation units (kern_rep.hip is compiled once per Rep with
// -DMPIGX_REP=<Rep> -DMPIGX_REP_NAME=<name>).
#pragma once
#include <hip/hip_runtime.h>

#include "common.hpp"

namespace mpigx {

using FoldLauncher = hipError_t (*)(int op, int nmax, int sched, dim3 grid, hipStream_t s, const FoldArgs& a);
using AccLauncher = hipError_t (*)(int op, dim3 grid, hipStream_t s, const AccArgs& a);
using ScanLauncher = hipError_t (*)(int op, dim3 grid, hipStream_t s, const ScanArgs& a);
using RingLauncher = hipError_t (*)(int op, dim3 grid, hipStream_t s, const RingArgs& a);

// ag: AG_PULL 0 / AG_PUSH 1 (kernels.hpp ar_zc_kernel)
using ArzcLauncher = hipError_t (*)(int op, int nmax, int shape, int ag, dim3 grid, hipStream_t s, const FoldArgs& a);
// resident blocks per CU of one spinning kernel: (op, kind 0 fold / 1 ar_zc /
// 2 ring / 3 scan / 4 ar_zc AG_PUSH, a, b) — kern_rep.hip occ_op
using OccQuery = int (*)(int op, int kind, int a, int b);

// ar_zc_kernel (kernels.hpp) instantiation for a communicator of n <= 8
// ranks and the planned fold (ntree leaves, rem pre-step pairs): NMAX = n
// rounded up to a power of two, SH_FULL when all NMAX leaves are present
// without a pre-step.  Returns false when the kernel does not apply (n > 8).
inline bool arzc_shape(int n, int ntree, int rem, int* nmax, int* shape) {
  if (n < 2 || n > 8) return false;
  *nmax = n <= 2 ? 2 : n <= 4 ? 4 : 8;
  *shape = (rem == 0 && ntree == *nmax) ? SH_FULL : SH_PRE;
  return true;
}

#define MPIGX_DECL_REP(NAME)                                                                     \
  hipError_t launch_arzc_##NAME(int op, int nmax, int shape, int ag, dim3 grid, hipStream_t s, const FoldArgs& a); \
  int occupancy_##NAME(int op, int kind, int a, int b); \
  hipError_t launch_fold_##NAME(int op, int nmax, int sched, dim3 grid, hipStream_t s, const FoldArgs& a); \
  hipError_t launch_scan_##NAME(int op, dim3 grid, hipStream_t s, const ScanArgs& a); \
  hipError_t launch_ring_##NAME(int op, dim3 grid, hipStream_t s, const RingArgs& a); \
  hipError_t launch_acc_##NAME(int op, dim3 grid, hipStream_t s, const AccArgs& a);
MPIGX_DECL_REP(i8) MPIGX_DECL_REP(u8) MPIGX_DECL_REP(i16) MPIGX_DECL_REP(u16)
MPIGX_DECL_REP(i32) MPIGX_DECL_REP(u32) MPIGX_DECL_REP(i64) MPIGX_DECL_REP(u64)
MPIGX_DECL_REP(f32) MPIGX_DECL_REP(f64) MPIGX_DECL_REP(c64) MPIGX_DECL_REP(c128)
MPIGX_DECL_REP(bf16)
#undef MPIGX_DECL_REP

hipError_t launch_copy(dim3 grid, hipStream_t s, const CopyArgs& a);
int occupancy_copy(int n);  // copy_kernel of an n-rank communicator
int occupancy_vx(int n);    // vx_kernel likewise
hipError_t launch_vx(dim3 grid, hipStream_t s, const VArgs& a);
hipError_t launch_xfer(hipStream_t s, const XferArgs& a);
hipError_t launch_pack(hipStream_t s, const PackArgs& a);
// read-only stream of nin (1, 2, 4, 8) buffers of `bytes` each (copy.hip; the
// per-box ceiling of config 2)
hipError_t launch_read_probe(const void* const* in, int nin, long long bytes, void* sink, hipStream_t s);
hipError_t launch_mix_probe(const void* const* in, int nin, long long bytes, void* out, hipStream_t s);

}  // namespace mpigx
