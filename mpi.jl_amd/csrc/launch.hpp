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

#define MPIGX_DECL_REP(NAME)                                                                     \
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
hipError_t launch_vx(dim3 grid, hipStream_t s, const VArgs& a);
hipError_t launch_xfer(hipStream_t s, const XferArgs& a);
hipError_t launch_pack(hipStream_t s, const PackArgs& a);

}  // namespace mpigx
