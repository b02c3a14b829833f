// kern_stub.cpp — development builds only (Makefile `dev` target): the
// launchers of one element representation with no kernels behind them; every
// launch fails with hipErrorInvalidValue (-> MPI_ERR_INTERN) and occupancy
// queries return 0.  Lets a protocol change be tried on the types a test uses
// without the full 91-object kernel build.  Never part of lib/libmpigx.so.
#include "launch.hpp"

#ifndef MPIGX_REP_NAME
#error "compile with -DMPIGX_REP_NAME=<name>"
#endif
#define MPIGX_CAT2(a, b) a##b
#define MPIGX_CAT(a, b) MPIGX_CAT2(a, b)

namespace mpigx {
hipError_t MPIGX_CAT(launch_arzc_, MPIGX_REP_NAME)(int, int, int, int, dim3, hipStream_t, const FoldArgs&) {
  return hipErrorInvalidValue;
}
int MPIGX_CAT(occupancy_, MPIGX_REP_NAME)(int, int, int, int) { return 0; }
hipError_t MPIGX_CAT(launch_fold_, MPIGX_REP_NAME)(int, int, int, dim3, hipStream_t, const FoldArgs&) {
  return hipErrorInvalidValue;
}
hipError_t MPIGX_CAT(launch_scan_, MPIGX_REP_NAME)(int, dim3, hipStream_t, const ScanArgs&) {
  return hipErrorInvalidValue;
}
hipError_t MPIGX_CAT(launch_ring_, MPIGX_REP_NAME)(int, dim3, hipStream_t, const RingArgs&) {
  return hipErrorInvalidValue;
}
hipError_t MPIGX_CAT(launch_acc_, MPIGX_REP_NAME)(int, dim3, hipStream_t, const AccArgs&) {
  return hipErrorInvalidValue;
}
}  // namespace mpigx
