// copy.hip — Bcast! / Allgather! / Alltoall! / Barrier (src/collective.jl:15-42,
// 295-335, 489-532): byte movement through the staging arenas, block b of
// every rank owning the same byte slice, peers pulled over xGMI.
#include "kernels.hpp"
#include "launch.hpp"

namespace mpigx {

__global__ __launch_bounds__(kThreads) void copy_kernel(CopyArgs A) {
  const PeerView& pv = A.pv;
  const int b = blockIdx.x, r = pv.rank, n = pv.n;
  uint64_t ep = pv.epoch;
  if (A.mode == C_BARRIER) {
    rank_barrier(pv, ep);
    return;
  }
  if (A.mode == C_PROBE_ALL || A.mode == C_PROBE_ONE) {
    // xGMI probe: pull A.bytes from every peer's staging (PROBE_ALL: all
    // links at once = aggregate ingress) or from rank r+1 only (one link);
    // loads are folded into a register so they stay live.
    if (!rank_barrier(pv, ep++)) return;
    const long long lo = lmin((long long)b * A.slice, A.bytes), hi = lmin(lo + A.slice, A.bytes);
    u32x4 acc = {0, 0, 0, 0};
    for (int k = 1; k < n; ++k) {
      if (A.mode == C_PROBE_ONE && k > 1) break;
      const u32x4* s = reinterpret_cast<const u32x4*>(pv.stage[(r + k) % n] + lo);
      const long long nv = (hi - lo) / 16;
      long long i = threadIdx.x;
      for (; i + 3 * (long long)blockDim.x < nv; i += 4 * (long long)blockDim.x)
        acc ^= ld16(s + i) ^ ld16(s + i + blockDim.x) ^ ld16(s + i + 2 * blockDim.x) ^ ld16(s + i + 3 * blockDim.x);
      for (; i < nv; i += blockDim.x) acc ^= ld16(s + i);
    }
    if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) reinterpret_cast<u32x4*>(pv.stage[r])[threadIdx.x] = acc;
    rank_barrier(pv, ep++);
    return;
  }
  const long long lo = lmin((long long)b * A.slice, A.bytes), hi = lmin(lo + A.slice, A.bytes);
  const long long len = hi - lo;
  char* mine = pv.stage[r];
  const char* send = (const char*)A.send;
  char* recv = (char*)A.recv;
  if (A.mode == C_BCAST) {
    if (r == A.root) block_copy(mine + lo, send + lo, len);
    if (!rank_barrier(pv, ep++)) return;
    if (r != A.root) block_copy(recv + lo, pv.stage[A.root] + lo, len);
    rank_barrier(pv, ep++);
    return;
  }
  if (A.mode == C_ALLGATHER) {
    block_copy(mine + lo, send + lo, len);
    if (!rank_barrier(pv, ep++)) return;
    for (int k = 0; k < n; ++k) {
      const int p = (r + k) % n;
      char* dst = recv + (long long)p * A.total + lo;
      if (p == r) {
        if (send + lo != dst) block_copy(dst, mine + lo, len);
      } else {
        block_copy(dst, pv.stage[p] + lo, len);
      }
    }
    rank_barrier(pv, ep++);
    return;
  }
  // C_ALLTOALL: block p of my send goes to rank p; block j of my recv comes
  // from rank j's block r.
  for (int p = 0; p < n; ++p) block_copy(mine + (long long)p * A.bytes + lo, send + (long long)p * A.total + lo, len);
  if (!rank_barrier(pv, ep++)) return;
  for (int k = 0; k < n; ++k) {
    const int p = (r + k) % n;
    block_copy(recv + (long long)p * A.total + lo, pv.stage[p] + (long long)r * A.bytes + lo, len);
  }
  rank_barrier(pv, ep++);
}

hipError_t launch_copy(dim3 grid, hipStream_t s, const CopyArgs& a) {
  hipLaunchKernelGGL(copy_kernel, grid, dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace mpigx
