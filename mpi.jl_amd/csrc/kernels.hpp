// kernels.hpp — the three kernel families of libmpigx.
//
//  fold_kernel<OP,T,NMAX,SCHED>: local multi-buffer reduce (config 2) and the
//      reducing collectives Allreduce! / Reduce! (src/collective.jl:605-714).
//  scan_kernel<OP,T>: Scan! / Exscan! (collective.jl:760-857) with MPICH's
//      recursive-doubling association and operand roles.
//  copy_kernel: Bcast! / Allgather! / Alltoall! / Barrier (collective.jl:15-42,
//      295-335, 489-532) — byte movement only.
//
// Data path of every collective (one launch per round, rounds bound the
// staging arena): block b of every rank owns the same element slice(s);
//   copy-in: my send slice(s) -> my staging arena (HBM, IPC-exported)
//   barrier(b): the slices are visible to every peer
//   compute: pull peer slices over xGMI (peer-mapped HBM), reduction fused
//            into the pull, write the result to my recvbuf (and staging)
//   barrier(b) ... final barrier(b): peers finished reading my staging.
#pragma once
#include "device.hpp"

namespace mpigx {

__device__ __forceinline__ long long lmin(long long a, long long b) { return a < b ? a : b; }

// Completion signal for blocking calls: every block counts itself on a
// device-memory counter after its last access; the block that completes the
// count stores the launch's sequence number to a host-mapped word (the host
// spins on it instead of paying a hipStreamSynchronize round trip).  One
// PCIe write per launch: per-block host atomics serialise (128 blocks cost
// ~65 us, tools/latency.py).
// The stored word is seq << 1 | aborted: a zero-copy launch's abort verdict
// (the same in every block, device.hpp zc_enter) travels in the completion
// store itself.
__device__ __forceinline__ void signal_done(const PeerView& pv, int aborted = 0) {
  if (pv.done) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long prev =
          __hip_atomic_fetch_add(pv.dcount, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      if (prev == pv.dbase + gridDim.x - 1) {
        __hip_atomic_store(pv.done, (pv.seq << 1) | (aborted ? 1ull : 0ull), __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        // push the word out now, not at some later system-scope release
        // (device.hpp flush_remote_stores): a host spinning on it saw it only
        // after its own hipStreamSynchronize fallback, 20 s late (r03r)
        flush_remote_stores();
      }
    }
  }
}

// Vectors per thread in flight for the collective folds: U 16-B vectors of
// 4-byte-or-wider elements, fewer where one vector takes more than 4 VGPRs
// (8- / 16-bit elements sit one per VGPR: 16 / 8 registers per vector), so
// the int8 kernels do not trade occupancy for loads they cannot hold.
template <class T>
constexpr int vec_regs() {
  using V = Vec<T, VecW<T>::v>;
  return V::N * (sizeof(typename V::S) >= 4 ? (int)(sizeof(typename V::S) / 4) : 1);
}
template <class T>
constexpr int zc_u(int U) {
  return U * 4 / vec_regs<T>() >= 1 ? U * 4 / vec_regs<T>() : 1;
}

template <class OP, class T, int NMAX, int SCHED>
__device__ __forceinline__ int fold_body(const FoldArgs& A);

template <class OP, class T, int NMAX, int SCHED>
__global__ __launch_bounds__(kThreads) void fold_kernel(FoldArgs A) {
  // The collective modes index FoldArgs with per-rank values (peer arenas,
  // mapped user buffers, fold sources).  Read from the kernarg segment, that
  // made the compiler copy the whole 864-B argument block to per-thread
  // scratch at entry in one instantiation family or another as the modes
  // grew (float MIN/MAX, NMAX 16, then every NMAX-8 kernel once the
  // zero-copy Reduce joined); every collective fold kernel therefore stages
  // it once per block in LDS (216 words, one pass of the block).
  __shared__ FoldArgs sA;
  static_assert(sizeof(FoldArgs) % 4 == 0, "FoldArgs word copy");
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&A);
  uint32_t* d = reinterpret_cast<uint32_t*>(&sA);
  for (unsigned i = threadIdx.x; i < sizeof(FoldArgs) / 4; i += blockDim.x) d[i] = w[i];
  __syncthreads();
  kernel_started(sA.pv);
  stamp(sA.pv, 0);
  const int ab = fold_body<OP, T, NMAX, SCHED>(sA);
  signal_done(sA.pv, ab);
}

// Config-2 local multi-buffer reduce in a kernel of its own: the collective
// modes index FoldArgs with per-rank values, which for the role-sensitive
// ops (float MIN/MAX) made the compiler copy the whole 840-B argument block
// to scratch in every thread at entry — 16 M threads x 840 B per 256 MiB
// call held f32 MAX at 0.67 TB/s.  This kernel touches only M_LOCAL fields.
//
// One pass: thread t of block b folds the U vectors (16 B of every input
// each) at vector indices (b*U + u)*kThreads + t, all U*ntree loads issued
// before any arithmetic; the grid covers the whole range (a grid-stride loop
// only takes over beyond 2^32 threads).  SHAPE: SH_PRE / SH_POW2 / SH_FULL.
template <class OP, class T, int NMAX, int SCHED, int SHAPE, int U>
__global__ __launch_bounds__(kThreads) void fold_local_kernel(FoldArgs A) {
  constexpr int W = VecW<T>::v;
  const T* const* src = reinterpret_cast<const T* const*>(A.src);
  const T* const* src2 = reinterpret_cast<const T* const*>(A.src2);
  T* out = (T*)A.recv;
  bool vec = ((uintptr_t)A.recv & 15) == 0;
#pragma unroll
  for (int s = 0; s < NMAX; ++s)
    if (s < A.ntree) vec &= ((uintptr_t)A.src[s] & 15) == 0;
  if constexpr (SHAPE == SH_PRE) {
#pragma unroll
    for (int s = 0; s < NMAX / 2; ++s)
      if (s < A.rem) vec &= ((uintptr_t)A.src2[s] & 15) == 0;
  }
  const long long tid = threadIdx.x;
  if (!vec) {
    const long long gt = (long long)blockIdx.x * kThreads + tid, gn = (long long)gridDim.x * kThreads;
    fold_range<OP, T, NMAX, SCHED, SHAPE>(A, src, src2, 0, A.count, out, nullptr, false, gt, gn);
    return;
  }
  const long long nv = A.count / W;
  const long long step = (long long)gridDim.x * (U * kThreads);
  for (long long v0 = (long long)blockIdx.x * (U * kThreads) + tid; v0 < nv; v0 += step) {
    if (v0 + (long long)(U - 1) * kThreads < nv) {
      Leaves<T, NMAX, SHAPE, W> L[U];
#pragma unroll
      for (int u = 0; u < U; ++u) load_leaves<T, NMAX, SCHED, SHAPE, W>(A, src, src2, (v0 + u * kThreads) * W, L[u]);
      // the block's output span (U * kThreads vectors), write-through stores
      const __amdgpu_buffer_rsrc_t span = span_rsrc(out + (v0 - tid) * W, U * kThreads * 16);
      unsigned strad = 0;  // vectors straddling a Rabenseifner block boundary
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long e = (v0 + u * kThreads) * W;
        Vec<T, W> r;
        if (fold_leaves<OP, T, NMAX, SCHED, SHAPE, W>(A, e, L[u], r)) stv_wt<T, W>(span, (int)(tid + u * kThreads) * 16, r);
        else strad |= 1u << u;
      }
#pragma unroll 1
      for (int u = 0; u < U; ++u)
        if ((strad >> u) & 1u) fold_elems<OP, T, NMAX, SCHED, SHAPE>(A, src, src2, (v0 + u * kThreads) * W, W, out, nullptr);
    } else {
#pragma unroll 1
      for (int u = 0; u < U; ++u)
        if (v0 + u * kThreads < nv) {
          const long long e = (v0 + u * kThreads) * W;
          Vec<T, W> r;
          if (fold_at<OP, T, NMAX, SCHED, SHAPE, W>(A, src, src2, e, r)) stv<T, W>(out + e, r);
          else fold_elems<OP, T, NMAX, SCHED, SHAPE>(A, src, src2, e, W, out, nullptr);
        }
    }
  }
  // ragged tail (count % W elements): the first thread of block 0
  if (blockIdx.x == 0 && tid == 0 && nv * W < A.count)
    fold_elems<OP, T, NMAX, SCHED, SHAPE>(A, src, src2, nv * W, (int)(A.count - nv * W), out, nullptr);
}

template <class OP, class T, int NMAX, int SCHED>
__device__ __forceinline__ int fold_body(const FoldArgs& A) {  // returns the zero-copy abort verdict
  // two vectors per thread in flight in every fold and gather of the
  // collective modes at n <= 8 (ar_zc_kernel goes further for the headline
  // zero-copy two-shot); NMAX 16 (n = 9..16) keeps one (VGPRs)
  constexpr int FU = NMAX <= 8 ? zc_u<T>(2) : 1;
  const T* const* src = reinterpret_cast<const T* const*>(A.src);
  const T* const* src2 = reinterpret_cast<const T* const*>(A.src2);
  const PeerView& pv = A.pv;
  constexpr int W = VecW<T>::v;
  const int b = blockIdx.x;
  const long long tid = threadIdx.x, nt = blockDim.x;

  T* recv = (T*)A.recv;
  T* mine = (T*)pv.stage[pv.rank];
  const char* send = (const char*)A.send;
  const bool recv_vec = ((uintptr_t)recv & 15) == 0;
  const int es = A.esize;
  uint64_t ep = pv.epoch;

  if (A.mode == M_AR_ZC) {
    // zero-copy two-shot: no staging; sources are the peers' send buffers
    // (skipped everywhere if any rank's view of the mappings is stale)
    const int n = pv.n, r = pv.rank;
    int ab;
    stamp(pv, 0);
    if (!zc_enter(pv, ep++, &ab)) return 0;  // every rank's send buffer is ready
    stamp(pv, 1);
    if (!ab) {
    const long long c0 = lmin((long long)r * A.chunk, A.count), c1 = lmin(c0 + A.chunk, A.count);
    const long long lo = lmin(c0 + (long long)b * A.slice, c1), hi = lmin(lo + A.slice, c1);
    bool vec = recv_vec;
#pragma unroll
    for (int s = 0; s < NMAX; ++s)
      if (s < A.ntree) vec &= ((uintptr_t)A.src[s] & 15) == 0;
#pragma unroll
    for (int s = 0; s < NMAX / 2; ++s)
      if (s < A.rem) vec &= ((uintptr_t)A.src2[s] & 15) == 0;
    fold_range<OP, T, NMAX, SCHED, SH_PRE, FU>(A, src, src2, lo, hi, recv, nullptr, vec, tid, nt);
    }
    stamp(pv, 2);
    if (!rank_barrier(pv, ep++, &ab)) return 0;  // every reduced chunk is in its owner's recvbuf
    stamp(pv, 3);
    if (!ab) {
    char* dsts[NMAX];
    const char* srcs[NMAX];
    long long lens[NMAX];
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
      dsts[j] = nullptr;
      srcs[j] = nullptr;
      lens[j] = 0;
      if (j + 1 < n) {
        const int p = (r + 1 + j) % n;
        const long long d0 = lmin((long long)p * A.chunk, A.count), d1 = lmin(d0 + A.chunk, A.count);
        const long long l2 = lmin(d0 + (long long)b * A.slice, d1), h2 = lmin(l2 + A.slice, d1);
        dsts[j] = (char*)(recv + l2);
        srcs[j] = A.zc_recv[p] + l2 * es;
        lens[j] = (h2 - l2) * es;
      }
    }
    block_gather_u<NMAX, FU>(dsts, srcs, lens, n - 1);
    }
    stamp(pv, 4);
    if (rank_barrier_exit(pv, ep++, &ab)) stamp(pv, 5);  // nobody reads my buffers any more
    return ab;
  }

  if (A.mode == M_RED_ZC) {
    // zero-copy Reduce: RS of my chunk straight from every rank's sendbuf;
    // non-roots keep it in their arena (slice b at the chunk-relative
    // offset), the root writes its own chunk into its recvbuf and then
    // gathers the others' from their arenas
    const int n = pv.n, r = pv.rank;
    int ab;
    if (!zc_enter(pv, ep++, &ab)) return 0;
    const long long c0 = lmin((long long)r * A.chunk, A.count), c1 = lmin(c0 + A.chunk, A.count);
    const long long lo = lmin(c0 + (long long)b * A.slice, c1), hi = lmin(lo + A.slice, c1);
    if (!ab) {
      bool vec = true;
#pragma unroll
      for (int s = 0; s < NMAX; ++s)
        if (s < A.ntree) vec &= ((uintptr_t)A.src[s] & 15) == 0;
#pragma unroll
      for (int s = 0; s < NMAX / 2; ++s)
        if (s < A.rem) vec &= ((uintptr_t)A.src2[s] & 15) == 0;
      // (two calls, not a select of the output pointer: selecting between
      // recv and the arena made the compiler copy FoldArgs to scratch)
      if (r == A.root)
        fold_range<OP, T, NMAX, SCHED, SH_PRE, FU>(A, src, src2, lo, hi, recv, nullptr, vec && recv_vec, tid, nt);
      else  // arena: element e of my chunk at e - c0 (c0 is a multiple of the vector width)
        fold_range<OP, T, NMAX, SCHED, SH_PRE, FU>(A, src, src2, lo, hi, mine - c0, nullptr, vec, tid, nt);
    }
    if (!rank_barrier(pv, ep++, &ab)) return 0;
    if (!ab && r == A.root) {
      char* dsts[NMAX];
      const char* srcs[NMAX];
      long long lens[NMAX];
#pragma unroll
      for (int j = 0; j < NMAX; ++j) {
        dsts[j] = nullptr;
        srcs[j] = nullptr;
        lens[j] = 0;
        if (j + 1 < n) {
          const int p = (r + 1 + j) % n;
          const long long d0 = lmin((long long)p * A.chunk, A.count), d1 = lmin(d0 + A.chunk, A.count);
          const long long l2 = lmin(d0 + (long long)b * A.slice, d1), h2 = lmin(l2 + A.slice, d1);
          dsts[j] = (char*)(recv + l2);
          srcs[j] = pv.stage[p] + (l2 - d0) * es;
          lens[j] = (h2 - l2) * es;
        }
      }
      block_gather_u<NMAX, FU>(dsts, srcs, lens, n - 1);
    }
    rank_barrier_exit(pv, ep++, &ab);  // nobody reads my sendbuf / arena any more
    return ab;
  }

  if (A.mode == M_AR_PUSH) {
    // push two-shot (the fold sources src[]/src2[] are my own arena slots and
    // my sendbuf, resolved on the host).  No entry barrier: phase 1 writes
    // only into the peers' arenas, which their previous launch (ended by a
    // barrier of every block) no longer reads; their recvbufs are written
    // only after barrier 1, i.e. after every rank entered this launch.
    const int n = pv.n, r = pv.rank;
    char* dsts[NMAX];
    const char* srcs[NMAX];
    long long lens[NMAX];
    {  // phase 1 stores into the peers' arenas before any barrier (zc_enter's checks)
      if (args_fault(pv)) {
        if (tid == 0) __hip_atomic_store(pv.err, kErrProtocol, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return 0;
      }
    }
    stamp(pv, 1);
    // phase 1: slice b of my chunk p -> rank p's slot [r], all peers at once
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
      dsts[j] = nullptr;
      srcs[j] = nullptr;
      lens[j] = 0;
      if (j + 1 < n) {
        const int p = (r + 1 + j) % n;
        const long long d0 = lmin((long long)p * A.chunk, A.count), d1 = lmin(d0 + A.chunk, A.count);
        const long long l2 = lmin(d0 + (long long)b * A.slice, d1), h2 = lmin(l2 + A.slice, d1);
        dsts[j] = pv.stage[p] + (long long)r * A.slot_bytes + (l2 - d0) * es;
        srcs[j] = send + l2 * es;
        lens[j] = (h2 - l2) * es;
      }
    }
    block_gather_u<NMAX, FU>(dsts, srcs, lens, n - 1);
    stamp(pv, 2);
    // phase 2 writes into the peers' recvbufs through the view's mappings:
    // the barrier checks every rank uses the same view (zc_enter)
    int ab = pv.zc_bad;
    if (!rank_barrier(pv, ep++, &ab, pv.zc_key, true)) return 0;
    stamp(pv, 3);
    if (!ab) {
    // phase 2: fold my chunk (slots = local HBM) into my recvbuf, then write
    // the reduced slice into every peer's recvbuf
    const long long c0 = lmin((long long)r * A.chunk, A.count), c1 = lmin(c0 + A.chunk, A.count);
    const long long lo = lmin(c0 + (long long)b * A.slice, c1), hi = lmin(lo + A.slice, c1);
    bool vec = recv_vec;
#pragma unroll
    for (int s = 0; s < NMAX; ++s)
      if (s < A.ntree) vec &= ((uintptr_t)A.src[s] & 15) == 0;
#pragma unroll
    for (int s = 0; s < NMAX / 2; ++s)
      if (s < A.rem) vec &= ((uintptr_t)A.src2[s] & 15) == 0;
    fold_range<OP, T, NMAX, SCHED, SH_PRE, FU>(A, src, src2, lo, hi, recv, nullptr, vec, tid, nt);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
      dsts[j] = nullptr;
      srcs[j] = nullptr;
      lens[j] = 0;
      if (j + 1 < n) {
        const int p = (r + 1 + j) % n;
        dsts[j] = A.zc_recv[p] + lo * es;
        srcs[j] = (const char*)(recv + lo);
        lens[j] = (hi - lo) * es;
      }
    }
    block_gather_u<NMAX, FU>(dsts, srcs, lens, n - 1);
    }
    stamp(pv, 4);
    if (rank_barrier(pv, ep++, &ab)) stamp(pv, 5);  // every slice of my recvbuf has arrived
    return ab;
  }

  if (A.mode == M_AR_LL || A.mode == M_RED_LL) {
    // small Allreduce in one step: every rank's slice b arrives as LL lines
    // in my own memory (device.hpp ll_exchange), unpacked into my arena slot
    // of its rank; the fold then reads local HBM only, with the same
    // schedule and leaf order as the one-shot (src[] = the unpack slots)
    const long long lo = lmin((long long)b * A.slice, A.count), hi = lmin(lo + A.slice, A.count);
    const long long bytes = A.count * es;
    const long long l0 = (lo * es) / 8, l1 = hi > lo ? (hi * es + 7) / 8 : l0;
    if (!ll_exchange(pv, A.zc_recv, A.ll_in, A.ll_stride, A.ll_flag, send, bytes, l0, l1, (char*)mine, A.slot_bytes,
                     pv.n, pv.rank, pv.err))
      return 0;
    if (A.mode == M_AR_LL || pv.rank == A.root)
      fold_range<OP, T, NMAX, SCHED, SH_PRE, FU>(A, src, src2, lo, hi, recv, nullptr, recv_vec, tid, nt);
    return 0;
  }

  if (A.mode == M_AR_LL2) {
    // LL two-shot (two-shot partition: chunk c, slice b of every chunk per
    // block).  Lines are chunk-relative; half 0 of every sender slot carries
    // the reduce-scatter, half 1 the allgather (common.hpp M_AR_LL2).  The
    // fold reads my own slice from my sendbuf and the peers' from my arena
    // slots (src[] is chunk-offset on the host, as for the push two-shot).
    const int n = pv.n, r = pv.rank;
    const unsigned flag = A.ll_flag;
    const long long half = A.ll_stride / 2;
    const uint64_t t0 = wall_clock64();
    uint64_t next = kCancelPoll;  // one cancel-word read per kCancelPoll of waiting
    bool ok = true;
    // chunk c: element offset, bytes, and this block's line range
    long long lo, hi;  // this block's elements of the chunk (chunk-relative)
    auto span = [&](int c, long long* c0, long long* cb, long long* l0, long long* l1) {
      *c0 = lmin((long long)c * A.chunk, A.count);
      const long long clen = lmin(*c0 + A.chunk, A.count) - *c0;
      lo = lmin((long long)b * A.slice, clen);
      hi = lmin(lo + A.slice, clen);
      *cb = clen * es;
      *l0 = lo * es / 8;
      *l1 = hi > lo ? (hi * es + 7) / 8 : *l0;
    };
    long long c0, cb, l0, l1;
    // reduce-scatter: slice b of chunk p -> rank p
    for (int p = 0; p < n; ++p) {
      if (p == r) continue;
      span(p, &c0, &cb, &l0, &l1);
      for (long long i = l0 + tid; i < l1; i += nt) ll_put(A.zc_recv[p], i, ll_pack8(send + c0 * es, i, cb), flag);
    }
    flush_remote_stores();
    long long r0, rb, rl0, rl1;
    span(r, &r0, &rb, &rl0, &rl1);
    const long long rlo = r0 + lo, rhi = r0 + hi;
    for (int p = 0; p < n && ok; ++p) {
      if (p == r) continue;
      for (long long i = rl0 + tid; i < rl1 && ok; i += nt) {
        uint64_t d;
        ok = ll_get(pv, ll_from(pv, A.ll_in, p, A.ll_stride), i, flag, t0, next, &d);
        if (ok) *reinterpret_cast<uint64_t*>((char*)mine + (long long)p * A.slot_bytes + 8 * i) = d;
      }
    }
    __syncthreads();
    if (__syncthreads_or(!ok)) {
      if (tid == 0) __hip_atomic_store(pv.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return 0;
    }
    bool vec = recv_vec;  // my own leaf is my sendbuf: alignment unknown
#pragma unroll
    for (int q = 0; q < NMAX; ++q)
      if (q < A.ntree) vec &= ((uintptr_t)A.src[q] & 15) == 0;
#pragma unroll
    for (int q = 0; q < NMAX / 2; ++q)
      if (q < A.rem) vec &= ((uintptr_t)A.src2[q] & 15) == 0;
    fold_range<OP, T, NMAX, SCHED, SH_PRE, FU>(A, src, src2, rlo, rhi, recv, nullptr, vec, tid, nt);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // allgather: my reduced slice -> every rank; slice b of chunk p <- rank p
    for (long long i = rl0 + tid; i < rl1; i += nt) {
      const uint64_t d = ll_pack8((const char*)recv + r0 * es, i, rb);
      for (int p = 0; p < n; ++p)
        if (p != r) ll_put(A.zc_recv[p] + half, i, d, flag);
    }
    flush_remote_stores();
    for (int p = 0; p < n && ok; ++p) {
      if (p == r) continue;
      span(p, &c0, &cb, &l0, &l1);
      for (long long i = l0 + tid; i < l1 && ok; i += nt) {
        uint64_t d;
        ok = ll_get(pv, ll_from(pv, A.ll_in, p, A.ll_stride) + half, i, flag, t0, next, &d);
        if (ok) ll_store8((char*)recv + c0 * es, i, cb, d);
      }
    }
    if (!ok) __hip_atomic_store(pv.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return 0;
  }

  if (A.mode == M_AR_ONESHOT || A.mode == M_RED_ONESHOT) {
    const long long lo = lmin((long long)b * A.slice, A.count), hi = lmin(lo + A.slice, A.count);
    block_copy((char*)(mine + lo), send + lo * es, (hi - lo) * es);
    if (!rank_barrier(pv, ep++)) return 0;
    if (A.mode == M_AR_ONESHOT || pv.rank == A.root)
      fold_range<OP, T, NMAX, SCHED, SH_PRE, FU>(A, src, src2, lo, hi, recv, nullptr, recv_vec, tid, nt);
    rank_barrier_exit(pv, ep++);
    return 0;
  }

  // two-shot: chunk c = [c*chunk, (c+1)*chunk) ∩ [0,count), block b owns
  // slice b of every chunk.
  const int n = pv.n, r = pv.rank;
  for (int c = 0; c < n; ++c) {
    const long long c0 = lmin((long long)c * A.chunk, A.count), c1 = lmin(c0 + A.chunk, A.count);
    const long long lo = lmin(c0 + (long long)b * A.slice, c1), hi = lmin(lo + A.slice, c1);
    block_copy((char*)(mine + lo), send + lo * es, (hi - lo) * es);
  }
  if (!rank_barrier(pv, ep++)) return 0;
  {
    const long long c0 = lmin((long long)r * A.chunk, A.count), c1 = lmin(c0 + A.chunk, A.count);
    const long long lo = lmin(c0 + (long long)b * A.slice, c1), hi = lmin(lo + A.slice, c1);
    // reduce-scatter: my chunk from every rank's staging; result into my
    // staging (for the peers' gather) and straight into my recvbuf.
    const bool want_recv = (A.mode == M_AR_TWOSHOT) || (r == A.root);
    if (want_recv)
      fold_range<OP, T, NMAX, SCHED, SH_PRE, FU>(A, src, src2, lo, hi, recv, mine, recv_vec, tid, nt);
    else
      fold_range<OP, T, NMAX, SCHED, SH_PRE, FU>(A, src, src2, lo, hi, mine, nullptr, true, tid, nt);
  }
  (void)W;
  if (!rank_barrier(pv, ep++)) return 0;
  if (A.mode == M_AR_TWOSHOT || r == A.root) {
    // allgather (or gather at root): every other rank's reduced chunk,
    // all peers interleaved per thread so every link is busy
    char* dsts[NMAX];
    const char* srcs[NMAX];
    long long lens[NMAX];
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
      dsts[j] = nullptr;
      srcs[j] = nullptr;
      lens[j] = 0;
      if (j + 1 < n) {
        const int p = (r + 1 + j) % n;
        const long long c0 = lmin((long long)p * A.chunk, A.count), c1 = lmin(c0 + A.chunk, A.count);
        const long long lo = lmin(c0 + (long long)b * A.slice, c1), hi = lmin(lo + A.slice, c1);
        dsts[j] = (char*)(recv + lo);
        srcs[j] = (const char*)((const T*)pv.stage[p] + lo);
        lens[j] = (hi - lo) * es;
      }
    }
    block_gather_u<NMAX, FU>(dsts, srcs, lens, n - 1);
  }
  rank_barrier_exit(pv, ep++);
  return 0;
}

// ---------------------------------------------------------------------------
// Zero-copy two-shot Allreduce (M_AR_ZC, the headline path >= MPIGX_ZC_MIN,
// MPICH tree schedule, n <= 8) in a kernel of its own, sized by the rank
// count.  The all-modes fold_kernel keeps ONE vector's leaves in flight per
// thread (n loads; 2 at n = 2) and gathers one vector per peer (1 load at
// n = 2): one 256-block grid then holds ~16 KB of loads in flight per CU,
// a third of what HBM needs (the n = 2 same-device two-shot ran at 0.46 of
// HBM against 0.79 for the local fold).  Here NMAX = n rounded
// up to a power of two (2, 4, 8) is a compile-time constant, and U = 16 /
// NMAX vectors per thread per iteration keep ~16 loads outstanding in both
// phases at every n:
//   entry barrier (zero-copy view check) -> RS: fold slice b of my chunk r
//   from every rank's sendbuf into my recvbuf -> barrier -> AG: slice b of
//   chunk p from rank p's recvbuf, every peer interleaved -> exit barrier.
// Same chunk / slice partition, barriers and fold schedule as fold_body's
// M_AR_ZC (identical bits; that path still serves LINEAR order and n > 8).
// SHAPE: SH_FULL (n = NMAX, no pre-step: every leaf present, no guards) or
// SH_PRE (pre-step partners and / or fewer leaves, guarded).
// AG: AG_PULL as above; AG_PUSH ("pullpush", MPIGX_ALGO=pullpush) stores each
// reduced slice straight into EVERY rank's recvbuf during the fold (peers'
// through the view's mappings) — no mid barrier, no allgather reads: per rank
// read S + write S instead of read 1.5 S + write S at n = 2 (2 S + 7/8 S
// reads at n = 8), the same xGMI bytes with the allgather half as posted
// writes.  Its exit barrier publishes those stores (full release / acquire).
// ---------------------------------------------------------------------------
template <class OP, class T, int NMAX, int SHAPE, int U, int AG = AG_PULL>
__global__ __launch_bounds__(kThreads) void ar_zc_kernel(FoldArgs A0) {
  __shared__ FoldArgs A;  // indexed by runtime ranks below (see fold_kernel)
  {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(&A0);
    uint32_t* d = reinterpret_cast<uint32_t*>(&A);
    for (unsigned i = threadIdx.x; i < sizeof(FoldArgs) / 4; i += blockDim.x) d[i] = w[i];
    __syncthreads();
  }
  const PeerView& pv = A.pv;
  const T* const* src = reinterpret_cast<const T* const*>(A.src);
  const T* const* src2 = reinterpret_cast<const T* const*>(A.src2);
  T* recv = (T*)A.recv;
  const int n = pv.n, r = pv.rank, b = blockIdx.x, es = A.esize;
  const long long tid = threadIdx.x, nt = blockDim.x;
  uint64_t ep = pv.epoch;
  int ab;
  kernel_started(pv);
  stamp(pv, 0);
  if (!zc_enter(pv, ep++, &ab)) {
    signal_done(pv, 0);
    return;
  }
  stamp(pv, 1);
  // my chunk: chunk r, except for the zero-copy Reduce, whose chunks belong
  // to the non-roots at n >= 3 (host reduce_zc_push)
  const int own = A.mode == M_RED_ZC ? A.own : r;
  const long long c0 = lmin((long long)own * A.chunk, A.count), c1 = lmin(c0 + A.chunk, A.count);
  bool vec = ((uintptr_t)recv & 15) == 0;
#pragma unroll
  for (int s = 0; s < NMAX; ++s)
    if (s < A.ntree) vec &= ((uintptr_t)A.src[s] & 15) == 0;
  if constexpr (SHAPE == SH_PRE) {
#pragma unroll
    for (int s = 0; s < NMAX / 2; ++s)
      if (s < A.rem) vec &= ((uintptr_t)A.src2[s] & 15) == 0;
  }
  if constexpr (AG == AG_PUSH) {
    // Allreduce: mine first, then the peers' recvbufs; Reduce (M_RED_ZC):
    // the root's recvbuf only
    const bool red = A.mode == M_RED_ZC;
    const int m = red ? 1 : n;
    T* outs[NMAX];
    bool fits = true;  // my chunk's end inside every recvbuf I store into (the view's exported sizes)
#pragma unroll
    for (int j = 0; j < NMAX; ++j) {
      const int q = red ? A.root : (r + j) % n;
      outs[j] = red ? (T*)A.zc_recv[A.root] : recv;
      if (!red && j > 0 && j < n) outs[j] = (T*)A.zc_recv[q];
      if (j < m) {
        vec &= ((uintptr_t)outs[j] & 15) == 0;
        fits &= outs[j] != nullptr && c1 * es <= A.zc_avail[q];
      }
    }
    if (!ab && !fits) {  // the same verdict in every block: the exit barrier's abort bit reaches every peer block
      ab = 1;
      if (tid == 0) __hip_atomic_store(pv.err, kErrProtocol, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (A.dyn) {
      // slices of my chunk handed out by a ticket counter (a block that
      // finishes early takes the next slice instead of idling until the
      // slowest block's static share is done); every block takes tickets
      // until one is past the end, so a launch consumes exactly
      // slices + grid tickets (mpigx.cpp allreduce_zc advances wbase by that)
      __shared__ long long s_tk;
      unsigned long long* tickets = pv.dcount + 1;
      const long long nsl = (c1 - c0 + A.slice - 1) / A.slice;
      if (tid == 0)
        s_tk = (long long)(__hip_atomic_fetch_add(tickets, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - pv.wbase);
      __syncthreads();
      long long tk = s_tk;
      while (tk < nsl) {
        long long nxt = 0;  // the next ticket, taken while this slice streams
        if (tid == 0)
          nxt = (long long)(__hip_atomic_fetch_add(tickets, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - pv.wbase);
        if (!ab) {
          const long long lo = c0 + tk * A.slice;
          fold_span_scatter<OP, T, NMAX, S_TREE, SHAPE, U>(A, src, src2, lo, lmin(lo + A.slice, c1), outs, m, vec);
        }
        __syncthreads();
        if (tid == 0) s_tk = nxt;
        __syncthreads();
        tk = s_tk;
      }
      stamp(pv, 2);
      stamp(pv, 3);
      stamp(pv, 4);
      if (rank_barrier_grid(pv, ep++, &ab)) stamp(pv, 5);  // every rank's blocks are done: my recvbuf is complete
    } else {
      if (!ab) {
        const long long lo = lmin(c0 + (long long)b * A.slice, c1), hi = lmin(lo + A.slice, c1);
        fold_span_scatter<OP, T, NMAX, S_TREE, SHAPE, U>(A, src, src2, lo, hi, outs, m, vec);
      }
      stamp(pv, 2);
      stamp(pv, 3);
      stamp(pv, 4);
      if (rank_barrier(pv, ep++, &ab)) stamp(pv, 5);  // every slice of my recvbuf has arrived
    }
    signal_done(pv, ab);
    return;
  }
  if (!ab) {
    const long long lo = lmin(c0 + (long long)b * A.slice, c1), hi = lmin(lo + A.slice, c1);
    if (vec) fold_span<OP, T, NMAX, S_TREE, SHAPE, U>(A, src, src2, lo, hi, recv, nullptr);
    else fold_range<OP, T, NMAX, S_TREE, SHAPE>(A, src, src2, lo, hi, recv, nullptr, false, tid, nt);
  }
  stamp(pv, 2);
  if (!rank_barrier(pv, ep++, &ab)) {  // every reduced chunk is in its owner's recvbuf
    signal_done(pv, 0);
    return;
  }
  stamp(pv, 3);
  if (!ab) {
    constexpr int MP = NMAX - 1;  // peers: n - 1 <= NMAX - 1
    char* dsts[MP];
    const char* srcs[MP];
    long long lens[MP];
#pragma unroll
    for (int j = 0; j < MP; ++j) {
      dsts[j] = nullptr;
      srcs[j] = nullptr;
      lens[j] = 0;
      if (j + 1 < n) {
        const int p = (r + 1 + j) % n;
        const long long d0 = lmin((long long)p * A.chunk, A.count), d1 = lmin(d0 + A.chunk, A.count);
        const long long l2 = lmin(d0 + (long long)b * A.slice, d1), h2 = lmin(l2 + A.slice, d1);
        dsts[j] = (char*)(recv + l2);
        srcs[j] = A.zc_recv[p] + l2 * es;
        lens[j] = (h2 - l2) * es;
      }
    }
    block_gather_u<MP, U>(dsts, srcs, lens, n - 1);
  }
  stamp(pv, 4);
  if (rank_barrier_exit(pv, ep++, &ab)) stamp(pv, 5);  // nobody reads my buffers any more
  signal_done(pv, ab);
}

// ---------------------------------------------------------------------------
// Ring reduce-scatter + allgather (RingArgs, common.hpp): the classic
// bandwidth-optimal schedule the north star names for large messages, here
// as a comparison against the all-peer direct two-shot.  Per ring every rank
// pulls from its left neighbour only (one xGMI link per direction per ring;
// nch rings of distinct strides use nch links).  Per step and block:
//   wait(left, step-1) -> pull + fold (RS) or pull (AG) -> signal(right)
// RS step s at ring position p folds chunk (p-s-1): its left neighbour's
// partial (its send buffer at s = 0) as inout with my contribution; the last
// RS step writes the final chunk (p+1) into my recvbuf.  AG step t copies
// chunk (p-t) out of the left neighbour's recvbuf.  Partials of the RS live
// in the staging arena at the chunk's element offset (one chunk per slot,
// written once per launch).  Signals are barrier words (device.hpp) stored
// into the right neighbour's slot [block][me]: monotone epochs, the sticky
// abort bit of the zero-copy entry.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void ring_signal(const PeerView& pv, int to, uint64_t ep, int ab) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t word = (ep << kSigShift) | ((uint64_t)(ab ? 1 : 0) << 24);
    __hip_atomic_store(pv.sig[to] + sig_index(blockIdx.x, pv.rank), word, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    flush_remote_stores();
  }
}
__device__ __forceinline__ bool ring_wait(const PeerView& pv, int from, uint64_t ep) {
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    const uint64_t* slot = sig_in(pv, from) + sig_index(blockIdx.x, from);
    const uint64_t t0 = wall_clock64();
    uint64_t next = kCancelPoll;
    int ok = 1;
    unsigned k = 0;
    while ((__hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >> kSigShift) < ep) {
      spin_pause(k);
      if (spin_expired(pv, t0, next)) {
        ok = 0;
        __hip_atomic_store(pv.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

// out[i] = OP(acc[i], mine[i]) over [0, len), the block cooperating
template <class OP, class T>
__device__ __forceinline__ void ring_fold(T* out, const T* acc, const T* mine, long long len) {
  constexpr int W = VecW<T>::v;
  long long i0 = 0;
  if (((((uintptr_t)out) | ((uintptr_t)acc) | ((uintptr_t)mine)) & 15) == 0) {
    const long long nv = len / W;
    for (long long v = threadIdx.x; v < nv; v += blockDim.x) {
      Vec<T, W> a, b;
      ldv<T, W>(a, acc + v * W);
      ldv<T, W>(b, mine + v * W);
      vapply<OP, T, W>(a, a, b);
      stv<T, W>(out + v * W, a);
    }
    i0 = nv * W;
  }
  for (long long i = i0 + threadIdx.x; i < len; i += blockDim.x) out[i] = OP::apply(acc[i], mine[i]);
}

template <class OP, class T>
__device__ __forceinline__ int ring_body(const RingArgs& A) {  // returns the abort verdict
  const PeerView& pv = A.pv;
  const int n = pv.n, r = pv.rank;
  const int k = blockIdx.x % A.nch, bc = blockIdx.x / A.nch;
  const int L = (r - A.stride[k] + n) % n, R = (r + A.stride[k]) % n, pos = A.pos[k];
  const long long p0 = lmin((long long)k * A.part, A.count), p1 = lmin(p0 + A.part, A.count);
  auto slice_of = [&](int c, long long* lo, long long* hi) {
    const long long c0 = lmin(p0 + (long long)c * A.chunk, p1), c1 = lmin(c0 + A.chunk, p1);
    *lo = lmin(c0 + (long long)bc * A.slice, c1);
    *hi = lmin(*lo + A.slice, c1);
  };
  const T* mine = (const T*)A.zsend[r];
  T* recv = (T*)A.zrecv[r];
  uint64_t ep = pv.epoch;
  int ab;
  if (!zc_enter(pv, ep++, &ab, false)) return 0;  // every rank's buffers ready, one view
  if (!ab) {
    // reduce-scatter: n-1 steps, forward signals ep .. ep+n-2
    for (int s = 0; s < n - 1; ++s) {
      const int c = (pos - s - 1 + 2 * n) % n;
      long long lo, hi;
      slice_of(c, &lo, &hi);
      const T* acc = s == 0 ? (const T*)A.zsend[L] : (const T*)pv.stage[L];
      T* out = s == n - 2 ? recv : (T*)pv.stage[r];
      if (s > 0 && !ring_wait(pv, L, ep + s - 1)) return 0;
      ring_fold<OP, T>(out + lo, acc + lo, mine + lo, hi - lo);
      ring_signal(pv, R, ep + s, 0);
      // my left neighbour's chunk `c` of its SEND buffer is read: tell it (with
      // IN_PLACE its allgather overwrites that chunk of the same buffer)
      if (s == 0) ring_signal(pv, L, ep, 0);
    }
    ep += n - 1;
    // allgather: n-1 steps, forward signals ep .. ep+n-3 (the last copy feeds nobody)
    for (int t = 0; t < n - 1; ++t) {
      if (!ring_wait(pv, L, t == 0 ? ep - 1 : ep + t - 1)) return 0;
      if (t == 0 && !ring_wait(pv, R, ep - (n - 1))) return 0;  // R read my chunk `pos` (its step 0)
      const int c = (pos - t + 2 * n) % n;
      long long lo, hi;
      slice_of(c, &lo, &hi);
      block_copy((char*)(recv + lo), (const char*)((const T*)A.zrecv[L] + lo), (hi - lo) * (long long)sizeof(T));
      if (t < n - 2) ring_signal(pv, R, ep + t, 0);
    }
    ep += n - 2;
  } else {
    ep += 2 * n - 3;  // every rank aborted at the entry: same epochs, no ring traffic
  }
  rank_barrier_exit(pv, ep++, &ab);  // nobody reads my buffers / arena any more
  return ab;
}

template <class OP, class T>
__global__ __launch_bounds__(kThreads) void ring_kernel(RingArgs A) {
  // per-block ring parameters are indexed by the block's channel: staged in
  // LDS like FoldArgs (kernarg arrays indexed at run time go to scratch)
  __shared__ RingArgs sA;
  static_assert(sizeof(RingArgs) % 4 == 0, "RingArgs word copy");
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&A);
  uint32_t* d = reinterpret_cast<uint32_t*>(&sA);
  for (unsigned i = threadIdx.x; i < sizeof(RingArgs) / 4; i += blockDim.x) d[i] = w[i];
  __syncthreads();
  kernel_started(sA.pv);
  const int ab = ring_body<OP, T>(sA);
  signal_done(sA.pv, ab);
}

// ---------------------------------------------------------------------------
// Scan / Exscan.  MPICH 3.3.2 MPIR_Scan/Exscan_intra_recursive_doubling: for
// rank q and every set bit m of q, the block total of the m ranks just below
// q's aligned 2m-block is folded in, in increasing m:
//   scan:   rec = x_q; rec = OP(rec, T_m) ...
//   exscan: ex  = T_m1; ex = OP(ex, T_m2) ...
// T(block, owner) is computed as on rank `owner`: OP(inout = half holding the
// owner, in = other half as computed on owner^half).
// ---------------------------------------------------------------------------
template <class OP, class T, int SIZE, int W>
__device__ __forceinline__ void blk_total(const char* const* src, int base, int owner, long long e, Vec<T, W>& out) {
  if constexpr (SIZE == 1) {
    ldv<T, W>(out, (const T*)src[base] + e);
  } else {
    constexpr int H = SIZE / 2;
    const bool hi_own = (owner - base) & H;
    Vec<T, W> a, c;
    blk_total<OP, T, H, W>(src, base, hi_own ? owner ^ H : owner, e, a);       // low half
    blk_total<OP, T, H, W>(src, base + H, hi_own ? owner : owner ^ H, e, c);   // high half
    if (hi_own) vapply<OP, T, W>(out, c, a);
    else vapply<OP, T, W>(out, a, c);
  }
}

template <class OP, class T, int W>
__device__ __forceinline__ void blk_total_rt(const char* const* src, int m, int base, int owner, long long e,
                                             Vec<T, W>& out) {
  switch (m) {
    case 1: blk_total<OP, T, 1, W>(src, base, owner, e, out); break;
    case 2: blk_total<OP, T, 2, W>(src, base, owner, e, out); break;
    case 4: blk_total<OP, T, 4, W>(src, base, owner, e, out); break;
    default: blk_total<OP, T, 8, W>(src, base, owner, e, out); break;
  }
}

template <class OP, class T, int W>
__device__ __forceinline__ void scan_at(const ScanArgs& A, long long e, Vec<T, W>& res, bool& have) {
  const int q = A.pv.rank;
  have = !A.exclusive;
  if (!A.exclusive) ldv<T, W>(res, (const T*)A.src[q] + e);
  for (int m = 1; m < A.pv.n; m <<= 1) {
    if (!(q & m)) continue;
    const int d = q ^ m;
    Vec<T, W> t;
    blk_total_rt<OP, T, W>(A.src, m, d & ~(m - 1), d, e, t);
    if (!have) {
      res = t;
      have = true;
    } else {
      vapply<OP, T, W>(res, res, t);
    }
  }
}

// ---------------------------------------------------------------------------
// Pull-push Scan / Exscan (zero-copy, n <= 8; ScanArgs.pp).  The staged and
// old zero-copy schedules have rank q read the contributions of ranks 0..q:
// sum over q of (q+1) S bytes of reads (36 S at n = 8), and the top rank
// pulls S from each of 7 peers over 7 links while rank 1 pulls from one.
// Here the message is cut into n chunks like the two-shot Allreduce and rank
// r owns chunk r for EVERY rank: it loads chunk r of all contributions once
// (leaves in registers) and stores rank q's prefix of it into rank q's
// recvbuf (peers' through the view), so every rank reads S and writes S and
// every link carries S/n each way: n S reads instead of n(n+1)/2 S.  The
// association per rank is the recursive-doubling one of scan_at above with
// compile-time leaf indices (identical bits).  In place is safe: element e is
// read (all leaves) and then written by one thread of its owner only.
// ---------------------------------------------------------------------------
template <class OP, class T, int W, int SIZE, int BASE, int OWNER>
__device__ __forceinline__ void blk_total_reg(const Vec<T, W>* x, Vec<T, W>& out) {
  if constexpr (SIZE == 1) {
    out = x[BASE];
  } else {
    constexpr int H = SIZE / 2;
    constexpr bool hi_own = ((OWNER - BASE) & H) != 0;
    Vec<T, W> a, c;
    blk_total_reg<OP, T, W, H, BASE, hi_own ? (OWNER ^ H) : OWNER>(x, a);       // low half
    blk_total_reg<OP, T, W, H, BASE + H, hi_own ? OWNER : (OWNER ^ H)>(x, c);   // high half
    if constexpr (hi_own) vapply<OP, T, W>(out, c, a);
    else vapply<OP, T, W>(out, a, c);
  }
}

// rank Q's result from leaves x[0..Q]: set bits M of Q in increasing order
template <class OP, class T, int W, int Q, int M, bool HAVE>
__device__ __forceinline__ void scan_reg_bits(const Vec<T, W>* x, Vec<T, W>& res) {
  if constexpr (M <= Q) {
    if constexpr ((Q & M) != 0) {
      constexpr int D = Q ^ M;
      Vec<T, W> t;
      blk_total_reg<OP, T, W, M, (D & ~(M - 1)), D>(x, t);
      if constexpr (HAVE) vapply<OP, T, W>(res, res, t);
      else res = t;
      scan_reg_bits<OP, T, W, Q, M * 2, true>(x, res);
    } else {
      scan_reg_bits<OP, T, W, Q, M * 2, HAVE>(x, res);
    }
  }
}

template <class OP, class T, int W, int Q, bool EXCL>
__device__ __forceinline__ void scan_reg(const Vec<T, W>* x, Vec<T, W>& res) {
  if constexpr (!EXCL) res = x[Q];
  scan_reg_bits<OP, T, W, Q, 1, !EXCL>(x, res);
}

// every rank's result at vector/element e of my chunk -> rank q's recvbuf
template <class OP, class T, int W, bool EXCL, int Q = 0>
__device__ __forceinline__ void scan_pp_store(const ScanArgs& A, const Vec<T, W>* x, long long e) {
  if constexpr (Q < 8) {
    if (Q < A.pv.n) {
      if constexpr (!(EXCL && Q == 0)) {
        Vec<T, W> r;
        scan_reg<OP, T, W, Q, EXCL>(x, r);
        stv<T, W>(wave_uniform((T*)A.zrecv[Q]) + e, r);
      }
      scan_pp_store<OP, T, W, EXCL, Q + 1>(A, x, e);
    }
  }
}

// [lo, hi) of my chunk.  Vector path: U 16-B vectors per thread, all 8 x U
// leaf loads issued before any arithmetic as buffer loads whose descriptor
// has no records for an absent leaf (rank >= n, or the top rank's own data in
// Exscan): such a load returns zeros without touching memory, so no branch
// sits between the loads.  Unaligned operands and the ragged tail go element
// by element.
template <class OP, class T, bool EXCL, int U>
__device__ __forceinline__ void scan_pp_span(const ScanArgs& A, long long lo, long long hi) {
  constexpr int W = VecW<T>::v;
  const int n = A.pv.n, nl = EXCL ? n - 1 : n;
  const long long tid = threadIdx.x, nt = blockDim.x, es = A.esize;
  bool vec = true;
#pragma unroll
  for (int s = 0; s < 8; ++s)
    if (s < n) vec &= ((((uintptr_t)A.src[s]) | ((uintptr_t)A.zrecv[s])) & 15) == 0;
  long long e0 = lo;
  if (vec) {
    // descriptors cover at most 1 GiB (32-bit offsets), rebuilt per piece
    constexpr long long kPiece = (1ll << 30) / 16;
    const long long nv_all = (hi - lo) / W;
    for (long long p0 = 0; p0 < nv_all; p0 += kPiece) {
      const long long nv = lmin(nv_all - p0, kPiece), base = lo + p0 * W;
      // descriptors from wave-uniform values (read from LDS, the compiler
      // cannot prove them uniform and would wrap every load in a waterfall loop)
      __amdgpu_buffer_rsrc_t rs[8];
      const int bytes = __builtin_amdgcn_readfirstlane((int)(nv * 16));
#pragma unroll
      for (int s = 0; s < 8; ++s)
        rs[s] = __builtin_amdgcn_make_buffer_rsrc((void*)wave_uniform(s < nl ? A.src[s] + base * es : A.src[0]), 0,
                                                  s < nl ? bytes : 0, 0x00020000);
      for (long long v0 = tid; v0 < nv; v0 += U * nt) {
        Vec<T, W> x[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int s = 0; s < 8; ++s)
            *reinterpret_cast<u32x4*>(x[u][s].x) =
                __builtin_amdgcn_raw_buffer_load_b128(rs[s], (int)((v0 + u * nt) * 16), 0, MPIGX_NT ? 2 : 0);
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (v0 + u * nt < nv) scan_pp_store<OP, T, W, EXCL>(A, x[u], base + (v0 + u * nt) * W);
      }
    }
    e0 = lo + nv_all * W;
  }
  for (long long e = e0 + tid; e < hi; e += nt) {
    Vec<T, 1> x[8] = {};
#pragma unroll
    for (int s = 0; s < 8; ++s)
      if (s < nl) x[s].x[0] = ((const T*)A.src[s])[e];
    scan_pp_store<OP, T, 1, EXCL>(A, x, e);
  }
}

template <class OP, class T>
__device__ __forceinline__ int scan_pp_body(const ScanArgs& A) {
  const PeerView& pv = A.pv;
  const int b = blockIdx.x, r = pv.rank;
  uint64_t ep = pv.epoch;
  int ab;
  if (!zc_enter(pv, ep++, &ab)) return 0;  // every rank's buffers ready, one view
  if (!ab) {
    const long long c0 = lmin((long long)r * A.chunk, A.count), c1 = lmin(c0 + A.chunk, A.count);
    const long long lo = lmin(c0 + (long long)b * A.slice, c1), hi = lmin(lo + A.slice, c1);
    // preconditions of every access below, checked instead of trusted (round
    // 3 saw an aperture violation in this kernel): the partition, non-null
    // operands, and the extents — my chunk's end inside every contribution I
    // load and every recvbuf I store into, against the sizes of the
    // allocations the peers exported for this view.  The verdict depends on
    // the chunk, not the block, so every block of this rank reaches it; a
    // violation stores nothing, fails the call here (MPI_ERR_INTERN) and sets
    // the abort bit of the exit barrier, which every block of every peer
    // receives — no rank completes with a chunk of its recvbuf unwritten.
    const int nl = A.exclusive ? pv.n - 1 : pv.n;
    const long long end = c1 * A.esize;
    bool sane = pv.n >= 2 && pv.n <= 8 && r < pv.n && 0 <= c0 && c0 <= lo && lo <= hi && hi <= c1 &&
                c1 <= A.count;
    for (int q = 0; q < pv.n; ++q)
      sane &= A.src[q] != nullptr && A.zrecv[q] != nullptr && end <= A.zr_avail[q] && (q >= nl || end <= A.zs_avail[q]);
    if (!sane) {
      ab = 1;
      if (threadIdx.x == 0) {
        __hip_atomic_store(pv.err, kErrProtocol, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (pv.stamps) pv.stamps[(size_t)b * 8 + 6] = 0xBAD0000000000000ull | (uint64_t)(hi - lo);
      }
    } else {
      constexpr int U = vec_regs<T>() <= 4 ? 2 : 1;
      if (A.exclusive) scan_pp_span<OP, T, true, U>(A, lo, hi);
      else scan_pp_span<OP, T, false, U>(A, lo, hi);
    }
  }
  rank_barrier(pv, ep++, &ab);  // publishes my stores into the peers' recvbufs
  return ab;
}

template <class OP, class T>
__device__ __forceinline__ int scan_body(const ScanArgs& A);

template <class OP, class T>
__global__ __launch_bounds__(kThreads) void scan_kernel(ScanArgs A) {
  // src[] / ll_push[] are indexed by rank at run time: staged in LDS like
  // FoldArgs (from the kernarg segment the compiler copied the whole block to
  // scratch in every thread)
  __shared__ ScanArgs sA;
  static_assert(sizeof(ScanArgs) % 4 == 0, "ScanArgs word copy");
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&A);
  uint32_t* d = reinterpret_cast<uint32_t*>(&sA);
  for (unsigned i = threadIdx.x; i < sizeof(ScanArgs) / 4; i += blockDim.x) d[i] = w[i];
  __syncthreads();
  kernel_started(sA.pv);
  stamp(sA.pv, 0);
  const int ab = sA.pp ? scan_pp_body<OP, T>(sA) : scan_body<OP, T>(sA);
  signal_done(sA.pv, ab);
}

template <class OP, class T>
__device__ __forceinline__ int scan_body(const ScanArgs& A) {  // returns the abort verdict
  constexpr int W = VecW<T>::v;
  const PeerView& pv = A.pv;
  const int b = blockIdx.x;
  const long long lo = lmin((long long)b * A.slice, A.count), hi = lmin(lo + A.slice, A.count);
  uint64_t ep = pv.epoch;
  int ab = 0;
  if (A.ll) {
    // small messages: every rank's slice b arrives as LL lines (device.hpp
    // ll_exchange; every rank sends to every rank so the area parities stay
    // safe), unpacked into my arena slots = src[]; no barrier at all
    const long long es = A.esize, bytes = A.count * es;
    const long long l0 = (lo * es) / 8, l1 = hi > lo ? (hi * es + 7) / 8 : l0;
    if (!ll_exchange(pv, A.ll_push, A.ll_in, A.ll_stride, A.ll_flag, (const char*)A.send, bytes, l0, l1,
                     pv.stage[pv.rank], A.ll_ustride, pv.n, pv.rank, pv.err))
      return 0;
  } else if (A.zc) {
    // zero-copy (out of place only): the operands are the ranks' sendbufs
    if (!zc_enter(pv, ep++, &ab)) return 0;
  } else {
    T* mine = (T*)pv.stage[pv.rank];
    block_copy((char*)(mine + lo), (const char*)A.send + lo * A.esize, (hi - lo) * A.esize);
    if (!rank_barrier(pv, ep++)) return 0;
  }
  T* recv = (T*)A.recv;
  const bool skip = ab || (A.exclusive && pv.rank == 0);  // rank 0's Exscan recvbuf untouched
  if (!skip) {
    const long long tid = threadIdx.x, nt = blockDim.x;
    long long s = lo;
    if (((uintptr_t)recv & 15) == 0) {
      const long long nv = (hi - lo) / W;
      for (long long i = tid; i < nv; i += nt) {
        Vec<T, W> r;
        bool have;
        scan_at<OP, T, W>(A, lo + i * W, r, have);
        stv<T, W>(recv + lo + i * W, r);
      }
      s = lo + nv * W;
    }
    for (long long e = s + tid; e < hi; e += nt) {
      Vec<T, 1> r;
      bool have;
      scan_at<OP, T, 1>(A, e, r, have);
      recv[e] = r.x[0];
    }
  }
  if (A.ll) return 0;
  rank_barrier_exit(pv, ep++, &ab);
  return ab;
}

}  // namespace mpigx

namespace mpigx {

// ---------------------------------------------------------------------------
// acc_kernel<OP,T>: RMA Accumulate / Get_accumulate / Fetch_and_op applied by
// the target rank to its own window (rma.cpp) — the origin's data is pulled
// over xGMI and the op is fused into the pull, so the only GPU writing the
// window is the one that owns it.  res (old values) is target-local scratch.
// ---------------------------------------------------------------------------
struct OpReplace { static constexpr int code = O_REPLACE; };
struct OpNoop { static constexpr int code = O_NOOP; };

template <class OP, class T>
__global__ __launch_bounds__(kThreads) void acc_kernel(AccArgs A) {
  const T* __restrict__ src = reinterpret_cast<const T*>(A.src);
  T* __restrict__ dst = reinterpret_cast<T*>(A.dst);
  T* __restrict__ res = reinterpret_cast<T*>(A.res);
  pull_acquire(A.coherent);
  const long long n = A.count, nt = (long long)gridDim.x * blockDim.x;
  constexpr int U = 4;  // independent elements in flight per thread
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * nt < n; i += U * nt) {
    T t[U], s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      t[u] = dst[i + u * nt];
      if constexpr (OP::code != O_NOOP) s[u] = src[i + u * nt];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (res) res[i + u * nt] = t[u];
      if constexpr (OP::code == O_REPLACE) dst[i + u * nt] = s[u];
      else if constexpr (OP::code != O_NOOP) dst[i + u * nt] = OP::apply(t[u], s[u]);
    }
  }
  for (; i < n; i += nt) {
    const T t = dst[i];
    if (res) res[i] = t;
    if constexpr (OP::code == O_REPLACE) dst[i] = src[i];
    else if constexpr (OP::code != O_NOOP) dst[i] = OP::apply(t, src[i]);
  }
  pull_release(A.coherent);
}

}  // namespace mpigx
