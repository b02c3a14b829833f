// common.hpp — definitions shared by the host runtime (mpigx.cpp) and the HIP
// kernels (kern_*.hip): element representations, op codes, kernel argument
// blocks.  The MPICH handle <-> representation mapping mirrors
// deps/consts_mpich.jl:47-72 and src/datatypes.jl:29-60.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "../../include/mpigx.h"

namespace mpigx {

constexpr int kMaxRanks = MPIGX_MAX_RANKS;
constexpr int kMaxBlocks = 1024;      // signal slots per rank per barrier
// One 128-B cache line per signal slot [block][rank]: a peer writes its slot
// through its IPC import of my array, which is not uncached there, and a
// line shared by several writers came back with one writer's stale copy of
// another's word (8 ranks on one GPU: rank 0 saw the root's previous epoch
// forever while every other rank saw its new one).
constexpr int kSigStride = 16;        // u64 words per slot
__host__ __device__ constexpr size_t sig_index(size_t block, int rank) {
  return (block * kMaxRanks + (size_t)rank) * kSigStride;
}
constexpr int kThreads = 256;         // threads per block of every kernel

// Element representations.  Several MPI handles share one (INT == INT32_T,
// LONG == INT64_T, CHAR == SIGNED_CHAR == INT8_T, BYTE == UINT8_T ...).
enum Rep : int {
  R_I8 = 0, R_U8, R_I16, R_U16, R_I32, R_U32, R_I64, R_U64,
  R_F32, R_F64, R_C64, R_C128, R_BF16, R_COUNT, R_NONE = -1
};

// Built-in ops (src/operators.jl:22-37), dense indices.
enum OpCode : int {
  O_SUM = 0, O_PROD, O_MIN, O_MAX, O_LAND, O_LOR, O_LXOR, O_BAND, O_BOR, O_BXOR, O_COUNT,
  O_NONE = -1
};

// RMA-only ops (MPI_REPLACE / MPI_NO_OP, mpi.h:322-323): accumulate kernels only.
constexpr int O_REPLACE = 16;
constexpr int O_NOOP = 17;

// Fold shapes (template parameter of the fold code): SH_PRE — pre-step
// partners possible (n not a power of two); SH_POW2 — none; SH_FULL — none
// and every one of the NMAX leaves present (no runtime guards at all).
enum Shape : int { SH_PRE = 0, SH_POW2 = 1, SH_FULL = 2 };

// Allgather half of the dedicated zero-copy two-shot (kernels.hpp
// ar_zc_kernel): pull the peers' reduced chunks, or have each owner store its
// reduced slice into every rank's recvbuf.
constexpr int AG_PULL = 0, AG_PUSH = 1;

// The local fold's shape and 16-B vectors per thread — ONE rule for the host
// (grid size, FoldArgs.lu) and the launcher (instantiation).  SH_FULL only at
// NMAX 8 (the 8-buffer headline; n = 16 takes SH_POW2).  U = 4 measured best
// or tied on three MI355X boxes at 256 MiB (tools/fold_tune.hip,
// profiles/r02_fold_tune*.json); bf16 MIN/MAX keep U = 1 (their
// owner-dispatched trees need the VGPRs).
constexpr int fold_shape(int sched, int nmax, int ntree, int rem) {
  return (sched == 0 && rem > 0) ? SH_PRE : (nmax == 8 && ntree == 8) ? SH_FULL : SH_POW2;
}
constexpr int local_u_max(int rep, int op, int shape) {
  return shape != SH_FULL ? 1 : (rep == R_BF16 && (op == O_MIN || op == O_MAX)) ? 1 : 4;
}
// ... and by size: at U = 4 a 1 MiB input made 64
// blocks of 256 threads, a quarter of the CUs.  Measured (graph-replayed
// launches, profiles/r06b_local_u_sweep.json, r06m_local_variant_u.json):
// U = 4 is fastest (or tied) from 4 MiB of f32 per input up — 256 blocks,
// one per CU — and U = 1 below (1 MiB: 2.3 vs 4.5 us); U = 2 was never the
// fastest at any size or for any (type, op).  So U = 4 from 256 Ki 16-B
// vectors per input, 1 below.
constexpr long long kLocalU4MinVec = 4ll * kThreads * 256;
constexpr int local_u(int rep, int op, int shape, long long nvec) {
  return (local_u_max(rep, op, shape) >= 4 && nvec >= kLocalU4MinVec) ? 4 : 1;
}

// Fold schedule (template parameter of the fold kernels).
enum Sched : int { S_TREE = 0, S_LINEAR = 1 };

// What one fold-kernel launch does (runtime, uniform).
enum FoldMode : int {
  M_LOCAL = 0,        // out = fold(src[*]) over [0,count): config 2, no peers
  M_AR_ONESHOT = 1,   // copy-in, barrier, every rank folds everything, barrier
  M_AR_TWOSHOT = 2,   // copy-in, barrier, RS (own chunk), barrier, AG, barrier
  M_RED_ONESHOT = 3,  // copy-in, barrier, root folds everything, barrier
  M_RED_TWOSHOT = 4,  // copy-in, barrier, RS (own chunk), barrier, root gathers, barrier
  M_AR_ZC = 5,        // zero-copy two-shot: barrier, RS straight from the peers' (IPC-
                      // registered) send buffers into my recvbuf, barrier, AG from the
                      // peers' recvbufs, barrier
  M_AR_PUSH = 6,      // push two-shot: write my chunk p into rank p's arena slot [me],
                      // barrier, fold my chunk from my own slots (local HBM), write the
                      // result into every rank's recvbuf (IPC-mapped), barrier
  M_RED_ZC = 7,       // zero-copy Reduce: barrier, RS of my chunk straight from every
                      // rank's sendbuf into my arena (the root: its recvbuf), barrier,
                      // the root gathers every chunk from the arenas, barrier
  M_AR_LL = 8,        // small Allreduce, no barrier: push my bytes as flag-carrying
                      // lines into every peer's LL area, poll my own area for every
                      // peer's lines, unpack them into my arena, fold locally
  M_RED_LL = 9,       // small Reduce: the same exchange (every rank receives from every
                      // rank, which keeps the area parities safe), only the root folds
  M_AR_LL2 = 10,      // medium Allreduce, two LL exchanges and no barrier: chunk p of
                      // my sendbuf -> rank p (LL half 0), fold my chunk, my reduced
                      // chunk -> every rank (LL half 1), unpacked into recvbuf
};

// LL ("low-latency") lines of M_AR_LL: 16 bytes = two 8-byte halves
// {4 payload bytes, 4-byte flag}, each stored with ONE 64-bit store, so a
// receiver that sees the launch's flag in a half has that half's payload —
// no fence and no separate signal.  A rank's LL area (uncached HBM,
// IPC-mapped by every peer) is [2 parities][kMaxRanks senders][ll_stride].
constexpr int kLLLine = 16;
// Payload bytes per block slice of an LL exchange are a multiple of this: 64
// payload bytes = 8 LL lines = one 128-B cache line of the receiver's area, so
// no two blocks of a sender (possibly on two XCDs, each with its own L2 copy
// of the line) write parts of one cache line.
constexpr int kLLAlign = 64;

// Copy-kernel modes (Bcast / Allgather / Alltoall / Barrier).
//   C_BCAST     : every non-root pulls the whole buffer from the root (small)
//   C_BCAST_SAG : scatter + allgather — rank q pulls chunk q from the root, then
//                 every rank pulls chunk p from rank p (large, n >= 3): each
//                 xGMI link carries <= 2S/n instead of each root link carrying S
enum CopyMode : int {
  C_BCAST = 0, C_ALLGATHER = 1, C_ALLTOALL = 2, C_BARRIER = 3, C_PROBE_ALL = 4, C_PROBE_ONE = 5,
  C_BCAST_SAG = 6,
  C_ALLTOALL_ZC = 7,  // zero-copy: pull block r straight from every rank's (IPC-mapped) sendbuf
  C_ALLGATHER_ZC = 8, // zero-copy: pull block p straight from rank p's sendbuf (or its recvbuf block p)
  C_BCAST_ZC = 9,     // zero-copy: every non-root pulls the root's buffer
  C_BCAST_SAG_ZC = 10, // zero-copy scatter + allgather between the user buffers
  // LL (small messages, no barrier; device.hpp ll_exchange's protocol): every
  // rank pushes lines into every peer's LL area — its data, or one token line
  // when it has nothing to send (Bcast non-roots), so every rank receives from
  // every rank and the area parities stay safe — and unpacks what it needs
  // straight into the user buffer
  C_BCAST_LL = 11, C_ALLGATHER_LL = 12, C_ALLTOALL_LL = 13,
  // zero-copy relay (large, n >= 3): the non-roots own the n - 1 chunks; the
  // owner of chunk i reads it from the root's buffer once and stores it into
  // its own and every other non-root's buffer in the same pass
  C_BCAST_RELAY_ZC = 14
};

// Per-call view of the communicator, passed by value to every kernel.
struct PeerView {
  int rank;
  int n;
  uint64_t epoch;              // first barrier epoch of this launch (monotone)
  uint64_t timeout_ticks;      // wall_clock64 ticks (100 MHz) before giving up
  uint64_t* sig[kMaxRanks];    // signal array [kMaxBlocks][kMaxRanks] of every rank
  unsigned* err;               // host-visible error word (0 = ok)
  unsigned long long* done;    // host-visible completion word (seq << 1 | aborted), or null
  unsigned long long* dcount;  // device-memory block arrival counter (monotone)
  unsigned long long dbase;    // dcount value before this launch
  unsigned long long seq;      // value the last block of this launch stores to *done
  char* stage[kMaxRanks];      // staging arena base of every rank (IPC-mapped)
  // zero-copy launches (mpigx.cpp zc_run)
  unsigned zc_key;             // id of the buffer-mapping view this launch uses
  int zc_bad;                  // 1: this rank has no valid view (the launch aborts everywhere)
  unsigned long long* stamps;  // diagnostic phase timestamps [block][8] (null: off)
  // dynamic slice hand-out (ar_zc_kernel AG_PUSH, dyn): monotone counters at
  // dcount[1] (tickets) and dcount[2] (finished blocks); their values before
  // this launch
  unsigned long long wbase;
  unsigned long long fbase;
  // Two signal arrays and two LL areas per rank (DESIGN §3 "one memory type
  // per pair"): peers on MY device write into my ordinary (cached, RW)
  // array, peers on other devices into my uncached one; bit q of rw_mask =
  // rank q is on my device (my own bit always set).  sig[q] above already
  // points at the array rank q expects from me.
  unsigned rw_mask;
  uint64_t* sig_uc;            // my uncached signal array (cross-device writers)
  uint64_t* sig_rw;            // my cached signal array (same-device writers and myself)
  const char* ll_rw;           // my cached LL area at this launch's parity (same-device senders)
  // Waiting for a late peer (round 5, DESIGN §3 "a late rank"): every
  // launch's polls give up only when its host stores a nonzero `cancel` word
  // (make_view sets it for every launch), never on time alone.  A blocking
  // call's host watches its peers while it waits (mpigx.cpp finish); a
  // stream-ordered launch's peers are watched by the process-wide watcher
  // (watch_peers).  Either cancels when a peer's process is gone, its
  // communicator failed, a peer's launch is stuck behind other communicators'
  // kernels (never started although enqueued), or — blocking calls — every
  // rank's kernel has sat in the launch past the timeout.  Block 0 stores
  // `kseq` (this launch's number, the same on every rank) into `started` at
  // entry, which tells the host — and through the shm block its peers —
  // which launch its GPU is in.
  unsigned long long kseq;
  unsigned long long* started;
  const unsigned* cancel;
  // Integrity of the argument block (zero-copy launches, device.hpp
  // zc_enter): a checksum over the block's first args_words 32-bit words (this
  // PeerView is its first member; the args_sum word itself counted as 0),
  // checked before any pointer in it is used.  0 words = unchecked.
  unsigned args_words;
  unsigned args_sum;
};
// Checksum of an argument block (host and device; mpigx.cpp seal_args,
// device.hpp args_fault): word i mixed with its index, summed — a permuted,
// stale or partly overwritten block does not match.
__host__ __device__ inline unsigned args_mix(unsigned w, unsigned i) {
  unsigned x = w ^ (i * 0x9E3779B9u);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// the array peer `from` writes its words for me into
__host__ __device__ inline uint64_t* sig_in(const PeerView& pv, int from) {
  return ((pv.rw_mask >> from) & 1u) ? pv.sig_rw : pv.sig_uc;
}
// sender p's LL lines for me at this launch's parity: `in` = my uncached area
__host__ __device__ inline const char* ll_from(const PeerView& pv, const char* in, int p, long long stride) {
  return (((pv.rw_mask >> p) & 1u) ? pv.ll_rw : in) + (long long)p * stride;
}

// Fold-kernel arguments.  Sources/partition are resolved on the host.
struct FoldArgs {
  PeerView pv;
  int mode;            // FoldMode
  int esize;           // element size in bytes
  long long count;     // elements in this launch (round)
  long long gbase;     // element offset of this round in the whole message
  long long chunk;     // elements per rank chunk (two-shot), multiple of vec
  long long slice;     // elements per block slice, multiple of vec
  // fold schedule
  int ntree;           // active tree leaves (binomial: n; pre-step tree: pof2)
  int rem;             // pre-step pairs (leaf s < rem folds src2[s] into src[s])
  int owner_mode;      // 0: lower subtree is inout (binomial); 1: Rabenseifner owner roles
  int pof2_log;        // log2(pof2) for owner computation
  long long blk_len;   // Rabenseifner block length (count_total / pof2)
  double blk_inv;      // 1.0 / blk_len (owner_block: reciprocal + one-step fix-up)
  int root;            // reduce root (rank)
  // leaf -> rank maps for collective modes (staging-sourced)
  signed char leaf_rank[kMaxRanks];
  signed char leaf2_rank[kMaxRanks];
  // LOCAL mode sources / destinations (user pointers)
  const void* src[kMaxRanks];
  const void* src2[kMaxRanks];
  const void* send;    // collective modes: my send buffer (may be == recv)
  void* recv;          // output
  char* zc_recv[kMaxRanks];  // M_AR_ZC / M_AR_PUSH: every rank's recvbuf (IPC-mapped; mine = recv)
  long long slot_bytes;      // M_AR_PUSH: arena bytes per source slot (chunk bytes, 16-B multiple);
                             // M_AR_LL: arena bytes per unpacked contribution
  // M_AR_LL: zc_recv[p] = rank p's LL area (this launch's parity) at my sender
  // slot; ll_in = my own area (same parity), sender q's lines at q * ll_stride
  const char* ll_in;
  long long ll_stride;
  unsigned ll_flag;    // this launch's flag (never 0, never a stale flag of the same parity)
  int dyn;             // ar_zc_kernel AG_PUSH: 1 = slices of `slice` elements handed out by a ticket counter
  int own;             // M_RED_ZC (ar_zc_kernel): index of the chunk this rank folds (root: none at n >= 3)
  // ar_zc_kernel AG_PUSH: bytes of rank q's allocation from zc_recv[q] to its
  // end (the agreed view's exported sizes): the remote stores are checked
  // against them before any is made
  long long zc_avail[kMaxRanks];
  int lu;              // M_LOCAL: 16-B vectors per thread the host sized the grid for (local_u)
};

// Ring reduce-scatter + allgather (MPIGX_ALGO=ring; kernels.hpp ring_kernel).
// The message is split into nch contiguous parts, part k travels its own ring
// of stride stride[k] (coprime with n: 0, s, 2s, ... visits every rank), and
// each part is cut into n chunks.  Chunk c of a part is folded along its
// ring starting at the rank in ring position c: partial = OP(partial, x_q),
// the partial as inout; the block of every rank that owns slice b of channel
// k synchronises only with block b of its two ring neighbours.
constexpr int kMaxRings = 4;
struct RingArgs {
  PeerView pv;
  int esize;
  int nch;                       // rings (channels): blocks b with b % nch == k run ring k
  int stride[kMaxRings];         // ring k: rank at position i is (i * stride[k]) mod n
  int pos[kMaxRings];            // my position in ring k
  long long count;               // elements in this launch (round)
  long long part;                // elements per ring part (multiple of n*vec)
  long long chunk;               // elements per chunk of a part (multiple of vec)
  long long slice;               // elements per block slice of a chunk (multiple of vec)
  const char* zsend[kMaxRanks];  // every rank's sendbuf (zero-copy view; + round offset)
  char* zrecv[kMaxRanks];        // every rank's recvbuf (zero-copy view; + round offset)
};

struct CopyArgs {
  PeerView pv;
  int mode;            // CopyMode
  int root;
  long long bytes;     // bytes per rank contribution (bcast: whole buffer)
  long long slice;     // bytes per block slice (multiple of 16)
  long long total;     // user-buffer stride between rank blocks (bytes of one full block)
  long long sstride;   // alltoall: staging stride between rank blocks (bytes rounded up to 16)
  long long chunk;     // bcast-sag: bytes per rank chunk (multiple of 16)
  const char* zsrc[kMaxRanks];  // alltoall-zc: every rank's sendbuf (IPC-mapped; mine = send)
  const void* send;
  void* recv;
  char* ll_push[kMaxRanks];     // LL modes: rank p's LL area (parity) at my sender slot
  const char* ll_in;            // my own LL area (parity)
  long long ll_stride;
  unsigned ll_flag;
  int ll_pad;
};

// Personalised exchange (Gather(v) / Scatter(v) / Allgatherv / Alltoallv):
// every rank stages up to n byte ranges of its send buffer into fixed slots
// of its arena (slot j at kSlotBase + j*R), then pulls from each peer p the
// range in p's slot p_slot[p].  Both ends of a transfer know its length, so
// both cut it into the same G per-block slices.  One launch = one round of
// at most R bytes of every range.
constexpr long long kSlotBase = 256;
struct VArgs {
  PeerView pv;
  long long R;          // slot size (bytes, multiple of 16)
  long long round_off;  // byte offset of this round inside every range
  int G;                // blocks (identical on every rank)
  int ncopy;            // copy-in ranges: send + c_src[j] (c_len[j] bytes total) -> my slot c_slot[j]
  int c_slot[kMaxRanks];
  long long c_src[kMaxRanks];
  long long c_len[kMaxRanks];
  long long p_len[kMaxRanks];  // bytes to pull from rank p (0: nothing)
  int p_slot[kMaxRanks];       // ... out of p's slot p_slot[p]
  long long p_dst[kMaxRanks];  // ... into recv + p_dst[p]
  const char* send;
  char* recv;
};

// Point-to-point batch: up to kMaxXfer matched messages per launch.
constexpr int kMaxXfer = 16;
struct XferArgs {
  int nseg;
  int coherent;  // system-scope acquire at start / release at end (pull_fences())
  int blk0[kMaxXfer + 1];       // first block of each segment (prefix sums)
  char* dst[kMaxXfer];
  const char* src[kMaxXfer];
  long long bytes[kMaxXfer];
};

// RMA accumulate applied by the TARGET to its own window memory (rma.cpp):
//   res[i] = dst[i] (Get_accumulate / Fetch_and_op), dst[i] = OP(dst[i], src[i])
// with dst = inout (the target) and src = in (the origin's buffer, pulled over
// xGMI), MPICH's operand roles for MPI_Accumulate.
struct AccArgs {
  const void* src;
  void* dst;
  void* res;  // may be null
  long long count;
  int coherent;  // system-scope acquire at start / release at end (pull_fences())
};

// Derived datatypes (types.cpp): n blocks of len bytes at off + i*stride.
struct TypeRun {
  long long off, len, n, stride;
};
// Pack (typed -> contiguous) or unpack (contiguous -> typed) `units` W-byte
// units of a packed stream of instances of one type (extent apart).
struct PackArgs {
  char* typed;
  char* contig;
  const TypeRun* runs;   // device copy, typemap order
  const long long* pfx;  // packed bytes before run r within one instance (nruns + 1)
  int nruns;
  int w;
  int unpack;
  int coherent;
  long long size, extent, units;
};

struct ScanArgs {
  PeerView pv;
  int exclusive;
  int esize;
  int zc;              // 1: operands straight from the peers' sendbufs (src[], zero-copy view)
  int ll;              // 1: LL exchange (FoldArgs M_AR_LL fields below), src[] = my unpack slots
  long long count;
  long long slice;
  const void* send;
  void* recv;
  const char* src[kMaxRanks];  // rank q's contribution: its staging arena, or its sendbuf (zc)
  char* ll_push[kMaxRanks];
  const char* ll_in;
  long long ll_stride;
  long long ll_ustride;
  unsigned ll_flag;
  int pp;              // 1: pull-push zero-copy (n <= 8): rank r computes EVERY rank's result for chunk r
  long long chunk;     // pp: elements per rank chunk (multiple of vec)
  char* zrecv[kMaxRanks];  // pp: every rank's recvbuf (zero-copy view)
  // pp: bytes of rank q's allocation from src[q] / zrecv[q] to its end (the
  // agreed view's exported sizes), checked before any load or store
  long long zs_avail[kMaxRanks];
  long long zr_avail[kMaxRanks];
};

}  // namespace mpigx
