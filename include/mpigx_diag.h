/*
 * mpigx_diag.h — diagnostic exports of libmpigx (not part of the MPI-facing
 * ABI in mpigx.h; nothing MPI.jl ccalls).  Used by bench.py, tools/ and the
 * GPU tests: per-block phase stamps, signal-slot / mapping checks, the
 * tuners' and zero-copy views' statistics, and bandwidth probes.
 */
#ifndef MPIGX_DIAG_H
#define MPIGX_DIAG_H

#include "mpigx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostic: per-block phase timestamps of the collective kernels (100 MHz
 * device wall clock).  stamps = device buffer of >= 1024 x 8 u64 (NULL
 * disables); slot [block][k]: 0 entry, 1 after the entry barrier, 2 after the
 * reduce-scatter, 3 after the middle barrier, 4 after the allgather, 5 after
 * the exit barrier.  Local (not collective). */
int mpigx_comm_set_stamps(mpigx_comm_t comm, void *stamps);
/* Diagnostic: barrier slot row `block` as this rank sees it.  mine[q] = the
 * word peer q last stored into MY signal array (my own mapping); theirs[q] =
 * the word I last stored into peer q's array, read back through MY mapping of
 * it.  A peer whose mine[] entry on its side differs from my theirs[] entry
 * for it sees another memory than the one I write.  Local. */
int mpigx_comm_diag_slots(mpigx_comm_t comm, int block, unsigned long long *mine, unsigned long long *theirs);
/* Diagnostic, local, never waits on the device (callable from a watchdog
 * thread): out[0] = my stream busy (0 idle, 1 busy, 2 error), [1] completion
 * word, [2] the word awaited, [3] blocks counted so far, [4] launch sequence,
 * [5] epoch, [6] my control-plane allgather sequence, [7] the lowest one any
 * rank has posted. */
int mpigx_comm_diag_state(mpigx_comm_t comm, unsigned long long *out);
/* Diagnostic, COLLECTIVE: every rank writes `nonce` ^ rank into its own
 * signal arrays (through its own mapping), then reads every peer's through
 * its IPC mapping of it.  *stale = bitmask of the ranks whose array some rank
 * (any) saw without the new nonce: that peer's mapping and the owner's no
 * longer alias one memory.  Every rank gets the same mask. */
int mpigx_comm_diag_mapcheck(mpigx_comm_t comm, unsigned long long nonce, unsigned *stale);
/* Which signalling protocol each peer pair runs (DESIGN §3 "one memory type
 * per writer / reader pair"): bit q of *rw_mask = rank q writes my
 * ordinary-memory signal array / LL area (a same-GPU peer); clear = my
 * uncached ones (a peer on another GPU, or every peer under
 * MPIGX_PEER_MEM=xdev).  Bit q of *same_device = rank q runs on my GPU.
 * Own bit set in both.  Local. */
int mpigx_comm_diag_peer_mem(mpigx_comm_t comm, unsigned *rw_mask, unsigned *same_device);
/* Fault injection (tests): mark this rank's communicator failed, as an
 * internal error would — every later call on it returns MPIGX_ERR_OTHER, and
 * the peers' waits on it (host gate, control-plane exchanges, a blocking
 * collective's watch) fail within a second instead of waiting for a rank
 * that will not come.  Local. */
int mpigx_comm_diag_break(mpigx_comm_t comm);
/* Read-only stream of `nin` (1, 2, 4 or 8) device buffers of `bytes` bytes
 * each (16-B aligned), in the layout of the config-2 fold kernel
 * (fold_local_kernel, 4 x 16 B per thread per input in flight) with the fold
 * and its stores removed: the box's own HBM read ceiling for that kernel,
 * which bench.py times beside it (roofline.peak_measured).  `sink` = a device
 * buffer of >= 4 KiB that is never written in practice.  Enqueued on
 * `stream` (hipStream_t; NULL = null stream), asynchronous. */
int mpigx_read_probe(const void *const *in, int nin, long long bytes, void *sink, void *stream);
/* The same stream with the fold's writes put back: reads the `nin` inputs in
 * the fold's layout and stores, per 16-B vector, the XOR of the nin loaded
 * vectors into `out` (`bytes` bytes, 16-B aligned) with the fold's
 * write-through stores — config 2's read/write mix (8 reads : 1 write) with
 * no arithmetic to speak of: the box's ceiling for that kernel
 * (roofline.peak_measured in bench.py).  Asynchronous on `stream`. */
int mpigx_mix_probe(const void *const *in, int nin, long long bytes, void *out, void *stream);
/* Zero-copy paths (user buffers mapped by the peers over IPC): how many
 * launches ran on a cached view without any host exchange, and how many
 * host exchanges of buffer registrations there were.  Diagnostic. */
int mpigx_comm_zc_stats(mpigx_comm_t comm, unsigned long long *optimistic_hits,
                        unsigned long long *exchanges);
/* Host time of the last collective call from its entry to its first kernel
 * launch (argument checks, planning, zero-copy view resolution).  Diagnostic. */
int mpigx_comm_host_stats(mpigx_comm_t comm, double *prelaunch_us);
/* Large (zero-copy-sized) Allreduce algorithm the communicator measured and
 * chose (MPIGX_AR_TUNE): *choice = -1 undecided, 0 pull two-shot, 1 push
 * two-shot, 2 pull-push two-shot (MPIGX_ALGO_PULLPUSH); *pull_ns_per_mib /
 * *push_ns_per_mib = this rank's measured device time per MiB of message
 * (0 = not measured).  Diagnostic. */
int mpigx_comm_ar_choice(mpigx_comm_t comm, int *choice, double *pull_ns_per_mib, double *push_ns_per_mib);
/* The same with every candidate's cost: ns_per_mib[0..2] = pull, push,
 * pull-push (this rank's device ns per MiB; 0 = not measured).  Diagnostic. */
int mpigx_comm_ar_costs(mpigx_comm_t comm, int *choice, double *ns_per_mib);
/* Smaller collectives (below the zero-copy size), size class
 * log2_bytes = floor(log2(message bytes)) + 64 * kind (kind 0 Allreduce,
 * 1 Bcast, 2 Allgather, 3 Alltoall; the byte movers' class is the per-rank
 * block): the algorithm the communicator measured and chose (*choice = -1
 * undecided / not tuned, 0 LL step, 1 staged one-shot (byte movers: the
 * staged copy), 2 staged two-shot, 3 LL two-shot) and this rank's best device
 * time per MiB of each (ns_per_mib[4], 0 = not a candidate or not measured).
 * Diagnostic. */
int mpigx_comm_tune_class(mpigx_comm_t comm, int log2_bytes, int *choice, double *ns_per_mib);

/* Diagnostic (bench roofline denominator): every rank pulls `bytes` from
 * every peer's staging arena at once (kind 0: aggregate xGMI ingress) or
 * from rank+1 only (kind 1: one link).  *seconds = device time of the pull
 * (includes one cross-rank barrier).  Collective. */
int mpigx_comm_probe(mpigx_comm_t comm, int kind, long long bytes, double *seconds);

#ifdef __cplusplus
}
#endif
#endif /* MPIGX_DIAG_H */
