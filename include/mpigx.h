/*
 * mpigx.h — C ABI of libmpigx, the MI355X-native collective engine that
 * replaces libmpi for device-resident buffers under MPI.jl.
 *
 * Boundary: every MPI.jl collective on the hot path is one
 * `ccall((:MPI_<Coll>, libmpi), Cint, ...)`.  Each entry point below takes the
 * same arguments in the same order as the MPI function it replaces (count is
 * a C int = Julia `Cint`, datatype/op are the MPICH handle values MPI.jl
 * already passes as `Datatype(T).val` / `op.val`, deps/consts_mpich.jl:30-72),
 * with the MPI_Comm replaced by an mpigx_comm_t.  Return values are MPI error
 * classes (mpi.h:782-809) so MPI.jl's `@mpichk` (src/error.jl:5-8) wraps them
 * unchanged.  Plain pointers and sizes only; no torch or HIP types.
 *
 * Semantics: blocking and collective, like MPI (results complete and visible
 * to the host and the comm's stream on return), unless the communicator was
 * switched to stream-ordered mode with mpigx_comm_set_blocking(comm, 0).
 * Work is ordered after prior work on the comm's stream (default: the HIP
 * null stream), which is how a caller's producer kernels are respected.
 */
#ifndef MPIGX_H
#define MPIGX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MPIGX_VERSION_MAJOR 0
#define MPIGX_VERSION_MINOR 1

#define MPIGX_MAX_RANKS 16
#define MPIGX_UNDEFINED (-32766) /* MPI_UNDEFINED */

/* ---- error classes: identical to MPICH's (mpi.h:782-809) ---------------- */
#define MPIGX_SUCCESS 0
#define MPIGX_ERR_BUFFER 1
#define MPIGX_ERR_COUNT 2
#define MPIGX_ERR_TYPE 3
#define MPIGX_ERR_COMM 5
#define MPIGX_ERR_ROOT 7
#define MPIGX_ERR_OP 9
#define MPIGX_ERR_ARG 12
#define MPIGX_ERR_OTHER 15
#define MPIGX_ERR_INTERN 16
#define MPIGX_ERR_NO_MEM 34

/* ---- sentinels (deps/consts_mpich.jl:105) -------------------------------- */
#define MPIGX_IN_PLACE ((void *)(intptr_t)-1)

/* ---- datatypes: MPICH handle values (deps/consts_mpich.jl:47-72) --------- */
#define MPIGX_CHAR 1275068673
#define MPIGX_UNSIGNED_CHAR 1275068674
#define MPIGX_BYTE 1275068685
#define MPIGX_SHORT 1275068931
#define MPIGX_UNSIGNED_SHORT 1275068932
#define MPIGX_INT 1275069445
#define MPIGX_UNSIGNED 1275069446
#define MPIGX_LONG 1275070471
#define MPIGX_UNSIGNED_LONG 1275070472
#define MPIGX_FLOAT 1275069450
#define MPIGX_DOUBLE 1275070475
#define MPIGX_SIGNED_CHAR 1275068696
#define MPIGX_WCHAR 1275069454
#define MPIGX_INT8_T 1275068727
#define MPIGX_INT16_T 1275068984
#define MPIGX_INT32_T 1275069497
#define MPIGX_INT64_T 1275070522
#define MPIGX_UINT8_T 1275068731
#define MPIGX_UINT16_T 1275068988
#define MPIGX_UINT32_T 1275069501
#define MPIGX_UINT64_T 1275070526
#define MPIGX_C_FLOAT_COMPLEX 1275070528
#define MPIGX_C_DOUBLE_COMPLEX 1275072577
/* Extension: bf16 (no MPICH handle; MPI.jl maps BFloat16 to UINT16_T by size,
 * datatypes.jl:281-284).  Encoded like an MPICH builtin of size 2 with an
 * unused index.  Computed in fp32, RNE-rounded to bf16 after every op. */
#define MPIGX_BFLOAT16 1275068912

/* ---- ops: MPICH handle values (deps/consts_mpich.jl:30-45) --------------- */
#define MPIGX_MAX 1476395009
#define MPIGX_MIN 1476395010
#define MPIGX_SUM 1476395011
#define MPIGX_PROD 1476395012
#define MPIGX_LAND 1476395013
#define MPIGX_BAND 1476395014
#define MPIGX_LOR 1476395015
#define MPIGX_BOR 1476395016
#define MPIGX_LXOR 1476395017
#define MPIGX_BXOR 1476395018

/* ---- reduction order (deterministic modes) ------------------------------- */
/* MPICH: bit-exact with MPICH 3.3.2 on one node (binomial tree to rank 0 for
 * <= 2 KiB or count < pof2, else Rabenseifner pre-step + recursive halving,
 * including MIN/MAX operand roles).  LINEAR: rank-ordered left fold
 * ((x0 op x1) op x2) ...  Both are deterministic and identical on all ranks. */
#define MPIGX_ORDER_MPICH 0
#define MPIGX_ORDER_LINEAR 1

typedef struct mpigx_comm *mpigx_comm_t;
typedef struct {
    char internal[128];
} mpigx_unique_id_t;

/* ---- library ------------------------------------------------------------- */
int mpigx_get_version(int *major, int *minor);
/* MPI_Error_string analogue (src/error.jl:11-19). `len` in/out like MPI. */
int mpigx_error_string(int errorcode, char *string, int *resultlen);
/* Thread level the engine provides (environment.jl:111-162 Init_thread /
 * Query_thread; MPICH values THREAD_SINGLE 0 .. THREAD_MULTIPLE 3): 3.
 * Point-to-point and RMA calls may come from any thread at once (one
 * process-wide lock; blocking p2p calls release it between polls, as in
 * test/test_threads.jl's threaded Isend / Irecv); collectives: one call at a
 * time per communicator, as MPI requires.  Needs no GPU. */
#define MPIGX_THREAD_SINGLE 0
#define MPIGX_THREAD_FUNNELED 1
#define MPIGX_THREAD_SERIALIZED 2
#define MPIGX_THREAD_MULTIPLE 3
int mpigx_query_thread(int *provided);
/* Host-only validation of (datatype, op): MPIGX_SUCCESS, MPIGX_ERR_TYPE or
 * MPIGX_ERR_OP following MPICH's op x type matrix.  Needs no GPU. */
int mpigx_op_valid(int datatype, int op);
/* MPI_Type_size analogue for the predefined types.  Needs no GPU. */
int mpigx_type_size(int datatype, int *size);

/* ---- communicator (src/comm.jl:6-115; rank -> GPU binding) -------------- */
/* Rank 0 creates an id and distributes it out of band (host MPI_Bcast of
 * 128 bytes, torch.distributed, a file ...); then every rank calls
 * mpigx_comm_init_rank.  All ranks must be on one node. */
int mpigx_get_unique_id(mpigx_unique_id_t *id);
int mpigx_comm_init_rank(mpigx_comm_t *comm, int nranks, const mpigx_unique_id_t *id,
                         int rank, int device);
int mpigx_comm_free(mpigx_comm_t comm);
/* Local release (no barrier; MPI.jl's GC finalizers, comm.jl:82): waits for
 * this rank's queued work on `comm`, then unmaps the peers' memory and frees
 * its own.  Valid once this rank's last call on `comm` has returned — every
 * collective's final barrier retires the peers' accesses to this rank's
 * memory — so ranks may release at different times.  mpigx_comm_free is the
 * collective form (a barrier first). */
int mpigx_comm_release(mpigx_comm_t comm);
/* MPI_Comm_split — comm.jl:92-105.  Collective; color = MPIGX_UNDEFINED
 * (-32766) gives *newcomm = NULL.  Members keep the parent's device. */
int mpigx_comm_split(mpigx_comm_t comm, int color, int key, mpigx_comm_t *newcomm);
int mpigx_comm_rank(mpigx_comm_t comm, int *rank);
int mpigx_comm_size(mpigx_comm_t comm, int *size);
int mpigx_comm_device(mpigx_comm_t comm, int *device);
/* HIP stream (hipStream_t as void*) the comm's work is ordered on; NULL =
 * the null stream. */
int mpigx_comm_set_stream(mpigx_comm_t comm, void *stream);
/* 1 (default): every call returns with results complete.  0: calls only
 * enqueue on the stream (RCCL-like); mpigx_comm_synchronize reports errors.
 * Every rank of a communicator must use the same mode (the zero-copy
 * protocol differs between the two). */
int mpigx_comm_set_blocking(mpigx_comm_t comm, int blocking);
int mpigx_comm_synchronize(mpigx_comm_t comm);
int mpigx_comm_set_reduce_order(mpigx_comm_t comm, int order);

/* Path-selecting settings ("knobs").  Each is read ONCE per communicator,
 * at mpigx_comm_init_rank, from the environment variable named beside it;
 * init compares every rank's values and fails with MPIGX_ERR_ARG on any
 * mismatch (a rank launching another kernel than its peers would otherwise
 * spin until the device timeout).  mpigx_comm_set_knob changes one later: it
 * is COLLECTIVE (every rank calls it with the same knob and value, in the same
 * order relative to its other calls on the communicator), checks that over
 * the control plane, and returns MPIGX_ERR_ARG on every rank, changing
 * nothing, when they differ.  The two init-only knobs (allocation sizes)
 * cannot be set. */
#define MPIGX_KNOB_ALGO 0             /* MPIGX_ALGO: MPIGX_ALGO_* below */
#define MPIGX_KNOB_BCAST 1            /* MPIGX_BCAST: 0 auto, 1 "direct", 2 "sag", 3 "relay" */
#define MPIGX_KNOB_RING_CHANNELS 2    /* MPIGX_RING_CHANNELS: rings of MPIGX_ALGO_RING (1-4) */
#define MPIGX_KNOB_MAX_BLOCKS 3       /* MPIGX_MAX_BLOCKS: grid cap of the collective kernels */
#define MPIGX_KNOB_ONESHOT_MAX 4      /* MPIGX_ONESHOT_MAX: bytes */
#define MPIGX_KNOB_ZC_MIN 5           /* MPIGX_ZC_MIN: bytes (0: no zero-copy paths) */
#define MPIGX_KNOB_BCAST_SAG_MIN 6    /* MPIGX_BCAST_SAG_MIN: bytes */
#define MPIGX_KNOB_ZC_REQUIRE 7       /* MPIGX_ZC_REQUIRE: 1 = error instead of the staged fallback */
#define MPIGX_KNOB_BYTES_PER_BLOCK 8  /* MPIGX_BYTES_PER_BLOCK */
#define MPIGX_KNOB_LL_AUTO 9          /* MPIGX_LL_AUTO: bytes (<= MPIGX_LL_MAX) */
#define MPIGX_KNOB_AR_TUNE 10         /* MPIGX_AR_TUNE: 0/1, the measured algorithm choices */
#define MPIGX_KNOB_ZC_OPTIMISTIC 11   /* MPIGX_ZC_OPTIMISTIC: 0/1 */
#define MPIGX_KNOB_SYNC_SPIN 12       /* MPIGX_SYNC_SPIN: 0/1 */
#define MPIGX_KNOB_STAGING_BYTES 13   /* MPIGX_STAGING_BYTES (init only) */
#define MPIGX_KNOB_LL_MAX 14          /* MPIGX_LL_MAX (init only) */
#define MPIGX_KNOB_AR_SLICES 15       /* MPIGX_AR_SLICES: pull-push two-shot / zero-copy Reduce slices per
                                         block handed out dynamically (0, default: one static slice per
                                         block; 1-64) */
#define MPIGX_KNOB_SCAN_PP 16        /* MPIGX_SCAN_PP: 0/1, pull-push Scan / Exscan at n <= 8 (default 1) */
#define MPIGX_KNOB_SHARE_HEADROOM 17 /* MPIGX_SHARE_HEADROOM: -1/0/1, ranks sharing a GPU leave one block per
                                        CU free in the spinning kernels' grid caps (default -1 = 1: whenever
                                        ranks share it; 0 only for measurements) */
#define MPIGX_KNOB_SHARED_GATE 18    /* MPIGX_SHARED_GATE: 0/1, ranks sharing a GPU drain their stream and meet
                                        on the host before each collective launch (default 1) */
#define MPIGX_KNOB_PEER_MEM 19       /* MPIGX_PEER_MEM: 0 "auto" (default), 1 "xdev": every peer is treated as
                                        on another GPU (uncached signal arrays and LL areas, the
                                        one-rank-per-GPU protocol) even when it shares this one; a test
                                        knob that runs the production signalling on a 1-GPU box (init only) */
#define MPIGX_KNOB_CONCURRENT_COMMS 20 /* MPIGX_CONCURRENT_COMMS: >= 1 (default 1), how many communicators'
                                        * collectives may run on a GPU at the same time (threads, or
                                        * stream-ordered launches on different streams); every spinning
                                        * kernel's grid is capped at 1/this of the device's resident blocks,
                                        * so all of them fit at once (init-only); too low for the
                                        * communicators in flight: the stuck call fails with
                                        * MPI_ERR_OTHER after MPIGX_TIMEOUT_MS */
#define MPIGX_KNOB_COUNT 21
#define MPIGX_ALGO_AUTO 0     /* unset: static rules + the measured choices */
#define MPIGX_ALGO_LL 1       /* "ll" */
#define MPIGX_ALGO_LL2 2      /* "ll2" */
#define MPIGX_ALGO_ONESHOT 3  /* "oneshot" */
#define MPIGX_ALGO_TWOSHOT 4  /* "twoshot" */
#define MPIGX_ALGO_PUSH 5     /* "push" */
#define MPIGX_ALGO_RING 6     /* "ring" */
#define MPIGX_ALGO_PULL 7     /* "pull": the zero-copy pull two-shot (no pull/push tuning) */
#define MPIGX_ALGO_PULL_GENERIC 8 /* "pull_generic": the same through the all-modes fold kernel
                                     (fewer vectors per thread in flight; comparison only) */
#define MPIGX_ALGO_PULLPUSH 9 /* "pullpush": zero-copy pull reduce-scatter that stores each reduced
                                 slice into every rank's recvbuf (no allgather phase) */
int mpigx_comm_set_knob(mpigx_comm_t comm, int knob, long long value);
int mpigx_comm_get_knob(mpigx_comm_t comm, int knob, long long *value);

/* Ranks sharing one GPU.  Collective kernels spin on their peers, so every
 * rank's grid must run at once: each launch caps its grid at
 * CUs x (resident blocks per CU of THAT kernel, from the occupancy API) /
 * (ranks on the most-loaded device), identical on every rank; init fails
 * with MPIGX_ERR_OTHER when more than MPIGX_MAX_RANKS_PER_DEVICE (environment,
 * default 10) ranks share a device (beyond that, some rank processes' kernels
 * were seen not to start while their peers spun).  *ranks = ranks on the
 * most-loaded device, *cap = compute units per rank there (a kernel's grid
 * cap is *cap x its resident blocks per CU). */
int mpigx_comm_device_share(mpigx_comm_t comm, int *ranks, int *cap);

/* The communicator's stall bound (default MPIGX_TIMEOUT_MS, 60000).  A call
 * waits for a late peer as long as that peer's process lives; it fails with
 * MPI_ERR_OTHER (the communicator marked broken) within about a second when
 * a peer is gone or its communicator failed, and after this bound when
 * every rank's GPU has sat in the same launch with none moving, or when a
 * peer's launch, enqueued but never started, is stuck behind other
 * communicators' kernels (MPIGX_CONCURRENT_COMMS).  Local; applies to later
 * calls.  ms >= 1. */
int mpigx_comm_set_timeout(mpigx_comm_t comm, long long ms);

/* Diagnostics (phase stamps, signal-slot and mapping checks, tuner and
 * zero-copy statistics, fabric probes): include/mpigx_diag.h. */

/* ---- collectives (src/collective.jl ccall sites) ------------------------- */
/* MPI_Barrier  — collective.jl:15-19 */
int mpigx_barrier(mpigx_comm_t comm);
/* MPI_Bcast    — collective.jl:29-37 */
int mpigx_bcast(void *buffer, int count, int datatype, int root, mpigx_comm_t comm);
/* MPI_Allgather — collective.jl:295-307 (sendbuf may be MPIGX_IN_PLACE) */
int mpigx_allgather(const void *sendbuf, int sendcount, int sendtype, void *recvbuf,
                    int recvcount, int recvtype, mpigx_comm_t comm);
/* MPI_Alltoall — collective.jl:489-501 (sendbuf may be MPIGX_IN_PLACE) */
int mpigx_alltoall(const void *sendbuf, int sendcount, int sendtype, void *recvbuf,
                   int recvcount, int recvtype, mpigx_comm_t comm);
/* v-collectives and rooted variants.  counts/displs are
 * host int arrays in elements, as MPI.jl passes them (Ptr{Cint}).
 * MPI_Gather   — collective.jl:230-246 (sendbuf IN_PLACE at root) */
int mpigx_gather(const void *sendbuf, int sendcount, int sendtype, void *recvbuf, int recvcount,
                 int recvtype, int root, mpigx_comm_t comm);
/* MPI_Gatherv  — collective.jl:363-382 (recvcounts/displs read at root) */
int mpigx_gatherv(const void *sendbuf, int sendcount, int sendtype, void *recvbuf,
                  const int *recvcounts, const int *displs, int recvtype, int root,
                  mpigx_comm_t comm);
/* MPI_Scatter  — collective.jl:90-106 (recvbuf IN_PLACE at root) */
int mpigx_scatter(const void *sendbuf, int sendcount, int sendtype, void *recvbuf, int recvcount,
                  int recvtype, int root, mpigx_comm_t comm);
/* MPI_Scatterv — collective.jl:156-175 (sendcounts/displs read at root) */
int mpigx_scatterv(const void *sendbuf, const int *sendcounts, const int *displs, int sendtype,
                   void *recvbuf, int recvcount, int recvtype, int root, mpigx_comm_t comm);
/* MPI_Allgatherv — collective.jl:424-437 (sendbuf may be MPIGX_IN_PLACE) */
int mpigx_allgatherv(const void *sendbuf, int sendcount, int sendtype, void *recvbuf,
                     const int *recvcounts, const int *displs, int recvtype, mpigx_comm_t comm);
/* MPI_Alltoallv — collective.jl:545-559 (sendbuf may be MPIGX_IN_PLACE) */
int mpigx_alltoallv(const void *sendbuf, const int *sendcounts, const int *sdispls, int sendtype,
                    void *recvbuf, const int *recvcounts, const int *rdispls, int recvtype,
                    mpigx_comm_t comm);
/* MPI_Reduce   — collective.jl:605-618 (IN_PLACE at root; recvbuf ignored
 * (may be NULL) elsewhere) */
int mpigx_reduce(const void *sendbuf, void *recvbuf, int count, int datatype, int op,
                 int root, mpigx_comm_t comm);
/* MPI_Allreduce — collective.jl:691-701 (sendbuf may be MPIGX_IN_PLACE) */
int mpigx_allreduce(const void *sendbuf, void *recvbuf, int count, int datatype, int op,
                    mpigx_comm_t comm);
/* MPI_Scan     — collective.jl:760-768 */
int mpigx_scan(const void *sendbuf, void *recvbuf, int count, int datatype, int op,
               mpigx_comm_t comm);
/* MPI_Exscan   — collective.jl:834-842 (rank 0's recvbuf is left untouched) */
int mpigx_exscan(const void *sendbuf, void *recvbuf, int count, int datatype, int op,
                 mpigx_comm_t comm);

/* ---- local ops (config 2; operators.jl built-in Op set on device) ------- */
/* MPI_Reduce_local (mpi.h:1357): inoutbuf[i] = op(inoutbuf[i], inbuf[i]).
 * Device pointers; blocking on the null stream. */
int mpigx_reduce_local(const void *inbuf, void *inoutbuf, int count, int datatype, int op);
/* out[i] = fold_{k<nin} in[k][i] in `order` (as if in[k] were rank k's
 * buffer of an nin-rank Allreduce).  Device pointers; enqueued on `stream`
 * (NULL = null stream), asynchronous.  nin in [1, MPIGX_MAX_RANKS]. */
int mpigx_reduce_local_multi(const void *const *in, int nin, void *out, long long count,
                             int datatype, int op, int order, void *stream);

/* ---- point-to-point (src/pointtopoint.jl) ----------
 * Device buffers, rendezvous protocol: the sender publishes an envelope
 * (tag, size, IPC handle of the allocation holding the buffer) in the
 * receiver's shm mailbox; the receiver matches it (MPI order: per source
 * FIFO, posted receives in post order, ANY_SOURCE / ANY_TAG) and pulls the
 * bytes with one copy kernel on its own transfer stream, then acknowledges.
 * Send buffers must be ready when the call is made (the comm's stream is
 * synchronised); receive buffers are written after prior work on the comm's
 * stream.  Progress happens inside every mpigx call on the communicator,
 * including blocking collectives.  Requests and statuses are the MPICH ones:
 * `int` request handles (MPIGX_REQUEST_NULL = MPI_REQUEST_NULL) and the
 * 20-byte MPI_Status layout (mpi.h:585-591, pointtopoint.jl:4-60). */
#define MPIGX_ERR_TAG 4
#define MPIGX_ERR_RANK 6
#define MPIGX_ERR_TRUNCATE 14
#define MPIGX_ERR_IN_STATUS 17
#define MPIGX_ERR_REQUEST 19
#define MPIGX_ANY_SOURCE (-2)
#define MPIGX_ANY_TAG (-1)
#define MPIGX_PROC_NULL (-1)
#define MPIGX_REQUEST_NULL 0x2c000000
#define MPIGX_TAG_UB 268435455 /* MPI_TAG_UB attribute of MPICH 3.3.2 ch3 */

typedef int mpigx_request_t;
typedef struct mpigx_status {
  int count_lo;               /* bytes received (low 31 bits), as MPICH */
  int count_hi_and_cancelled; /* bit 0: cancelled */
  int MPI_SOURCE;
  int MPI_TAG;
  int MPI_ERROR;
} mpigx_status_t;
#define MPIGX_STATUS_IGNORE ((mpigx_status_t *)1)

/* MPI_Send / MPI_Isend — pointtopoint.jl:188-198, :221-232 */
int mpigx_send(const void *buf, int count, int datatype, int dest, int tag, mpigx_comm_t comm);
int mpigx_isend(const void *buf, int count, int datatype, int dest, int tag, mpigx_comm_t comm,
                mpigx_request_t *request);
/* MPI_Recv / MPI_Irecv — pointtopoint.jl:266-273, :325-336 */
int mpigx_recv(void *buf, int count, int datatype, int source, int tag, mpigx_comm_t comm,
               mpigx_status_t *status);
int mpigx_irecv(void *buf, int count, int datatype, int source, int tag, mpigx_comm_t comm,
                mpigx_request_t *request);
/* MPI_Sendrecv — pointtopoint.jl:370-386 */
int mpigx_sendrecv(const void *sendbuf, int sendcount, int sendtype, int dest, int sendtag,
                   void *recvbuf, int recvcount, int recvtype, int source, int recvtag,
                   mpigx_comm_t comm, mpigx_status_t *status);
/* MPI_Probe / MPI_Iprobe — pointtopoint.jl:107-115, :126-137 */
int mpigx_probe(int source, int tag, mpigx_comm_t comm, mpigx_status_t *status);
int mpigx_iprobe(int source, int tag, mpigx_comm_t comm, int *flag, mpigx_status_t *status);
/* MPI_Get_count — pointtopoint.jl:150-156 (MPIGX_UNDEFINED if not a multiple) */
int mpigx_get_count(const mpigx_status_t *status, int datatype, int *count);
/* MPI_Test_cancelled */
int mpigx_test_cancelled(const mpigx_status_t *status, int *flag);
/* MPI_Wait / Test / Waitall / Testall / Waitany / Testany / Waitsome /
 * Testsome / Cancel / Request_free — pointtopoint.jl:398-681.  Completed
 * requests are freed and set to MPIGX_REQUEST_NULL; null entries are
 * skipped and report the empty status (source ANY_SOURCE, tag ANY_TAG). */
int mpigx_wait(mpigx_request_t *request, mpigx_status_t *status);
int mpigx_test(mpigx_request_t *request, int *flag, mpigx_status_t *status);
int mpigx_waitall(int count, mpigx_request_t *requests, mpigx_status_t *statuses);
int mpigx_testall(int count, mpigx_request_t *requests, int *flag, mpigx_status_t *statuses);
int mpigx_waitany(int count, mpigx_request_t *requests, int *index, mpigx_status_t *status);
int mpigx_testany(int count, mpigx_request_t *requests, int *index, int *flag,
                  mpigx_status_t *status);
int mpigx_waitsome(int incount, mpigx_request_t *requests, int *outcount, int *indices,
                   mpigx_status_t *statuses);
int mpigx_testsome(int incount, mpigx_request_t *requests, int *outcount, int *indices,
                   mpigx_status_t *statuses);
int mpigx_cancel(mpigx_request_t *request);
int mpigx_request_free(mpigx_request_t *request);

/* ---- one-sided communication (src/onesided.jl) -----
 * Windows over device memory.  Get is pulled by the origin straight from the
 * target's (IPC-mapped) window; Put / Accumulate / Get_accumulate /
 * Fetch_and_op are posted as envelopes to the target, which applies them to
 * its own memory — pulling the origin buffer over xGMI with the op fused into
 * the pull — so only the GPU that owns a window ever writes it (the same
 * coherence rule as the collectives).  Consequence, as for MPICH ch3 on
 * non-shared windows: passive-target operations complete when the target
 * makes progress, i.e. is inside any mpigx call on the communicator
 * (blocking collectives, Wait, Barrier, Win_* ...).  Accumulates to one
 * target are applied in one stream, so they are atomic per element and
 * ordered per origin, as MPI requires.  Operand roles: window = inout,
 * origin = in (MPICH's MPI_Accumulate), pinned by tests/golden/rma_golden.json.
 * Handles are opaque pointers (MPI.jl's Win wraps MPI_Win the same way,
 * onesided.jl:1-3); errors are MPI error classes. */
#define MPIGX_ERR_WIN 45
#define MPIGX_ERR_BASE 46
#define MPIGX_ERR_LOCKTYPE 47
#define MPIGX_ERR_RMA_SYNC 50
#define MPIGX_ERR_SIZE 51
#define MPIGX_ERR_DISP 52
#define MPIGX_ERR_RMA_RANGE 55
#define MPIGX_ERR_RMA_ATTACH 56
#define MPIGX_ERR_RMA_FLAVOR 58
#define MPIGX_REPLACE 1476395021 /* MPI_REPLACE (mpi.h:322) */
#define MPIGX_NO_OP 1476395022   /* MPI_NO_OP   (mpi.h:323) */
#define MPIGX_LOCK_EXCLUSIVE 234
#define MPIGX_LOCK_SHARED 235
#define MPIGX_MODE_NOCHECK 1024
#define MPIGX_WIN_FLAVOR_CREATE 1
#define MPIGX_WIN_FLAVOR_ALLOCATE 2 /* (not produced) */
#define MPIGX_WIN_FLAVOR_DYNAMIC 3
#define MPIGX_WIN_FLAVOR_SHARED 4

typedef struct mpigx_win *mpigx_win_t;

/* MPI_Win_create — onesided.jl:24-34 (base: device pointer; size in bytes) */
int mpigx_win_create(void *base, long long size, int disp_unit, mpigx_comm_t comm, mpigx_win_t *win);
/* MPI_Win_create_dynamic — onesided.jl:47-56 */
int mpigx_win_create_dynamic(mpigx_comm_t comm, mpigx_win_t *win);
/* MPI_Win_allocate_shared — onesided.jl:72-83: device memory owned by this
 * rank (uncached HBM, zero-filled), IPC-mapped by every peer */
int mpigx_win_allocate_shared(long long size, int disp_unit, mpigx_comm_t comm, void *baseptr,
                              mpigx_win_t *win);
/* MPI_Win_shared_query — onesided.jl:98-108 (baseptr: this process's mapping
 * of `rank`'s segment; rank = MPIGX_PROC_NULL: first non-empty segment) */
int mpigx_win_shared_query(mpigx_win_t win, int rank, long long *size, int *disp_unit, void *baseptr);
/* MPI_Win_free — onesided.jl:85-92 (collective; *win set to NULL) */
int mpigx_win_free(mpigx_win_t *win);
/* MPI_Win_attach / MPI_Win_detach — onesided.jl:110-122 (dynamic windows:
 * target_disp is the absolute device address, MPI_Get_address) */
int mpigx_win_attach(mpigx_win_t win, void *base, long long size);
int mpigx_win_detach(mpigx_win_t win, const void *base);
/* MPI_Win_fence / flush / sync / lock / unlock — onesided.jl:124-148 */
int mpigx_win_fence(int assert_, mpigx_win_t win);
int mpigx_win_flush(int rank, mpigx_win_t win);
int mpigx_win_sync(mpigx_win_t win);
int mpigx_win_lock(int lock_type, int rank, int assert_, mpigx_win_t win);
int mpigx_win_unlock(int rank, mpigx_win_t win);
/* MPI_Win_get_attr(MPI_WIN_CREATE_FLAVOR) analogue */
int mpigx_win_get_flavor(mpigx_win_t win, int *flavor);
/* MPI_Get / MPI_Put — onesided.jl:150-184 */
int mpigx_get(void *origin_addr, int origin_count, int origin_datatype, int target_rank,
              long long target_disp, int target_count, int target_datatype, mpigx_win_t win);
int mpigx_put(const void *origin_addr, int origin_count, int origin_datatype, int target_rank,
              long long target_disp, int target_count, int target_datatype, mpigx_win_t win);
/* MPI_Fetch_and_op — onesided.jl:186-195 */
int mpigx_fetch_and_op(const void *origin_addr, void *result_addr, int datatype, int target_rank,
                       long long target_disp, int op, mpigx_win_t win);
/* MPI_Accumulate — onesided.jl:197-206 */
int mpigx_accumulate(const void *origin_addr, int origin_count, int origin_datatype, int target_rank,
                     long long target_disp, int target_count, int target_datatype, int op,
                     mpigx_win_t win);
/* MPI_Get_accumulate — onesided.jl:208-219 */
int mpigx_get_accumulate(const void *origin_addr, int origin_count, int origin_datatype,
                         void *result_addr, int result_count, int result_datatype, int target_rank,
                         long long target_disp, int target_count, int target_datatype, int op,
                         mpigx_win_t win);

/* ---- derived datatypes (src/datatypes.jl:62-318) ---
 * The MPI_Type_* constructors MPI.Types ccalls, for device buffers: handles
 * are `int`s in libmpigx's own space (0x3d000000 | generation << 16 | slot,
 * never issued by MPICH: an MPICH derived type is rejected with
 * MPI_ERR_TYPE, not aliased), usable
 * wherever a datatype is taken once committed — point-to-point (strided and
 * dense SubArrays, buffers.jl:104-117; padded isbits structs,
 * datatypes.jl:269-316) and the byte-moving collectives (Bcast, Allgather,
 * Alltoall, Gather, Scatter), which pack non-contiguous types on device
 * (pack_kernel) around the contiguous algorithm.  Reductions accept derived
 * types that are contiguous runs of one predefined type.  lb / extent /
 * sizes follow MPICH 3.3.2 (tests/golden/types_golden.json). */
#define MPIGX_ORDER_C 56
#define MPIGX_ORDER_FORTRAN 57
#define MPIGX_DATATYPE_NULL 0x0c000000
int mpigx_type_contiguous(int count, int oldtype, int *newtype);
int mpigx_type_vector(int count, int blocklength, int stride, int oldtype, int *newtype);
int mpigx_type_create_hvector(int count, int blocklength, long long stride, int oldtype, int *newtype);
int mpigx_type_create_subarray(int ndims, const int *sizes, const int *subsizes, const int *starts, int order,
                               int oldtype, int *newtype);
int mpigx_type_create_struct(int count, const int *blocklengths, const long long *displacements,
                             const int *types, int *newtype);
int mpigx_type_create_resized(int oldtype, long long lb, long long extent, int *newtype);
int mpigx_type_commit(int *datatype);
int mpigx_type_free(int *datatype);
int mpigx_type_get_extent(int datatype, long long *lb, long long *extent);
int mpigx_type_get_true_extent(int datatype, long long *true_lb, long long *true_extent);
int mpigx_type_size_x(int datatype, long long *size);
/* MPI_Pack / MPI_Unpack / MPI_Pack_size on device buffers (stream: hipStream_t
 * or NULL; blocking).  Pack layout = MPI's (typemap order, no padding). */
int mpigx_pack_size(int incount, int datatype, long long *size);
int mpigx_pack(const void *inbuf, int incount, int datatype, void *outbuf, long long outsize,
               long long *position, void *stream);
int mpigx_unpack(const void *inbuf, long long insize, long long *position, void *outbuf, int outcount,
                 int datatype, void *stream);

/* ---- user-defined ops (operators.jl:56-88 OpWrapper) --
 * MPI_Op_create analogues.  Handles live in libmpigx's own space
 * (0x3c000000 | generation << 16 | slot: MPICH never issues a kind-00 handle
 * with a non-zero payload), so an op MPI.jl created in libmpi (MPICH user op
 * 0x98000000 | k) is rejected with MPI_ERR_OP instead of aliasing one of
 * these; a freed handle is rejected too.  Accepted by Allreduce / Reduce /
 * Scan / Exscan for predefined and contiguous derived types.  The engine gathers
 * the contributions with its own kernels and folds in rank order,
 * inout = x_q (op) inout from the highest contributing rank down.
 *   host callback   — MPI_User_function on HOST copies (what MPI.jl's
 *                     @cfunction(OpWrapper) is); operands staged via pinned memory
 *   device callback — device pointers + the comm's stream (hipStream_t as
 *                     void*); the callee enqueues its own kernels. */
typedef void(mpigx_user_function)(void *invec, void *inoutvec, int *len, int *datatype);
typedef void(mpigx_device_function)(const void *invec, void *inoutvec, long long len, int datatype,
                                    void *stream);
int mpigx_op_create(mpigx_user_function *user_fn, int commute, int *op);
int mpigx_op_create_device(mpigx_device_function *device_fn, int commute, int *op);
int mpigx_op_free(int *op);
int mpigx_op_commutative(int op, int *commute);

/* ---- device buffers (north-star subsystem 1: the ROCBuffer backing) ----- */
int mpigx_malloc(void **ptr, size_t bytes);
int mpigx_free(void *ptr);
int mpigx_memcpy(void *dst, const void *src, size_t bytes); /* any direction, blocking */

#ifdef __cplusplus
}
#endif
#endif /* MPIGX_H */
