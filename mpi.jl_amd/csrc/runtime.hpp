// runtime.hpp — host-runtime internals shared by mpigx.cpp (communicators,
// collectives) and p2p.cpp (point-to-point): the shm rendezvous block, the
// communicator object and the few helpers both sides call.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "common.hpp"

namespace mpigx {

// ---------------------------------------------------------------------------
// shm block (one per communicator, mapped by every rank)
// ---------------------------------------------------------------------------
constexpr uint64_t kMagic = 0x6d70696778763036ull;  // "mpigxv06"

constexpr uint64_t kSigCanary = 0x6d70696778c0ffeeull;  // signal-array canary (mpigx.cpp comm_init)

struct ShmRank {
  int pid;
  int device;
  int pci_bus;
  int pci_dev;
  int pci_domain;
  int cus;                       // compute units of my device
  int max_share;                 // MPIGX_MAX_RANKS_PER_DEVICE of this rank (the minimum over ranks applies)
  long long knobs[MPIGX_KNOB_COUNT];  // path-selecting settings read at init (must agree)
  unsigned long long epoch0;          // first barrier epoch (MPIGX_EPOCH_BASE; must agree)
  unsigned long long stage_bytes;
  unsigned long long stage_ptr;  // raw pointer (same-process peers)
  unsigned long long sig_ptr;
  unsigned long long sig_rw_ptr;
  unsigned long long ll_rw_ptr;
  hipIpcMemHandle_t stage_h;
  hipIpcMemHandle_t sig_h;
  hipIpcMemHandle_t sig_rw_h;
  hipIpcMemHandle_t ll_rw_h;
  unsigned long long ll_bytes;   // LL area size (0: none; must agree on every rank)
  unsigned long long ll_ptr;
  hipIpcMemHandle_t ll_h;
  // liveness of the rank's side of the protocol, read by its peers' host
  // waits (mpigx.cpp finish / host_allgather_wait): `broken` = its
  // communicator failed (it will never join another collective), `kseq_enq`
  // = the last collective launch it enqueued, `kseq_run` = the last one its
  // device reported started (kernels' `started` word), `proc_busy` = how many
  // communicators of its PROCESS have a collective in flight (this one
  // included; mpigx.cpp busy_comms) — a launch enqueued long ago that its GPU
  // never started while other communicators' kernels run is stuck, not late
  // (mpigx.cpp stuck_peer)
  std::atomic<int> broken;
  std::atomic<uint64_t> kseq_enq;
  std::atomic<uint64_t> kseq_run;
  std::atomic<int> proc_busy;
  // host control-plane exchange (host_allgather): double-buffered blobs
  std::atomic<uint64_t> xseq;
  char xbuf[2][256];
};

// Point-to-point envelope: written by the sender into the (sender, receiver)
// mailbox, consumed in order by the receiver.  `posted` = message seq + 1
// once the fields are valid; `done` = seq + 1 once the receiver has pulled
// the bytes (the slot may then be reused and the send request completes).
constexpr int kP2PSlots = 32;
struct alignas(64) P2PEnvelope {
  std::atomic<uint64_t> posted;
  std::atomic<uint64_t> done;
  int tag;
  int pad;
  long long bytes;
  unsigned long long buf_id;     // HIP buffer id of the allocation holding the data
  long long off;                 // offset of the data in that allocation
  unsigned long long raw;        // sender's own pointer (self-sends)
  hipIpcMemHandle_t h;           // IPC handle of the allocation
};
struct P2PMailbox {
  P2PEnvelope slot[kP2PSlots];
};

// One-sided (RMA) windows (rma.cpp).  Envelopes travel origin -> target in
// the [origin][target] box of the window's slot; the TARGET applies Put /
// Accumulate to its own memory (pulling the origin's buffer over xGMI) and
// stores done = seq + 1.  Lock words are per target rank: 0 free, > 0 shared
// holders, -1 exclusive.  Dynamic windows publish attached regions in
// dyn[rank][*] (gen odd while being written).
constexpr int kMaxWins = 16;
constexpr int kRmaSlots = 16;
constexpr int kMaxAttach = 16;
struct alignas(64) RmaEnvelope {
  std::atomic<uint64_t> posted;
  std::atomic<uint64_t> done;
  int kind;     // RmaKind (rma.cpp)
  int op;       // OpCode / O_REPLACE / O_NOOP
  int rep;      // element representation
  int err;      // target-side result (MPI error class), valid once done
  long long tdisp;  // byte offset into the target window (dynamic: absolute address)
  long long count;  // elements (bytes for PUT)
  long long res_off;  // GACC: byte offset of the old values in the target's scratch
  unsigned long long buf_id;  // origin allocation (HIP buffer id), offset and handle
  long long off;
  unsigned long long raw;     // origin pointer (same-process origin)
  hipIpcMemHandle_t h;
};
struct RmaBox {
  RmaEnvelope slot[kRmaSlots];
};
struct DynRegion {
  std::atomic<uint64_t> gen;
  unsigned long long addr, size, buf_id;
  long long off;
  hipIpcMemHandle_t h;
};
struct WinShm {
  std::atomic<int> lock[kMaxRanks];
  RmaBox box[kMaxRanks][kMaxRanks];  // [origin][target]
  DynRegion dyn[kMaxRanks][kMaxAttach];
};

struct ShmBlock {
  std::atomic<uint64_t> magic;
  int nranks;
  std::atomic<int> arrived;
  std::atomic<int> connected;
  std::atomic<int> failed;
  ShmRank ranks[kMaxRanks];
  P2PMailbox box[kMaxRanks][kMaxRanks];  // [sender][receiver]
  WinShm win[kMaxWins];
};

struct P2PState;  // p2p.cpp
struct RmaState;  // rma.cpp

}  // namespace mpigx

// ---------------------------------------------------------------------------
// communicator
// ---------------------------------------------------------------------------
struct mpigx_comm {
  int rank = 0, n = 1, device = 0;
  hipStream_t stream = nullptr;
  int blocking = 1;
  int order = MPIGX_ORDER_MPICH;
  bool broken = false;
  uint64_t epoch = 1;
  uint64_t timeout_ticks = 0;
  // local resources
  char* stage = nullptr;
  size_t stage_bytes = 0;
  uint64_t* sig = nullptr;     // signal array, uncached: words from peers on OTHER devices
  uint64_t* sig_rw = nullptr;  // signal array, ordinary memory: words from peers on MY device (and mine)
  char* ll = nullptr;          // LL area (uncached): [2 parities][kMaxRanks senders][ll_stride]
  char* ll_rw = nullptr;       // LL area, ordinary memory: lines from peers on my device
  unsigned rw_mask = 0;        // bit q: rank q is on my device (bit rank always set)
  long long ll_max = 0;        // MPIGX_LL_MAX: LL capacity per sender (bytes; 0: no LL area)
  long long ll_auto = 0;       // MPIGX_LL_AUTO: largest message that takes LL by default
  long long ll_stride = 0;     // bytes of one sender's lines (2 x ll_max rounded to 16)
  unsigned long long ll_seq = 0;  // LL launches so far (parity = ll_seq & 1; same on every rank)
  bool ll_unfenced = false;       // an LL launch (no exit barrier) since the last push two-shot
  // large-Allreduce algorithm chosen by measurement (mpigx.cpp ar_tune_*):
  // -1 undecided, 0 pull two-shot, 1 push two-shot, 2 pull-push two-shot
  int ar_choice = -1;
  int ar_tune = 1;                // MPIGX_AR_TUNE
  int ar_step = 0;                // zero-copy Allreduces seen while undecided
  double ar_spb[3] = {0, 0, 0};   // device seconds per byte: pull, push, pull-push (this rank)
  int ar_slices = 0;              // MPIGX_AR_SLICES: dynamic pull-push slices per block (0: static)
  // dynamic slice hand-out counters (dcount_dev[1] tickets, [2] finished
  // blocks): totals of every launch so far, the next launch's bases
  unsigned long long wtickets = 0, wfinished = 0;
  hipEvent_t ar_ev[2] = {nullptr, nullptr};
  // small / medium Allreduce tuner (mpigx.cpp mt_*): per size class
  // (floor(log2 bytes)) the measured choice among LL / one-shot / two-shot
  // (kind 0 Allreduce: LL / one-shot / two-shot; kinds 1-3 Bcast / Allgather
  // / Alltoall: LL / staged), slot = kind * kTuneClasses + class
  static constexpr int kTuneClasses = 40;
  static constexpr int kTuneKinds = 4;
  signed char mt_choice[kTuneKinds * kTuneClasses];     // -1 undecided
  unsigned char mt_step[kTuneKinds * kTuneClasses] = {};
  double mt_spb[kTuneKinds * kTuneClasses][4] = {};     // min device s/byte per variant (0: none)
  unsigned* err = nullptr;  // host-pinned, device-written
  unsigned* err_dev = nullptr;
  // completion counter for blocking calls (host-pinned; kernels add 1 per block)
  volatile unsigned long long* done = nullptr;
  unsigned long long* done_dev = nullptr;
  // late-peer protocol (PeerView.started / .cancel): the launch my GPU last
  // reported started, and the word that makes a blocking launch give up
  volatile unsigned long long* started = nullptr;
  unsigned long long* started_dev = nullptr;
  volatile unsigned* cancel = nullptr;
  unsigned* cancel_dev = nullptr;
  unsigned long long kseq = 0;  // collective launches so far (the same on every rank)
  unsigned long long kseq_done = 0;  // launches known complete (kseq when the last finish() returned)
  // stuck-peer tracking (mpigx.cpp stuck_peer): since when rank q has been
  // seen enqueued-but-not-started in the awaited launch (0: not seen so)
  double stuck_since[mpigx::kMaxRanks] = {};   // finish()'s (the calling thread)
  double wstuck_since[mpigx::kMaxRanks] = {};  // the watcher thread's (stream-ordered launches)
  // the watcher's view of a stream-ordered communicator: the launch its GPU
  // last reported started, since when, and whether its stream had work
  unsigned long long watch_seen = 0;
  double watch_moved = 0;
  bool watch_busy = false;
  hipEvent_t so_ev = nullptr;  // recorded after every stream-ordered launch (note_launch)
  unsigned long long done_target = 0;  // launch sequence the host waits for
  unsigned long long* dcount_dev = nullptr;
  unsigned long long dcount_total = 0;  // blocks counted on dcount so far
  unsigned long long launch_seq = 0;
  bool unflagged = false;  // work enqueued without the counter (stream-ordered mode)
  int sync_mode = 1;       // 1: spin on the counter, 0: hipStreamSynchronize
  uint64_t xseq = 0;       // host_allgather sequence
  // zero-copy registration caches (user buffers exported / peers' imported)
  struct LocalReg {
    unsigned long long id;
    char* base;
    size_t size;  // allocation size (a reallocation at the same base with another size is another allocation)
    hipIpcMemHandle_t h;
  };
  struct Import {
    int peer;
    unsigned long long id;
    char* base;
    unsigned long long tick;
    int pins;  // RMA windows holding this mapping (never evicted while > 0)
    hipIpcMemHandle_t h;
  };
  // zero-copy views (mpigx.cpp zc_run): my recent (send, recv) registrations
  // and the agreed peer mappings of recent exchanges
  struct ZcTuple {
    char* base[2];
    unsigned long long id[2];
    long long off[2];
    hipIpcMemHandle_t h[2];
    unsigned serial;
    unsigned long long tick;
  };
  struct ZcView {
    unsigned id;                            // exchange sequence number (the launch key)
    unsigned serial[mpigx::kMaxRanks];      // every rank's registration serial
    const char* ps[mpigx::kMaxRanks];       // every rank's sendbuf, mapped here
    char* pr[mpigx::kMaxRanks];             // every rank's recvbuf, mapped here
    long long as[mpigx::kMaxRanks];         // bytes of each rank's send / recv allocation from the pointer
    long long ar[mpigx::kMaxRanks];         // to its end (exported sizes; kernels check remote stores against them)
    unsigned long long tick;
  };
  std::vector<ZcTuple> ztuples;
  std::vector<ZcView> zviews;
  unsigned zserial = 0, zview_seq = 0;
  bool last_aborted = false;         // the last completed launch's zero-copy abort verdict
  double t_entry = 0, last_prelaunch_s = 0;  // host time from API entry to the first launch
  bool launch_pending = false;
  bool zc_optimistic = true;         // MPIGX_ZC_OPTIMISTIC (blocking calls only)
  unsigned long long zstat_hits = 0, zstat_exchanges = 0;
  std::vector<LocalReg> lreg;
  std::vector<std::pair<long long, char*>> tmp_free, tmp_used;  // derived-type pack temporaries
  std::vector<Import> imports;
  unsigned long long tick = 0;
  long long zc_min = 16ll << 20;  // bytes; 0 disables
  bool zc_require = false;        // MPIGX_ZC_REQUIRE=1: error instead of the staged fallback
  // peers (index = rank; self included)
  char* peer_stage[mpigx::kMaxRanks] = {};
  uint64_t* peer_sig[mpigx::kMaxRanks] = {};
  uint64_t* peer_sig_rw[mpigx::kMaxRanks] = {};  // every rank's ordinary-memory signal array (IPC-mapped)
  char* peer_ll_rw[mpigx::kMaxRanks] = {};
  bool peer_rw_opened[mpigx::kMaxRanks] = {};
  bool peer_opened[mpigx::kMaxRanks] = {};      // peer_stage[q] is an IPC mapping of ours
  bool peer_sig_opened[mpigx::kMaxRanks] = {};  // peer_sig[q] likewise
  char* peer_ll[mpigx::kMaxRanks] = {};         // every rank's LL area (IPC-mapped)
  bool peer_ll_opened[mpigx::kMaxRanks] = {};
  bool same_device[mpigx::kMaxRanks] = {};      // rank q runs on my GPU (PCI bus/device id)
  mpigx::ShmBlock* shm = nullptr;
  // point-to-point engine (created on first use)
  mpigx::P2PState* p2p = nullptr;
  // one-sided engine (created by the first window)
  mpigx::RmaState* rma = nullptr;
  bool in_progress = false;  // re-entrancy guard of rt::progress_all
  // tuning (the path-selecting knobs, include/mpigx.h MPIGX_KNOB_*: read once
  // at init, checked to agree on every rank, changed only collectively)
  int max_blocks = 256;
  int cus_min = 256;                       // compute units of the smallest device (agreed at init)
  int dev_share = 1;                       // ranks on the most-loaded device (grid caps: kernel_cap)
  long long oneshot_max = 256 << 10;
  long long bcast_sag_min = 256 << 10;  // Bcast: scatter+allgather from this size (n >= 3)
  long long bytes_per_block = 64 << 10;
  int algo = MPIGX_ALGO_AUTO;           // MPIGX_ALGO
  int bcast_mode = 0;                   // MPIGX_BCAST: 0 auto, 1 direct, 2 sag
  int ring_channels = 1;                // MPIGX_RING_CHANNELS
  unsigned long long* stamps = nullptr; // diagnostic phase timestamps (mpigx_comm_set_stamps)
  int share_headroom = -1;              // MPIGX_SHARE_HEADROOM: ranks sharing a device leave one block per CU free (-1 auto: >= 4 ranks)
  bool scan_pp = true;                  // MPIGX_SCAN_PP: pull-push Scan / Exscan (kernels.hpp scan_pp_body)
  bool shared_gate = true;              // MPIGX_SHARED_GATE: ranks sharing a device meet on the host first
  int concurrent_comms = 1;             // MPIGX_CONCURRENT_COMMS: grid caps divided by it (kernel_cap)
  int peer_mem = 0;                     // MPIGX_PEER_MEM: 0 auto (memory type per pair), 1 xdev (every peer as
                                        // if on another GPU: uncached signal / LL arrays; test knob)
  bool diag_trace = false;              // MPIGX_DIAG_TRACE: one stderr line per launch (diagnostic)
  unsigned ll_gen = 0;                  // LL flag generation (epoch >> 31) the LL area was cleared for
  int test_import_fail = 0;             // MPIGX_TEST_IMPORT_FAIL: fail that many peer imports (tests)
  // Largest allocation this rank IPC-exports (zero-copy views, p2p, RMA);
  // 0 = no limit.  HIP runtimes before 7.2 (e.g. the 7.0 runtime PyTorch
  // bundles, which a torch process loads instead of the system's) never
  // return from hipIpcOpenMemHandle of an allocation >= 2 GiB (DESIGN §13,
  // tools/ipc_torch.py); MPIGX_IPC_ALLOC_MAX overrides (tests).
  long long ipc_alloc_max = 0;
  int hip_runtime = 0;                  // hipRuntimeGetVersion of the runtime this process loaded
  // Registered with the process-wide peer watcher (mpigx.cpp watch_peers)
  // at the first stream-ordered launch, unregistered in comm_release.
  bool watched = false;
  std::mutex mu;
};

namespace mpigx {
namespace rt {
// mpigx.cpp
int comm_check(mpigx_comm* c);
void comm_mark_broken(mpigx_comm* c);  // broken, and published to the peers (ShmRank.broken)
int dtype_size(int datatype);  // bytes, or -1 if not a valid datatype handle
bool export_buf(mpigx_comm* c, const void* p, unsigned long long* id, long long* off, hipIpcMemHandle_t* h);
char* import_buf(mpigx_comm* c, int peer, unsigned long long id, const hipIpcMemHandle_t& h);
// as import_buf, and pin (+1) / unpin (-1) the mapping for a window's lifetime
char* import_pinned(mpigx_comm* c, int peer, unsigned long long id, const hipIpcMemHandle_t& h);
void unpin(mpigx_comm* c, char* base);
int host_allgather(mpigx_comm* c, const void* mine, int len, void* out);
// every engine's progress (p2p + RMA target side); safe to call anywhere
void progress_all(mpigx_comm* c);
// MPI_THREAD_MULTIPLE (mpigx_query_thread): one process-wide recursive lock,
// taken by every non-blocking point-to-point call, every RMA call and every
// progress pass.  Blocking point-to-point calls (Wait*, Send, Recv, Probe)
// loop over their non-blocking forms, so they release it between polls and a
// thread blocked in Wait never holds up another thread's Isend.  Collectives
// take it only for their progress passes (one call at a time per
// communicator, as MPI requires).
// Recursive, and YIELDABLE: a thread that waits inside a locked call (an RMA
// fence or lock, a host exchange) gives the lock up while it polls
// (yield_big_lock), so that e.g. one thread in Win_fence never blocks another
// thread's Isend that a peer needs before it can reach the fence.
struct BigLock {
  std::mutex m;
  std::atomic<std::thread::id> owner{};
  int depth = 0;
  void lock() {
    if (owner.load(std::memory_order_relaxed) == std::this_thread::get_id()) {
      ++depth;
      return;
    }
    m.lock();
    owner.store(std::this_thread::get_id(), std::memory_order_relaxed);
    depth = 1;
  }
  void unlock() {
    if (--depth == 0) {
      owner.store(std::thread::id(), std::memory_order_relaxed);
      m.unlock();
    }
  }
};
BigLock& big_lock();
// In a wait loop: if this thread holds the big lock, release it completely,
// let other threads in, and take it back at the same depth.
void yield_big_lock();
// Some peer of c can no longer take part: its process is gone or its
// communicator failed (shm flags).  Point-to-point and RMA waits use it as
// their only way out: like the collectives they wait for a live late peer.
bool peer_dead(const mpigx_comm* c);
// RMA accumulate (datatype, op) check incl. REPLACE / NO_OP: rep, size, op code
int acc_check(int datatype, int op, int* rep, int* esize, int* oc);
double wall();
int pull_fences();  // MPIGX_PULL_FENCES (default 1): coherent flag of p2p / RMA pull kernels
// p2p.cpp
void p2p_progress(mpigx_comm* c);
void p2p_sync(mpigx_comm* c);     // drain the transfer stream
void p2p_destroy(mpigx_comm* c);
// types.cpp
struct TypeDesc {
  long long size;    // packed bytes per element
  long long extent;  // bytes between consecutive elements in memory
  int basic;         // predefined type every byte belongs to (0: mixed)
  bool derived;
  bool contig;       // count elements = count*size contiguous bytes from the pointer
};
int type_info(int datatype, TypeDesc* d);  // MPIGX_ERR_TYPE for unknown / uncommitted
// pack (unpack=0: typed -> contig) or unpack the first `bytes` packed bytes of
// `count` elements; enqueued on `s` (device `device`)
int type_pack(int datatype, const void* typed, long long count, void* contig, long long bytes, int unpack, int device,
              hipStream_t s);
// rma.cpp
void rma_progress(mpigx_comm* c);
void rma_destroy(mpigx_comm* c);
void rma_sync(mpigx_comm* c);  // drain the RMA stream
}  // namespace rt
}  // namespace mpigx
