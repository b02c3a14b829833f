// mpigx.cpp — host runtime of libmpigx: the C ABI declared in include/mpigx.h.
//
// Replaces, for device-resident buffers, the libmpi that MPI.jl ccalls
// (src/collective.jl ccall sites :17 :34 :304 :498 :615 :698 :765 :839).
// Responsibilities:
//   * MPICH handle -> element representation / op mapping and the MPICH
//     op x type validity matrix (returns MPI_ERR_OP like MPICH);
//   * communicator bootstrap (src/comm.jl rank -> GPU binding): a POSIX shm
//     rendezvous keyed by a unique id exchanges hipIpc handles of every rank's
//     staging arena (HBM) and signal array (uncached HBM);
//   * per-call planning: MPICH-compatible fold schedule (binomial vs
//     Rabenseifner regime, operand roles), one-shot vs two-shot algorithm,
//     grid and slice sizes, rounds that bound the staging arena;
//   * blocking MPI semantics on a HIP stream with device-side timeouts turned
//     into MPI error classes.
#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mpigx_diag.h"
#include "common.hpp"
#include "handles.hpp"
#include "launch.hpp"
#include "runtime.hpp"

using namespace mpigx;

namespace {

// ---------------------------------------------------------------------------
// datatypes / ops (deps/consts_mpich.jl:30-72; src/datatypes.jl:29-60)
// ---------------------------------------------------------------------------
struct TypeInfo {
  int handle;
  Rep rep;
  int size;
  int kind;  // 0 int, 1 float, 2 complex, 3 byte (bitwise only), 4 none (copies only)
};
const TypeInfo kTypes[] = {
    {MPIGX_INT8_T, R_I8, 1, 0},          {MPIGX_UINT8_T, R_U8, 1, 0},
    {MPIGX_INT16_T, R_I16, 2, 0},        {MPIGX_UINT16_T, R_U16, 2, 0},
    {MPIGX_INT32_T, R_I32, 4, 0},        {MPIGX_UINT32_T, R_U32, 4, 0},
    {MPIGX_INT64_T, R_I64, 8, 0},        {MPIGX_UINT64_T, R_U64, 8, 0},
    {MPIGX_BYTE, R_U8, 1, 3},            {MPIGX_SHORT, R_I16, 2, 0},
    {MPIGX_UNSIGNED_SHORT, R_U16, 2, 0}, {MPIGX_INT, R_I32, 4, 0},
    {MPIGX_UNSIGNED, R_U32, 4, 0},       {MPIGX_LONG, R_I64, 8, 0},
    {MPIGX_UNSIGNED_LONG, R_U64, 8, 0},  {MPIGX_CHAR, R_I8, 1, 0},
    {MPIGX_SIGNED_CHAR, R_I8, 1, 0},     {MPIGX_UNSIGNED_CHAR, R_U8, 1, 0},
    {MPIGX_WCHAR, R_I32, 4, 4},          {MPIGX_FLOAT, R_F32, 4, 1},
    {MPIGX_DOUBLE, R_F64, 8, 1},         {MPIGX_C_FLOAT_COMPLEX, R_C64, 8, 2},
    {MPIGX_C_DOUBLE_COMPLEX, R_C128, 16, 2},
    {MPIGX_BFLOAT16, R_BF16, 2, 1},
};

const TypeInfo* find_type(int h) {
  for (const auto& t : kTypes)
    if (t.handle == h) return &t;
  return nullptr;
}

int op_code(int h) {
  switch (h) {
    case MPIGX_SUM: return O_SUM;
    case MPIGX_PROD: return O_PROD;
    case MPIGX_MIN: return O_MIN;
    case MPIGX_MAX: return O_MAX;
    case MPIGX_LAND: return O_LAND;
    case MPIGX_LOR: return O_LOR;
    case MPIGX_LXOR: return O_LXOR;
    case MPIGX_BAND: return O_BAND;
    case MPIGX_BOR: return O_BOR;
    case MPIGX_BXOR: return O_BXOR;
    default: return O_NONE;
  }
}

// MPICH 3.3.2 op x type matrix (probed with MPI_Reduce_local, pinned in
// tests/golden/op_type_matrix.json).
int validate(int dtype, int op, const TypeInfo** ti, int* oc) {
  const TypeInfo* t = find_type(dtype);
  if (!t) return MPIGX_ERR_TYPE;
  const int o = op_code(op);
  if (o == O_NONE) return MPIGX_ERR_OP;
  bool ok = false;
  switch (t->kind) {
    case 0: ok = true; break;
    case 1: ok = !(o == O_BAND || o == O_BOR || o == O_BXOR); break;
    case 2: ok = (o == O_SUM || o == O_PROD); break;
    case 3: ok = (o == O_BAND || o == O_BOR || o == O_BXOR); break;
    default: ok = false;
  }
  if (!ok) return MPIGX_ERR_OP;
  if (ti) *ti = t;
  if (oc) *oc = o;
  return MPIGX_SUCCESS;
}

FoldLauncher fold_launcher(Rep r) {
  switch (r) {
    case R_I8: return launch_fold_i8;
    case R_U8: return launch_fold_u8;
    case R_I16: return launch_fold_i16;
    case R_U16: return launch_fold_u16;
    case R_I32: return launch_fold_i32;
    case R_U32: return launch_fold_u32;
    case R_I64: return launch_fold_i64;
    case R_U64: return launch_fold_u64;
    case R_F32: return launch_fold_f32;
    case R_F64: return launch_fold_f64;
    case R_C64: return launch_fold_c64;
    case R_C128: return launch_fold_c128;
    case R_BF16: return launch_fold_bf16;
    default: return nullptr;
  }
}
RingLauncher ring_launcher(Rep r) {
  switch (r) {
    case R_I8: return launch_ring_i8;
    case R_U8: return launch_ring_u8;
    case R_I16: return launch_ring_i16;
    case R_U16: return launch_ring_u16;
    case R_I32: return launch_ring_i32;
    case R_U32: return launch_ring_u32;
    case R_I64: return launch_ring_i64;
    case R_U64: return launch_ring_u64;
    case R_F32: return launch_ring_f32;
    case R_F64: return launch_ring_f64;
    case R_C64: return launch_ring_c64;
    case R_C128: return launch_ring_c128;
    case R_BF16: return launch_ring_bf16;
    default: return nullptr;
  }
}
ArzcLauncher arzc_launcher(Rep r) {
  switch (r) {
    case R_I8: return launch_arzc_i8;
    case R_U8: return launch_arzc_u8;
    case R_I16: return launch_arzc_i16;
    case R_U16: return launch_arzc_u16;
    case R_I32: return launch_arzc_i32;
    case R_U32: return launch_arzc_u32;
    case R_I64: return launch_arzc_i64;
    case R_U64: return launch_arzc_u64;
    case R_F32: return launch_arzc_f32;
    case R_F64: return launch_arzc_f64;
    case R_C64: return launch_arzc_c64;
    case R_C128: return launch_arzc_c128;
    case R_BF16: return launch_arzc_bf16;
    default: return nullptr;
  }
}
// Resident 256-thread blocks per CU of ONE kernel that spins on its peers
// (hipOccupancyMaxActiveBlocksPerMultiprocessor; process-wide cache): kind
// 0 fold_kernel (a = nmax, b = sched), 1 ar_zc_kernel (a = nmax, b = shape),
// 2 ring_kernel, 3 scan_kernel, 4 ar_zc_kernel AG_PUSH (kern_rep.hip
// occ_op), 10 copy_kernel and
// 11 vx_kernel of an a-rank communicator (copy.hip).
enum OccKind { OK_FOLD = 0, OK_ARZC = 1, OK_RING = 2, OK_SCAN = 3, OK_ARZC_PUSH = 4, OK_COPY = 10, OK_VX = 11 };
int kernel_occ(int rep, int op, int kind, int a, int b) {
  static std::mutex mu;
  static std::vector<std::pair<unsigned long long, int>> cache;
  const unsigned long long key = ((unsigned long long)(rep + 1) << 40) | ((unsigned long long)(op + 1) << 32) |
                                 ((unsigned long long)kind << 16) | ((unsigned long long)a << 8) | (unsigned)b;
  std::lock_guard<std::mutex> g(mu);
  for (auto& e : cache)
    if (e.first == key) return e.second;
  static const OccQuery qs[R_COUNT] = {occupancy_i8,  occupancy_u8,  occupancy_i16, occupancy_u16, occupancy_i32,
                                       occupancy_u32, occupancy_i64, occupancy_u64, occupancy_f32, occupancy_f64,
                                       occupancy_c64, occupancy_c128, occupancy_bf16};
  int v = 0;
  if (kind == OK_COPY) v = occupancy_copy(a);
  else if (kind == OK_VX) v = occupancy_vx(a);
  else if (rep >= 0 && rep < R_COUNT) v = qs[rep](op, kind, a, b);
  cache.push_back({key, v});
  return v;
}
ScanLauncher scan_launcher(Rep r) {
  switch (r) {
    case R_I8: return launch_scan_i8;
    case R_U8: return launch_scan_u8;
    case R_I16: return launch_scan_i16;
    case R_U16: return launch_scan_u16;
    case R_I32: return launch_scan_i32;
    case R_U32: return launch_scan_u32;
    case R_I64: return launch_scan_i64;
    case R_U64: return launch_scan_u64;
    case R_F32: return launch_scan_f32;
    case R_F64: return launch_scan_f64;
    case R_C64: return launch_scan_c64;
    case R_C128: return launch_scan_c128;
    case R_BF16: return launch_scan_bf16;
    default: return nullptr;
  }
}

long long env_ll(const char* name, long long dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  return strtoll(v, nullptr, 0);
}

int pof2_of(int n) {
  int p = 1;
  while (p * 2 <= n) p *= 2;
  return p;
}
int log2i(int p) {
  int l = 0;
  while ((1 << l) < p) ++l;
  return l;
}
long long cdiv(long long a, long long b) { return (a + b - 1) / b; }
long long rup(long long a, long long b) { return cdiv(a, b) * b; }

// ---------------------------------------------------------------------------
// shm rendezvous
// ---------------------------------------------------------------------------
// (ShmBlock / ShmRank: runtime.hpp)

// Unique id payload (fits in mpigx_unique_id_t::internal).
struct IdPayload {
  char name[64];
  uint64_t magic;
};

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

}  // namespace

// (struct mpigx_comm: runtime.hpp)

namespace {

#define HIPCK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "[mpigx] %s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return MPIGX_ERR_INTERN;                                                     \
    }                                                                              \
  } while (0)

int host_allgather_wait(mpigx_comm* c, const void* mine, int len, void* out, bool until_gone);
bool peer_gone(const mpigx_comm* c, int q);

// A failed communicator never joins another collective: say so in the shm
// block, where every peer's host wait (finish, host_allgather_wait) looks, so
// the peers fail at once instead of waiting for a rank that will not come.
void mark_broken(mpigx_comm* c) {
  c->broken = true;
  if (c->shm) c->shm->ranks[c->rank].broken.store(1, std::memory_order_release);
}
// the first peer whose communicator failed, or -1
int peer_broken(const mpigx_comm* c) {
  if (!c->shm) return -1;
  for (int q = 0; q < c->n; ++q)
    if (q != c->rank && c->shm->ranks[q].broken.load(std::memory_order_acquire)) return q;
  return -1;
}

// Ranks sharing a GPU (the test box; one rank per GPU never takes this):
// before a collective kernel is enqueued, this rank's earlier work on the
// stream has finished and every rank has got that far (a host barrier over
// the shm control plane), so the ranks' kernels start together and spin for
// microseconds.  Without it, ranks that arrived early spin on the device that
// the late rank's own kernels need: with 8 ranks on one GPU a late rank's
// torch compare (nonzero) took 5.7 s and a device synchronize over a minute
// while its peers spun (r04k), and calls timed out.  The wait has no time
// limit while the late rank's process lives: its own stream can stay busy
// for over a minute with torch work alone when 8 processes share the GPU
// (r04q: a rank's torch.nonzero kernels, no collective kernel of anyone
// running), and a collective must not fail for a late peer.  Blocking
// communicators only (stream-ordered ones cannot wait); MPIGX_SHARED_GATE=0
// disables it.
int shared_gate(mpigx_comm* c) {
  if (c->dev_share <= 1 || !c->blocking || !c->shared_gate || c->n == 1) return MPIGX_SUCCESS;
  // poll first: a drained (or nearly drained) stream is the common case in a
  // loop of collectives, and the query costs far less than a synchronize
  const double t0 = now_s();
  hipError_t q;
  while ((q = hipStreamQuery(c->stream)) == hipErrorNotReady && now_s() - t0 < 2e-3) {
  }
  if (q == hipErrorNotReady) HIPCK(hipStreamSynchronize(c->stream));
  else if (q != hipSuccess) HIPCK(q);
  int z = 0, all[kMaxRanks];
  return host_allgather_wait(c, &z, sizeof z, all, true);
}

// Late or stuck.  Every spinning kernel needs its whole
// grid resident together with its peers' grids.  Collectives of several
// communicators in flight at once (threads, or streams) can fill a GPU with
// grids whose partners are resident nowhere: GPU 0 holds A and B, GPU 1 B
// and C, GPU 2 A and C, each waiting for a grid its peer cannot make
// resident.  Such a peer looks like a late one (its GPU has not reached the
// launch), and a late peer is waited for without limit — so the cycle never
// ended.  What separates the two: the stuck peer's HOST enqueued the launch
// long ago (kseq_enq), its GPU has not started it (kseq_run), and its
// process has another communicator's collective in flight (proc_busy >= 2).
// The same holds when two communicators' streams share one hardware queue
// (HIP maps streams onto GPU_MAX_HW_QUEUES queues, 4 by default): a launch
// queued behind another communicator's spinning kernel cannot start until
// that kernel ends, and the queue order differs from rank to rank (r06b).
// busy_comms() is that count for this process: blocking calls inside
// finish()'s wait, plus stream-ordered communicators whose stream the watcher
// last found busy.
namespace {
std::atomic<int> g_live_comms{0};     // communicators of this process (init .. release)
std::atomic<int> g_busy_blocking{0};  // finish() waits in progress
std::atomic<int> g_busy_streams{0};   // watched stream-ordered communicators with work queued
struct BusyWait {
  BusyWait() { g_busy_blocking.fetch_add(1, std::memory_order_relaxed); }
  ~BusyWait() { g_busy_blocking.fetch_sub(1, std::memory_order_relaxed); }
};
}  // namespace
int busy_comms() {
  return g_busy_blocking.load(std::memory_order_relaxed) + g_busy_streams.load(std::memory_order_relaxed);
}
// The first peer that has been stuck in launch L (enqueued, never started,
// other communicators busy in its process) for longer than tmo seconds, or
// -1.  since[q] remembers when q was first seen so; any other state resets
// it.  Called every 0.25 s, by finish() with c->stuck_since and by the
// watcher thread with c->wstuck_since (a communicator can have both: a
// blocking call after stream-ordered launches).
int stuck_peer(mpigx_comm* c, unsigned long long L, double t, double tmo, double* since) {
  int who = -1;
  for (int q = 0; q < c->n; ++q) {
    if (q == c->rank) continue;
    const ShmRank& sr = c->shm->ranks[q];
    const bool s = sr.kseq_enq.load(std::memory_order_relaxed) >= L &&
                   sr.kseq_run.load(std::memory_order_acquire) < L && sr.proc_busy.load(std::memory_order_relaxed) >= 2;
    if (!s) {
      since[q] = 0;
      continue;
    }
    if (since[q] == 0) since[q] = t;
    if (who < 0 && t - since[q] > tmo) who = q;
  }
  return who;
}
void note_stuck(mpigx_comm* c, int who, double t, const double* since) {
  fprintf(stderr, "[mpigx] rank %d: rank %d enqueued this launch %.0f s ago but its GPU never started it while "
          "other communicators' collectives run in its process: more communicators are in flight at once than "
          "the GPU holds resident together (set MPIGX_CONCURRENT_COMMS to their number), or their streams share "
          "a hardware queue (GPU_MAX_HW_QUEUES at least the number of streams in use)\n", c->rank, who,
          t - since[who]);
}

// Stream-ordered (RCCL-style) launches wait for a late peer too (round 5):
// like ncclAllReduce they have no time limit — nobody waits on the host for
// them — and one process-wide watcher thread does for every communicator
// that has made a stream-ordered launch what finish() does for a blocking
// call: it publishes the launch this rank's GPU has reached
// (ShmRank.kseq_run) and whether its stream has work (proc_busy), and stores
// the cancel word when the wait cannot end, i.e. when a peer's communicator
// failed or its process is gone, or when a peer is stuck in the launch this
// GPU has sat in past the timeout (stuck_peer; checked every 0.25 s).  The
// cancelled kernels record a timeout in the error word, which the next
// synchronizing call reports (mpigx_comm_synchronize / any blocking call),
// breaking the communicator.  The every-rank-in-the-launch stall rule
// applies only while other communicators' collectives are in flight (the
// partial-residency deadlock); otherwise a stream-ordered launch that never
// completes for a protocol reason hangs, as an RCCL kernel would.
// One thread for the process however many communicators there are (an
// application with hundreds of Comm_split results must not get hundreds of
// 100 Hz threads); it runs while at least one communicator is registered
// and exits by itself when the last is released.  The registry is never
// destroyed (a static destructor at exit would race the detached thread).
namespace {
struct PeerWatch {
  std::mutex m;
  std::vector<mpigx_comm*> comms;
  bool running = false;
};
PeerWatch& peer_watch() {
  static PeerWatch* w = new PeerWatch;
  return *w;
}
void watch_one(mpigx_comm* c, bool check) {
  if (!c->shm) return;
  const unsigned long long st = *c->started;
  ShmRank& me = c->shm->ranks[c->rank];
  me.kseq_run.store(st, std::memory_order_release);
  me.proc_busy.store(busy_comms(), std::memory_order_relaxed);
  if (!check || __atomic_load_n(c->cancel, __ATOMIC_ACQUIRE)) return;  // already cancelled (finish or here)
  const double t = now_s();
  if (st != c->watch_seen || c->watch_moved == 0) {
    c->watch_seen = st;
    c->watch_moved = t;
  }
  int who = peer_broken(c);
  const char* why = who >= 0 ? "its communicator failed" : nullptr;
  for (int q = 0; !why && q < c->n; ++q)
    if (q != c->rank && peer_gone(c, q)) {
      who = q;
      why = "its process is gone";
    }
  // a peer stuck in the launch my GPU has sat in past the timeout (my stream
  // still has work: launch st has not completed here)
  const double tmo = c->timeout_ticks / 1e8;
  if (!why && st > 0 && c->watch_busy && t - c->watch_moved > tmo) {
    who = stuck_peer(c, st, t, tmo, c->wstuck_since);
    if (who >= 0) {
      note_stuck(c, who, t, c->wstuck_since);
      why = "stuck behind other communicators' kernels";
    } else if (me.kseq_enq.load(std::memory_order_relaxed) == st) {
      // partial residency: launch st is the last this rank enqueued (so my
      // stream holds no later work I could be late with), every rank's GPU
      // is in it, none has left it for the timeout, and other
      // communicators' collectives run somewhere — their grids hold the
      // slots this launch's missing blocks need.  Without other
      // communicators in flight a stream-ordered launch keeps RCCL's rule
      // and waits.
      bool all_in = true, others = busy_comms() >= 2;
      for (int q = 0; q < c->n; ++q) {
        if (q == c->rank) continue;
        all_in &= c->shm->ranks[q].kseq_run.load(std::memory_order_acquire) == st;
        others |= c->shm->ranks[q].proc_busy.load(std::memory_order_relaxed) >= 2;
      }
      if (all_in && others) {
        who = c->rank;
        why = "every rank's GPU is in this launch and none has left it while other communicators' collectives "
              "run (their grids do not fit on the GPU together: set MPIGX_CONCURRENT_COMMS to the number of "
              "communicators in flight at once)";
      }
    }
  }
  if (why) {
    fprintf(stderr, "[mpigx] rank %d: cancelling stream-ordered waits: rank %d: %s\n", c->rank, who, why);
    __atomic_store_n(c->cancel, 1u, __ATOMIC_RELEASE);
  }
}
void watch_peers() {
  PeerWatch& w = peer_watch();
  for (unsigned tick = 1;; ++tick) {
    usleep(10000);
    std::lock_guard<std::mutex> g(w.m);
    if (w.comms.empty()) {
      w.running = false;
      g_busy_streams.store(0, std::memory_order_relaxed);
      return;
    }
    const bool check = tick % 25 == 0;
    if (check) {  // which watched communicators have a launch not yet complete (proc_busy)
      int busy = 0;
      for (mpigx_comm* c : w.comms) {
        // the event recorded after the communicator's last stream-ordered
        // launch (note_launch; the comm's own, unlike the caller's stream)
        const hipError_t q = c->so_ev ? hipEventQuery(c->so_ev) : hipSuccess;
        if (q != hipSuccess && q != hipErrorNotReady) (void)hipGetLastError();
        c->watch_busy = q == hipErrorNotReady;
        busy += c->watch_busy;
      }
      g_busy_streams.store(busy, std::memory_order_relaxed);
    }
    for (mpigx_comm* c : w.comms) watch_one(c, check);
  }
}
// make_view of a stream-ordered launch: register c (once)
void watch_register(mpigx_comm* c) {
  PeerWatch& w = peer_watch();
  std::lock_guard<std::mutex> g(w.m);
  if (c->watched) return;
  c->watched = true;
  w.comms.push_back(c);
  if (!w.running) {
    w.running = true;
    std::thread(watch_peers).detach();
  }
  static const bool at_exit = [] {
    // a process that exits without freeing its communicators: stop watching
    // before the runtime frees the pinned words the watcher reads (exit
    // handlers run in reverse order, and the HIP runtime registered its own
    // before this one)
    std::atexit([] {
      PeerWatch& pw = peer_watch();
      std::lock_guard<std::mutex> l(pw.m);
      for (mpigx_comm* x : pw.comms) x->watched = false;
      pw.comms.clear();
    });
    return true;
  }();
  (void)at_exit;
}
// comm_release: once this returns the watcher never touches c again
void watch_unregister(mpigx_comm* c) {
  if (!c->watched) return;
  PeerWatch& w = peer_watch();
  std::lock_guard<std::mutex> g(w.m);
  w.comms.erase(std::remove(w.comms.begin(), w.comms.end(), c), w.comms.end());
  c->watched = false;
}
}  // namespace

PeerView make_view(mpigx_comm* c) {
  if (c->diag_trace) {  // before every launch: the peers' canaries through my mappings of their signal arrays
    for (int q = 0; q < c->n; ++q) {
      uint64_t* arr = ((c->rw_mask >> q) & 1u) ? c->peer_sig_rw[q] : c->peer_sig[q];
      if (q == c->rank || !arr) continue;
      uint64_t w = 0;
      void* base = nullptr;
      size_t size = 0;
      (void)hipMemcpy(&w, arr + sig_index(kMaxBlocks + 1, 0), sizeof w, hipMemcpyDeviceToHost);
      (void)hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)arr);
      (void)hipGetLastError();
      if (w != (kSigCanary ^ (uint64_t)q) || base != (void*)arr)
        fprintf(stderr, "[trace r%d] MAPPING of peer %d's signal array at %p: canary %llx (want %llx), "
                "allocation base %p size %zu\n", c->rank, q, (void*)arr, (unsigned long long)w,
                (unsigned long long)(kSigCanary ^ (uint64_t)q), base, size);
    }
  }
  // a failed gate (a peer never reached it) breaks the communicator; the
  // launch that follows then gives up at its first barrier
  const bool gate_ok = shared_gate(c) == MPIGX_SUCCESS;
  if (!gate_ok) mark_broken(c);
  PeerView pv;
  memset(&pv, 0, sizeof pv);
  pv.rank = c->rank;
  pv.n = c->n;
  pv.epoch = c->epoch;
  pv.timeout_ticks = gate_ok ? c->timeout_ticks : 0;
  pv.err = c->err_dev;
  pv.done = (c->blocking && c->sync_mode == 1) ? c->done_dev : nullptr;
  pv.dcount = c->dcount_dev;
  pv.dbase = c->dcount_total;
  pv.wbase = c->wtickets;
  pv.fbase = c->wfinished;
  pv.seq = c->launch_seq + 1;
  pv.kseq = c->kseq + 1;
  pv.started = c->started_dev;
  // every launch waits for a late peer until its host cancels: a blocking
  // call's host watches the peers while it waits (finish), a stream-ordered
  // launch's peers are watched by watch_peers (started here, once)
  pv.cancel = c->cancel_dev;
  if (!pv.done && c->n > 1 && c->shm && !c->watched) watch_register(c);
  pv.stamps = c->stamps;
  // each peer gets its words in the array of ITS memory type for me: ordinary
  // memory between ranks of one device, uncached across devices (one memory
  // type per writer / reader pair)
  pv.rw_mask = c->rw_mask;
  pv.sig_uc = c->sig;
  pv.sig_rw = c->sig_rw;
  for (int p = 0; p < c->n; ++p) {
    pv.sig[p] = ((c->rw_mask >> p) & 1u) ? c->peer_sig_rw[p] : c->peer_sig[p];
    pv.stage[p] = c->peer_stage[p];
  }
  return pv;
}

// Account for one launch of `grid` blocks made with view `pv`.
void note_launch(mpigx_comm* c, const PeerView& pv, unsigned grid) {
  if (c->diag_trace)  // diagnostic launch trace (MPIGX_DIAG_TRACE, read at init)
    fprintf(stderr, "[trace r%d] t=%.6f launch epoch=%llu grid=%u key=%u bad=%d dbase=%llu seq=%llu\n", c->rank,
            now_s(), (unsigned long long)pv.epoch, grid, pv.zc_key, pv.zc_bad, (unsigned long long)pv.dbase,
            (unsigned long long)pv.seq);
  if (c->launch_pending) {
    c->last_prelaunch_s = now_s() - c->t_entry;
    c->launch_pending = false;
  }
  c->kseq += 1;
  if (c->shm) c->shm->ranks[c->rank].kseq_enq.store(c->kseq, std::memory_order_relaxed);
  if (pv.done) {
    c->dcount_total += grid;
    c->launch_seq += 1;
    c->done_target = c->launch_seq;
  } else {
    c->unflagged = true;
    // completion marker of a stream-ordered launch for the watcher (is this
    // communicator busy: proc_busy / stuck_peer); ~1 us of host time, spent
    // only while the process has another communicator (alone, this one can
    // never make proc_busy reach 2)
    if (c->n > 1 && c->shm && g_live_comms.load(std::memory_order_relaxed) >= 2) {
      if (!c->so_ev && hipEventCreateWithFlags(&c->so_ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        c->so_ev = nullptr;
      }
      if (c->so_ev && hipEventRecord(c->so_ev, c->stream) != hipSuccess) (void)hipGetLastError();
    }
  }
}

int barrier_launch(mpigx_comm* c);

// After enqueueing: in blocking mode wait and translate device errors.  The
// wait spins on the host-mapped completion counter (every block of every
// launch adds 1 after its last access) — ~13 us less than
// hipStreamSynchronize per call (tools/latency.py); stream-ordered work
// enqueued earlier without the counter falls back to a stream sync.
int finish(mpigx_comm* c) {
  if (!c->blocking) return MPIGX_SUCCESS;
  bool cancelled = false;
  if (c->unflagged || c->sync_mode != 1) {
    HIPCK(hipStreamSynchronize(c->stream));
    c->unflagged = false;
    if (c->sync_mode == 1 && c->launch_seq) {
      const unsigned long long w = *c->done;  // complete: the last flagged launch's word
      c->last_aborted = (w >> 1) == c->launch_seq && (w & 1) != 0;
    }
    // stream-ordered launches the watcher cancelled (watch_one)
    cancelled = __atomic_load_n(c->cancel, __ATOMIC_ACQUIRE) != 0;
  } else {
    // While the kernels run, this host watches the peers (round 5, VERDICT
    // r04 item 2): MPI_Allreduce (collective.jl:698-700) waits for a late
    // rank as long as it takes, so the kernels' polls do not give up on time
    // (PeerView.cancel).  The host stores the cancel word — and the call
    // fails, MPI_ERR_OTHER — only when the wait cannot end:
    //   * a peer's communicator failed (ShmRank.broken) or its process is
    //     gone: checked every 0.25 s, so a vanished peer fails the call in
    //     about a second;
    //   * a peer is stuck, not late (round 6, VERDICT r05 item 2,
    //     stuck_peer): its host enqueued the launch my GPU is in, its GPU has
    //     not started it for longer than the timeout, and its process has
    //     other communicators' collectives in flight — their grids hold the
    //     GPU, so this one can never become resident;
    //   * my GPU has been in one of THIS wait's launches for longer than the
    //     timeout and every peer's GPU has reached that launch too
    //     (ShmRank.kseq_run): nobody is late, the protocol itself is stuck.
    // A peer whose GPU has not reached the launch yet (its host is in a long
    // host phase, or its stream still runs earlier work) is late: waited for,
    // with one note to stderr once the timeout has passed.  So am I, while my
    // own GPU has not started any launch of this wait (my stream still runs
    // the caller's earlier work: ADVICE r05) — my peers wait for me, and I
    // declare nothing.
    BusyWait busy;  // this process has a collective in flight (proc_busy)
    const double t0 = now_s();
    const double tmo = c->timeout_ticks / 1e8;
    double next_watch = t0 + 0.25, t_moved = t0;
    unsigned long long seen = *c->started;
    bool noted = false;
    unsigned spins = 0;
    unsigned long long w;
    for (int q = 0; q < c->n; ++q) c->stuck_since[q] = 0;
    while (((w = *c->done) >> 1) < c->done_target) {
      // keep point-to-point rendezvous moving while blocked here (a peer may
      // wait on our acknowledgement before it joins this collective)
      if ((spins & 63) == 0) rt::progress_all(c);
      if ((++spins & 1023) == 0) {
        const double t = now_s(), el = t - t0;
        const unsigned long long st = *c->started;
        if (st != seen) {
          seen = st;
          t_moved = t;
        }
        if (c->shm) {
          c->shm->ranks[c->rank].kseq_run.store(st, std::memory_order_release);
          c->shm->ranks[c->rank].proc_busy.store(busy_comms(), std::memory_order_relaxed);
        }
        // The completion word is the only source of the zero-copy verdict, so
        // it is never replaced by an older one.  A stream that drained without
        // it (every block of the last launch counts itself and the last one
        // stores the word before the kernel ends) means the word is lost —
        // a protocol failure, reported, not guessed past.
        if (el > 0.05 && hipStreamQuery(c->stream) == hipSuccess) {
          HIPCK(hipStreamSynchronize(c->stream));
          const double t1 = now_s();
          while (((w = *c->done) >> 1) < c->done_target && now_s() - t1 < 1.0) sched_yield();
          if ((w >> 1) < c->done_target) {
            fprintf(stderr, "[mpigx] rank %d: completion word %llu never arrived for launch %llu (stream drained)\n",
                    c->rank, (unsigned long long)(w >> 1), (unsigned long long)c->done_target);
            mark_broken(c);
            c->last_aborted = false;
            return MPIGX_ERR_INTERN;
          }
          break;
        }
        if (!cancelled && t >= next_watch && c->shm) {
          next_watch = t + 0.25;
          int who = peer_broken(c);
          const char* why = who >= 0 ? "its communicator failed" : nullptr;
          for (int q = 0; !why && q < c->n; ++q)
            if (q != c->rank && peer_gone(c, q)) {
              who = q;
              why = "its process is gone";
            }
          // my GPU is in a launch of this wait (seen > kseq_done); the late /
          // stuck / stall rules below judge the peers against THAT launch
          const bool mine_running = seen > c->kseq_done;
          if (!why && mine_running) {
            const int stuck = stuck_peer(c, seen, t, tmo, c->stuck_since);
            if (stuck >= 0) {
              note_stuck(c, stuck, t, c->stuck_since);
              who = stuck;
              why = "stuck behind other communicators' kernels";
            }
          }
          if (!why && mine_running && t - t_moved > tmo) {
            int late = -1;
            for (int q = 0; q < c->n && late < 0; ++q)
              if (q != c->rank && c->shm->ranks[q].kseq_run.load(std::memory_order_acquire) < seen) late = q;
            if (late < 0) {
              // partial residency: every rank's block 0 started but not all
              // blocks are resident — the same cause as a stuck peer when
              // other communicators' collectives are in flight somewhere
              bool others = busy_comms() >= 2;
              for (int q = 0; q < c->n && !others; ++q)
                others = c->shm->ranks[q].proc_busy.load(std::memory_order_relaxed) >= 2;
              who = c->rank;  // (the message names no peer: every rank is in the launch)
              why = others ? "every rank's GPU is in this launch and none has moved while other communicators' "
                             "collectives run (their grids do not fit on the GPU together: set "
                             "MPIGX_CONCURRENT_COMMS to the number of communicators in flight at once)"
                           : "every rank's GPU is in this launch and none has moved (protocol stall)";
            } else if (!noted) {
              noted = true;
              fprintf(stderr, "mpigx: rank %d has waited %.0f s for rank %d to reach the collective\n", c->rank, el,
                      late);
            }
          } else if (!why && !mine_running && el > tmo && !noted) {
            noted = true;
            fprintf(stderr, "mpigx: rank %d has waited %.0f s for its own stream to reach the collective\n", c->rank,
                    el);
          }
          if (why) {
            fprintf(stderr, "[mpigx] rank %d: cancelling launch %llu: rank %d: %s\n", c->rank, seen, who, why);
            __atomic_store_n(c->cancel, 1u, __ATOMIC_RELEASE);
            cancelled = true;
          }
        }
        // a long wait: leave the host cores to the late rank
        if (el > 0.05 && !cancelled) usleep(50);
      }
    }
    if (c->shm) c->shm->ranks[c->rank].kseq_run.store(*c->started, std::memory_order_release);
    // the last launch's zero-copy verdict (kernels.hpp signal_done): only
    // from the word of exactly that launch
    c->last_aborted = (w >> 1) == c->done_target && (w & 1) != 0;
  }
  if (const unsigned e = __atomic_load_n(c->err, __ATOMIC_ACQUIRE)) {
    // device.hpp kErrTimeout (a peer did not arrive / the wait was
    // cancelled) / kErrProtocol
    mark_broken(c);
    return e == 2 ? MPIGX_ERR_INTERN : MPIGX_ERR_OTHER;
  }
  if (cancelled) {
    // the cancel word stays set (every later wait would give up after 1 ms)
    // and it was stored because the wait could not end: the call fails and
    // the communicator with it, even if every block happened to finish
    // 
    mark_broken(c);
    return MPIGX_ERR_OTHER;
  }
  c->kseq_done = c->kseq;
  return MPIGX_SUCCESS;
}

// Grid cap of a kernel whose blocks spin on their peers: every rank's grid
// must be resident at once, so at most CUs x (resident blocks per CU of THAT
// kernel) / (ranks sharing the most-loaded device).  The occupancy API can
// admit one block per CU more than the hardware where SGPRs bind (>= 6 blocks
// of 256 threads, MI355X_MICROARCH.md "Residency"): one fewer there;
// VGPR-bound counts (<= 5) are exact.  The same on every rank (same kernel,
// agreed cus_min / dev_share).
// Ranks sharing a device (the 1-GPU test box) never fill it: every rank's
// grids at exactly the occupancy limit (e.g. 4 x 256 blocks of a 126-VGPR
// kernel at n = 4) timed out in one run of three, all ranks launching the
// same grid at the same epoch within a millisecond (tools/scan_repro.py,
// DESIGN §3 "Ranks sharing a GPU") — some blocks of some rank never became
// resident while the others spun.  So at most occupancy - 1 blocks per CU
// in total there (three quarters of the CUs at occupancy 1).  One rank per
// GPU is unaffected (its 256-block grid is at most one block per CU).
// The rule holds at EVERY share count > 1 (round 5; round 4 applied it from
// 4 ranks up): r04u recorded, at 8 ranks with grids filling every CU slot,
// one rank's scan blocks becoming resident only when the other ranks' blocks
// gave up 30 s later; nothing about 2 ranks makes that impossible — any other
// resident kernel (a peer's torch work) takes the slot a spinning grid needs.
// MPIGX_SHARE_HEADROOM = 0 turns it off (measurement only).
// Concurrent communicators (MPIGX_CONCURRENT_COMMS = K, agreed): collectives
// of K communicators may spin on one GPU at once (threads, or stream-ordered
// launches on separate streams); a kernel's blocks wait only for the same
// blocks of ITS peers, so all K kernels must fit together or a GPU can fill up
// with blocks whose partners are not resident anywhere (seen with 3 ranks x 3
// communicators on one GPU: every rank's GPU in a launch, none moving).  The
// share of every communicator is therefore one K-th of the device.
int kernel_cap(mpigx_comm* c, int occ) {
  const long long share = (long long)(c->dev_share > 0 ? c->dev_share : 1) * (c->concurrent_comms > 0 ? c->concurrent_comms : 1);
  long long cap;
  const bool headroom = c->share_headroom != 0;
  if (share > 1 && headroom)
    cap = occ >= 2 ? (long long)c->cus_min * (occ - 1) / share : (long long)c->cus_min * 3 / (4 * share);
  else if (share > 1)
    cap = (long long)c->cus_min * (occ >= 6 ? occ - 1 : occ > 0 ? occ : 1) / share;
  else
    cap = (long long)c->cus_min * (occ >= 6 ? occ - 1 : occ > 0 ? occ : 1);
  return (int)(cap < 1 ? 1 : cap > kMaxBlocks ? kMaxBlocks : cap);
}
int cap_fold(mpigx_comm* c, const TypeInfo* t, int oc, int nmax, int sched) {
  return kernel_cap(c, kernel_occ(t->rep, oc, OK_FOLD, nmax, sched));
}
int cap_arzc(mpigx_comm* c, const TypeInfo* t, int oc, int nmax, int shape, int ag) {
  return kernel_cap(c, kernel_occ(t->rep, oc, ag == AG_PUSH ? OK_ARZC_PUSH : OK_ARZC, nmax, shape));
}
int cap_ring(mpigx_comm* c, const TypeInfo* t, int oc) { return kernel_cap(c, kernel_occ(t->rep, oc, OK_RING, 0, 0)); }
int cap_scan(mpigx_comm* c, const TypeInfo* t, int oc) { return kernel_cap(c, kernel_occ(t->rep, oc, OK_SCAN, 0, 0)); }
int cap_copy(mpigx_comm* c) { return kernel_cap(c, kernel_occ(-1, -1, OK_COPY, c->n, 0)); }
int cap_vx(mpigx_comm* c) { return kernel_cap(c, kernel_occ(-1, -1, OK_VX, c->n, 0)); }

int grid_for(mpigx_comm* c, long long bytes, int cap) {
  long long g = cdiv(bytes, c->bytes_per_block);
  if (g < 1) g = 1;
  if (g > c->max_blocks) g = c->max_blocks;
  if (g > cap) g = cap;
  return (int)g;
}

// Fold schedule for an n-leaf reduction (MPICH single-node semantics):
//   small (count*size <= 2048 or count < pof2): binomial tree over relative
//   ranks (rel = (rank - root) mod n), lower subtree = inout;
//   large: Rabenseifner as MPICH's Reduce runs it (reduce_scatter_gather;
//   one node's Allreduce = Reduce to rank 0 + Bcast) — even rank 2i folds
//   odd rank 2i+1 (pre-step, inout = even), then the pairwise tree over
//   newranks with owner-based operand roles.  The pre-step roles matter for
//   MIN/MAX with NaN / +-0 only; the large-count MPICH fixtures pin them
//   (tests/golden/mpich_large.npz, n = 5: an odd-inout pre-step differs).
// `ptrs[k]` is what leaf k reads for rank k (staging base or user pointer).
void plan_schedule(mpigx_comm* c, FoldArgs& a, int n, int root, long long count_total, int esize,
                   const void* const* ptrs, int* nmax, int* sched, int order) {
  a.rem = 0;
  a.owner_mode = 0;
  a.pof2_log = 0;
  a.blk_len = 1;
  a.blk_inv = 1.0;
  (void)c;
  if (order == MPIGX_ORDER_LINEAR) {
    *sched = S_LINEAR;
    *nmax = n <= 8 ? 8 : 16;
    a.ntree = n;
    for (int k = 0; k < n; ++k) a.src[k] = ptrs[k];
    return;
  }
  *sched = S_TREE;
  const int pof2 = pof2_of(n);
  if (count_total * esize <= 2048 || count_total < pof2) {
    a.ntree = n;
    for (int k = 0; k < n; ++k) a.src[k] = ptrs[(k + root) % n];
    *nmax = n <= 8 ? 8 : 16;
  } else {
    const int rem = n - pof2;
    a.ntree = pof2;
    a.rem = rem;
    for (int s = 0; s < pof2; ++s) {
      if (s < rem) {
        a.src[s] = ptrs[2 * s];       // inout
        a.src2[s] = ptrs[2 * s + 1];  // in
      } else {
        a.src[s] = ptrs[s + rem];
      }
    }
    a.owner_mode = 1;
    a.pof2_log = log2i(pof2);
    a.blk_len = count_total / pof2;
    a.blk_inv = 1.0 / (double)a.blk_len;
    // NMAX from n, not pof2: n = 9..15 has pof2 = 8 but up to 7 pre-step
    // partners (the fold reads src2[s] for s < NMAX/2) and n-1 peers to
    // gather from (the gather phases cover j < NMAX)
    *nmax = n <= 8 ? 8 : 16;
  }
}

int host_allgather(mpigx_comm* c, const void* mine, int len, void* out);

// ---- zero-copy registration ---------------------------------------------
// A user buffer is exported by the IPC handle of the allocation that holds it
// (hipMemGetAddressRange base) plus an offset; allocations are identified by
// HIP's unique buffer id, so a freed-and-reused address never aliases a stale
// import.  Peers' allocations are opened once and kept (LRU-bounded).
constexpr size_t kZcCache = 64;
constexpr size_t kZcTuples = 32;
constexpr size_t kZcViews = 8;

bool zc_export(mpigx_comm* c, const void* p, char** pbase, unsigned long long* id, long long* off,
               hipIpcMemHandle_t* h, size_t* asize = nullptr) {
  void* base = nullptr;
  size_t size = 0;
  unsigned long long bid = 0;
  if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p) != hipSuccess || !base ||
      hipPointerGetAttribute(&bid, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  // an allocation the loaded HIP runtime cannot map into a peer
  // (runtime.hpp ipc_alloc_max): not exportable — zero-copy calls take the
  // staged path on every rank, p2p stages the message in a pooled temporary
  if (c->ipc_alloc_max > 0 && (long long)size > c->ipc_alloc_max) {
    if (c->diag_trace)
      fprintf(stderr, "[trace r%d] not exporting %zu-byte allocation (IPC limit %lld, HIP runtime %d)\n", c->rank,
              size, c->ipc_alloc_max, c->hip_runtime);
    return false;
  }
  *pbase = (char*)base;
  *id = bid;
  *off = (const char*)p - (const char*)base;
  if (asize) *asize = size;
  // (base, buffer id, size): HIP may recycle a buffer id for a new allocation
  // at a freed one's address; one of another size is certainly another
  // allocation, whose handle this cache must not hand out
  for (auto& r : c->lreg)
    if (r.id == bid && r.base == base && r.size == size) {
      *h = r.h;
      return true;
    }
  hipIpcMemHandle_t hh;
  if (hipIpcGetMemHandle(&hh, base) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (c->lreg.size() >= kZcCache) c->lreg.erase(c->lreg.begin());
  c->lreg.push_back({bid, (char*)base, size, hh});
  if (c->diag_trace)
    fprintf(stderr, "[trace r%d] export base=%p size=%zu end=%p id=%llu\n", c->rank, base, size,
            (char*)base + size, bid);
  *h = hh;
  return true;
}

char* zc_import(mpigx_comm* c, int peer, unsigned long long id, const hipIpcMemHandle_t& h) {
  // keyed by the handle too: the HIP runtime may hand a recycled buffer id to
  // a new allocation (seen with free/alloc of equal sizes), whose handle differs
  for (auto& im : c->imports)
    if (im.peer == peer && im.id == id && !memcmp(&im.h, &h, sizeof h)) {
      im.tick = ++c->tick;
      return im.base;
    }
  void* ptr = nullptr;
  if (c->test_import_fail > 0) {  // fault injection (MPIGX_TEST_IMPORT_FAIL, tests only)
    --c->test_import_fail;
    return nullptr;
  }
  if (c->diag_trace) fprintf(stderr, "[trace r%d] zc import peer %d id=%llu: opening\n", c->rank, peer, id);
  if (hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (c->imports.size() >= kZcCache) {
    long oldest = -1;
    for (size_t i = 0; i < c->imports.size(); ++i)
      if (c->imports[i].pins == 0 && (oldest < 0 || c->imports[i].tick < c->imports[oldest].tick)) oldest = (long)i;
    if (oldest >= 0) {
      // a queued launch of mine may still read the evicted mapping
      (void)hipStreamSynchronize(c->stream);
      rt::p2p_sync(c);
      rt::rma_sync(c);
      (void)hipIpcCloseMemHandle(c->imports[oldest].base);
      c->imports.erase(c->imports.begin() + oldest);
      c->zviews.clear();  // views may point into the closed mapping
    }
  }
  c->imports.push_back({peer, id, (char*)ptr, ++c->tick, 0, h});
  if (c->diag_trace) fprintf(stderr, "[trace r%d] zc import peer %d id=%llu at %p\n", c->rank, peer, id, ptr);
  return (char*)ptr;
}

// ---- zero-copy views ---------------------------------------------------------
// A zero-copy launch reads / writes the peers' USER buffers through IPC
// mappings.  Which mappings is agreed in an exchange over the shm control
// plane (every rank's {buffer id, offset, IPC handle} of send and recv); the
// result is a VIEW: an id (the exchange's sequence number, the same on every
// rank) and every rank's mapped pointers, cached per rank with the serial
// number of each rank's (send, recv) registration.
//
// Blocking calls do not exchange again when the buffers repeat: every rank
// launches at once with the most recent view whose entry for itself matches
// its current buffers, or flagged bad if it has none.  The launch's entry
// barrier carries the view id and the flag (device.hpp rank_barrier): a
// mismatch or a flag anywhere aborts the launch on every rank before any
// peer byte is touched; the host then sees the abort, all ranks exchange and
// the launch is repeated on the fresh view.  The steady state (the same
// buffers call after call, as in any training or benchmark loop) costs no
// host round trip; a change costs one empty launch.  Stream-ordered calls
// cannot wait for that verdict and always exchange first.
struct ZcBlob {
  int ok;
  unsigned serial;
  unsigned long long id[2];
  long long off[2];
  long long avail[2];         // bytes of the allocation from the buffer to its end
  unsigned long long raw[2];  // the owner's own pointers (launch trace only)
  hipIpcMemHandle_t h[2];
};
static_assert(sizeof(ZcBlob) <= 256, "control-plane blob");

// Serial number of my (send, recv) registration; 0 = not exportable.
unsigned zc_register(mpigx_comm* c, const void* send, void* recv, ZcBlob* mine) {
  memset(mine, 0, sizeof *mine);
  char* base[2];
  size_t asz[2] = {0, 0};
  if (!zc_export(c, send, &base[0], &mine->id[0], &mine->off[0], &mine->h[0], &asz[0]) ||
      !zc_export(c, recv, &base[1], &mine->id[1], &mine->off[1], &mine->h[1], &asz[1]))
    return 0;
  mine->ok = 1;
  for (int k = 0; k < 2; ++k) mine->avail[k] = (long long)asz[k] - mine->off[k];
  mine->raw[0] = (unsigned long long)(uintptr_t)send;
  mine->raw[1] = (unsigned long long)(uintptr_t)recv;
  for (auto& t : c->ztuples)
    if (t.id[0] == mine->id[0] && t.id[1] == mine->id[1] && t.off[0] == mine->off[0] && t.off[1] == mine->off[1] &&
        t.base[0] == base[0] && t.base[1] == base[1] && !memcmp(t.h, mine->h, sizeof t.h)) {
      t.tick = ++c->tick;
      mine->serial = t.serial;
      return t.serial;
    }
  if (c->ztuples.size() >= kZcTuples) {
    size_t old = 0;
    for (size_t i = 1; i < c->ztuples.size(); ++i)
      if (c->ztuples[i].tick < c->ztuples[old].tick) old = i;
    c->ztuples.erase(c->ztuples.begin() + old);
  }
  mpigx_comm::ZcTuple t;
  memset(&t, 0, sizeof t);
  for (int k = 0; k < 2; ++k) {
    t.base[k] = base[k];
    t.id[k] = mine->id[k];
    t.off[k] = mine->off[k];
    t.h[k] = mine->h[k];
  }
  t.serial = ++c->zserial;
  t.tick = ++c->tick;
  c->ztuples.push_back(t);
  mine->serial = t.serial;
  return t.serial;
}

struct ZcLaunch {
  const char* ps[kMaxRanks];
  char* pr[kMaxRanks];
  long long as[kMaxRanks];  // bytes from ps[q] / pr[q] to the end of rank q's allocation
  long long ar[kMaxRanks];
  unsigned key;
  int bad;
};

// One line per rank of a view (MPIGX_DIAG_TRACE): the pointer this rank uses
// for every peer's buffers, its allocation's end, and what the owner said.
void zc_trace_view(const mpigx_comm* c, const char* what, const ZcLaunch& z, const ZcBlob* all) {
  if (!c->diag_trace) return;
  for (int q = 0; q < c->n; ++q)
    fprintf(stderr,
            "[trace r%d] %s key=%u bad=%d rank %d: send %p (+%lld B) recv %p (+%lld B)%s owner send %llx recv %llx "
            "id %llu/%llu off %lld/%lld\n",
            c->rank, what, z.key, z.bad, q, (const void*)z.ps[q], z.as[q], (void*)z.pr[q], z.ar[q],
            all ? "" : " (cached view)", all ? all[q].raw[0] : 0ull, all ? all[q].raw[1] : 0ull,
            all ? all[q].id[0] : 0ull, all ? all[q].id[1] : 0ull, all ? all[q].off[0] : 0ll, all ? all[q].off[1] : 0ll);
}

// The optimistic launch's pointers: the most recent view in which my entry
// is my current registration; bad = 1 (the launch aborts) if there is none.
void zc_optimistic(mpigx_comm* c, const void* send, void* recv, ZcLaunch* z) {
  memset(z, 0, sizeof *z);
  ZcBlob mine;
  const unsigned ser = zc_register(c, send, recv, &mine);
  const mpigx_comm::ZcView* best = nullptr;
  if (ser)
    for (auto& v : c->zviews)
      if (v.serial[c->rank] == ser && (!best || v.tick > best->tick)) best = &v;
  if (!best) {
    z->bad = 1;
    return;
  }
  for (int q = 0; q < c->n; ++q) {
    z->ps[q] = best->ps[q];
    z->pr[q] = best->pr[q];
    z->as[q] = best->as[q];
    z->ar[q] = best->ar[q];
  }
  z->ps[c->rank] = (const char*)send;
  z->pr[c->rank] = (char*)recv;
  z->as[c->rank] = mine.avail[0];
  z->ar[c->rank] = mine.avail[1];
  z->key = best->id;
  zc_trace_view(c, "optimistic", *z, nullptr);
}

// Exchange: every rank's registration, imports, a new view.  Returns 1 =
// launch with *z, 0 = some rank's buffer is not exportable or some rank could
// not import a peer's (every rank takes the staged path: a second 4-byte
// exchange agrees on the import results, so no rank launches a zero-copy
// kernel that a peer aborts — in stream-ordered mode nobody would learn of
// that abort and recvbuf would stay unwritten), < 0 = -error.
int zc_exchange(mpigx_comm* c, const void* send, void* recv, ZcLaunch* z) {
  memset(z, 0, sizeof *z);
  const int n = c->n;
  ZcBlob mine;
  if (c->diag_trace) fprintf(stderr, "[trace r%d] exchange: registering\n", c->rank);
  zc_register(c, send, recv, &mine);
  if (c->diag_trace) fprintf(stderr, "[trace r%d] exchange: registered ok=%d serial=%u\n", c->rank, mine.ok, mine.serial);
  ZcBlob all[kMaxRanks];
  const int rc = host_allgather(c, &mine, sizeof mine, all);
  if (rc) return -rc;
  c->zstat_exchanges++;
  const unsigned id = (++c->zview_seq) & 0xffffffu;
  for (int q = 0; q < n; ++q)
    if (!all[q].ok) return 0;
  mpigx_comm::ZcView v;
  memset(&v, 0, sizeof v);
  v.id = id;
  bool ok = true;
  for (int q = 0; q < n; ++q) {
    v.serial[q] = all[q].serial;
    v.as[q] = all[q].avail[0];
    v.ar[q] = all[q].avail[1];
    if (q == c->rank) {
      v.ps[q] = (const char*)send;
      v.pr[q] = (char*)recv;
      continue;
    }
    char* sb = zc_import(c, q, all[q].id[0], all[q].h[0]);
    char* rb = all[q].id[1] == all[q].id[0] ? sb : zc_import(c, q, all[q].id[1], all[q].h[1]);
    if (!sb || !rb) {
      ok = false;
      break;
    }
    v.ps[q] = sb + all[q].off[0];
    v.pr[q] = rb + all[q].off[1];
  }
  int iok = ok ? 1 : 0, iall[kMaxRanks];
  const int rc2 = host_allgather(c, &iok, sizeof iok, iall);
  if (rc2) return -rc2;
  for (int q = 0; q < n; ++q)
    if (!iall[q]) return 0;
  v.tick = ++c->tick;
  if (c->zviews.size() >= kZcViews) {
    size_t old = 0;
    for (size_t i = 1; i < c->zviews.size(); ++i)
      if (c->zviews[i].tick < c->zviews[old].tick) old = i;
    c->zviews.erase(c->zviews.begin() + old);
  }
  c->zviews.push_back(v);
  for (int q = 0; q < n; ++q) {
    z->ps[q] = v.ps[q];
    z->pr[q] = v.pr[q];
    z->as[q] = v.as[q];
    z->ar[q] = v.ar[q];
  }
  z->key = id;
  zc_trace_view(c, "exchange", *z, all);
  return 1;
}

bool zc_take_stale(mpigx_comm* c) {
  const bool a = c->last_aborted;
  c->last_aborted = false;
  return a;
}

// Runs one zero-copy collective: `launch(z)` enqueues its kernel(s) with
// view z on every rank (identical grids everywhere).  Returns an error, or
// MPIGX_SUCCESS with *staged = true when the caller must run the staged
// algorithm instead (some rank's buffer cannot be exported).
template <class F>
int zc_run(mpigx_comm* c, const void* send, void* recv, bool* staged, F&& launch) {
  *staged = false;
  ZcLaunch z;
  // the optimistic launch needs the abort verdict before returning: blocking
  // calls completed through the completion word (MPIGX_SYNC_SPIN=1, default)
  if (c->blocking && c->sync_mode == 1 && c->zc_optimistic) {
    zc_optimistic(c, send, recv, &z);
    int rc = launch(z);
    if (!rc) rc = finish(c);
    if (c->diag_trace) fprintf(stderr, "[trace r%d] optimistic launch finished rc=%d aborted=%d\n", c->rank, rc, c->last_aborted ? 1 : 0);
    if (rc) return rc;
    if (!zc_take_stale(c)) {
      c->zstat_hits++;
      return MPIGX_SUCCESS;
    }
  }
  const int r = zc_exchange(c, send, recv, &z);
  if (r < 0) return -r;
  if (r == 0) {
    *staged = true;
    return MPIGX_SUCCESS;
  }
  int rc = launch(z);
  if (!rc) rc = finish(c);
  // every rank imported every mapping (agreed above), so an abort here means
  // a broken protocol, not a missing mapping
  if (!rc && zc_take_stale(c)) rc = MPIGX_ERR_INTERN;
  return rc;
}

void zc_apply(PeerView& pv, const ZcLaunch& z) {
  pv.zc_key = z.key;
  pv.zc_bad = z.bad;
}
// Extents of a zero-copy byte-mover launch (Bcast / Allgather / Alltoall),
// checked on the host against the view's exported allocation sizes — the
// same numbers on every rank, so the same verdict everywhere: every rank's
// region the launch reads holds `src_bytes` from the view's pointer, every
// region it may store into `dst_bytes`.  A failure marks the launch bad, and
// its entry barrier aborts it on every rank before any peer byte is touched
// (ar_zc_kernel and scan_pp_body check the same sizes on the device).
void zc_extents(PeerView& pv, const ZcLaunch& z, int n, long long src_bytes, long long dst_bytes) {
  for (int q = 0; q < n; ++q)
    if (z.as[q] < src_bytes || z.ar[q] < dst_bytes) pv.zc_bad = 1;
}

// Seals a zero-copy launch's argument block (device.hpp args_fault): its
// size in words and the checksum of those words with args_sum itself 0.
// The block must be complete (and its padding zero: every caller memsets it).
template <class Args>
void seal_args(Args& a) {
  static_assert(offsetof(Args, pv) == 0, "the PeerView opens every argument block");
  static_assert(sizeof(Args) % 4 == 0, "word checksum");
  a.pv.args_words = (unsigned)(sizeof(Args) / 4);
  a.pv.args_sum = 0;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&a);
  unsigned sum = 0;
  for (unsigned i = 0; i < a.pv.args_words; ++i) sum += args_mix(w[i], i);
  a.pv.args_sum = sum;
}

// Zero-copy two-shot Allreduce over the whole message (no rounds: nothing is
// staged).  Same chunk/slice partition and fold schedule as M_AR_TWOSHOT.
// push_ag: the pull-push variant (ar_zc_kernel AG_PUSH: the reduce-scatter
// stores into every rank's recvbuf); it needs the dedicated kernel (n <= 8,
// MPICH tree order), otherwise the pull two-shot runs.
int allreduce_zc(mpigx_comm* c, const ZcLaunch& z, long long count, const TypeInfo* t, int oc, bool push_ag) {
  const int n = c->n, es = t->size;
  const int vec = es >= 16 ? 1 : 16 / es;
  FoldArgs a;
  memset(&a, 0, sizeof a);
  a.pv = make_view(c);
  zc_apply(a.pv, z);
  a.mode = M_AR_ZC;
  a.esize = es;
  a.count = count;
  a.gbase = 0;
  a.send = z.ps[c->rank];
  a.recv = z.pr[c->rank];
  for (int p = 0; p < n; ++p) a.zc_recv[p] = z.pr[p];
  int nmax, sched;
  const void* ptrs[kMaxRanks];
  for (int p = 0; p < n; ++p) ptrs[p] = z.ps[p];
  plan_schedule(c, a, n, 0, count, es, ptrs, &nmax, &sched, c->order);
  a.chunk = rup(cdiv(count, n), vec);
  // the dedicated kernel (kernels.hpp ar_zc_kernel) for the MPICH tree at
  // n <= 8; the all-modes fold_kernel for LINEAR order and n > 8 (same bits)
  int znmax, zshape;
  const bool dedicated =
      sched == S_TREE && c->algo != MPIGX_ALGO_PULL_GENERIC && arzc_shape(n, a.ntree, a.rem, &znmax, &zshape);
  // (not from the pointers: a rank whose optimistic view is stale launches
  // with null ones, and every rank must pick the same kernel; unaligned
  // buffers take the kernels' scalar paths)
  const int ag = (push_ag && dedicated) ? AG_PUSH : AG_PULL;
  const int grid = grid_for(c, a.chunk * es, dedicated ? cap_arzc(c, t, oc, znmax, zshape, ag)
                                                        : cap_fold(c, t, oc, nmax, sched));
  a.slice = rup(cdiv(a.chunk, grid), vec);
  long long tickets = 0;
  if (ag == AG_PUSH && c->ar_slices > 0) {
    // dynamic hand-out: ar_slices slices per block (at least 32 KiB each);
    // the kernel consumes my chunk's slices + one past-the-end ticket per block
    a.dyn = 1;
    a.slice = rup(cdiv(a.chunk, (long long)grid * c->ar_slices), vec);
    const long long min_slice = rup(cdiv(32 << 10, es), vec);
    if (a.slice < min_slice) a.slice = min_slice;
    const long long c0 = std::min((long long)c->rank * a.chunk, count), c1 = std::min(c0 + a.chunk, count);
    tickets = cdiv(c1 - c0, a.slice) + grid;
  }
  for (int p = 0; p < n; ++p) a.zc_avail[p] = z.ar[p];
  seal_args(a);
  if (dedicated)
    HIPCK(arzc_launcher(t->rep)(oc, znmax, zshape, ag, dim3(grid), c->stream, a));
  else
    HIPCK(fold_launcher(t->rep)(oc, nmax, sched, dim3(grid), c->stream, a));
  note_launch(c, a.pv, grid);
  if (a.dyn) {
    c->wtickets += tickets;
    c->wfinished += grid;
  }
  c->epoch += ag == AG_PUSH ? 2 : 3;
  return MPIGX_SUCCESS;
}

// Zero-copy Reduce straight into the root's recvbuf: every rank folds its
// chunk from every rank's sendbuf and stores it into chunk r of the root's
// recvbuf through the view's mapping (ar_zc_kernel AG_PUSH in M_RED_ZC mode:
// one output), dynamic slices and the whole-launch exit barrier as for the
// pull-push Allreduce.  No arena, no rounds, no gather by the root.  Returns
// -1 (nothing launched) where the dedicated kernel does not apply (n > 8,
// LINEAR order, MPIGX_ALGO=pull_generic) — the caller runs the arena path
// (M_RED_ZC in fold_kernel).
int reduce_zc_push(mpigx_comm* c, const ZcLaunch& z, long long count, const TypeInfo* t, int oc, int root) {
  const int n = c->n, es = t->size;
  const int vec = es >= 16 ? 1 : 16 / es;
  if (c->algo == MPIGX_ALGO_PULL_GENERIC) return -1;
  FoldArgs a;
  memset(&a, 0, sizeof a);
  a.pv = make_view(c);
  zc_apply(a.pv, z);
  a.mode = M_RED_ZC;
  a.esize = es;
  a.count = count;
  a.gbase = 0;
  a.root = root;
  a.send = z.ps[c->rank];
  a.recv = z.pr[c->rank];
  for (int p = 0; p < n; ++p) a.zc_recv[p] = z.pr[p];
  int nmax, sched;
  const void* ptrs[kMaxRanks];
  for (int p = 0; p < n; ++p) ptrs[p] = z.ps[p];
  plan_schedule(c, a, n, root, count, es, ptrs, &nmax, &sched, c->order);
  // chunks: at n >= 3 only the non-roots own one (n - 1 chunks, root + 1 + i
  // owns chunk i).  With a chunk of its own the root's incoming links carry
  // its peers' pushes AND its own pulls (2S/n each); without, S/(n - 1): at
  // n = 8 S/4 -> S/7 per root link.  At n = 2 the split stays (S per link
  // direction either way, and both ranks' blocks share the work).
  const bool xroot = n >= 3;
  const int owners = xroot ? n - 1 : n;
  a.own = xroot ? (c->rank == root ? n - 1 : (c->rank - root - 1 + n) % n) : c->rank;
  a.chunk = rup(cdiv(count, owners), vec);
  int znmax, zshape;
  // decided from agreed settings only, never from the view's pointers (a
  // stale optimistic view is all null on its rank; see allreduce_zc)
  if (sched != S_TREE || !arzc_shape(n, a.ntree, a.rem, &znmax, &zshape)) return -1;
  const int grid = grid_for(c, a.chunk * es, cap_arzc(c, t, oc, znmax, zshape, AG_PUSH));
  a.slice = rup(cdiv(a.chunk, grid), vec);
  long long tickets = 0;
  if (c->ar_slices > 0) {
    a.dyn = 1;
    a.slice = rup(cdiv(a.chunk, (long long)grid * c->ar_slices), vec);
    const long long min_slice = rup(cdiv(32 << 10, es), vec);
    if (a.slice < min_slice) a.slice = min_slice;
    const long long c0 = std::min((long long)a.own * a.chunk, count), c1 = std::min(c0 + a.chunk, count);
    tickets = cdiv(c1 - c0, a.slice) + grid;
  }
  for (int p = 0; p < n; ++p) a.zc_avail[p] = z.ar[p];
  seal_args(a);
  HIPCK(arzc_launcher(t->rep)(oc, znmax, zshape, AG_PUSH, dim3(grid), c->stream, a));
  note_launch(c, a.pv, grid);
  if (a.dyn) {
    c->wtickets += tickets;
    c->wfinished += grid;
  }
  c->epoch += 2;
  return MPIGX_SUCCESS;
}

// Push two-shot Allreduce (MPIGX_ALGO=push; needs the zero-copy mapping of
// every rank's recvbuf).  Rounds of at most n slots of one chunk each fit the
// arena; per round: my chunk p -> rank p's slot [me] (remote stores), barrier,
// fold my chunk from my slots + my sendbuf (same schedule as every other
// path, so the same bits), result -> every rank's recvbuf, barrier.
int allreduce_push(mpigx_comm* c, const ZcLaunch& z, const void* send, long long count, const TypeInfo* t, int oc) {
  const int n = c->n, r = c->rank, es = t->size;
  const int vec = es >= 16 ? 1 : 16 / es;
  long long round = (long long)(c->stage_bytes / es);
  round = (round / (n * (long long)vec)) * n * vec;
  if (c->ll_unfenced) {
    // the push writes into the peers' arenas before any barrier, relying on
    // their previous launch having ended with one; an LL launch does not (a
    // peer may still be unpacking into its arena), so barrier first.  The
    // flag follows the same collective sequence on every rank.
    const int rc = barrier_launch(c);
    if (rc) return rc;
    c->ll_unfenced = false;
  }
  for (long long off = 0; off < count; off += round) {
    const long long cnt = count - off < round ? count - off : round;
    FoldArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    zc_apply(a.pv, z);
    a.mode = M_AR_PUSH;
    a.esize = es;
    a.count = cnt;
    a.gbase = off;
    a.send = (const char*)send + off * es;
    a.recv = z.pr[r] + off * es;
    for (int p = 0; p < n; ++p) a.zc_recv[p] = z.pr[p] ? z.pr[p] + off * es : nullptr;
    a.chunk = rup(cdiv(cnt, n), vec);
    a.slot_bytes = a.chunk * es;
    // leaf q of my chunk: slot q of my arena holds rank q's copy of it
    // (indexed by the round-relative element e: slot base - c0), my own
    // contribution is read straight from my sendbuf
    const long long c0 = (long long)r * a.chunk;
    const void* ptrs[kMaxRanks];
    for (int q = 0; q < n; ++q)
      ptrs[q] = q == r ? (const void*)a.send : (const void*)(c->stage + (long long)q * a.slot_bytes - c0 * es);
    int nmax, sched;
    plan_schedule(c, a, n, 0, count, es, ptrs, &nmax, &sched, c->order);
    const int grid = grid_for(c, a.chunk * es, cap_fold(c, t, oc, nmax, sched));
    a.slice = rup(cdiv(a.chunk, grid), vec);
    seal_args(a);
    HIPCK(fold_launcher(t->rep)(oc, nmax, sched, dim3(grid), c->stream, a));
    note_launch(c, a.pv, grid);
    c->epoch += 2;
  }
  return MPIGX_SUCCESS;
}

// Ring strides: candidates 1, n-1, 2, n-2, ... coprime with n (each a ring
// through every rank), distinct, at most `want` (oracle/mpich_model.py
// ring_strides is the same rule).
int ring_strides(int n, int want, int* st) {
  int m = 0;
  for (int d = 1; d < n && m < want; ++d) {
    const int cand[2] = {d, n - d};
    for (int j = 0; j < 2 && m < want; ++j) {
      int a = cand[j], b = n;
      while (b) {
        const int t = a % b;
        a = b;
        b = t;
      }
      bool dup = false;
      for (int i = 0; i < m; ++i) dup |= st[i] == cand[j];
      if (a == 1 && !dup) st[m++] = cand[j];
    }
  }
  return m;
}

// Ring reduce-scatter + allgather (MPIGX_ALGO=ring, zero-copy mapping of
// every rank's buffers; kernels.hpp ring_kernel).  MPIGX_RING_CHANNELS rings
// of distinct strides each carry one contiguous part of the message.  Rounds
// bound the partials kept in the staging arena (a round's elements in all).
int allreduce_ring(mpigx_comm* c, const ZcLaunch& z, long long count, const TypeInfo* t, int oc) {
  const int n = c->n, r = c->rank, es = t->size;
  const int vec = es >= 16 ? 1 : 16 / es;
  const int want = c->ring_channels;  // 1..kMaxRings (knob)
  int st[kMaxRings];
  const int nch = ring_strides(n, want, st);
  RingLauncher L = ring_launcher(t->rep);
  long long round = (long long)(c->stage_bytes / es);
  round = (round / ((long long)nch * n * vec)) * nch * n * vec;
  for (long long off = 0; off < count; off += round) {
    const long long cnt = count - off < round ? count - off : round;
    RingArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    zc_apply(a.pv, z);
    a.esize = es;
    a.nch = nch;
    for (int k = 0; k < nch; ++k) {
      a.stride[k] = st[k];
      for (int p = 0; p < n; ++p)
        if ((long long)p * st[k] % n == r) a.pos[k] = p;
    }
    a.count = cnt;
    a.part = rup(cdiv(cnt, nch), (long long)n * vec);
    a.chunk = a.part / n;
    // nch rings share the grid: the whole grid within MAX_BLOCKS and the cap
    const int rcap = cap_ring(c, t, oc);
    int gc = grid_for(c, a.chunk * es, rcap);
    const int lim = c->max_blocks < rcap ? c->max_blocks : rcap;
    if (gc * nch > lim) gc = lim / nch > 0 ? lim / nch : 1;
    a.slice = rup(cdiv(a.chunk, gc), vec);
    for (int q = 0; q < n; ++q) {
      a.zsend[q] = z.ps[q] ? z.ps[q] + off * es : nullptr;
      a.zrecv[q] = z.pr[q] ? z.pr[q] + off * es : nullptr;
    }
    seal_args(a);
    HIPCK(L(oc, dim3(gc * nch), c->stream, a));
    note_launch(c, a.pv, gc * nch);
    c->epoch += 2 * n - 1;
  }
  return MPIGX_SUCCESS;
}

// Shared driver for Allreduce / Reduce.
// LL exchange (device.hpp ll_exchange) for a `bytes`-byte message: taken by
// small Allreduce / Reduce / Scan / Exscan unless MPIGX_ALGO forces the
// staged one-/two-shot.  The decision is identical on every rank (same count,
// knobs that init checked to agree and that only change collectively).
// MPIGX_ALGO=ll takes it up to the area's capacity (MPIGX_LL_MAX), otherwise
// up to MPIGX_LL_AUTO.
bool ll_fits(mpigx_comm* c, long long bytes) {
  if (c->algo == MPIGX_ALGO_ONESHOT || c->algo == MPIGX_ALGO_TWOSHOT) return false;
  const bool forced = c->algo == MPIGX_ALGO_LL;
  return c->ll && bytes <= (forced ? c->ll_max : c->ll_auto);
}
bool ll_take(mpigx_comm* c, long long bytes) {
  return ll_fits(c, bytes) && (long long)c->n * rup(c->ll_max, 16) <= (long long)c->stage_bytes;
}
// This launch's LL pointers: push[p] = rank p's area (parity) at my sender
// slot, *in = my own area (parity), and a flag no earlier launch of the same
// parity used (the epoch is monotone and equal on every rank).
// The flag carries the epoch's low 31 bits; when the epoch enters a new
// 2^31 generation (epoch >> 31 changes, on every rank at the same call) a
// line last written exactly one generation earlier could carry the current
// flag, so the area is cleared first: barrier (no rank still reads or writes
// LL lines of earlier launches), every rank zeroes its own area, barrier (no
// rank pushes before every area is clear); a zero line never matches a flag
// (top bit set).  `pv` (the launch's view, made before this call) is renewed
// after those launches.
int barrier_launch(mpigx_comm* c);
int ll_fill(mpigx_comm* c, PeerView& pv, char** push, const char** in, long long* stride, unsigned* flag) {
  if ((unsigned)(c->epoch >> 31) != c->ll_gen) {
    int rc = barrier_launch(c);
    if (rc) return rc;
    if (c->ll) HIPCK(hipMemsetAsync(c->ll, 0, (size_t)2 * kMaxRanks * c->ll_stride, c->stream));
    if (c->ll_rw) HIPCK(hipMemsetAsync(c->ll_rw, 0, (size_t)2 * kMaxRanks * c->ll_stride, c->stream));
    if ((rc = barrier_launch(c))) return rc;
    c->ll_gen = (unsigned)(c->epoch >> 31);
    const unsigned key = pv.zc_key;
    const int bad = pv.zc_bad;
    pv = make_view(c);
    pv.zc_key = key;
    pv.zc_bad = bad;
  }
  const long long par = (long long)(c->ll_seq & 1) * kMaxRanks * c->ll_stride;
  for (int p = 0; p < c->n; ++p) {
    char* area = ((c->rw_mask >> p) & 1u) ? c->peer_ll_rw[p] : c->peer_ll[p];
    push[p] = area ? area + par + (long long)c->rank * c->ll_stride : nullptr;
  }
  *in = c->ll ? c->ll + par : nullptr;
  pv.ll_rw = c->ll_rw ? c->ll_rw + par : nullptr;
  *stride = c->ll_stride;
  *flag = (unsigned)(c->epoch & 0x7fffffffu) | 0x80000000u;
  return MPIGX_SUCCESS;
}
// one cross-rank barrier launch (copy_kernel C_BARRIER, one block)
int barrier_launch(mpigx_comm* c) {
  CopyArgs b;
  memset(&b, 0, sizeof b);
  b.pv = make_view(c);
  b.mode = C_BARRIER;
  HIPCK(launch_copy(dim3(1), c->stream, b));
  note_launch(c, b.pv, 1);
  c->epoch += 1;
  return MPIGX_SUCCESS;
}
void ll_launched(mpigx_comm* c) {
  c->epoch += 1;
  c->ll_seq += 1;
  c->ll_unfenced = true;
}
// Bcast / Allgather / Alltoall: LL for blocks up to MPIGX_LL_MAX bytes
// (MPIGX_ALGO=oneshot/twoshot keeps the staged copy, as for the reductions)
bool copy_ll_take(mpigx_comm* c, long long bytes) { return ll_fits(c, bytes); }

// Large-Allreduce tuner.  Whether pulling peer data over xGMI (two-shot,
// M_AR_ZC), pushing it (M_AR_PUSH) or pulling the reduce-scatter and pushing
// the allgather (ar_zc_kernel AG_PUSH) moves more bytes per second depends on
// the fabric, so the communicator measures the three on its first
// zero-copy-sized Allreduces (blocking calls only: the host then knows the
// launch finished) and keeps the fastest.  Device time of the launch, max
// over ranks (one host exchange), per byte; another variant must beat the
// pull by 3 % to replace it.  All give the same bits (same fold schedule),
// so the choice never changes results.  Returns the variant to time on this
// call (0 pull, 1 push, 2 pull-push) or -1 and sets *variant to the one to
// run.  Every rank sees the same calls and outcomes (blocking mode,
// MPIGX_AR_TUNE and the zero-copy verdict agree), so the exchange in
// ar_tune_note is collective.
// the pull-push two-shot exists only as the dedicated kernel (n <= 8, MPICH
// tree order); elsewhere allreduce_zc runs the pull for it, so it is not timed
bool ar_pullpush_ok(const mpigx_comm* c) { return c->n >= 2 && c->n <= 8 && c->order != MPIGX_ORDER_LINEAR; }

int ar_tune_pick(mpigx_comm* c, int* variant) {
  if (c->ar_choice >= 0) {
    *variant = c->ar_choice;
    return -1;
  }
  *variant = 0;
  if (!c->ar_tune || !c->blocking || c->sync_mode != 1 || !c->ar_ev[0]) return -1;
  const int step = c->ar_step++;
  if (step == 0) return -1;  // registration call (host exchange, first imports)
  // pull, push, pull-push (again if a call fell back to staging)
  *variant = (step - 1) % (ar_pullpush_ok(c) ? 3 : 2);
  return *variant;
}
int ar_tune_note(mpigx_comm* c, int variant, long long bytes) {
  float ms = 0;
  // the completion word arrives before the stream reaches the end event
  HIPCK(hipEventSynchronize(c->ar_ev[1]));
  HIPCK(hipEventElapsedTime(&ms, c->ar_ev[0], c->ar_ev[1]));
  c->ar_spb[variant] = (ms / 1e3) / (double)bytes;
  const bool pp = ar_pullpush_ok(c);
  if (variant != (pp ? 2 : 1) || c->ar_spb[0] <= 0 || c->ar_spb[1] <= 0) return MPIGX_SUCCESS;
  if (!pp) c->ar_spb[2] = -1;  // not available: never chosen, reported as -1
  double mine[3] = {c->ar_spb[0], c->ar_spb[1], c->ar_spb[2]}, all[kMaxRanks][3];
  const int rc = host_allgather(c, mine, sizeof mine, all);
  if (rc) return rc;
  double w[3] = {0, 0, 0};
  for (int q = 0; q < c->n; ++q)
    for (int k = 0; k < 3; ++k) w[k] = all[q][k] > w[k] ? all[q][k] : w[k];
  int best = (!pp || w[1] < w[2]) ? 1 : 2;
  c->ar_choice = w[best] < 0.97 * w[0] ? best : 0;
  return MPIGX_SUCCESS;
}

// Small / medium Allreduce tuner (below the zero-copy size).  The LL step,
// the staged one-shot and the staged two-shot all fold with the same schedule
// (same bits), and which is fastest at a given size depends on the fabric
// (xGMI latency vs bytes) — so, like the pull/push choice above, each
// communicator measures them: per size class k = floor(log2 bytes), the
// candidates valid for the whole class run twice each in turn on the first
// calls of that class (device time on the comm stream, min of the two), one
// host exchange takes the max over ranks, and the class keeps the fastest
// (another than the static default only if >= 3 % faster).
// The byte movers (Bcast / Allgather / Alltoall, kinds 1-3) are tuned the
// same way between their LL step and their staged algorithm (V_ONE), the size
// class taken from the per-rank block.
enum MidVariant { V_LL = 0, V_ONE = 1, V_TWO = 2, V_LL2 = 3 };
// LL two-shot: a chunk (count/n, rounded to vectors) fits half a sender slot
bool ll2_fits(mpigx_comm* c, long long bytes, int es) {
  const int vec = es >= 16 ? 1 : 16 / es;
  const long long chunk = rup(cdiv(bytes / es, c->n), vec) * es;
  return c->ll && c->n > 1 && chunk <= rup(c->ll_max, 16) / 2 &&
         (long long)c->n * rup(c->ll_max, 16) <= (long long)c->stage_bytes;
}
enum TuneKind { TK_ALLREDUCE = 0, TK_BCAST = 1, TK_ALLGATHER = 2, TK_ALLTOALL = 3 };
int mt_cands(mpigx_comm* c, int kind, int k, int* cand) {
  const long long lo = 1ll << k, hi = (2ll << k) - 1;
  int m = 0;
  if (kind != TK_ALLREDUCE) {
    if (c->ll && hi <= c->ll_max) cand[m++] = V_LL;
    cand[m++] = V_ONE;
    return m;
  }
  if (c->ll && hi <= c->ll_max && (long long)c->n * rup(c->ll_max, 16) <= (long long)c->stage_bytes) cand[m++] = V_LL;
  if (hi <= (4ll << 20) && hi <= (long long)c->stage_bytes) cand[m++] = V_ONE;
  if (lo >= (4ll << 10)) cand[m++] = V_TWO;
  // LL two-shot where a whole class's chunk fits (16-B rounding: +16 per rank)
  if (lo >= (4ll << 10) && c->ll && cdiv(hi, c->n) + 16 <= rup(c->ll_max, 16) / 2 &&
      (long long)c->n * rup(c->ll_max, 16) <= (long long)c->stage_bytes)
    cand[m++] = V_LL2;
  return m;
}
// -1: no forced variant (static rules); else the variant to run.  *timed =
// the variant if this call is a tuning sample, *cls its class.
int mt_pick(mpigx_comm* c, int kind, long long bytes, int* timed, int* cls) {
  *timed = -1;
  if (!c->ar_tune || !c->blocking || c->sync_mode != 1 || !c->ar_ev[0] || bytes <= 0) return -1;
  const int k = 63 - __builtin_clzll((unsigned long long)bytes);
  if (k >= mpigx_comm::kTuneClasses) return -1;
  const int slot = kind * mpigx_comm::kTuneClasses + k;
  *cls = slot;
  if (c->mt_choice[slot] >= 0) return c->mt_choice[slot];
  int cand[4];
  const int m = mt_cands(c, kind, k, cand);
  if (m <= 1) return -1;
  const int s = c->mt_step[slot];
  if (s >= 2 * m) return -1;  // a sample failed: keep the static rules
  c->mt_step[slot] = (unsigned char)(s + 1);
  *timed = cand[s % m];
  return *timed;
}
bool copy_ll_take(mpigx_comm* c, long long bytes);
int mt_default(mpigx_comm* c, int kind, long long bytes) {
  if (kind != TK_ALLREDUCE) return copy_ll_take(c, bytes) ? V_LL : V_ONE;
  return ll_take(c, bytes) ? V_LL : bytes <= c->oneshot_max ? V_ONE : V_TWO;
}
int mt_note(mpigx_comm* c, int slot, int variant, long long bytes) {
  const int kind = slot / mpigx_comm::kTuneClasses, k = slot % mpigx_comm::kTuneClasses;
  float ms = 0;
  HIPCK(hipEventSynchronize(c->ar_ev[1]));
  HIPCK(hipEventElapsedTime(&ms, c->ar_ev[0], c->ar_ev[1]));
  const double spb = (ms / 1e3) / (double)bytes;
  double& best = c->mt_spb[slot][variant];
  if (best <= 0 || spb < best) best = spb;
  int cand[4];
  const int m = mt_cands(c, kind, k, cand);
  if (c->mt_step[slot] != 2 * m) return MPIGX_SUCCESS;
  double all[kMaxRanks][4];
  const int rc = host_allgather(c, c->mt_spb[slot], sizeof(double) * 4, all);
  if (rc) return rc;
  double w[4] = {0, 0, 0, 0};
  for (int q = 0; q < c->n; ++q)
    for (int v = 0; v < 4; ++v) w[v] = all[q][v] > w[v] ? all[q][v] : w[v];
  const int def = mt_default(c, kind, 1ll << k);
  int best_v = -1;
  for (int i = 0; i < m; ++i)
    if (w[cand[i]] > 0 && (best_v < 0 || w[cand[i]] < w[best_v])) best_v = cand[i];
  if (best_v >= 0 && w[def] > 0 && !(w[best_v] < 0.97 * w[def])) best_v = def;
  c->mt_choice[slot] = (signed char)(best_v >= 0 ? best_v : def);
  return MPIGX_SUCCESS;
}

// finish() of a call that may be a tuning sample (mt_pick)
int mt_finish(mpigx_comm* c, int timed, int cls, long long bytes) {
  if (timed >= 0) HIPCK(hipEventRecord(c->ar_ev[1], c->stream));
  int rc = finish(c);
  if (!rc && timed >= 0) rc = mt_note(c, cls, timed, bytes);
  return rc;
}

int reduce_common(mpigx_comm* c, const void* send, void* recv, long long count, const TypeInfo* t,
                  int oc, int root, bool all) {
  const int n = c->n, es = t->size;
  const int vec = es >= 16 ? 1 : 16 / es;
  FoldLauncher L = fold_launcher(t->rep);
  // elements per round: staging holds a whole round
  long long round = (long long)(c->stage_bytes / es);
  round = (round / (n * (long long)vec)) * n * vec;
  const int algo = c->algo;  // knob: identical on every rank
  // count and the thresholds are identical on every rank, so is this test
  if (all && n > 1 && c->zc_min > 0 && count * es >= c->zc_min && algo != MPIGX_ALGO_ONESHOT) {
    int variant = algo == MPIGX_ALGO_PUSH ? 1 : algo == MPIGX_ALGO_PULLPUSH ? 2 : 0;
    const bool ring = algo == MPIGX_ALGO_RING;
    // no MPIGX_ALGO: the pull, push or pull-push two-shot, whichever measured
    // fastest on this communicator (ar_tune_*); undecided, calls 2-4 time
    // them in turn (call 1 registers the buffers)
    const int timed = algo != MPIGX_ALGO_AUTO ? -1 : ar_tune_pick(c, &variant);
    bool staged;
    const int rc = zc_run(c, send, recv, &staged, [&](const ZcLaunch& z) {
      if (ring) return allreduce_ring(c, z, count, t, oc);
      if (timed >= 0) HIPCK(hipEventRecord(c->ar_ev[0], c->stream));
      const int lr = variant == 1 ? allreduce_push(c, z, send, count, t, oc)
                                  : allreduce_zc(c, z, count, t, oc, variant == 2);
      if (timed >= 0 && !lr) HIPCK(hipEventRecord(c->ar_ev[1], c->stream));
      return lr;
    });
    if (!rc && !staged && timed >= 0) {
      const int trc = ar_tune_note(c, timed, count * es);
      if (trc) return trc;
    }
    if (rc || !staged) return rc;
    if (c->zc_require) return MPIGX_ERR_INTERN;  // tests: the path must not fall back
  }
  if (!all && n > 1 && c->zc_min > 0 && count * es >= c->zc_min) {
    // zero-copy Reduce: no copy-in; the reduced chunks wait in the arenas
    // (rounds of n chunks of at most one arena each) for the root to gather
    bool staged;
    const int rc = zc_run(c, send, recv ? recv : (void*)send, &staged, [&](const ZcLaunch& z) {
      const int pr = reduce_zc_push(c, z, count, t, oc, root);
      if (pr != -1) return pr;
      long long zround = (long long)(c->stage_bytes / es) / vec * vec * n;
      for (long long off = 0; off < count; off += zround) {
        const long long cnt = count - off < zround ? count - off : zround;
        FoldArgs a;
        memset(&a, 0, sizeof a);
        a.pv = make_view(c);
        zc_apply(a.pv, z);
        a.mode = M_RED_ZC;
        a.esize = es;
        a.count = cnt;
        a.gbase = off;
        a.root = root;
        a.recv = recv ? (char*)recv + off * es : nullptr;
        int nmax, sched;
        const void* ptrs[kMaxRanks];
        for (int p = 0; p < n; ++p) ptrs[p] = z.ps[p] ? z.ps[p] + off * es : nullptr;
        plan_schedule(c, a, n, root, count, es, ptrs, &nmax, &sched, c->order);
        a.chunk = rup(cdiv(cnt, n), vec);
        const int grid = grid_for(c, a.chunk * es, cap_fold(c, t, oc, nmax, sched));
        a.slice = rup(cdiv(a.chunk, grid), vec);
        seal_args(a);
        HIPCK(L(oc, nmax, sched, dim3(grid), c->stream, a));
        note_launch(c, a.pv, grid);
        c->epoch += 3;
      }
      return MPIGX_SUCCESS;
    });
    if (rc || !staged) return rc;
    if (c->zc_require) return MPIGX_ERR_INTERN;
  }
  // below the zero-copy size: the measured variant for Allreduce (mt_*)
  int timed = -1, cls = -1;
  int force = (all && algo == MPIGX_ALGO_AUTO) ? mt_pick(c, TK_ALLREDUCE, count * es, &timed, &cls) : -1;
  if (all && algo == MPIGX_ALGO_LL2) force = V_LL2;
  if (force == V_LL2 && !ll2_fits(c, count * es, es)) force = -1;
  if (timed >= 0) HIPCK(hipEventRecord(c->ar_ev[0], c->stream));
  if (force == V_LL2) {
    // medium Allreduce: LL two-shot (kernels.hpp M_AR_LL2) — two LL
    // exchanges, no barrier; the peers' chunk-r slices land in my arena slots
    const long long ustride = rup(c->ll_max, 16);
    FoldArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    a.mode = M_AR_LL2;
    a.esize = es;
    a.count = count;
    a.send = send;
    a.recv = recv;
    if (int e = ll_fill(c, a.pv, a.zc_recv, &a.ll_in, &a.ll_stride, &a.ll_flag)) return e;
    a.slot_bytes = ustride;
    a.chunk = rup(cdiv(count, n), vec);
    const long long c0 = (long long)c->rank * a.chunk < count ? (long long)c->rank * a.chunk : count;
    int nmax, sched;
    const void* ptrs[kMaxRanks];
    for (int q = 0; q < n; ++q)
      ptrs[q] = q == c->rank ? send : (const void*)(c->stage + q * ustride - c0 * es);
    plan_schedule(c, a, n, 0, count, es, ptrs, &nmax, &sched, c->order);
    const int grid = grid_for(c, a.chunk * es, cap_fold(c, t, oc, nmax, sched));
    a.slice = rup(cdiv(a.chunk, grid), kLLAlign / es);  // whole 128-B lines of LL area per block
    HIPCK(L(oc, nmax, sched, dim3(grid), c->stream, a));
    note_launch(c, a.pv, grid);
    ll_launched(c);
    return mt_finish(c, timed, cls, count * es);
  }
  // small Allreduce / Reduce: one LL step (no barrier, kernels.hpp M_AR_LL /
  // M_RED_LL); the unpacked contributions take n slots of my arena
  if (force >= 0 ? force == V_LL : ll_take(c, count * es)) {
    const long long ustride = rup(c->ll_max, 16);
    FoldArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    a.mode = all ? M_AR_LL : M_RED_LL;
    a.esize = es;
    a.count = count;
    a.root = root;
    a.send = send;
    a.recv = recv;
    if (int e = ll_fill(c, a.pv, a.zc_recv, &a.ll_in, &a.ll_stride, &a.ll_flag)) return e;
    a.slot_bytes = ustride;
    int nmax, sched;
    const void* ptrs[kMaxRanks];
    for (int p = 0; p < n; ++p) ptrs[p] = c->stage + p * ustride;
    plan_schedule(c, a, n, root, count, es, ptrs, &nmax, &sched, c->order);
    const int grid = grid_for(c, count * es, cap_fold(c, t, oc, nmax, sched));
    a.slice = rup(cdiv(count, grid), kLLAlign / es);  // whole 128-B lines of LL area per block
    HIPCK(L(oc, nmax, sched, dim3(grid), c->stream, a));
    note_launch(c, a.pv, grid);
    ll_launched(c);
    return mt_finish(c, timed, cls, count * es);
  }
  for (long long off = 0; off < count; off += round) {
    const long long cnt = count - off < round ? count - off : round;
    FoldArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    a.esize = es;
    a.count = cnt;
    a.gbase = off;
    a.root = root;
    a.send = (const char*)send + off * es;
    a.recv = recv ? (char*)recv + off * es : nullptr;
    int nmax, sched;
    const void* ptrs[kMaxRanks];
    for (int p = 0; p < n; ++p) ptrs[p] = c->peer_stage[p];
    plan_schedule(c, a, n, root, count, es, ptrs, &nmax, &sched, c->order);
    bool oneshot = cnt * es <= c->oneshot_max;
    if (algo == MPIGX_ALGO_ONESHOT) oneshot = true;
    if (algo == MPIGX_ALGO_TWOSHOT) oneshot = false;
    if (force == V_ONE || force == V_TWO) oneshot = force == V_ONE;
    int grid, nbar;
    if (oneshot) {
      a.mode = all ? M_AR_ONESHOT : M_RED_ONESHOT;
      grid = grid_for(c, cnt * es, cap_fold(c, t, oc, nmax, sched));
      a.slice = rup(cdiv(cnt, grid), vec);
      nbar = 2;
    } else {
      a.mode = all ? M_AR_TWOSHOT : M_RED_TWOSHOT;
      a.chunk = rup(cdiv(cnt, n), vec);
      grid = grid_for(c, a.chunk * es, cap_fold(c, t, oc, nmax, sched));
      a.slice = rup(cdiv(a.chunk, grid), vec);
      nbar = 3;
    }
    HIPCK(L(oc, nmax, sched, dim3(grid), c->stream, a));
    note_launch(c, a.pv, grid);
    c->epoch += nbar;
  }
  return mt_finish(c, timed, cls, count * es);
}

int check_comm(mpigx_comm* c) {
  if (!c) return MPIGX_ERR_COMM;
  if (c->broken) return MPIGX_ERR_OTHER;
  // A call cannot be captured into a HIP graph: every launch carries a fresh
  // epoch and argument block, which a replay would repeat (the peers would
  // wait for epochs that never come), and blocking calls wait on the host.
  // Refused before anything is enqueued, so the capture and the
  // communicator both stay usable.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(c->stream, &cap) != hipSuccess) (void)hipGetLastError();
  else if (cap != hipStreamCaptureStatusNone) {
    fprintf(stderr, "[mpigx] rank %d: the stream is being captured into a HIP graph; mpigx calls cannot be "
            "captured (issue them outside the capture)\n", c->rank);
    return MPIGX_ERR_OTHER;
  }
  c->t_entry = now_s();  // host-cost diagnostic (mpigx_comm_host_stats)
  c->launch_pending = true;
  if (hipSetDevice(c->device) != hipSuccess) return MPIGX_ERR_INTERN;
  return MPIGX_SUCCESS;
}

// Pooled device temporaries for derived-type packing in collectives (used on
// the comm's stream only, so stream order makes reuse safe).
char* tmp_get(mpigx_comm* c, long long bytes) {
  size_t best = c->tmp_free.size();
  for (size_t i = 0; i < c->tmp_free.size(); ++i)
    if (c->tmp_free[i].first >= bytes && (best == c->tmp_free.size() || c->tmp_free[i].first < c->tmp_free[best].first))
      best = i;
  if (best < c->tmp_free.size()) {
    char* p = c->tmp_free[best].second;
    c->tmp_used.push_back(c->tmp_free[best]);
    c->tmp_free.erase(c->tmp_free.begin() + best);
    return p;
  }
  const long long cap = (bytes + (1 << 20) - 1) & ~((1ll << 20) - 1);
  char* p = nullptr;
  if (hipMalloc(&p, cap) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  c->tmp_used.push_back({cap, p});
  return p;
}
void tmp_put(mpigx_comm* c, char* p, long long) {
  for (size_t i = 0; i < c->tmp_used.size(); ++i)
    if (c->tmp_used[i].second == p) {
      c->tmp_free.push_back(c->tmp_used[i]);
      c->tmp_used.erase(c->tmp_used.begin() + i);
      return;
    }
}

int copy_n1(mpigx_comm* c, void* dst, const void* src, size_t bytes) {
  if (dst != src && bytes) HIPCK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream));
  return finish(c);
}

// Host control plane: allgather of <= 64-byte blobs through the shm block
// (double-buffered by sequence parity: a rank can only reuse a buffer after
// every peer posted the next sequence, i.e. finished reading it).
// A peer process that no longer runs: gone, or exited and not yet reaped by
// its parent (a zombie still answers kill(pid, 0)).  A live one we may not
// signal counts as alive.
bool peer_gone(const mpigx_comm* c, int q) {
  const int pid = c->shm->ranks[q].pid;
  if (pid <= 0) return false;
  if (kill(pid, 0) != 0) return errno == ESRCH;
  char path[64], buf[256];
  snprintf(path, sizeof path, "/proc/%d/stat", pid);
  FILE* f = fopen(path, "r");
  if (!f) return false;
  const size_t len = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[len] = 0;
  const char* e = strrchr(buf, ')');  // "pid (comm) S ..."
  return e && e[1] == ' ' && (e[2] == 'Z' || e[2] == 'X');
}

// until_gone: wait for as long as the peer's process lives (MPI semantics: a
// collective waits for a late rank) instead of failing after the
// communicator's timeout; a note goes to stderr once that timeout has passed.
int host_allgather_wait(mpigx_comm* c, const void* mine, int len, void* out, bool until_gone) {
  if (len > 256) return MPIGX_ERR_INTERN;
  if (c->n == 1 || !c->shm) {
    memcpy(out, mine, len);
    return MPIGX_SUCCESS;
  }
  const uint64_t k = ++c->xseq;
  ShmRank& me = c->shm->ranks[c->rank];
  memcpy(me.xbuf[k & 1], mine, len);
  me.xseq.store(k, std::memory_order_release);
  const double t0 = now_s(), limit = c->timeout_ticks / 1e8;
  bool noted = false;
  double next_check = t0 + 1.0;
  for (int q = 0; q < c->n; ++q) {
    unsigned spins = 0;
    while (c->shm->ranks[q].xseq.load(std::memory_order_acquire) < k) {
      if ((spins & 63) == 0) {
        rt::progress_all(c);
        rt::yield_big_lock();  // a Win_fence / Comm_split caller lets other threads' p2p through
      }
      if ((++spins & 4095) == 0) {
        const double t = now_s();
        if (!until_gone && t - t0 > limit) {
          mark_broken(c);
          return MPIGX_ERR_OTHER;
        }
        if (c->shm->ranks[q].broken.load(std::memory_order_acquire)) {
          fprintf(stderr, "mpigx: rank %d: rank %d's communicator failed; it will not join\n", c->rank, q);
          mark_broken(c);
          return MPIGX_ERR_OTHER;
        }
        if (until_gone && t > next_check) {
          next_check = t + 1.0;
          if (peer_gone(c, q)) {
            fprintf(stderr, "mpigx: rank %d: rank %d's process is gone\n", c->rank, q);
            mark_broken(c);
            return MPIGX_ERR_OTHER;
          }
          if (!noted && t - t0 > limit) {
            noted = true;
            fprintf(stderr, "mpigx: rank %d has waited %.0f s for rank %d to reach the collective\n", c->rank,
                    t - t0, q);
          }
        }
        // a long wait: leave the host cores to the late rank (with several
        // ranks per GPU the waiters would otherwise spin on every core)
        if (until_gone && t - t0 > 0.05) usleep(200);
      }
    }
    memcpy((char*)out + (size_t)q * len, c->shm->ranks[q].xbuf[k & 1], len);
  }
  return MPIGX_SUCCESS;
}
// Every host exchange of a collective (zero-copy view agreement, the
// v-collectives' round agreement, tuner verdicts, knob changes, RMA fences,
// Comm_split) waits for a late rank as long as its process lives and its
// communicator has not failed (round 5): MPI's collectives block until every
// rank arrives (collective.jl:698-700), so a rank that spends longer than
// MPIGX_TIMEOUT_MS in a checkpoint or a host phase before a Gatherv or a
// stream-ordered first call must not break the communicator.
int host_allgather(mpigx_comm* c, const void* mine, int len, void* out) {
  return host_allgather_wait(c, mine, len, out, true);
}

// Per-rank description of a personalised exchange (see VArgs in common.hpp).
struct VSpec {
  int ncopy = 0;
  int c_slot[kMaxRanks] = {};
  long long c_src[kMaxRanks] = {};
  long long c_len[kMaxRanks] = {};
  long long p_len[kMaxRanks] = {};
  int p_slot[kMaxRanks] = {};
  long long p_dst[kMaxRanks] = {};
  const char* send = nullptr;
  char* recv = nullptr;
};

// Drives Gather(v)/Scatter(v)/Allgatherv/Alltoallv: agrees on the longest
// range across ranks (host control plane), then runs ceil(max/R) rounds of
// vx_kernel with an identical grid on every rank.
int vexchange(mpigx_comm* c, const VSpec& s) {
  const int n = c->n;
  long long mx = 0;
  for (int j = 0; j < s.ncopy; ++j) mx = s.c_len[j] > mx ? s.c_len[j] : mx;
  for (int p = 0; p < n; ++p) mx = s.p_len[p] > mx ? s.p_len[p] : mx;
  long long all[kMaxRanks];
  int rc = host_allgather(c, &mx, sizeof mx, all);
  if (rc) return rc;
  long long gmax = 0;
  for (int q = 0; q < n; ++q) gmax = all[q] > gmax ? all[q] : gmax;
  if (gmax == 0) return finish(c);
  const long long R = ((long long)(c->stage_bytes - kSlotBase) / n) & ~15ll;
  if (R < 16) return MPIGX_ERR_NO_MEM;
  const long long per_round = gmax < R ? gmax : R;
  const int G = grid_for(c, per_round * n, cap_vx(c));
  for (long long off = 0; off < gmax; off += R) {
    VArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    a.R = R;
    a.round_off = off;
    a.G = G;
    a.ncopy = s.ncopy;
    for (int j = 0; j < s.ncopy; ++j) {
      a.c_slot[j] = s.c_slot[j];
      a.c_src[j] = s.c_src[j];
      a.c_len[j] = s.c_len[j];
    }
    for (int p = 0; p < n; ++p) {
      a.p_len[p] = s.p_len[p];
      a.p_slot[p] = s.p_slot[p];
      a.p_dst[p] = s.p_dst[p];
    }
    a.send = s.send;
    a.recv = s.recv;
    HIPCK(launch_vx(dim3(G), c->stream, a));
    note_launch(c, a.pv, G);
    c->epoch += 2;
  }
  return finish(c);
}

}  // namespace

// Runtime services for p2p.cpp (runtime.hpp).
namespace mpigx {
namespace rt {
int comm_check(mpigx_comm* c) { return check_comm(c); }
void comm_mark_broken(mpigx_comm* c) { mark_broken(c); }
int dtype_size(int datatype) {
  const TypeInfo* t = find_type(datatype);
  return t ? t->size : -1;
}
bool export_buf(mpigx_comm* c, const void* p, unsigned long long* id, long long* off, hipIpcMemHandle_t* h) {
  char* base;
  return zc_export(c, p, &base, id, off, h);
}
char* import_buf(mpigx_comm* c, int peer, unsigned long long id, const hipIpcMemHandle_t& h) {
  return zc_import(c, peer, id, h);
}
char* import_pinned(mpigx_comm* c, int peer, unsigned long long id, const hipIpcMemHandle_t& h) {
  char* p = zc_import(c, peer, id, h);
  if (p)
    for (auto& im : c->imports)
      if (im.base == p) ++im.pins;
  return p;
}
void unpin(mpigx_comm* c, char* base) {
  for (auto& im : c->imports)
    if (im.base == base && im.pins > 0) {
      --im.pins;
      return;
    }
}
int host_allgather(mpigx_comm* c, const void* mine, int len, void* out) {
  return ::host_allgather(c, mine, len, out);
}
int acc_check(int datatype, int op, int* rep, int* esize, int* oc) {
  const TypeInfo* t = find_type(datatype);
  if (!t) return MPIGX_ERR_TYPE;
  int o;
  if (op == MPIGX_REPLACE) o = O_REPLACE;
  else if (op == MPIGX_NO_OP) o = O_NOOP;
  else {
    const int rc = validate(datatype, op, &t, &o);
    if (rc) return rc;
  }
  *rep = t->rep;
  *esize = t->size;
  *oc = o;
  return MPIGX_SUCCESS;
}
bool peer_dead(const mpigx_comm* c) {
  if (!c || !c->shm || c->n <= 1) return false;
  if (peer_broken(c) >= 0) return true;
  for (int q = 0; q < c->n; ++q)
    if (q != c->rank && peer_gone(c, q)) return true;
  return false;
}
BigLock& big_lock() {
  static BigLock m;
  return m;
}
void yield_big_lock() {
  BigLock& b = big_lock();
  if (b.owner.load(std::memory_order_relaxed) != std::this_thread::get_id()) return;
  const int d = b.depth;
  b.depth = 0;
  b.owner.store(std::thread::id(), std::memory_order_relaxed);
  b.m.unlock();
  sched_yield();
  b.m.lock();
  b.owner.store(std::this_thread::get_id(), std::memory_order_relaxed);
  b.depth = d;
}
void progress_all(mpigx_comm* c) {
  std::lock_guard<BigLock> g(big_lock());
  if (c->in_progress) return;
  c->in_progress = true;
  if (c->p2p) p2p_progress(c);
  if (c->rma) rma_progress(c);
  c->in_progress = false;
}
double wall() { return now_s(); }
int pull_fences() {
  static const int v = (int)env_ll("MPIGX_PULL_FENCES", 1);
  return v;
}
}  // namespace rt
}  // namespace mpigx

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int mpigx_get_version(int* major, int* minor) {
  if (major) *major = MPIGX_VERSION_MAJOR;
  if (minor) *minor = MPIGX_VERSION_MINOR;
  return MPIGX_SUCCESS;
}

int mpigx_query_thread(int* provided) {
  if (!provided) return MPIGX_ERR_ARG;
  *provided = MPIGX_THREAD_MULTIPLE;  // rt::big_lock (runtime.hpp)
  return MPIGX_SUCCESS;
}
int mpigx_error_string(int code, char* str, int* len) {
  const char* s;
  switch (code) {
    case MPIGX_SUCCESS: s = "No MPI error"; break;
    case MPIGX_ERR_BUFFER: s = "Invalid buffer pointer"; break;
    case MPIGX_ERR_COUNT: s = "Invalid count argument"; break;
    case MPIGX_ERR_TYPE: s = "Invalid datatype argument"; break;
    case MPIGX_ERR_COMM: s = "Invalid communicator"; break;
    case MPIGX_ERR_ROOT: s = "Invalid root"; break;
    case MPIGX_ERR_OP: s = "Invalid MPI_Op (not defined for this datatype)"; break;
    case MPIGX_ERR_ARG: s = "Invalid argument"; break;
    case MPIGX_ERR_OTHER: s = "Other MPI error (mpigx: peer did not arrive / communicator broken)"; break;
    case MPIGX_ERR_INTERN: s = "Internal MPI error (mpigx: HIP runtime failure)"; break;
    case MPIGX_ERR_NO_MEM: s = "Out of memory"; break;
    default: s = "Unknown error"; break;
  }
  if (str) {
    strncpy(str, s, 511);
    str[511] = 0;
  }
  if (len) *len = (int)strlen(s);
  return MPIGX_SUCCESS;
}

int mpigx_op_valid(int datatype, int op) { return validate(datatype, op, nullptr, nullptr); }

int mpigx_type_size(int datatype, int* size) {
  const TypeInfo* t = find_type(datatype);
  if (!t) {
    long long s = 0;
    const int rc = mpigx_type_size_x(datatype, &s);
    if (rc) return rc;
    if (size) *size = s > 0x7fffffff ? MPIGX_UNDEFINED : (int)s;
    return MPIGX_SUCCESS;
  }
  if (size) *size = t->size;
  return MPIGX_SUCCESS;
}

int mpigx_get_unique_id(mpigx_unique_id_t* id) {
  if (!id) return MPIGX_ERR_ARG;
  memset(id, 0, sizeof *id);
  IdPayload p;
  memset(&p, 0, sizeof p);
  unsigned long long r = 0;
  FILE* f = fopen("/dev/urandom", "rb");
  if (f) {
    if (fread(&r, sizeof r, 1, f) != 1) r = 0;
    fclose(f);
  }
  r ^= (unsigned long long)getpid() << 32 ^ (unsigned long long)(now_s() * 1e9);
  snprintf(p.name, sizeof p.name, "/mpigx-%d-%016llx", (int)getpid(), r);
  p.magic = kMagic;
  memcpy(id->internal, &p, sizeof p);
  return MPIGX_SUCCESS;
}

}  // extern "C"

namespace {

// ---- knobs (include/mpigx.h MPIGX_KNOB_*) ----------------------------------
// Every path-selecting setting is read ONCE, here, per communicator; init
// compares every rank's values (comm_init) and mpigx_comm_set_knob changes
// them only collectively, so all ranks always take the same branch.
const char* const kAlgoNames[] = {"",     "ll",   "ll2",  "oneshot",      "twoshot",
                                  "push", "ring", "pull", "pull_generic", "pullpush"};
const char* const kKnobEnv[MPIGX_KNOB_COUNT] = {
    "MPIGX_ALGO",   "MPIGX_BCAST",      "MPIGX_RING_CHANNELS", "MPIGX_MAX_BLOCKS",     "MPIGX_ONESHOT_MAX",
    "MPIGX_ZC_MIN", "MPIGX_BCAST_SAG_MIN", "MPIGX_ZC_REQUIRE", "MPIGX_BYTES_PER_BLOCK", "MPIGX_LL_AUTO",
    "MPIGX_AR_TUNE", "MPIGX_ZC_OPTIMISTIC", "MPIGX_SYNC_SPIN", "MPIGX_STAGING_BYTES",  "MPIGX_LL_MAX",
    "MPIGX_AR_SLICES", "MPIGX_SCAN_PP", "MPIGX_SHARE_HEADROOM", "MPIGX_SHARED_GATE", "MPIGX_PEER_MEM",
    "MPIGX_CONCURRENT_COMMS"};

long long knob_value(const mpigx_comm* c, int k) {
  switch (k) {
    case MPIGX_KNOB_ALGO: return c->algo;
    case MPIGX_KNOB_BCAST: return c->bcast_mode;
    case MPIGX_KNOB_RING_CHANNELS: return c->ring_channels;
    case MPIGX_KNOB_MAX_BLOCKS: return c->max_blocks;
    case MPIGX_KNOB_ONESHOT_MAX: return c->oneshot_max;
    case MPIGX_KNOB_ZC_MIN: return c->zc_min;
    case MPIGX_KNOB_BCAST_SAG_MIN: return c->bcast_sag_min;
    case MPIGX_KNOB_ZC_REQUIRE: return c->zc_require ? 1 : 0;
    case MPIGX_KNOB_BYTES_PER_BLOCK: return c->bytes_per_block;
    case MPIGX_KNOB_LL_AUTO: return c->ll_auto;
    case MPIGX_KNOB_AR_TUNE: return c->ar_tune;
    case MPIGX_KNOB_ZC_OPTIMISTIC: return c->zc_optimistic ? 1 : 0;
    case MPIGX_KNOB_SYNC_SPIN: return c->sync_mode;
    case MPIGX_KNOB_STAGING_BYTES: return (long long)c->stage_bytes;
    case MPIGX_KNOB_LL_MAX: return c->ll_max;
    case MPIGX_KNOB_AR_SLICES: return c->ar_slices;
    case MPIGX_KNOB_SCAN_PP: return c->scan_pp ? 1 : 0;
    case MPIGX_KNOB_SHARE_HEADROOM: return c->share_headroom;
    case MPIGX_KNOB_SHARED_GATE: return c->shared_gate ? 1 : 0;
    case MPIGX_KNOB_PEER_MEM: return c->peer_mem;
    case MPIGX_KNOB_CONCURRENT_COMMS: return c->concurrent_comms;
    default: return -1;
  }
}

// Validates and applies one knob (init = true: the two allocation sizes may
// be set too).  MPIGX_ERR_ARG for an unknown knob or an out-of-range value.
int knob_apply(mpigx_comm* c, int k, long long v, bool init) {
  auto in = [&](long long lo, long long hi) { return v >= lo && v <= hi; };
  switch (k) {
    case MPIGX_KNOB_ALGO:
      if (!in(MPIGX_ALGO_AUTO, MPIGX_ALGO_PULLPUSH)) return MPIGX_ERR_ARG;
      c->algo = (int)v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_BCAST:
      if (!in(0, 3)) return MPIGX_ERR_ARG;
      c->bcast_mode = (int)v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_RING_CHANNELS:
      if (!in(1, kMaxRings)) return MPIGX_ERR_ARG;
      c->ring_channels = (int)v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_MAX_BLOCKS: {
      if (!in(1, kMaxBlocks)) return MPIGX_ERR_ARG;
      c->max_blocks = (int)v;
      return MPIGX_SUCCESS;
    }
    case MPIGX_KNOB_ONESHOT_MAX:
      if (v < 0) return MPIGX_ERR_ARG;
      c->oneshot_max = v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_ZC_MIN:
      if (v < 0) return MPIGX_ERR_ARG;
      c->zc_min = v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_BCAST_SAG_MIN:
      if (v < 0) return MPIGX_ERR_ARG;
      c->bcast_sag_min = v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_ZC_REQUIRE:
      if (!in(0, 1)) return MPIGX_ERR_ARG;
      c->zc_require = v != 0;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_BYTES_PER_BLOCK:
      if (v < 16) return MPIGX_ERR_ARG;
      c->bytes_per_block = v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_LL_AUTO:
      if (v < 0) return MPIGX_ERR_ARG;
      c->ll_auto = v < c->ll_max ? v : c->ll_max;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_AR_TUNE:
      if (!in(0, 1)) return MPIGX_ERR_ARG;
      if (v && !init && !c->ar_ev[0]) {  // the tuners' events (comm_init creates them when on)
        HIPCK(hipEventCreate(&c->ar_ev[0]));
        HIPCK(hipEventCreate(&c->ar_ev[1]));
      }
      c->ar_tune = (int)v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_ZC_OPTIMISTIC:
      if (!in(0, 1)) return MPIGX_ERR_ARG;
      c->zc_optimistic = v != 0;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_SYNC_SPIN:
      if (!in(0, 1)) return MPIGX_ERR_ARG;
      c->sync_mode = (int)v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_STAGING_BYTES:
      if (!init || v < 4096) return MPIGX_ERR_ARG;
      c->stage_bytes = ((size_t)v + 4095) & ~(size_t)4095;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_LL_MAX:
      if (!init) return MPIGX_ERR_ARG;
      c->ll_max = v < 0 ? 0 : v > (4ll << 20) ? (4ll << 20) : v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_AR_SLICES:
      if (!in(0, 64)) return MPIGX_ERR_ARG;
      c->ar_slices = (int)v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_SCAN_PP:
      if (!in(0, 1)) return MPIGX_ERR_ARG;
      c->scan_pp = v != 0;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_SHARE_HEADROOM:
      if (!in(-1, 1)) return MPIGX_ERR_ARG;
      c->share_headroom = (int)v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_SHARED_GATE:
      if (!in(0, 1)) return MPIGX_ERR_ARG;
      c->shared_gate = v != 0;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_PEER_MEM:  // selects the arrays the peers map at init
      if (!init || !in(0, 1)) return MPIGX_ERR_ARG;
      c->peer_mem = (int)v;
      return MPIGX_SUCCESS;
    case MPIGX_KNOB_CONCURRENT_COMMS:  // init-only: the grids of every launch depend on it
      if (!init || !in(1, 64)) return MPIGX_ERR_ARG;
      c->concurrent_comms = (int)v;
      return MPIGX_SUCCESS;
    default: return MPIGX_ERR_ARG;
  }
}

// Defaults, then the environment.  Numeric knobs out of range are clamped as
// before the knobs existed; an unknown MPIGX_ALGO / MPIGX_BCAST name fails
// init (it used to be ignored silently on the rank that had it).
int knobs_from_env(mpigx_comm* c) {
  c->algo = MPIGX_ALGO_AUTO;
  const char* a = getenv("MPIGX_ALGO");
  if (a && *a) {
    int v = -1;
    for (int i = 1; i < (int)(sizeof kAlgoNames / sizeof kAlgoNames[0]); ++i)
      if (!strcmp(a, kAlgoNames[i])) v = i;
    if (v < 0) {
      fprintf(stderr, "[mpigx] MPIGX_ALGO=%s: unknown algorithm\n", a);
      return MPIGX_ERR_ARG;
    }
    c->algo = v;
  }
  c->bcast_mode = 0;
  const char* bc = getenv("MPIGX_BCAST");
  if (bc && *bc) {
    if (!strcmp(bc, "direct")) c->bcast_mode = 1;
    else if (!strcmp(bc, "sag")) c->bcast_mode = 2;
    else if (!strcmp(bc, "relay")) c->bcast_mode = 3;
    else {
      fprintf(stderr, "[mpigx] MPIGX_BCAST=%s: expected direct, sag or relay\n", bc);
      return MPIGX_ERR_ARG;
    }
  }
  long long rc_ = env_ll("MPIGX_RING_CHANNELS", 1);
  c->ring_channels = (int)(rc_ < 1 ? 1 : rc_ > kMaxRings ? kMaxRings : rc_);
  long long mb = env_ll("MPIGX_MAX_BLOCKS", 256);
  c->max_blocks = (int)(mb < 1 ? 1 : mb > kMaxBlocks ? kMaxBlocks : mb);
  c->oneshot_max = env_ll("MPIGX_ONESHOT_MAX", 256 << 10);
  c->zc_min = env_ll("MPIGX_ZC_MIN", 16ll << 20);
  c->bcast_sag_min = env_ll("MPIGX_BCAST_SAG_MIN", 256 << 10);
  c->zc_require = env_ll("MPIGX_ZC_REQUIRE", 0) != 0;
  // 8 KiB of message per block: 64 KiB one-shot drops 19.5 -> 6.7 us and
  // 1 MiB two-shot 31 -> 19 us vs 64 KiB per block (tools/latency.py, 2 ranks)
  c->bytes_per_block = env_ll("MPIGX_BYTES_PER_BLOCK", 8 << 10);
  if (c->bytes_per_block < 16) c->bytes_per_block = 16;
  c->stage_bytes = (size_t)env_ll("MPIGX_STAGING_BYTES", 512ll << 20);
  c->stage_bytes = (c->stage_bytes + 4095) & ~(size_t)4095;
  if (c->stage_bytes < 4096) c->stage_bytes = 4096;
  c->ll_max = env_ll("MPIGX_LL_MAX", 256 << 10);
  if (c->ll_max < 0) c->ll_max = 0;
  if (c->ll_max > (4ll << 20)) c->ll_max = 4ll << 20;
  // static default: the staged one-shot (same-device LL measured slower than
  // it, r03s: 59 vs 32 us at 8 KiB); blocking communicators still time LL
  // among the candidates of every small size class (mt_cands) and keep it
  // where it wins on the fabric they run on
  c->ll_auto = env_ll("MPIGX_LL_AUTO", 0);
  if (c->ll_auto > c->ll_max) c->ll_auto = c->ll_max;
  if (c->ll_auto < 0) c->ll_auto = 0;
  c->ar_tune = env_ll("MPIGX_AR_TUNE", 1) != 0 ? 1 : 0;
  c->zc_optimistic = env_ll("MPIGX_ZC_OPTIMISTIC", 1) != 0;
  c->sync_mode = env_ll("MPIGX_SYNC_SPIN", 1) != 0 ? 1 : 0;
  // static slices by default: on ranks sharing one GPU the ticket hand-out
  // moved the straggler tail but not the span (profiles/r03e_coll_n2_1gpu.json)
  const long long sl = env_ll("MPIGX_AR_SLICES", 0);
  c->ar_slices = (int)(sl < 0 ? 0 : sl > 64 ? 64 : sl);
  // pull-push Scan / Exscan: on since round 4 (the round-3 n = 8 fault did
  // not recur with the kernel's checked preconditions: the GPU suite with it
  // forced and the 8-rank headline / sequence / large-count cases, r04n)
  c->scan_pp = env_ll("MPIGX_SCAN_PP", 1) != 0;
  // residency headroom (-1 = auto and 1: on whenever ranks share the GPU;
  // 0 off, for measurements only; kernel_cap)
  {
    const long long h = env_ll("MPIGX_SHARE_HEADROOM", -1);
    c->share_headroom = h < 0 ? -1 : h > 0 ? 1 : 0;
  }
  c->shared_gate = env_ll("MPIGX_SHARED_GATE", 1) != 0;
  {
    const long long cc = env_ll("MPIGX_CONCURRENT_COMMS", 1);
    c->concurrent_comms = (int)(cc < 1 ? 1 : cc > 64 ? 64 : cc);
  }
  // "xdev": every peer takes the cross-device protocol (uncached signal
  // arrays and LL areas, comm_init) — what one rank per GPU runs, exercised
  // on the 1-GPU test box
  c->peer_mem = 0;
  const char* pm = getenv("MPIGX_PEER_MEM");
  if (pm && *pm) {
    if (!strcmp(pm, "xdev") || !strcmp(pm, "1")) c->peer_mem = 1;
    else if (strcmp(pm, "auto") && strcmp(pm, "0")) {
      fprintf(stderr, "[mpigx] MPIGX_PEER_MEM=%s: expected auto or xdev\n", pm);
      return MPIGX_ERR_ARG;
    }
  }
  return MPIGX_SUCCESS;
}

// Frees whatever a (possibly half-built) communicator holds: the device
// allocations, the pinned page, peer mappings and the shm block.  Used by
// mpigx_comm_free after its closing barrier and by every failed init.
void comm_release(mpigx_comm* c) {
  g_live_comms.fetch_sub(1, std::memory_order_relaxed);
  (void)hipSetDevice(c->device);
  if (c->stream || c->launch_seq) (void)hipStreamSynchronize(c->stream);
  watch_unregister(c);  // after the drain: a waiting stream-ordered launch needs the watcher to be cancelled
  rt::rma_destroy(c);
  rt::p2p_destroy(c);
  for (int q = 0; q < c->n; ++q) {
    if (c->peer_opened[q]) (void)hipIpcCloseMemHandle(c->peer_stage[q]);
    if (c->peer_sig_opened[q]) (void)hipIpcCloseMemHandle(c->peer_sig[q]);
    if (c->peer_ll_opened[q]) (void)hipIpcCloseMemHandle(c->peer_ll[q]);
    if (c->peer_rw_opened[q]) {
      (void)hipIpcCloseMemHandle(c->peer_sig_rw[q]);
      if (c->peer_ll_rw[q]) (void)hipIpcCloseMemHandle(c->peer_ll_rw[q]);
    }
  }
  for (auto& im : c->imports) (void)hipIpcCloseMemHandle(im.base);
  if (c->shm) munmap(c->shm, sizeof(ShmBlock));
  for (auto& b : c->tmp_free) (void)hipFree(b.second);
  for (auto& b : c->tmp_used) (void)hipFree(b.second);
  if (c->stage) (void)hipFree(c->stage);
  if (c->sig) (void)hipFree(c->sig);
  if (c->sig_rw) (void)hipFree(c->sig_rw);
  if (c->ll) (void)hipFree(c->ll);
  if (c->ll_rw) (void)hipFree(c->ll_rw);
  if (c->dcount_dev) (void)hipFree(c->dcount_dev);
  for (auto& e : c->ar_ev)
    if (e) (void)hipEventDestroy(e);
  if (c->so_ev) (void)hipEventDestroy(c->so_ev);  // after watch_unregister: the watcher no longer queries it
  if (c->err) (void)hipHostFree(c->err);
  (void)hipGetLastError();
  delete c;
}

// Builds communicator c (allocations, then the shm rendezvous and the IPC
// mappings of every peer's arena and signal array).  On failure returns the
// error with c holding whatever was acquired so far; *shm_created tells the
// caller it must unlink the shm name (rank 0 before every rank mapped it).
int comm_init(mpigx_comm* c, const IdPayload& p, bool* shm_created) {
  const int rank = c->rank, nranks = c->n, device = c->device;
  int krc = knobs_from_env(c);
  if (krc) return krc;
  c->timeout_ticks = (uint64_t)(env_ll("MPIGX_TIMEOUT_MS", 60000) * 100000ll);  // 100 MHz clock
  c->epoch = (uint64_t)env_ll("MPIGX_EPOCH_BASE", 1);  // test hook (LL flag generations); must agree
  if (c->epoch < 1) c->epoch = 1;
  c->ll_gen = (unsigned)(c->epoch >> 31);
  c->test_import_fail = (int)env_ll("MPIGX_TEST_IMPORT_FAIL", 0);
  // diagnostic only (selects no path, so not an agreed knob): one stderr line
  // per launch with its epoch, grid, view key and completion sequence
  c->diag_trace = env_ll("MPIGX_DIAG_TRACE", 0) != 0;  // per rank: fault injection, not a knob
  // IPC export size limit (runtime.hpp ipc_alloc_max): selects no kernel —
  // whether a buffer is exportable is agreed per exchange (zc_exchange: every
  // rank takes the staged path if any rank cannot export)
  (void)hipRuntimeGetVersion(&c->hip_runtime);
  c->ipc_alloc_max = c->hip_runtime < 70200000 ? (1ll << 31) - 1 : 0;
  c->ipc_alloc_max = env_ll("MPIGX_IPC_ALLOC_MAX", c->ipc_alloc_max);

  if (c->ipc_alloc_max > 0 && (long long)c->stage_bytes > c->ipc_alloc_max) {
    // every peer maps the arena: one the loaded runtime cannot IPC-map would
    // hang the rendezvous (runtime.hpp ipc_alloc_max)
    fprintf(stderr, "[mpigx] MPIGX_STAGING_BYTES=%zu exceeds what HIP runtime %d can IPC-map (%lld bytes)\n",
            (size_t)c->stage_bytes, c->hip_runtime, c->ipc_alloc_max);
    return MPIGX_ERR_ARG;
  }
  HIPCK(hipMalloc(&c->stage, c->stage_bytes));
  // rows [0, kMaxBlocks): per-block barriers; row kMaxBlocks: whole-launch
  // barrier (device.hpp rank_barrier_grid)
  // + one row: word 0 of row kMaxBlocks + 1 holds this rank's canary
  // (kSigCanary ^ rank), which the launch trace reads through every peer's
  // mapping to check that the mapping still aliases the peer's array
  // Two of each (DESIGN §3 "one memory type per writer / reader pair"): a
  // peer on ANOTHER device stores into my uncached array (its mapping of my
  // memory reaches HBM over xGMI, my polls read HBM); a peer on MY device
  // stores into my ordinary-memory array.  Its IPC import of my memory is an
  // ordinary cached mapping whatever my allocation's flags, so a store it
  // makes into my UNCACHED array stays a dirty line in its XCD's L2 that its
  // release does not write back and my uncached polls never see (8 ranks on
  // one GPU: the root's entry word never reached rank 0; an atomic read of
  // the slot on rank 0 saw the old word too, r04e/r04h) — between two
  // cached mappings of ordinary memory the hardware keeps the XCDs' L2s
  // coherent as within one process.
  const size_t sig_bytes = sig_index(kMaxBlocks + 2, 0) * sizeof(uint64_t);
  HIPCK(hipExtMallocWithFlags((void**)&c->sig, sig_bytes, hipDeviceMallocUncached));
  HIPCK(hipMalloc((void**)&c->sig_rw, sig_bytes));
  HIPCK(hipMemset(c->sig, 0, sig_bytes));
  HIPCK(hipMemset(c->sig_rw, 0, sig_bytes));
  {
    const uint64_t canary = kSigCanary ^ (uint64_t)rank;
    HIPCK(hipMemcpy(c->sig + sig_index(kMaxBlocks + 1, 0), &canary, sizeof canary, hipMemcpyHostToDevice));
    HIPCK(hipMemcpy(c->sig_rw + sig_index(kMaxBlocks + 1, 0), &canary, sizeof canary, hipMemcpyHostToDevice));
  }
  // LL areas for small messages (M_AR_LL ...): the same two memory types
  c->ll_stride = rup(c->ll_max, 16) / 8 * kLLLine;
  // events of the measured algorithm choices (MPIGX_AR_TUNE)
  for (auto& x : c->mt_choice) x = -1;
  if (c->ar_tune) {
    HIPCK(hipEventCreate(&c->ar_ev[0]));
    HIPCK(hipEventCreate(&c->ar_ev[1]));
  }
  if (c->ll_max > 0 && nranks > 1) {
    const size_t llb = (size_t)2 * kMaxRanks * c->ll_stride;
    HIPCK(hipExtMallocWithFlags((void**)&c->ll, llb, hipDeviceMallocUncached));
    HIPCK(hipMalloc((void**)&c->ll_rw, llb));
    HIPCK(hipMemset(c->ll, 0, llb));
    HIPCK(hipMemset(c->ll_rw, 0, llb));
  }
  HIPCK(hipHostMalloc((void**)&c->err, 64, hipHostMallocCoherent | hipHostMallocMapped));
  memset(c->err, 0, 64);
  HIPCK(hipHostGetDevicePointer((void**)&c->err_dev, c->err, 0));
  c->done = (volatile unsigned long long*)(c->err + 8);  // same pinned page, own 32-B slot
  HIPCK(hipHostGetDevicePointer((void**)&c->done_dev, (void*)c->done, 0));
  // and the late-peer words: the launch my GPU last started, the cancel word
  c->started = (volatile unsigned long long*)(c->err + 4);
  c->cancel = (volatile unsigned*)(c->err + 6);
  HIPCK(hipHostGetDevicePointer((void**)&c->started_dev, (void*)c->started, 0));
  HIPCK(hipHostGetDevicePointer((void**)&c->cancel_dev, (void*)c->cancel, 0));
  HIPCK(hipMalloc((void**)&c->dcount_dev, 64));
  HIPCK(hipMemset(c->dcount_dev, 0, 64));
  HIPCK(hipDeviceSynchronize());
  c->peer_stage[rank] = c->stage;
  c->peer_sig[rank] = c->sig;
  c->peer_ll[rank] = c->ll;
  c->peer_sig_rw[rank] = c->sig_rw;
  c->peer_ll_rw[rank] = c->ll_rw;
  c->rw_mask = 1u << rank;
  {
    int cus = 0;
    HIPCK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    c->cus_min = cus > 0 ? cus : 1;
    c->dev_share = 1;
  }
  if (nranks == 1) return MPIGX_SUCCESS;

  // rendezvous
  const double t0 = now_s();
  const double limit = env_ll("MPIGX_INIT_TIMEOUT_MS", 120000) / 1000.0;
  int fd = -1;
  if (rank == 0) {
    fd = shm_open(p.name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd >= 0) *shm_created = true;
    if (fd < 0 || ftruncate(fd, sizeof(ShmBlock)) != 0) {
      fprintf(stderr, "[mpigx] shm_open(%s): %s\n", p.name, strerror(errno));
      if (fd >= 0) close(fd);
      return MPIGX_ERR_INTERN;
    }
  } else {
    while ((fd = shm_open(p.name, O_RDWR, 0600)) < 0) {
      if (now_s() - t0 > limit) return MPIGX_ERR_OTHER;
      usleep(1000);
    }
    struct stat st;
    while (fstat(fd, &st) == 0 && (size_t)st.st_size < sizeof(ShmBlock)) {
      if (now_s() - t0 > limit) {
        close(fd);
        return MPIGX_ERR_OTHER;
      }
      usleep(1000);
    }
  }
  void* m = mmap(nullptr, sizeof(ShmBlock), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return MPIGX_ERR_INTERN;
  c->shm = (ShmBlock*)m;
  if (rank == 0) {
    c->shm->nranks = nranks;
    c->shm->magic.store(kMagic, std::memory_order_release);
  } else {
    while (c->shm->magic.load(std::memory_order_acquire) != kMagic) {
      if (now_s() - t0 > limit) return MPIGX_ERR_OTHER;
      usleep(1000);
    }
    if (c->shm->nranks != nranks) return MPIGX_ERR_ARG;
  }
  ShmRank& me = c->shm->ranks[rank];
  me.pid = getpid();
  me.device = device;
  hipDeviceProp_t prop;
  HIPCK(hipGetDeviceProperties(&prop, device));
  me.pci_bus = prop.pciBusID;
  me.pci_dev = prop.pciDeviceID;
  me.pci_domain = prop.pciDomainID;
  me.cus = prop.multiProcessorCount;
  me.max_share = (int)env_ll("MPIGX_MAX_RANKS_PER_DEVICE", 10);
  for (int k = 0; k < MPIGX_KNOB_COUNT; ++k) me.knobs[k] = knob_value(c, k);
  me.epoch0 = c->epoch;
  me.stage_bytes = c->stage_bytes;
  me.stage_ptr = (unsigned long long)(uintptr_t)c->stage;
  me.sig_ptr = (unsigned long long)(uintptr_t)c->sig;
  me.sig_rw_ptr = (unsigned long long)(uintptr_t)c->sig_rw;
  HIPCK(hipIpcGetMemHandle(&me.stage_h, c->stage));
  HIPCK(hipIpcGetMemHandle(&me.sig_h, c->sig));
  HIPCK(hipIpcGetMemHandle(&me.sig_rw_h, c->sig_rw));
  me.ll_bytes = c->ll ? (unsigned long long)c->ll_max : 0;
  me.ll_ptr = (unsigned long long)(uintptr_t)c->ll;
  me.ll_rw_ptr = (unsigned long long)(uintptr_t)c->ll_rw;
  if (c->ll) HIPCK(hipIpcGetMemHandle(&me.ll_h, c->ll));
  if (c->ll_rw) HIPCK(hipIpcGetMemHandle(&me.ll_rw_h, c->ll_rw));
  c->shm->arrived.fetch_add(1, std::memory_order_acq_rel);
  while (c->shm->arrived.load(std::memory_order_acquire) < nranks) {
    if (now_s() - t0 > limit) return MPIGX_ERR_OTHER;
    usleep(200);
  }
  // every path-selecting knob must agree (a rank taking another branch than
  // its peers would launch another kernel and spin until the device timeout)
  for (int q = 0; q < nranks; ++q) {
    const ShmRank& pr = c->shm->ranks[q];
    for (int k = 0; k < MPIGX_KNOB_COUNT; ++k)
      if (pr.knobs[k] != me.knobs[k]) {
        fprintf(stderr, "[mpigx] rank %d: %s differs between ranks (%lld on rank %d, %lld on rank %d)\n", rank,
                kKnobEnv[k], me.knobs[k], rank, pr.knobs[k], q);
        return MPIGX_ERR_ARG;
      }
    if (pr.epoch0 != me.epoch0) return MPIGX_ERR_ARG;  // MPIGX_EPOCH_BASE likewise
  }
  // ranks sharing a device: every rank's grid of a spinning kernel must be
  // resident at once (kernel_cap: per launched kernel, from cus_min and
  // dev_share; include/mpigx.h mpigx_comm_device_share)
  {
    int share = 1, cus = me.cus;
    long long limit_share = me.max_share;
    for (int q = 0; q < nranks; ++q) {
      const ShmRank& a = c->shm->ranks[q];
      if (a.max_share < limit_share) limit_share = a.max_share;  // every rank applies the same limit
      int k = 0;
      for (int j = 0; j < nranks; ++j) {
        const ShmRank& b = c->shm->ranks[j];
        k += b.pci_domain == a.pci_domain && b.pci_bus == a.pci_bus && b.pci_dev == a.pci_dev;
      }
      share = k > share ? k : share;
      cus = a.cus < cus ? a.cus : cus;
    }
    c->dev_share = share;
    c->cus_min = cus;
    if (share > limit_share) {
      fprintf(stderr,
              "[mpigx] %d ranks share one GPU (limit MPIGX_MAX_RANKS_PER_DEVICE=%lld): more rank processes than "
              "that did not all get hardware queues at once; bind ranks to distinct GPUs\n",
              share, limit_share);
      return MPIGX_ERR_OTHER;
    }
  }
  for (int q = 0; q < nranks; ++q) {
    if (q == rank) continue;
    const ShmRank& pr = c->shm->ranks[q];
    c->same_device[q] = pr.pci_domain == me.pci_domain && pr.pci_bus == me.pci_bus && pr.pci_dev == me.pci_dev;
    // same device: the ordinary-memory arrays, unless MPIGX_PEER_MEM=xdev
    // makes this pair run the cross-device protocol (the device share, and so
    // the grid caps, still count it)
    if (c->same_device[q] && c->peer_mem == 0) c->rw_mask |= 1u << q;
    if (pr.pid == me.pid) {
      c->peer_stage[q] = (char*)(uintptr_t)pr.stage_ptr;
      c->peer_sig[q] = (uint64_t*)(uintptr_t)pr.sig_ptr;
      c->peer_ll[q] = (char*)(uintptr_t)pr.ll_ptr;
      c->peer_sig_rw[q] = (uint64_t*)(uintptr_t)pr.sig_rw_ptr;
      c->peer_ll_rw[q] = (char*)(uintptr_t)pr.ll_rw_ptr;
    } else {
      void* ps = nullptr;
      HIPCK(hipIpcOpenMemHandle(&ps, pr.stage_h, hipIpcMemLazyEnablePeerAccess));
      c->peer_stage[q] = (char*)ps;
      c->peer_opened[q] = true;
      // only the signal array / LL area of the memory type this pair uses
      void* pg = nullptr;
      void* pl = nullptr;
      if ((c->rw_mask >> q) & 1u) {
        HIPCK(hipIpcOpenMemHandle(&pg, pr.sig_rw_h, hipIpcMemLazyEnablePeerAccess));
        c->peer_sig_rw[q] = (uint64_t*)pg;
        c->peer_rw_opened[q] = true;
        if (c->ll) {
          HIPCK(hipIpcOpenMemHandle(&pl, pr.ll_rw_h, hipIpcMemLazyEnablePeerAccess));
          c->peer_ll_rw[q] = (char*)pl;
        }
      } else {
        HIPCK(hipIpcOpenMemHandle(&pg, pr.sig_h, hipIpcMemLazyEnablePeerAccess));
        c->peer_sig[q] = (uint64_t*)pg;
        c->peer_sig_opened[q] = true;
        if (c->ll) {
          HIPCK(hipIpcOpenMemHandle(&pl, pr.ll_h, hipIpcMemLazyEnablePeerAccess));
          c->peer_ll[q] = (char*)pl;
          c->peer_ll_opened[q] = true;
        }
      }
      if (c->diag_trace)
        fprintf(stderr, "[trace r%d] import peer %d (%s) sig=%p ll=%p stage=%p\n", rank, q,
                ((c->rw_mask >> q) & 1u) ? "same device: ordinary memory"
                : c->same_device[q]      ? "same device, xdev protocol: uncached"
                                         : "other device: uncached",
                pg, pl, ps);
    }
  }
  c->shm->connected.fetch_add(1, std::memory_order_acq_rel);
  while (c->shm->connected.load(std::memory_order_acquire) < nranks) {
    if (now_s() - t0 > limit) return MPIGX_ERR_OTHER;
    usleep(200);
  }
  if (rank == 0) {
    shm_unlink(p.name);  // every rank has it mapped now
    *shm_created = false;
  }
  return MPIGX_SUCCESS;
}

}  // namespace

extern "C" {

int mpigx_comm_init_rank(mpigx_comm_t* out, int nranks, const mpigx_unique_id_t* id, int rank, int device) {
  if (!out || !id) return MPIGX_ERR_ARG;
  if (nranks < 1 || nranks > kMaxRanks) return MPIGX_ERR_ARG;
  if (rank < 0 || rank >= nranks) return MPIGX_ERR_ARG;
  IdPayload p;
  memcpy(&p, id->internal, sizeof p);
  if (p.magic != kMagic) return MPIGX_ERR_ARG;
  HIPCK(hipSetDevice(device));
  mpigx_comm* c = new mpigx_comm();
  g_live_comms.fetch_add(1, std::memory_order_relaxed);  // comm_release (every exit path) takes it back
  c->rank = rank;
  c->n = nranks;
  c->device = device;
  bool created = false;
  const int rc = comm_init(c, p, &created);
  if (rc) {
    // nothing outlives a failed init: no allocation, mapping or shm name
    if (created) shm_unlink(p.name);
    mark_broken(c);
    comm_release(c);
    return rc;
  }
  *out = c;
  return MPIGX_SUCCESS;
}

int mpigx_comm_release(mpigx_comm_t c) {
  // No barrier: every collective kernel's last barrier retires the peers'
  // accesses to this rank's arena, signal array, LL area and buffers before
  // it completes here, so once this rank's queued work has drained nothing
  // of this rank is touched by a peer any more (for the communicator, which
  // its peers release the same way).
  if (!c) return MPIGX_ERR_COMM;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  comm_release(c);
  return MPIGX_SUCCESS;
}

int mpigx_comm_free(mpigx_comm_t c) {
  if (!c) return MPIGX_ERR_COMM;
  (void)hipSetDevice(c->device);
  int rc = MPIGX_SUCCESS;
  if (c->n > 1 && !c->broken) {
    // make sure no peer still reads our staging
    const int b = c->blocking;
    c->blocking = 1;
    rc = mpigx_barrier(c);
    c->blocking = b;
  }
  (void)hipStreamSynchronize(c->stream);
  comm_release(c);
  return rc;
}

// MPI_Comm_split (comm.jl:92-105): (color, key) are agreed over the host
// control plane; the lowest (key, rank) member of each color creates the
// group's unique id, a second exchange hands it out, then every member joins
// its group with mpigx_comm_init_rank (groups rendezvous independently).
int mpigx_comm_split(mpigx_comm_t c, int color, int key, mpigx_comm_t* out) {
  int rc = check_comm(c);
  if (rc) return rc;
  if (!out) return MPIGX_ERR_ARG;
  if (color < 0 && color != MPIGX_UNDEFINED) return MPIGX_ERR_ARG;
  const int n = c->n;
  int mine[2] = {color, key}, all[kMaxRanks][2];
  rc = host_allgather(c, mine, sizeof mine, all);
  if (rc) return rc;
  int members[kMaxRanks], m = 0;
  for (int q = 0; q < n; ++q)
    if (color != MPIGX_UNDEFINED && all[q][0] == color) members[m++] = q;
  // MPI order: by key, ties by rank in the parent
  for (int i = 1; i < m; ++i)
    for (int j = i; j > 0 && (all[members[j]][1] < all[members[j - 1]][1]); --j) {
      const int t = members[j];
      members[j] = members[j - 1];
      members[j - 1] = t;
    }
  int sub = -1;
  for (int i = 0; i < m; ++i)
    if (members[i] == c->rank) sub = i;
  mpigx_unique_id_t id;
  memset(&id, 0, sizeof id);
  if (sub == 0) {
    rc = mpigx_get_unique_id(&id);
    if (rc) return rc;
  }
  static_assert(sizeof(mpigx_unique_id_t) <= 256, "control-plane blob");
  std::vector<mpigx_unique_id_t> ids(n);
  rc = host_allgather(c, &id, sizeof id, ids.data());
  if (rc) return rc;
  if (sub < 0) {
    *out = nullptr;
    return MPIGX_SUCCESS;
  }
  mpigx_comm_t nc = nullptr;
  rc = mpigx_comm_init_rank(&nc, m, &ids[members[0]], sub, c->device);
  if (rc) return rc;
  nc->stream = c->stream;
  nc->blocking = c->blocking;
  nc->order = c->order;
  *out = nc;
  return MPIGX_SUCCESS;
}

int mpigx_comm_rank(mpigx_comm_t c, int* rank) {
  if (!c) return MPIGX_ERR_COMM;
  if (rank) *rank = c->rank;
  return MPIGX_SUCCESS;
}
int mpigx_comm_size(mpigx_comm_t c, int* size) {
  if (!c) return MPIGX_ERR_COMM;
  if (size) *size = c->n;
  return MPIGX_SUCCESS;
}
int mpigx_comm_device(mpigx_comm_t c, int* device) {
  if (!c) return MPIGX_ERR_COMM;
  if (device) *device = c->device;
  return MPIGX_SUCCESS;
}
int mpigx_comm_set_stream(mpigx_comm_t c, void* stream) {
  if (!c) return MPIGX_ERR_COMM;
  c->stream = (hipStream_t)stream;
  return MPIGX_SUCCESS;
}
int mpigx_comm_set_blocking(mpigx_comm_t c, int blocking) {
  if (!c) return MPIGX_ERR_COMM;
  c->blocking = blocking ? 1 : 0;
  return MPIGX_SUCCESS;
}
int mpigx_comm_synchronize(mpigx_comm_t c) {
  int rc = check_comm(c);
  if (rc) return rc;
  const int b = c->blocking;
  c->blocking = 1;
  rc = finish(c);
  c->blocking = b;
  return rc;
}
int mpigx_comm_zc_stats(mpigx_comm_t c, unsigned long long* optimistic_hits, unsigned long long* exchanges) {
  if (!c) return MPIGX_ERR_COMM;
  if (optimistic_hits) *optimistic_hits = c->zstat_hits;
  if (exchanges) *exchanges = c->zstat_exchanges;
  return MPIGX_SUCCESS;
}
int mpigx_comm_host_stats(mpigx_comm_t c, double* prelaunch_us) {
  if (!c) return MPIGX_ERR_COMM;
  if (prelaunch_us) *prelaunch_us = c->last_prelaunch_s * 1e6;
  return MPIGX_SUCCESS;
}
int mpigx_comm_ar_choice(mpigx_comm_t c, int* choice, double* pull_ns_per_mib, double* push_ns_per_mib) {
  if (!c) return MPIGX_ERR_COMM;
  if (choice) *choice = c->ar_choice;
  if (pull_ns_per_mib) *pull_ns_per_mib = c->ar_spb[0] * 1e9 * 1048576.0;
  if (push_ns_per_mib) *push_ns_per_mib = c->ar_spb[1] * 1e9 * 1048576.0;
  return MPIGX_SUCCESS;
}
int mpigx_comm_ar_costs(mpigx_comm_t c, int* choice, double* ns_per_mib) {
  if (!c) return MPIGX_ERR_COMM;
  if (choice) *choice = c->ar_choice;
  if (ns_per_mib)
    for (int k = 0; k < 3; ++k) ns_per_mib[k] = c->ar_spb[k] < 0 ? -1.0 : c->ar_spb[k] * 1e9 * 1048576.0;
  return MPIGX_SUCCESS;
}
int mpigx_comm_tune_class(mpigx_comm_t c, int log2_bytes, int* choice, double* ns_per_mib) {
  if (!c) return MPIGX_ERR_COMM;
  // log2_bytes + 64 * kind (0 Allreduce, 1 Bcast, 2 Allgather, 3 Alltoall)
  const int kind = log2_bytes / 64, k = log2_bytes % 64;
  if (log2_bytes < 0 || kind >= mpigx_comm::kTuneKinds || k >= mpigx_comm::kTuneClasses) return MPIGX_ERR_ARG;
  const int slot = kind * mpigx_comm::kTuneClasses + k;
  if (choice) *choice = c->mt_choice[slot];
  if (ns_per_mib)
    for (int v = 0; v < 4; ++v) ns_per_mib[v] = c->mt_spb[slot][v] * 1e9 * 1048576.0;
  return MPIGX_SUCCESS;
}
int mpigx_comm_set_reduce_order(mpigx_comm_t c, int order) {
  if (!c) return MPIGX_ERR_COMM;
  if (order != MPIGX_ORDER_MPICH && order != MPIGX_ORDER_LINEAR) return MPIGX_ERR_ARG;
  c->order = order;
  return MPIGX_SUCCESS;
}

// Collective: every rank's (knob, value) over the control plane; any
// difference -> MPIGX_ERR_ARG everywhere and nothing changes.
int mpigx_comm_set_knob(mpigx_comm_t c, int knob, long long value) {
  if (!c) return MPIGX_ERR_COMM;
  if (c->broken) return MPIGX_ERR_OTHER;
  struct {
    long long knob, value;
  } mine = {knob, value}, all[kMaxRanks];
  if (c->n > 1) {
    const int rc = host_allgather(c, &mine, sizeof mine, all);
    if (rc) return rc;
    for (int q = 0; q < c->n; ++q)
      if (all[q].knob != mine.knob || all[q].value != mine.value) return MPIGX_ERR_ARG;
  }
  if (knob < 0 || knob >= MPIGX_KNOB_COUNT) return MPIGX_ERR_ARG;
  return knob_apply(c, knob, value, false);
}
int mpigx_comm_get_knob(mpigx_comm_t c, int knob, long long* value) {
  if (!c) return MPIGX_ERR_COMM;
  if (knob < 0 || knob >= MPIGX_KNOB_COUNT || !value) return MPIGX_ERR_ARG;
  *value = knob_value(c, knob);
  return MPIGX_SUCCESS;
}
int mpigx_comm_device_share(mpigx_comm_t c, int* ranks, int* cap) {
  if (!c) return MPIGX_ERR_COMM;
  if (ranks) *ranks = c->dev_share;
  if (cap) *cap = c->cus_min / (c->dev_share > 0 ? c->dev_share : 1);
  return MPIGX_SUCCESS;
}
int mpigx_comm_diag_break(mpigx_comm_t c) {
  if (!c) return MPIGX_ERR_COMM;
  mark_broken(c);
  return MPIGX_SUCCESS;
}
int mpigx_read_probe(const void* const* in, int nin, long long bytes, void* sink, void* stream) {
  if (!in || !sink || bytes < 16 || (nin != 1 && nin != 2 && nin != 4 && nin != 8)) return MPIGX_ERR_ARG;
  for (int k = 0; k < nin; ++k)
    if (!in[k] || ((uintptr_t)in[k] & 15)) return MPIGX_ERR_BUFFER;
  HIPCK(launch_read_probe(in, nin, bytes, sink, (hipStream_t)stream));
  return MPIGX_SUCCESS;
}
int mpigx_mix_probe(const void* const* in, int nin, long long bytes, void* out, void* stream) {
  if (!in || !out || bytes < 16 || (nin != 1 && nin != 2 && nin != 4 && nin != 8)) return MPIGX_ERR_ARG;
  if ((uintptr_t)out & 15) return MPIGX_ERR_BUFFER;
  for (int k = 0; k < nin; ++k)
    if (!in[k] || ((uintptr_t)in[k] & 15)) return MPIGX_ERR_BUFFER;
  HIPCK(launch_mix_probe(in, nin, bytes, out, (hipStream_t)stream));
  return MPIGX_SUCCESS;
}
int mpigx_comm_diag_peer_mem(mpigx_comm_t c, unsigned* rw_mask, unsigned* same_device) {
  if (!c) return MPIGX_ERR_COMM;
  unsigned sd = 1u << c->rank;
  for (int q = 0; q < c->n; ++q)
    if (c->same_device[q]) sd |= 1u << q;
  if (rw_mask) *rw_mask = c->rw_mask;
  if (same_device) *same_device = sd;
  return MPIGX_SUCCESS;
}
int mpigx_comm_set_stamps(mpigx_comm_t c, void* stamps) {
  if (!c) return MPIGX_ERR_COMM;
  c->stamps = (unsigned long long*)stamps;
  return MPIGX_SUCCESS;
}
int mpigx_comm_diag_slots(mpigx_comm_t c, int block, unsigned long long* mine, unsigned long long* theirs) {
  if (!c) return MPIGX_ERR_COMM;
  if (block < 0 || block > kMaxBlocks || !mine || !theirs) return MPIGX_ERR_ARG;
  (void)hipSetDevice(c->device);
  for (int q = 0; q < c->n; ++q) {
    mine[q] = theirs[q] = 0;
    const bool rw = (c->rw_mask >> q) & 1u;
    if (hipMemcpy(&mine[q], (rw ? c->sig_rw : c->sig) + sig_index(block, q), 8, hipMemcpyDeviceToHost) !=
            hipSuccess ||
        hipMemcpy(&theirs[q], (rw ? c->peer_sig_rw[q] : c->peer_sig[q]) + sig_index(block, c->rank), 8,
                  hipMemcpyDeviceToHost) != hipSuccess) {
      (void)hipGetLastError();
      return MPIGX_ERR_INTERN;
    }
  }
  return MPIGX_SUCCESS;
}
int mpigx_comm_diag_state(mpigx_comm_t c, unsigned long long* out) {
  if (!c || !out) return MPIGX_ERR_COMM;
  // no call here waits on the device: safe from a watchdog thread while the
  // owner is blocked in a synchronize
  const hipError_t q = hipStreamQuery(c->stream);
  (void)hipGetLastError();
  out[0] = q == hipSuccess ? 0 : (q == hipErrorNotReady ? 1 : 2);
  out[1] = c->done ? *c->done : 0;
  out[2] = c->done_target;
  out[3] = c->dcount_total;
  out[4] = c->launch_seq;
  out[5] = c->epoch;
  out[6] = c->xseq;
  unsigned long long mn = ~0ull;
  if (c->shm)
    for (int q2 = 0; q2 < c->n; ++q2) {
      const unsigned long long s = c->shm->ranks[q2].xseq.load(std::memory_order_acquire);
      mn = s < mn ? s : mn;
    }
  out[7] = c->shm ? mn : 0;
  return MPIGX_SUCCESS;
}
int mpigx_comm_diag_mapcheck(mpigx_comm_t c, unsigned long long nonce, unsigned* stale) {
  if (!c || !stale) return MPIGX_ERR_COMM;
  *stale = 0;
  if (c->n == 1) return MPIGX_SUCCESS;
  (void)hipSetDevice(c->device);
  HIPCK(hipStreamSynchronize(c->stream));
  const uint64_t mine = nonce ^ (uint64_t)c->rank;
  const size_t at = sig_index(kMaxBlocks + 1, 0);
  HIPCK(hipMemcpy(c->sig + at, &mine, 8, hipMemcpyHostToDevice));
  HIPCK(hipMemcpy(c->sig_rw + at, &mine, 8, hipMemcpyHostToDevice));
  int dummy = 0, all_dummy[kMaxRanks];
  int rc = host_allgather(c, &dummy, sizeof dummy, all_dummy);  // every rank has written
  if (rc) return rc;
  unsigned seen_stale = 0;
  for (int q = 0; q < c->n; ++q) {
    if (q == c->rank) continue;
    uint64_t* arr = ((c->rw_mask >> q) & 1u) ? c->peer_sig_rw[q] : c->peer_sig[q];
    uint64_t w = 0;
    HIPCK(hipMemcpy(&w, arr + at, 8, hipMemcpyDeviceToHost));
    if (w != (nonce ^ (uint64_t)q)) seen_stale |= 1u << q;
  }
  unsigned all[kMaxRanks];
  rc = host_allgather(c, &seen_stale, sizeof seen_stale, all);
  if (rc) return rc;
  for (int q = 0; q < c->n; ++q) *stale |= all[q];
  return MPIGX_SUCCESS;
}
int mpigx_comm_set_timeout(mpigx_comm_t c, long long ms) {
  if (!c) return MPIGX_ERR_COMM;
  if (ms < 1) return MPIGX_ERR_ARG;
  c->timeout_ticks = (uint64_t)ms * 100000ull;  // 100 MHz device clock
  return MPIGX_SUCCESS;
}

// ---------------------------------------------------------------------------
int mpigx_barrier(mpigx_comm_t c) {
  int rc = check_comm(c);
  if (rc) return rc;
  if (c->n == 1) return finish(c);
  CopyArgs a;
  memset(&a, 0, sizeof a);
  a.pv = make_view(c);
  a.mode = C_BARRIER;
  HIPCK(launch_copy(dim3(1), c->stream, a));
  note_launch(c, a.pv, 1);
  c->epoch += 1;
  return finish(c);
}

int mpigx_comm_probe(mpigx_comm_t c, int kind, long long bytes, double* seconds) {
  int rc = check_comm(c);
  if (rc) return rc;
  if (c->n == 1 || bytes <= 0) return MPIGX_ERR_ARG;
  if ((size_t)bytes > c->stage_bytes) bytes = (long long)c->stage_bytes;
  bytes &= ~15ll;
  CopyArgs a;
  memset(&a, 0, sizeof a);
  a.pv = make_view(c);
  a.mode = kind == 1 ? C_PROBE_ONE : C_PROBE_ALL;
  a.bytes = bytes;
  const int g = c->max_blocks < cap_copy(c) ? c->max_blocks : cap_copy(c);
  a.slice = rup(cdiv(bytes, g), 16);
  hipEvent_t e0, e1;
  HIPCK(hipEventCreate(&e0));
  HIPCK(hipEventCreate(&e1));
  HIPCK(hipEventRecord(e0, c->stream));
  HIPCK(launch_copy(dim3(g), c->stream, a));
  note_launch(c, a.pv, g);
  HIPCK(hipEventRecord(e1, c->stream));
  c->epoch += 2;
  HIPCK(hipEventSynchronize(e1));
  float ms = 0;
  HIPCK(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (seconds) *seconds = ms / 1e3;
  return finish(c);
}

static int bcast_impl(void* buf, int count, int datatype, int root, mpigx_comm_t c) {
  int rc = check_comm(c);
  if (rc) return rc;
  const TypeInfo* t = find_type(datatype);
  if (!t) return MPIGX_ERR_TYPE;
  if (count < 0) return MPIGX_ERR_COUNT;
  if (root < 0 || root >= c->n) return MPIGX_ERR_ROOT;
  if (count == 0) return MPIGX_SUCCESS;
  if (!buf) return MPIGX_ERR_BUFFER;
  if (c->n == 1) return finish(c);
  const long long bytes = (long long)count * t->size;
  const long long round = (long long)(c->stage_bytes & ~(size_t)15);
  // direct pull from the root (one barrier less) for small messages or two
  // ranks; scatter + allgather when the root's links would be the bottleneck.
  // The choice depends only on (bytes, n, env), identical on every rank.
  const bool env = c->bcast_mode != 0;  // MPIGX_BCAST knob: 1 direct, 2 sag, 3 relay
  bool sag = c->n >= 3 && bytes >= c->bcast_sag_min;
  if (c->bcast_mode == 1) sag = false;
  if (c->bcast_mode >= 2) sag = c->n >= 2;
  // zero-copy: the relay replaces the pull scatter + allgather (n >= 3)
  // unless "sag" is asked for by name
  const bool relay = sag && c->n >= 3 && c->bcast_mode != 2;
  // (zero-copy first when the size asks for it: tests force it at every size)
  // below the zero-copy size: LL or the staged copy, measured (mt_*)
  const bool zc_size = c->zc_min > 0 && bytes >= c->zc_min;
  int timed = -1, cls = -1;
  const int force = (!env && c->algo == MPIGX_ALGO_AUTO && !zc_size) ? mt_pick(c, TK_BCAST, bytes, &timed, &cls) : -1;
  if (timed >= 0) HIPCK(hipEventRecord(c->ar_ev[0], c->stream));
  if (force >= 0 ? force == V_LL : (!env && copy_ll_take(c, bytes) && !zc_size)) {
    // small: the root's lines straight into every peer's LL area (C_BCAST_LL)
    CopyArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    a.mode = C_BCAST_LL;
    a.root = root;
    a.bytes = bytes;
    a.send = buf;
    a.recv = buf;
    if (int e = ll_fill(c, a.pv, a.ll_push, &a.ll_in, &a.ll_stride, &a.ll_flag)) return e;
    const int g = grid_for(c, bytes, cap_copy(c));
    a.slice = rup(cdiv(bytes, g), kLLAlign);
    HIPCK(launch_copy(dim3(g), c->stream, a));
    note_launch(c, a.pv, g);
    ll_launched(c);
    return mt_finish(c, timed, cls, bytes);
  }
  if (c->zc_min > 0 && bytes >= c->zc_min) {
    // zero-copy: the non-roots pull straight from the root's buffer, no
    // copy-in at the root; large (n >= 3): the relay, each non-root pulling
    // its chunk once and storing it into every non-root's buffer
    bool staged;
    const int rc = zc_run(c, buf, buf, &staged, [&](const ZcLaunch& z) {
      CopyArgs a;
      memset(&a, 0, sizeof a);
      a.pv = make_view(c);
      zc_apply(a.pv, z);
      a.root = root;
      a.bytes = bytes;
      a.recv = buf;
      for (int p = 0; p < c->n; ++p) a.zsrc[p] = z.ps[p];
      zc_extents(a.pv, z, c->n, bytes, (relay || sag) ? bytes : 0);  // relay / sag store into peers' buffers
      int g;
      if (relay) {
        a.mode = C_BCAST_RELAY_ZC;
        a.chunk = rup(cdiv(bytes, c->n - 1), 16);
        g = grid_for(c, a.chunk, cap_copy(c));
        a.slice = rup(cdiv(a.chunk, g), 16);
      } else if (sag) {
        a.mode = C_BCAST_SAG_ZC;
        a.chunk = rup(cdiv(bytes, c->n), 16);
        g = grid_for(c, a.chunk, cap_copy(c));
        a.slice = rup(cdiv(a.chunk, g), 16);
      } else {
        a.mode = C_BCAST_ZC;
        g = grid_for(c, bytes, cap_copy(c));
        a.slice = rup(cdiv(bytes, g), 16);
      }
      seal_args(a);
      HIPCK(launch_copy(dim3(g), c->stream, a));
      note_launch(c, a.pv, g);
      c->epoch += (sag && !relay) ? 3 : 2;
      return MPIGX_SUCCESS;
    });
    if (rc || !staged) return rc;
    if (c->zc_require) return MPIGX_ERR_INTERN;
  }
  for (long long off = 0; off < bytes; off += round) {
    const long long len = bytes - off < round ? bytes - off : round;
    CopyArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    a.root = root;
    a.bytes = len;
    a.send = (const char*)buf + off;
    a.recv = (char*)buf + off;
    int g;
    if (sag) {
      a.mode = C_BCAST_SAG;
      a.chunk = rup(cdiv(len, c->n), 16);
      g = grid_for(c, a.chunk, cap_copy(c));
      a.slice = rup(cdiv(a.chunk, g), 16);
    } else {
      a.mode = C_BCAST;
      g = grid_for(c, len, cap_copy(c));
      a.slice = rup(cdiv(len, g), 16);
    }
    HIPCK(launch_copy(dim3(g), c->stream, a));
    note_launch(c, a.pv, g);
    c->epoch += sag ? 3 : 2;
  }
  return mt_finish(c, timed, cls, bytes);
}

static int gather_like(const void* send, int scount, int stype, void* recv, int rcount, int rtype,
                       mpigx_comm_t c, bool alltoall) {
  int rc = check_comm(c);
  if (rc) return rc;
  const TypeInfo* rt = find_type(rtype);
  if (!rt) return MPIGX_ERR_TYPE;
  if (rcount < 0) return MPIGX_ERR_COUNT;
  const bool inplace = send == MPIGX_IN_PLACE;
  if (!inplace) {
    const TypeInfo* st = find_type(stype);
    if (!st) return MPIGX_ERR_TYPE;
    if (scount < 0) return MPIGX_ERR_COUNT;
    if ((long long)scount * st->size != (long long)rcount * rt->size) return MPIGX_ERR_ARG;
  }
  const long long bytes = (long long)rcount * rt->size;  // per rank block
  if (bytes == 0) return MPIGX_SUCCESS;
  if (!recv || (!inplace && !send)) return MPIGX_ERR_BUFFER;
  const int n = c->n, r = c->rank;
  const char* s = inplace ? (alltoall ? (const char*)recv : (const char*)recv + (long long)r * bytes)
                          : (const char*)send;
  if (n == 1) return copy_n1(c, alltoall ? recv : (char*)recv, s, bytes);
  // below the zero-copy size: LL or the staged copy, measured (mt_*)
  const bool zc_size = c->zc_min > 0 && bytes * n >= c->zc_min && (!alltoall || !inplace);
  int timed = -1, cls = -1;
  const int force = (c->algo == MPIGX_ALGO_AUTO && !zc_size)
                        ? mt_pick(c, alltoall ? TK_ALLTOALL : TK_ALLGATHER, bytes, &timed, &cls) : -1;
  if (timed >= 0) HIPCK(hipEventRecord(c->ar_ev[0], c->stream));
  if (force >= 0 ? force == V_LL : (copy_ll_take(c, bytes) && !zc_size)) {
    // small: every rank's block(s) as LL lines, unpacked straight into recvbuf
    CopyArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    a.mode = alltoall ? C_ALLTOALL_LL : C_ALLGATHER_LL;
    a.bytes = bytes;
    a.total = bytes;
    a.send = s;
    a.recv = recv;
    if (int e = ll_fill(c, a.pv, a.ll_push, &a.ll_in, &a.ll_stride, &a.ll_flag)) return e;
    const int g = grid_for(c, bytes, cap_copy(c));
    a.slice = rup(cdiv(bytes, g), kLLAlign);
    HIPCK(launch_copy(dim3(g), c->stream, a));
    note_launch(c, a.pv, g);
    ll_launched(c);
    return mt_finish(c, timed, cls, bytes);
  }
  // large out-of-place Alltoall: pull straight from the peers' sendbufs (no
  // copy-in, no rounds).  IN_PLACE is given by every rank or none (MPI), and
  // (bytes, n, thresholds) agree, so every rank takes the same branch.
  if (alltoall && !inplace && c->zc_min > 0 && bytes * n >= c->zc_min) {
    bool staged;
    const int rc = zc_run(c, s, recv, &staged, [&](const ZcLaunch& z) {
      CopyArgs a;
      memset(&a, 0, sizeof a);
      a.pv = make_view(c);
      zc_apply(a.pv, z);
      a.mode = C_ALLTOALL_ZC;
      a.bytes = bytes;
      a.total = bytes;
      for (int p = 0; p < n; ++p) a.zsrc[p] = z.ps[p];
      zc_extents(a.pv, z, n, bytes * n, 0);
      const int g = grid_for(c, bytes * n, cap_copy(c));
      a.slice = rup(cdiv(bytes, g), 16);
      a.send = s;
      a.recv = recv;
      seal_args(a);
      HIPCK(launch_copy(dim3(g), c->stream, a));
      note_launch(c, a.pv, g);
      c->epoch += 2;
      return MPIGX_SUCCESS;
    });
    if (rc || !staged) return rc;
    if (c->zc_require) return MPIGX_ERR_INTERN;
  }
  if (!alltoall && c->zc_min > 0 && bytes * n >= c->zc_min) {
    // zero-copy Allgather: block p straight from rank p's sendbuf (IN_PLACE:
    // from block p of its recvbuf — the registration of `s` points there)
    bool staged;
    const int rc = zc_run(c, s, recv, &staged, [&](const ZcLaunch& z) {
      CopyArgs a;
      memset(&a, 0, sizeof a);
      a.pv = make_view(c);
      zc_apply(a.pv, z);
      a.mode = C_ALLGATHER_ZC;
      a.bytes = bytes;
      a.total = bytes;
      for (int p = 0; p < n; ++p) a.zsrc[p] = z.ps[p];
      zc_extents(a.pv, z, n, bytes, 0);
      const int g = grid_for(c, bytes, cap_copy(c));
      a.slice = rup(cdiv(bytes, g), 16);
      a.send = s;
      a.recv = recv;
      seal_args(a);
      HIPCK(launch_copy(dim3(g), c->stream, a));
      note_launch(c, a.pv, g);
      c->epoch += 2;
      return MPIGX_SUCCESS;
    });
    if (rc || !staged) return rc;
    if (c->zc_require) return MPIGX_ERR_INTERN;
  }
  // rounds: allgather stages `bytes` per rank; alltoall stages n*round
  const long long cap = alltoall ? (long long)(c->stage_bytes / n) & ~15ll : (long long)c->stage_bytes & ~15ll;
  for (long long off = 0; off < bytes; off += cap) {
    const long long len = bytes - off < cap ? bytes - off : cap;
    CopyArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    a.mode = alltoall ? C_ALLTOALL : C_ALLGATHER;
    a.bytes = len;
    a.total = bytes;
    a.sstride = rup(len, 16);
    const int g = grid_for(c, len * (alltoall ? n : 1), cap_copy(c));
    a.slice = rup(cdiv(len, g), 16);
    if (alltoall) {
      a.send = s + off;
      a.recv = (char*)recv + off;
      // staging layout for the round: block p at p*len
    } else {
      a.send = s + off;
      a.recv = (char*)recv + off;
    }
    HIPCK(launch_copy(dim3(g), c->stream, a));
    note_launch(c, a.pv, g);
    c->epoch += 2;
  }
  return mt_finish(c, timed, cls, bytes);
}

// ---------------------------------------------------------------------------
// Derived datatypes in the byte-moving collectives: a
// contiguous derived type travels as bytes; any other one is packed on device
// (types.cpp pack_kernel) into a pooled temporary on the comm's stream, moved
// by the contiguous algorithm as MPI_BYTE, and unpacked on the same stream.
// ---------------------------------------------------------------------------
static bool derived(int h) { return rt::dtype_size(h) < 0; }

static int bytes_of(int type, long long count, rt::TypeDesc* d, int* out) {
  if (rt::type_info(type, d)) return MPIGX_ERR_TYPE;
  if (count < 0) return MPIGX_ERR_COUNT;
  const long long b = count * d->size;
  if (b > 0x7fffffff) return MPIGX_ERR_COUNT;
  *out = (int)b;
  return MPIGX_SUCCESS;
}

static int pack_on(mpigx_comm* c, int type, const void* typed, long long count, char* tmp, long long bytes,
                   int unpack) {
  const int rc = rt::type_pack(type, typed, count, tmp, bytes, unpack, c->device, c->stream);
  if (!rc) c->unflagged = true;  // the final finish() drains the stream
  return rc;
}

int mpigx_bcast(void* buf, int count, int datatype, int root, mpigx_comm_t c) {
  if (!derived(datatype)) return bcast_impl(buf, count, datatype, root, c);
  int rc = check_comm(c);
  if (rc) return rc;
  rt::TypeDesc d;
  int nb;
  if ((rc = bytes_of(datatype, count, &d, &nb))) return rc;
  if (d.contig) return bcast_impl(buf, nb, MPIGX_BYTE, root, c);
  if (root < 0 || root >= c->n) return MPIGX_ERR_ROOT;
  if (nb == 0) return MPIGX_SUCCESS;
  char* tmp = tmp_get(c, nb);
  if (!tmp) return MPIGX_ERR_NO_MEM;
  if (c->rank == root) rc = pack_on(c, datatype, buf, count, tmp, nb, 0);
  if (!rc) rc = bcast_impl(tmp, nb, MPIGX_BYTE, root, c);
  if (!rc && c->rank != root) rc = pack_on(c, datatype, buf, count, tmp, nb, 1);
  if (!rc) rc = finish(c);
  tmp_put(c, tmp, nb);
  return rc;
}

static int gather_like_any(const void* sendbuf, int sendcount, int sendtype, void* recvbuf, int recvcount,
                           int recvtype, mpigx_comm_t c, bool alltoall) {
  const bool inplace = sendbuf == MPIGX_IN_PLACE;
  if (!derived(recvtype) && (inplace || !derived(sendtype)))
    return gather_like(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype, c, alltoall);
  int rc = check_comm(c);
  if (rc) return rc;
  const int n = c->n, r = c->rank;
  rt::TypeDesc rd, sd;
  int rb, sb = 0;
  if ((rc = bytes_of(recvtype, recvcount, &rd, &rb))) return rc;  // bytes per rank block
  if (!inplace && (rc = bytes_of(sendtype, sendcount, &sd, &sb))) return rc;
  if (!inplace && sb != rb) return MPIGX_ERR_ARG;
  if (rb == 0) return MPIGX_SUCCESS;
  const long long ninst = (long long)n * recvcount;  // recv elements in the whole buffer
  // receive side: the typed buffer, or a packed temporary of n blocks
  char* rtmp = nullptr;
  char* rdst = (char*)recvbuf;
  if (!rd.contig) {
    if (!(rtmp = tmp_get(c, (long long)n * rb))) return MPIGX_ERR_NO_MEM;
    rdst = rtmp;
  }
  const void* src = sendbuf;
  char* stmp = nullptr;
  if (inplace) {
    if (rtmp) {  // my block(s) of the typed recvbuf -> the packed temporary
      if (alltoall) rc = pack_on(c, recvtype, recvbuf, ninst, rtmp, (long long)n * rb, 0);
      else rc = pack_on(c, recvtype, (const char*)recvbuf + (long long)r * recvcount * rd.extent, recvcount,
                        rtmp + (long long)r * rb, rb, 0);
    }
  } else if (derived(sendtype) && !sd.contig) {
    const long long sinst = alltoall ? (long long)n * sendcount : sendcount;
    if (!(stmp = tmp_get(c, sinst * sd.size))) rc = MPIGX_ERR_NO_MEM;
    else rc = pack_on(c, sendtype, sendbuf, sinst, stmp, sinst * sd.size, 0);
    src = stmp;
  }
  if (!rc) rc = gather_like(src, rb, MPIGX_BYTE, rdst, rb, MPIGX_BYTE, c, alltoall);
  if (!rc && rtmp) rc = pack_on(c, recvtype, recvbuf, ninst, rtmp, (long long)n * rb, 1);
  if (!rc) rc = finish(c);
  if (stmp) tmp_put(c, stmp, 0);
  if (rtmp) tmp_put(c, rtmp, 0);
  return rc;
}

int mpigx_allgather(const void* sendbuf, int sendcount, int sendtype, void* recvbuf, int recvcount, int recvtype,
                    mpigx_comm_t c) {
  return gather_like_any(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype, c, false);
}
int mpigx_alltoall(const void* sendbuf, int sendcount, int sendtype, void* recvbuf, int recvcount, int recvtype,
                   mpigx_comm_t c) {
  return gather_like_any(sendbuf, sendcount, sendtype, recvbuf, recvcount, recvtype, c, true);
}

// ---------------------------------------------------------------------------
// v-collectives and rooted variants (collective.jl:90-578)
// ---------------------------------------------------------------------------
// Element size for the v-collectives: predefined types and contiguous derived
// types (displacements are in extents, equal to sizes only then).
static int vsize(int dtype, int* out) {
  rt::TypeDesc d;
  if (rt::type_info(dtype, &d) || !d.contig || d.size > 0x7fffffff) return MPIGX_ERR_TYPE;
  *out = (int)d.size;
  return MPIGX_SUCCESS;
}

static int type_bytes(int dtype, long long count, long long* out) {
  int sz;
  if (vsize(dtype, &sz)) return MPIGX_ERR_TYPE;
  if (count < 0) return MPIGX_ERR_COUNT;
  *out = count * sz;
  return MPIGX_SUCCESS;
}

// MPI_Gather / MPI_Gatherv (collective.jl:230-246, 363-382).  counts/displs
// (in recvtype elements) are read at the root only; NULL => equal blocks.
static int gather_common(const void* send, int scount, int stype, void* recv, int rcount, const int* rcounts,
                         const int* displs, int rtype, int root, mpigx_comm_t c) {
  int rc = check_comm(c);
  if (rc) return rc;
  const int n = c->n, r = c->rank;
  if (root < 0 || root >= n) return MPIGX_ERR_ROOT;
  const bool isroot = r == root, inplace = send == MPIGX_IN_PLACE;
  if (inplace && !isroot) return MPIGX_ERR_BUFFER;
  VSpec s;
  int rsz = 0;
  if (isroot) {
    if ((rc = vsize(rtype, &rsz))) return rc;
    if (!recv) return MPIGX_ERR_BUFFER;
    for (int p = 0; p < n; ++p) {
      const long long cnt = rcounts ? rcounts[p] : rcount;
      if (cnt < 0) return MPIGX_ERR_COUNT;
      const long long dsp = rcounts ? displs[p] : (long long)p * rcount;
      s.p_len[p] = cnt * rsz;
      s.p_slot[p] = 0;
      s.p_dst[p] = dsp * rsz;
    }
    if (inplace) s.p_len[r] = 0;
  }
  if (!inplace) {
    long long sb;
    if ((rc = type_bytes(stype, scount, &sb))) return rc;
    if (sb && !send) return MPIGX_ERR_BUFFER;
    s.ncopy = 1;
    s.c_slot[0] = 0;
    s.c_src[0] = 0;
    s.c_len[0] = sb;
  }
  s.send = (const char*)send;
  s.recv = (char*)recv;
  return vexchange(c, s);
}

int mpigx_gather(const void* sendbuf, int sendcount, int sendtype, void* recvbuf, int recvcount, int recvtype,
                 int root, mpigx_comm_t c) {
  const bool inplace = sendbuf == MPIGX_IN_PLACE;
  int rc = check_comm(c);
  if (rc) return rc;
  if (root < 0 || root >= c->n) return MPIGX_ERR_ROOT;
  const bool isroot = c->rank == root;
  if ((inplace || !derived(sendtype)) && (!isroot || !derived(recvtype)))
    return gather_common(sendbuf, sendcount, sendtype, recvbuf, recvcount, nullptr, nullptr, recvtype, root, c);
  // derived types: pack my contribution / receive packed blocks at the root
  rt::TypeDesc sd, rd;
  int sb = 0, rb = 0;
  if (!inplace && (rc = bytes_of(sendtype, sendcount, &sd, &sb))) return rc;
  if (isroot && (rc = bytes_of(recvtype, recvcount, &rd, &rb))) return rc;
  if (!isroot) rb = sb;
  const int n = c->n;
  char *stmp = nullptr, *rtmp = nullptr;
  const void* src = sendbuf;
  void* dst = recvbuf;
  if (!inplace && !sd.contig) {
    if (!(stmp = tmp_get(c, sb > 0 ? sb : 1))) return MPIGX_ERR_NO_MEM;
    rc = pack_on(c, sendtype, sendbuf, sendcount, stmp, sb, 0);
    src = stmp;
  }
  if (!rc && isroot && !rd.contig) {
    if (!(rtmp = tmp_get(c, (long long)n * rb > 0 ? (long long)n * rb : 1))) rc = MPIGX_ERR_NO_MEM;
    else if (inplace)
      rc = pack_on(c, recvtype, (const char*)recvbuf + (long long)root * recvcount * rd.extent, recvcount,
                   rtmp + (long long)root * rb, rb, 0);
    dst = rtmp;
  }
  if (!rc) rc = gather_common(src, inplace ? 0 : sb, MPIGX_BYTE, dst, rb, nullptr, nullptr, MPIGX_BYTE, root, c);
  if (!rc && rtmp) rc = pack_on(c, recvtype, recvbuf, (long long)n * recvcount, rtmp, (long long)n * rb, 1);
  if (!rc) rc = finish(c);
  if (stmp) tmp_put(c, stmp, 0);
  if (rtmp) tmp_put(c, rtmp, 0);
  return rc;
}
int mpigx_gatherv(const void* sendbuf, int sendcount, int sendtype, void* recvbuf, const int* recvcounts,
                  const int* displs, int recvtype, int root, mpigx_comm_t c) {
  if (c && c->rank == root && (!recvcounts || !displs)) return MPIGX_ERR_ARG;
  return gather_common(sendbuf, sendcount, sendtype, recvbuf, 0, recvcounts, displs, recvtype, root, c);
}

// MPI_Scatter / MPI_Scatterv (collective.jl:90-106, 156-175).
static int scatter_common(const void* send, int scount, const int* scounts, const int* displs, int stype, void* recv,
                          int rcount, int rtype, int root, mpigx_comm_t c) {
  int rc = check_comm(c);
  if (rc) return rc;
  const int n = c->n, r = c->rank;
  if (root < 0 || root >= n) return MPIGX_ERR_ROOT;
  const bool isroot = r == root, inplace = recv == MPIGX_IN_PLACE;
  if (inplace && !isroot) return MPIGX_ERR_BUFFER;
  VSpec s;
  if (isroot) {
    int ssz = 0;
    if ((rc = vsize(stype, &ssz))) return rc;
    if (!send) return MPIGX_ERR_BUFFER;
    s.ncopy = n;
    for (int q = 0; q < n; ++q) {
      const long long cnt = scounts ? scounts[q] : scount;
      if (cnt < 0) return MPIGX_ERR_COUNT;
      const long long dsp = scounts ? displs[q] : (long long)q * scount;
      s.c_slot[q] = q;
      s.c_src[q] = dsp * ssz;
      s.c_len[q] = (inplace && q == r) ? 0 : cnt * ssz;
    }
  }
  if (!inplace) {
    long long rb;
    if ((rc = type_bytes(rtype, rcount, &rb))) return rc;
    if (rb && !recv) return MPIGX_ERR_BUFFER;
    s.p_len[root] = rb;
    s.p_slot[root] = r;
    s.p_dst[root] = 0;
  }
  s.send = (const char*)send;
  s.recv = (char*)recv;
  return vexchange(c, s);
}

int mpigx_scatter(const void* sendbuf, int sendcount, int sendtype, void* recvbuf, int recvcount, int recvtype,
                  int root, mpigx_comm_t c) {
  const bool inplace = recvbuf == MPIGX_IN_PLACE;
  int rc = check_comm(c);
  if (rc) return rc;
  if (root < 0 || root >= c->n) return MPIGX_ERR_ROOT;
  const bool isroot = c->rank == root;
  if ((!isroot || !derived(sendtype)) && (inplace || !derived(recvtype)))
    return scatter_common(sendbuf, sendcount, nullptr, nullptr, sendtype, recvbuf, recvcount, recvtype, root, c);
  rt::TypeDesc sd, rd;
  int sb = 0, rb = 0;
  if (!inplace && (rc = bytes_of(recvtype, recvcount, &rd, &rb))) return rc;
  if (isroot && (rc = bytes_of(sendtype, sendcount, &sd, &sb))) return rc;
  if (!isroot) sb = rb;
  const int n = c->n;
  char *stmp = nullptr, *rtmp = nullptr;
  const void* src = sendbuf;
  void* dst = recvbuf;
  if (isroot && !sd.contig) {
    if (!(stmp = tmp_get(c, (long long)n * sb > 0 ? (long long)n * sb : 1))) return MPIGX_ERR_NO_MEM;
    rc = pack_on(c, sendtype, sendbuf, (long long)n * sendcount, stmp, (long long)n * sb, 0);
    src = stmp;
  }
  if (!rc && !inplace && !rd.contig) {
    if (!(rtmp = tmp_get(c, rb > 0 ? rb : 1))) rc = MPIGX_ERR_NO_MEM;
    dst = rtmp;
  }
  if (!rc) rc = scatter_common(src, sb, nullptr, nullptr, MPIGX_BYTE, dst, inplace ? 0 : rb, MPIGX_BYTE, root, c);
  if (!rc && rtmp) rc = pack_on(c, recvtype, recvbuf, recvcount, rtmp, rb, 1);
  if (!rc) rc = finish(c);
  if (stmp) tmp_put(c, stmp, 0);
  if (rtmp) tmp_put(c, rtmp, 0);
  return rc;
}
int mpigx_scatterv(const void* sendbuf, const int* sendcounts, const int* displs, int sendtype, void* recvbuf,
                   int recvcount, int recvtype, int root, mpigx_comm_t c) {
  if (c && c->rank == root && (!sendcounts || !displs)) return MPIGX_ERR_ARG;
  return scatter_common(sendbuf, 0, sendcounts, displs, sendtype, recvbuf, recvcount, recvtype, root, c);
}

// MPI_Allgatherv (collective.jl:424-437)
int mpigx_allgatherv(const void* sendbuf, int sendcount, int sendtype, void* recvbuf, const int* recvcounts,
                     const int* displs, int recvtype, mpigx_comm_t c) {
  int rc = check_comm(c);
  if (rc) return rc;
  if (!recvcounts || !displs) return MPIGX_ERR_ARG;
  const int n = c->n, r = c->rank;
  int rsz = 0;
  if ((rc = vsize(recvtype, &rsz))) return rc;
  const bool inplace = sendbuf == MPIGX_IN_PLACE;
  VSpec s;
  for (int p = 0; p < n; ++p) {
    if (recvcounts[p] < 0) return MPIGX_ERR_COUNT;
    s.p_len[p] = (long long)recvcounts[p] * rsz;
    s.p_slot[p] = 0;
    s.p_dst[p] = (long long)displs[p] * rsz;
  }
  if (!recvbuf && s.p_len[r]) return MPIGX_ERR_BUFFER;
  s.ncopy = 1;
  s.c_slot[0] = 0;
  if (inplace) {
    s.send = (const char*)recvbuf;
    s.c_src[0] = s.p_dst[r];
    s.c_len[0] = s.p_len[r];
    s.p_len[r] = 0;
  } else {
    long long sb;
    if ((rc = type_bytes(sendtype, sendcount, &sb))) return rc;
    if (sb && !sendbuf) return MPIGX_ERR_BUFFER;
    s.send = (const char*)sendbuf;
    s.c_src[0] = 0;
    s.c_len[0] = sb;
  }
  s.recv = (char*)recvbuf;
  return vexchange(c, s);
}

// MPI_Alltoallv (collective.jl:545-559); MPI-2.2 IN_PLACE takes the send
// layout from recvcounts/rdispls.
int mpigx_alltoallv(const void* sendbuf, const int* sendcounts, const int* sdispls, int sendtype, void* recvbuf,
                    const int* recvcounts, const int* rdispls, int recvtype, mpigx_comm_t c) {
  int rc = check_comm(c);
  if (rc) return rc;
  if (!recvcounts || !rdispls) return MPIGX_ERR_ARG;
  const int n = c->n, r = c->rank;
  const bool inplace = sendbuf == MPIGX_IN_PLACE;
  int rsz = 0, ssz = 0;
  if ((rc = vsize(recvtype, &rsz))) return rc;
  if (!inplace) {
    if (!sendcounts || !sdispls) return MPIGX_ERR_ARG;
    if ((rc = vsize(sendtype, &ssz))) return rc;
  }
  VSpec s;
  s.ncopy = n;
  for (int q = 0; q < n; ++q) {
    const long long sc = inplace ? recvcounts[q] : sendcounts[q];
    const long long sd = inplace ? rdispls[q] : sdispls[q];
    if (sc < 0 || recvcounts[q] < 0) return MPIGX_ERR_COUNT;
    s.c_slot[q] = q;
    s.c_src[q] = sd * (inplace ? rsz : ssz);
    s.c_len[q] = sc * (inplace ? rsz : ssz);
    s.p_len[q] = (long long)recvcounts[q] * rsz;
    s.p_slot[q] = r;
    s.p_dst[q] = (long long)rdispls[q] * rsz;
  }
  s.send = inplace ? (const char*)recvbuf : (const char*)sendbuf;
  s.recv = (char*)recvbuf;
  return vexchange(c, s);
}

// ---------------------------------------------------------------------------
// User-defined ops (operators.jl:56-88 OpWrapper, MPI_Op_create; SURVEY §8f
// row 4).  Two kinds of callback:
//   host   (mpigx_op_create): MPI_User_function on HOST memory — what MPI.jl's
//          @cfunction(OpWrapper) is; operands are staged device -> pinned host
//   device (mpigx_op_create_device): called with DEVICE pointers and the
//          comm's stream; it enqueues its own kernels (no staging)
// Algorithm: the contributions are gathered with the engine's Allgather /
// Gather kernels, then folded in rank order with inout = x_q (op) inout from
// the highest rank down — x0 o (x1 o (... o x_{n-1})), MPI's canonical order
// for non-commutative ops (identical for any associative op).
// ---------------------------------------------------------------------------
struct UserOp {
  mpigx_user_function* host_fn;
  mpigx_device_function* dev_fn;
  int commute;
};
// libmpigx's own op handle space (handles.hpp): an op MPI.jl created in libmpi
// (MPICH user op 0x98000000 | k) never resolves to one of ours — it is not a
// predefined op either, so it is rejected with MPI_ERR_OP
static Registry<UserOp, HS_OP> g_userops;

static UserOp* user_op(int h) { return g_userops.get(h); }

// Fold the n contributions x_0..x_{n-1} of `len` elements each, stored in
// slots `slot` bytes apart at `all` (device), into slot n-1:
// inout = x_q o inout for q = n-2 .. 0 (the rank order user_reduce uses).
static int user_fold_slots(mpigx_comm* c, UserOp* u, char* all, long long slot, int n, int len, int dt) {
  if (len == 0 || n < 2) return MPIGX_SUCCESS;
  char* inout = all + (long long)(n - 1) * slot;
  if (u->dev_fn) {
    for (int q = n - 2; q >= 0; --q) u->dev_fn(all + q * slot, inout, (long long)len, dt, (void*)c->stream);
    return hipGetLastError() == hipSuccess ? MPIGX_SUCCESS : MPIGX_ERR_OTHER;
  }
  char* h = nullptr;
  if (hipHostMalloc((void**)&h, (size_t)n * slot, 0) != hipSuccess) {
    (void)hipGetLastError();
    return MPIGX_ERR_NO_MEM;
  }
  int rc = MPIGX_SUCCESS;
  if (hipMemcpyAsync(h, all, (size_t)n * slot, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    rc = MPIGX_ERR_INTERN;
  for (int q = n - 2; !rc && q >= 0; --q) u->host_fn(h + q * slot, h + (n - 1) * slot, &len, &dt);
  if (!rc && (hipMemcpyAsync(inout, h + (n - 1) * slot, (size_t)slot, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
              hipStreamSynchronize(c->stream) != hipSuccess))
    rc = MPIGX_ERR_INTERN;
  if (rc) (void)hipGetLastError();
  (void)hipHostFree(h);
  return rc;
}

// Allreduce (kind 0) / Reduce (kind 1) with a user op: reduce-scatter +
// allgather / gather, so each rank receives (n-1)/n of the message, runs n-1
// callbacks on ITS chunk only and sends its chunk back out — O(S) bytes and
// O(S) callback work per rank instead of gathering all n contributions
// (n·S) and folding all of them everywhere.  Chunk k = datatype elements
// [k·ce, (k+1)·ce), ce = ceil(count/n); every element still sees
// inout = x_q o inout for q = n-2 .. 0, so results are bit-identical to the
// all-gather fold (and MPI's canonical order for non-commutative ops).
static int user_reduce_rs(mpigx_comm* c, UserOp* u, const void* mine, void* recv, int count, int datatype,
                          long long esz, int root, int kind) {
  const int n = c->n, r = c->rank;
  const long long ce = (count + (long long)n - 1) / n;
  int cnt[kMaxRanks], dsp[kMaxRanks], rcnt[kMaxRanks], rdsp[kMaxRanks];
  for (int k = 0; k < n; ++k) {
    const long long lo = std::min((long long)k * ce, (long long)count), hi = std::min(lo + ce, (long long)count);
    cnt[k] = (int)((hi - lo) * esz);
    dsp[k] = (int)(lo * esz);
  }
  const long long slot = cnt[r];
  for (int q = 0; q < n; ++q) {
    rcnt[q] = (int)slot;
    rdsp[q] = (int)(q * slot);
  }
  char* all = tmp_get(c, std::max(16ll, (long long)n * slot));
  if (!all) return MPIGX_ERR_NO_MEM;
  // reduce-scatter: chunk r of every rank's contribution -> slot q of `all`
  int rc = mpigx_alltoallv(mine, cnt, dsp, MPIGX_BYTE, all, rcnt, rdsp, MPIGX_BYTE, c);
  if (!rc) rc = user_fold_slots(c, u, all, slot, n, (int)(slot / esz), datatype);
  char* res = all + (long long)(n - 1) * slot;
  if (!rc && kind == 0) {
    if (slot && hipMemcpyAsync((char*)recv + dsp[r], res, (size_t)slot, hipMemcpyDeviceToDevice, c->stream) != hipSuccess) {
      (void)hipGetLastError();
      rc = MPIGX_ERR_INTERN;
    }
    // (stream order: the allgather's flagged launch completes after the copy)
    if (!rc) rc = mpigx_allgatherv(MPIGX_IN_PLACE, 0, MPIGX_BYTE, recv, cnt, dsp, MPIGX_BYTE, c);
  } else if (!rc) {
    rc = mpigx_gatherv(res, (int)slot, MPIGX_BYTE, recv, cnt, dsp, MPIGX_BYTE, root, c);
  }
  tmp_put(c, all, 0);
  return rc;
}

// kind: 0 allreduce, 1 reduce, 2 scan, 3 exscan
static int user_reduce(mpigx_comm* c, UserOp* u, const void* send, void* recv, int count, int datatype, int root, int kind) {
  rt::TypeDesc d;
  if (rt::type_info(datatype, &d) || !d.contig) return MPIGX_ERR_TYPE;
  if (count < 0) return MPIGX_ERR_COUNT;
  if (count == 0) return MPIGX_SUCCESS;
  const int n = c->n, r = c->rank;
  if (kind == 1 && (root < 0 || root >= n)) return MPIGX_ERR_ROOT;
  const long long eb = (long long)count * d.size;
  if (eb > 0x7fffffff) return MPIGX_ERR_COUNT;
  const void* mine = send == MPIGX_IN_PLACE ? recv : send;
  if (!mine || (!recv && (kind != 1 || r == root))) return MPIGX_ERR_BUFFER;
  if (kind <= 1 && n > 1) return user_reduce_rs(c, u, mine, recv, count, datatype, d.size, root, kind);
  // every contribution needed here: all (allreduce), at the root (reduce), ranks <= r (scans)
  char* all = tmp_get(c, (long long)n * eb);
  if (!all) return MPIGX_ERR_NO_MEM;
  int rc;
  if (kind == 1)
    rc = gather_common(mine, (int)eb, MPIGX_BYTE, all, (int)eb, nullptr, nullptr, MPIGX_BYTE, root, c);
  else
    rc = gather_like(mine, (int)eb, MPIGX_BYTE, all, (int)eb, MPIGX_BYTE, c, false);
  int hi = n - 1;  // fold x_lo .. x_hi
  bool skip = false;
  if (kind == 1 && r != root) skip = true;
  if (kind == 2) hi = r;
  if (kind == 3) {
    hi = r - 1;
    if (r == 0) skip = true;  // rank 0's exscan result is untouched
  }
  if (!rc && !skip) {
    int len = count, dt = datatype;
    if (u->dev_fn) {
      if (hipMemcpyAsync(recv, all + hi * eb, eb, hipMemcpyDeviceToDevice, c->stream) != hipSuccess) rc = MPIGX_ERR_INTERN;
      for (int q = hi - 1; !rc && q >= 0; --q) u->dev_fn(all + q * eb, recv, (long long)len, dt, (void*)c->stream);
      c->unflagged = true;
      if (!rc) rc = finish(c);
      if (!rc && hipGetLastError() != hipSuccess) rc = MPIGX_ERR_OTHER;
    } else {
      char* h = nullptr;
      if (hipHostMalloc((void**)&h, (size_t)(hi + 1) * eb, 0) != hipSuccess) {
        (void)hipGetLastError();
        rc = MPIGX_ERR_NO_MEM;
      } else {
        if (hipMemcpyAsync(h, all, (size_t)(hi + 1) * eb, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess) {
          (void)hipGetLastError();
          rc = MPIGX_ERR_INTERN;
        }
        for (int q = hi - 1; !rc && q >= 0; --q) u->host_fn(h + q * eb, h + hi * eb, &len, &dt);
        if (!rc && (hipMemcpyAsync(recv, h + hi * eb, eb, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
                    hipStreamSynchronize(c->stream) != hipSuccess)) {
          (void)hipGetLastError();
          rc = MPIGX_ERR_INTERN;
        }
        (void)hipHostFree(h);
      }
    }
  } else if (!rc) {
    rc = finish(c);
  }
  tmp_put(c, all, 0);
  return rc;
}

// Reductions over a derived type: only contiguous runs of ONE predefined type
// (MPI allows predefined ops on such types; they reduce element-wise).
static int lower_reduce_type(int* datatype, int* count) {
  if (!derived(*datatype)) return MPIGX_SUCCESS;
  rt::TypeDesc d;
  if (rt::type_info(*datatype, &d)) return MPIGX_ERR_TYPE;
  const int bs = rt::dtype_size(d.basic);
  if (!d.contig || d.basic == 0 || bs <= 0 || d.size % bs) return MPIGX_ERR_TYPE;
  const long long n = (long long)*count * (d.size / bs);
  if (n > 0x7fffffff) return MPIGX_ERR_COUNT;
  *datatype = d.basic;
  *count = (int)n;
  return MPIGX_SUCCESS;
}

int mpigx_allreduce(const void* sendbuf, void* recvbuf, int count, int datatype, int op, mpigx_comm_t c) {
  int rc = check_comm(c);
  if (rc) return rc;
  if (UserOp* u = user_op(op)) return user_reduce(c, u, sendbuf, recvbuf, count, datatype, 0, 0);
  if ((rc = lower_reduce_type(&datatype, &count))) return rc;
  const TypeInfo* t;
  int oc;
  if ((rc = validate(datatype, op, &t, &oc))) return rc;
  if (count < 0) return MPIGX_ERR_COUNT;
  if (count == 0) return MPIGX_SUCCESS;
  if (!recvbuf || !sendbuf) return MPIGX_ERR_BUFFER;
  const void* s = sendbuf == MPIGX_IN_PLACE ? recvbuf : sendbuf;
  if (c->n == 1) return copy_n1(c, recvbuf, s, (size_t)count * t->size);
  return reduce_common(c, s, recvbuf, count, t, oc, 0, true);
}

int mpigx_reduce(const void* sendbuf, void* recvbuf, int count, int datatype, int op, int root, mpigx_comm_t c) {
  int rc = check_comm(c);
  if (rc) return rc;
  if (UserOp* u = user_op(op)) return user_reduce(c, u, sendbuf, recvbuf, count, datatype, root, 1);
  if ((rc = lower_reduce_type(&datatype, &count))) return rc;
  const TypeInfo* t;
  int oc;
  if ((rc = validate(datatype, op, &t, &oc))) return rc;
  if (count < 0) return MPIGX_ERR_COUNT;
  if (root < 0 || root >= c->n) return MPIGX_ERR_ROOT;
  if (count == 0) return MPIGX_SUCCESS;
  const bool isroot = c->rank == root;
  if (isroot && !recvbuf) return MPIGX_ERR_BUFFER;
  if (!sendbuf || (sendbuf == MPIGX_IN_PLACE && !isroot)) return MPIGX_ERR_BUFFER;
  const void* s = sendbuf == MPIGX_IN_PLACE ? recvbuf : sendbuf;
  if (c->n == 1) return copy_n1(c, recvbuf, s, (size_t)count * t->size);
  return reduce_common(c, s, isroot ? recvbuf : nullptr, count, t, oc, root, false);
}

static int scan_common(const void* sendbuf, void* recvbuf, int count, int datatype, int op, mpigx_comm_t c,
                       int exclusive) {
  int rc = check_comm(c);
  if (rc) return rc;
  if (UserOp* u = user_op(op)) return user_reduce(c, u, sendbuf, recvbuf, count, datatype, 0, exclusive ? 3 : 2);
  if ((rc = lower_reduce_type(&datatype, &count))) return rc;
  const TypeInfo* t;
  int oc;
  if ((rc = validate(datatype, op, &t, &oc))) return rc;
  if (count < 0) return MPIGX_ERR_COUNT;
  if (count == 0) return MPIGX_SUCCESS;
  if (!recvbuf || !sendbuf) return MPIGX_ERR_BUFFER;
  const void* s = sendbuf == MPIGX_IN_PLACE ? recvbuf : sendbuf;
  const int es = t->size;
  if (c->n == 1) {
    if (exclusive) return finish(c);
    return copy_n1(c, recvbuf, s, (size_t)count * es);
  }
  ScanLauncher L = scan_launcher(t->rep);
  const int vec = es >= 16 ? 1 : 16 / es;
  // pull-push (n <= 8): rank r computes every rank's result for chunk r
  // (kernels.hpp scan_pp_body) — in place too, since each element is read
  // and written by one thread of its owner only; n > 8 keeps the pull
  // schedule, out of place (with IN_PLACE my recvbuf, which I overwrite,
  // would be the operand the higher ranks read)
  // On by default (agreed knob MPIGX_SCAN_PP, c->scan_pp = 1).  Round 3 saw
  // one aperture violation (n = 8 ranks on one GPU, 64 Mi-element headline
  // case) and wrong words on one rank in another run; since round 5 the
  // kernel checks its argument block (checksum + launch freshness) and every
  // load / store extent against the view's exported allocation sizes before
  // touching a peer's buffer, and a failed check aborts every rank's launch
  // (DESIGN §13 "The round-3 aperture violation").
  const bool pp = c->scan_pp && c->n <= 8;
  if ((pp || sendbuf != MPIGX_IN_PLACE) && c->zc_min > 0 && (long long)count * es >= c->zc_min) {
    // zero-copy: no copy-in, no rounds
    bool staged;
    const int rc = zc_run(c, s, recvbuf, &staged, [&](const ZcLaunch& z) {
      ScanArgs a;
      memset(&a, 0, sizeof a);
      a.pv = make_view(c);
      zc_apply(a.pv, z);
      a.zc = 1;
      a.exclusive = exclusive;
      a.esize = es;
      a.count = count;
      int g;
      if (pp) {
        a.pp = 1;
        a.chunk = rup(cdiv(count, c->n), vec);
        g = grid_for(c, a.chunk * es, cap_scan(c, t, oc));
        a.slice = rup(cdiv(a.chunk, g), vec);
        for (int p = 0; p < c->n; ++p) {
          a.zrecv[p] = z.pr[p];
          a.zs_avail[p] = z.as[p];
          a.zr_avail[p] = z.ar[p];
        }
      } else {
        g = grid_for(c, (long long)count * es, cap_scan(c, t, oc));
        a.slice = rup(cdiv(count, g), vec);
      }
      a.send = s;
      a.recv = recvbuf;
      for (int p = 0; p < c->n; ++p) a.src[p] = z.ps[p];
      seal_args(a);
      HIPCK(L(oc, dim3(g), c->stream, a));
      note_launch(c, a.pv, g);
      c->epoch += 2;
      return MPIGX_SUCCESS;
    });
    if (rc || !staged) return rc;
    if (c->zc_require) return MPIGX_ERR_INTERN;
  }
  if (ll_take(c, (long long)count * es)) {
    // small Scan / Exscan: one LL step, the operands are my arena's unpack
    // slots (IN_PLACE-safe: my own contribution is copied there too)
    ScanArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    a.ll = 1;
    a.exclusive = exclusive;
    a.esize = es;
    a.count = count;
    const int g = grid_for(c, (long long)count * es, cap_scan(c, t, oc));
    a.slice = rup(cdiv(count, g), kLLAlign / es);
    a.send = s;
    a.recv = recvbuf;
    a.ll_ustride = rup(c->ll_max, 16);
    for (int p = 0; p < c->n; ++p) a.src[p] = c->stage + p * a.ll_ustride;
    if (int e = ll_fill(c, a.pv, a.ll_push, &a.ll_in, &a.ll_stride, &a.ll_flag)) return e;
    HIPCK(L(oc, dim3(g), c->stream, a));
    note_launch(c, a.pv, g);
    ll_launched(c);
    return finish(c);
  }
  long long round = (long long)(c->stage_bytes / es) / vec * vec;
  for (long long off = 0; off < count; off += round) {
    const long long cnt = count - off < round ? count - off : round;
    ScanArgs a;
    memset(&a, 0, sizeof a);
    a.pv = make_view(c);
    for (int p = 0; p < c->n; ++p) a.src[p] = c->peer_stage[p];
    a.exclusive = exclusive;
    a.esize = es;
    a.count = cnt;
    const int g = grid_for(c, cnt * es, cap_scan(c, t, oc));
    a.slice = rup(cdiv(cnt, g), vec);
    a.send = (const char*)s + off * es;
    a.recv = (char*)recvbuf + off * es;
    HIPCK(L(oc, dim3(g), c->stream, a));
    note_launch(c, a.pv, g);
    c->epoch += 2;
  }
  return finish(c);
}

int mpigx_scan(const void* sendbuf, void* recvbuf, int count, int datatype, int op, mpigx_comm_t c) {
  return scan_common(sendbuf, recvbuf, count, datatype, op, c, 0);
}
int mpigx_exscan(const void* sendbuf, void* recvbuf, int count, int datatype, int op, mpigx_comm_t c) {
  return scan_common(sendbuf, recvbuf, count, datatype, op, c, 1);
}

// ---------------------------------------------------------------------------
// local ops
// ---------------------------------------------------------------------------
int mpigx_reduce_local_multi(const void* const* in, int nin, void* out, long long count, int datatype, int op,
                             int order, void* stream) {
  const TypeInfo* t;
  int oc;
  int rc = validate(datatype, op, &t, &oc);
  if (rc) return rc;
  if (nin < 1 || nin > kMaxRanks) return MPIGX_ERR_ARG;
  if (order != MPIGX_ORDER_MPICH && order != MPIGX_ORDER_LINEAR) return MPIGX_ERR_ARG;
  if (count < 0) return MPIGX_ERR_COUNT;
  if (count == 0) return MPIGX_SUCCESS;
  if (!in || !out) return MPIGX_ERR_BUFFER;
  for (int k = 0; k < nin; ++k)
    if (!in[k]) return MPIGX_ERR_BUFFER;
  FoldArgs a;
  memset(&a, 0, sizeof a);
  a.mode = M_LOCAL;
  a.esize = t->size;
  a.count = count;
  a.recv = out;
  int nmax, sched;
  plan_schedule(nullptr, a, nin, 0, count, t->size, in, &nmax, &sched, order);
  // grid: U 16-byte vectors per thread (fold_shape / local_u, the rule the
  // launcher instantiates with), the whole range in ONE pass.  Measured on MI355X
  // (tools/local_tune.hip, 8 x 256 MiB f32): one pass 6.0-6.1 TB/s vs
  // 4.8-5.6 TB/s for grid-stride loops over 1792-16384 blocks — short-lived
  // waves dispatched in address order keep the 9 streams sequential in DRAM.
  // The kernel strides over the grid only past HIP's 2^32-thread limit.
  // U by size (local_u): fewer vectors per thread for small inputs, so the
  // grid covers the CUs (MPIGX_LOCAL_U = 1 / 2 / 4 forces one, measurement)
  const int vec = t->size >= 16 ? 1 : 16 / t->size;
  const int shape = fold_shape(sched, nmax, a.ntree, a.rem);
  int u = local_u(t->rep, oc, shape, cdiv(count, vec));
  const long long force_u = env_ll("MPIGX_LOCAL_U", 0);
  if (force_u == 1 || force_u == 2 || force_u == 4) u = (int)force_u <= local_u_max(t->rep, oc, shape) ? (int)force_u : u;
  a.lu = u;
  long long g = cdiv(cdiv(count, vec), (long long)kThreads * u);
  long long cap = env_ll("MPIGX_LOCAL_MAX_BLOCKS", 0xffffffffll / kThreads);
  if (cap > 0xffffffffll / kThreads) cap = 0xffffffffll / kThreads;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  FoldLauncher L = fold_launcher(t->rep);
  hipError_t e = L(oc, nmax, sched, dim3((unsigned)g), (hipStream_t)stream, a);
  if (e != hipSuccess) {
    fprintf(stderr, "[mpigx] reduce_local_multi launch: %s\n", hipGetErrorString(e));
    return MPIGX_ERR_INTERN;
  }
  return MPIGX_SUCCESS;
}

int mpigx_reduce_local(const void* inbuf, void* inoutbuf, int count, int datatype, int op) {
  if (count < 0) return MPIGX_ERR_COUNT;
  const void* ptrs[2] = {inoutbuf, inbuf};  // leaf 0 = inout (lower subtree), leaf 1 = in
  int rc = mpigx_reduce_local_multi(ptrs, 2, inoutbuf, count, datatype, op, MPIGX_ORDER_LINEAR, nullptr);
  if (rc) return rc;
  HIPCK(hipStreamSynchronize(nullptr));
  return MPIGX_SUCCESS;
}

static int op_register(UserOp* u, int* op) {
  const int h = g_userops.add(u);
  if (!h) {
    delete u;
    return MPIGX_ERR_NO_MEM;
  }
  *op = h;
  return MPIGX_SUCCESS;
}
int mpigx_op_create(mpigx_user_function* fn, int commute, int* op) {
  if (!fn || !op) return MPIGX_ERR_ARG;
  return op_register(new UserOp{fn, nullptr, commute}, op);
}
int mpigx_op_create_device(mpigx_device_function* fn, int commute, int* op) {
  if (!fn || !op) return MPIGX_ERR_ARG;
  return op_register(new UserOp{nullptr, fn, commute}, op);
}
int mpigx_op_free(int* op) {
  if (!op) return MPIGX_ERR_ARG;
  UserOp* u = g_userops.remove(*op);
  if (!u) return MPIGX_ERR_OP;  // predefined, foreign or already freed
  delete u;
  *op = 0x18000000;  // MPI_OP_NULL
  return MPIGX_SUCCESS;
}
int mpigx_op_commutative(int op, int* commute) {
  if (!commute) return MPIGX_ERR_ARG;
  if (UserOp* u = user_op(op)) {
    *commute = u->commute;
    return MPIGX_SUCCESS;
  }
  if (op_code(op) == O_NONE) return MPIGX_ERR_OP;
  *commute = 1;
  return MPIGX_SUCCESS;
}

int mpigx_malloc(void** ptr, size_t bytes) {
  if (!ptr) return MPIGX_ERR_ARG;
  if (hipMalloc(ptr, bytes ? bytes : 1) != hipSuccess) return MPIGX_ERR_NO_MEM;
  return MPIGX_SUCCESS;
}
int mpigx_free(void* ptr) {
  if (ptr && hipFree(ptr) != hipSuccess) return MPIGX_ERR_INTERN;
  return MPIGX_SUCCESS;
}
int mpigx_memcpy(void* dst, const void* src, size_t bytes) {
  if (!bytes) return MPIGX_SUCCESS;
  HIPCK(hipMemcpy(dst, src, bytes, hipMemcpyDefault));
  return MPIGX_SUCCESS;
}

}  // extern "C"
