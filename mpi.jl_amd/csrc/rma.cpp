// rma.cpp — one-sided communication on device windows:
// the MPI_Win_* / Get / Put / Accumulate / Get_accumulate / Fetch_and_op
// family that src/onesided.jl ccalls (:24-219).
//
// Data path (the collectives' rule: a GPU only ever WRITES its own HBM;
// every cross-GPU byte moves by a reader's pull over xGMI):
//   Get            origin pulls from the target's IPC-mapped window (xfer
//                  kernel on the RMA stream), completes at flush / unlock /
//                  fence.
//   Put, Acc, GAcc origin publishes an envelope {kind, op, type, target
//                  offset, count, IPC handle of the origin buffer} in slot
//                  seq % 16 of the window's [origin][target] shm box; the
//                  TARGET's progress pulls the origin buffer and applies it
//                  to its own window in order (xfer kernel for Put,
//                  acc_kernel<OP,T> with the op fused into the pull for
//                  Accumulate), writes old values of Get_accumulate /
//                  Fetch_and_op into its scratch slot for that origin, drains
//                  the stream and stores done = seq + 1.  The origin then
//                  pulls the old values from that slot.
// One stream applies every envelope a target receives, so accumulates are
// atomic per element and ordered per origin (MPI-3 §11.7.1 defaults).
// Progress runs inside every mpigx call that waits (collectives' host spin,
// host control plane, p2p waits, and every Win_* call), as with MPICH ch3 on
// non-shared windows.
//
// Synchronisation: lock words in shm (0 free, > 0 shared holders, -1
// exclusive); Win_unlock / Win_flush wait for the target's done stores; a
// fence = flush everything + a host barrier during which progress applies
// the incoming envelopes, so on return every rank's window holds every
// operation of the closed epoch.  Local window accesses are ordered by
// draining the communicator's stream at unlock(self) / fence / sync.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <vector>

#include "launch.hpp"
#include "runtime.hpp"

using namespace mpigx;

namespace {

enum RmaKind { RK_PUT = 1, RK_ACC = 2, RK_GACC = 3 };

AccLauncher acc_launcher(int rep) {
  switch (rep) {
    case R_I8: return launch_acc_i8;
    case R_U8: return launch_acc_u8;
    case R_I16: return launch_acc_i16;
    case R_U16: return launch_acc_u16;
    case R_I32: return launch_acc_i32;
    case R_U32: return launch_acc_u32;
    case R_I64: return launch_acc_i64;
    case R_U64: return launch_acc_u64;
    case R_F32: return launch_acc_f32;
    case R_F64: return launch_acc_f64;
    case R_C64: return launch_acc_c64;
    case R_C128: return launch_acc_c128;
    case R_BF16: return launch_acc_bf16;
    default: return nullptr;
  }
}

long long env_ll(const char* name, long long dflt) {
  const char* v = getenv(name);
  return (v && *v) ? strtoll(v, nullptr, 0) : dflt;
}

}  // namespace

struct mpigx_win {
  mpigx_comm* c = nullptr;
  int slot = -1;
  int flavor = MPIGX_WIN_FLAVOR_CREATE;
  char* base = nullptr;
  long long size = 0;
  int disp_unit = 1;
  char* shared_alloc = nullptr;  // SHARED: this rank's uncached segment
  // every rank's window as seen from this process (self: base)
  char* peer_base[kMaxRanks] = {};
  long long peer_size[kMaxRanks] = {};
  int peer_du[kMaxRanks] = {};
  // Get_accumulate scratch (the communicator's, RmaState): slot_bytes per origin
  char* scratch = nullptr;
  long long slot_bytes = 0;
  char* peer_scratch[kMaxRanks] = {};
  std::vector<char*> pinned;  // imported allocations to unpin at free
  uint64_t sseq[kMaxRanks] = {};  // origin: envelopes posted per target
  uint64_t rseq[kMaxRanks] = {};  // target: envelopes applied per origin
  int lock_held[kMaxRanks] = {};  // 0 none, 1 shared, 2 exclusive, 3 NOCHECK
  bool gets_pending = false;
  bool ready = false;  // every rank reset its rows of the slot (first exchange done)
  int err = MPIGX_SUCCESS;        // first deferred (target-side) error
  struct Attach {
    char* base;
    long long size;
    int idx;
  };
  std::vector<Attach> attached;
};

namespace mpigx {
struct RmaState {
  hipStream_t ws = nullptr;  // origin Gets and target-side applies
  hipEvent_t ev = nullptr;
  unsigned used = 0;  // window slots in use (identical on every rank)
  std::vector<mpigx_win*> wins;
  WinShm* local = nullptr;  // single-rank communicator (no shm block)
  // Get_accumulate / Fetch_and_op old values: one slot per origin, allocated
  // and exchanged once (with the first window) and shared by all windows —
  // an origin has at most one such operation in flight (acc_common waits).
  char* scratch = nullptr;
  long long slot_bytes = 0;
  char* peer_scratch[kMaxRanks] = {};
  std::vector<char*> pinned;
};
}  // namespace mpigx

namespace {

WinShm* wshm(mpigx_win* w) {
  mpigx_comm* c = w->c;
  return c->shm ? &c->shm->win[w->slot] : &c->rma->local[w->slot];
}

bool same_process(mpigx_comm* c, int q) {
  return q == c->rank || (c->shm && c->shm->ranks[q].pid == getpid());
}

int state_of(mpigx_comm* c, RmaState** out) {
  if (!c->rma) {
    RmaState* R = new RmaState();
    if (hipStreamCreateWithFlags(&R->ws, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&R->ev, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      delete R;
      return MPIGX_ERR_INTERN;
    }
    if (!c->shm) R->local = (WinShm*)calloc(kMaxWins, sizeof(WinShm));
    c->rma = R;
  }
  *out = c->rma;
  return MPIGX_SUCCESS;
}

// RMA waits (a target's apply, a lock, a fence) last as long as the peers
// live, like every other wait (p2p.cpp Deadline): they give up only when a
// peer's process is gone or its communicator failed (checked every 0.25 s).
struct Deadline {
  mpigx_comm* c;
  double t0, lim, next;
  unsigned spins = 0;
  bool noted = false;
  explicit Deadline(mpigx_comm* cc) : c(cc), t0(rt::wall()), lim(cc->timeout_ticks / 1e8), next(t0 + 0.25) {}
  bool expired() {
    if ((++spins & 1023) != 0) return false;
    const double t = rt::wall();
    if (t < next) return false;
    next = t + 0.25;
    if (rt::peer_dead(c)) return true;
    if (!noted && t - t0 > lim) {
      noted = true;
      fprintf(stderr, "mpigx: an RMA wait has lasted %.0f s; still waiting for the peer\n", t - t0);
    }
    return false;
  }
};

// ---------------------------------------------------------------------------
// target side: apply the envelopes addressed to me
// ---------------------------------------------------------------------------
// My window memory for [disp, disp+bytes) (disp: byte offset, or the absolute
// address for dynamic windows); null if out of range.
char* local_target(mpigx_win* w, long long disp, long long bytes) {
  if (w->flavor == MPIGX_WIN_FLAVOR_DYNAMIC) {
    const uintptr_t a = (uintptr_t)disp;
    for (auto& r : w->attached)
      if (a >= (uintptr_t)r.base && a + bytes <= (uintptr_t)r.base + r.size) return (char*)a;
    return nullptr;
  }
  if (disp < 0 || disp + bytes > w->size) return nullptr;
  return w->base + disp;
}

int apply_one(mpigx_win* w, int o, RmaEnvelope* e, hipStream_t ws) {
  mpigx_comm* c = w->c;
  int rep = e->rep, esize = 1;
  if (e->kind != RK_PUT) {
    static const int kSize[R_COUNT] = {1, 1, 2, 2, 4, 4, 8, 8, 4, 8, 8, 16, 2};
    if (rep < 0 || rep >= R_COUNT) return MPIGX_ERR_TYPE;
    esize = kSize[rep];
  }
  const long long bytes = e->count * esize;
  char* dst = local_target(w, e->tdisp, bytes);
  if (!dst) return MPIGX_ERR_RMA_RANGE;
  const char* src;
  if (same_process(c, o)) {
    src = (const char*)(uintptr_t)e->raw;
  } else if (e->op == O_NOOP && e->kind != RK_PUT) {
    src = nullptr;  // fetch only: the origin buffer is not read
  } else {
    char* b = rt::import_buf(c, o, e->buf_id, e->h);
    if (!b) return MPIGX_ERR_INTERN;
    src = b + e->off;
  }
  if (e->kind == RK_PUT) {
    XferArgs a;
    memset(&a, 0, sizeof a);
    a.nseg = 1;
    a.coherent = rt::pull_fences();
    long long g = (bytes + (64 << 10) - 1) / (64 << 10);
    a.blk0[1] = (int)std::max(1ll, std::min(g, 256ll));
    a.dst[0] = dst;
    a.src[0] = src;
    a.bytes[0] = bytes;
    return launch_xfer(ws, a) == hipSuccess ? MPIGX_SUCCESS : MPIGX_ERR_INTERN;
  }
  AccArgs a;
  a.src = src;
  a.dst = dst;
  a.res = nullptr;
  a.count = e->count;
  a.coherent = rt::pull_fences();
  if (e->kind == RK_GACC) {
    if (e->res_off < 0 || e->res_off + bytes > w->slot_bytes * c->n) return MPIGX_ERR_INTERN;
    a.res = w->scratch + e->res_off;
  }
  AccLauncher L = acc_launcher(rep);
  if (!L) return MPIGX_ERR_TYPE;
  long long g = (e->count + 4 * 256 - 1) / (4 * 256);
  g = std::max(1ll, std::min(g, 1024ll));
  return L(e->op, dim3((unsigned)g), ws, a) == hipSuccess ? MPIGX_SUCCESS : MPIGX_ERR_INTERN;
}

void apply_incoming(mpigx_win* w) {
  mpigx_comm* c = w->c;
  if (!w->ready) return;  // a peer may not have cleared the slot's previous envelopes yet
  WinShm* S = wshm(w);
  struct Done {
    RmaEnvelope* e;
    uint64_t seq;
    int err;
  };
  Done batch[kMaxRanks * kRmaSlots];
  int nb = 0;
  for (int o = 0; o < c->n; ++o) {
    for (int k = 0; k < kRmaSlots; ++k) {
      RmaEnvelope* e = &S->box[o][c->rank].slot[w->rseq[o] % kRmaSlots];
      if (e->posted.load(std::memory_order_acquire) != w->rseq[o] + 1) break;
      batch[nb++] = {e, w->rseq[o], apply_one(w, o, e, c->rma->ws)};
      w->rseq[o] += 1;
    }
  }
  if (!nb) return;
  int serr = MPIGX_SUCCESS;
  if (hipStreamSynchronize(c->rma->ws) != hipSuccess) {
    (void)hipGetLastError();
    serr = MPIGX_ERR_INTERN;
  }
  for (int i = 0; i < nb; ++i) {
    batch[i].e->err = batch[i].err ? batch[i].err : serr;
    batch[i].e->done.store(batch[i].seq + 1, std::memory_order_release);
  }
}

// ---------------------------------------------------------------------------
// origin side
// ---------------------------------------------------------------------------
int spin_progress(mpigx_win* w, Deadline& d) {
  rt::progress_all(w->c);
  rt::yield_big_lock();  // other threads' calls go on while this one waits
  if (d.expired()) {
    rt::comm_mark_broken(w->c);
    return MPIGX_ERR_OTHER;
  }
  return MPIGX_SUCCESS;
}

int post(mpigx_win* w, int t, int kind, int op, int rep, long long tdisp, long long count, const void* origin,
         long long res_off, uint64_t* seq_out) {
  mpigx_comm* c = w->c;
  RmaEnvelope tmp;
  memset((void*)&tmp, 0, sizeof tmp);
  tmp.raw = (unsigned long long)(uintptr_t)origin;
  const bool needs_src = !(kind != RK_PUT && op == O_NOOP);
  if (needs_src && !same_process(c, t) &&
      !rt::export_buf(c, origin, &tmp.buf_id, &tmp.off, &tmp.h))
    return MPIGX_ERR_BUFFER;
  // Claim the sequence number before anything can yield the big lock
  // (spin_progress): under THREAD_MULTIPLE another thread's Put to the same
  // target may post while this one waits for its slot, and reading sseq
  // before the wait and advancing it after let two threads fill one
  // envelope.  Claimed numbers are posted in any order; the
  // target applies them in sequence order (rma_progress polls slot rseq).
  const uint64_t seq = w->sseq[t]++;
  RmaEnvelope* e = &wshm(w)->box[c->rank][t].slot[seq % kRmaSlots];
  Deadline d(c);
  // the slot is mine once ITS previous envelope (seq - 16) was posted and
  // applied — not just any earlier one: with claims outstanding, seq + 16
  // waits on the same slot and must not take it before seq has used it
  const uint64_t prev_posted = seq >= (uint64_t)kRmaSlots ? seq + 1 - kRmaSlots : 0;
  for (;;) {
    const uint64_t pp = e->posted.load(std::memory_order_acquire);
    if (pp == prev_posted && e->done.load(std::memory_order_acquire) == pp) break;
    int rc = spin_progress(w, d);
    if (rc) return rc;
  }
  if (seq >= (uint64_t)kRmaSlots && e->err && !w->err) w->err = e->err;
  e->kind = kind;
  e->op = op;
  e->rep = rep;
  e->err = 0;
  e->tdisp = tdisp;
  e->count = count;
  e->res_off = res_off;
  e->buf_id = tmp.buf_id;
  e->off = tmp.off;
  e->raw = tmp.raw;
  e->h = tmp.h;
  e->posted.store(seq + 1, std::memory_order_release);
  if (seq_out) *seq_out = seq;
  return MPIGX_SUCCESS;
}

// Wait until envelope `seq` to target t was applied; its error class.
int wait_done(mpigx_win* w, int t, uint64_t seq) {
  RmaEnvelope* e = &wshm(w)->box[w->c->rank][t].slot[seq % kRmaSlots];
  Deadline d(w->c);
  while (e->done.load(std::memory_order_acquire) < seq + 1) {
    int rc = spin_progress(w, d);
    if (rc) return rc;
  }
  return e->err;
}

int flush_target(mpigx_win* w, int t) {
  const uint64_t n = w->sseq[t];
  if (n == 0) return MPIGX_SUCCESS;
  int rc = wait_done(w, t, n - 1);
  if (rc) return rc;
  // in-order application: every earlier envelope is applied too; collect
  // the errors still visible in the ring
  RmaEnvelope* slots = wshm(w)->box[w->c->rank][t].slot;
  const uint64_t lo = n > (uint64_t)kRmaSlots ? n - kRmaSlots : 0;
  for (uint64_t s = lo; s < n; ++s) {
    const int e = slots[s % kRmaSlots].err;
    if (e && !w->err) w->err = e;
  }
  return MPIGX_SUCCESS;
}

int sync_gets(mpigx_win* w) {
  if (!w->gets_pending) return MPIGX_SUCCESS;
  w->gets_pending = false;
  if (hipStreamSynchronize(w->c->rma->ws) != hipSuccess) {
    (void)hipGetLastError();
    return MPIGX_ERR_INTERN;
  }
  return MPIGX_SUCCESS;
}

int take_err(mpigx_win* w) {
  const int e = w->err;
  w->err = MPIGX_SUCCESS;
  return e;
}

int sync_stream(mpigx_comm* c) {
  if (hipStreamSynchronize(c->stream) != hipSuccess) {
    (void)hipGetLastError();
    return MPIGX_ERR_INTERN;
  }
  return MPIGX_SUCCESS;
}

// The target's memory for [disp, disp+bytes) as mapped in this process (Get).
const char* remote_target(mpigx_win* w, int t, long long disp, long long bytes) {
  mpigx_comm* c = w->c;
  if (w->flavor != MPIGX_WIN_FLAVOR_DYNAMIC) {
    const long long off = disp * w->peer_du[t];
    if (disp < 0 || off + bytes > w->peer_size[t] || !w->peer_base[t]) return nullptr;
    return w->peer_base[t] + off;
  }
  const unsigned long long a = (unsigned long long)disp;
  if (t == c->rank) return local_target(w, disp, bytes);
  WinShm* S = wshm(w);
  for (int k = 0; k < kMaxAttach; ++k) {
    DynRegion& r = S->dyn[t][k];
    const uint64_t g = r.gen.load(std::memory_order_acquire);
    if (g == 0 || (g & 1)) continue;
    const unsigned long long ra = r.addr, rs = r.size, id = r.buf_id;
    const long long off = r.off;
    const hipIpcMemHandle_t h = r.h;
    if (r.gen.load(std::memory_order_acquire) != g) continue;  // rewritten meanwhile
    if (a < ra || a + bytes > ra + rs) continue;
    if (same_process(c, t)) return (const char*)(uintptr_t)a;
    char* b = rt::import_buf(c, t, id, h);
    if (!b) return nullptr;
    return b + off + (a - ra);
  }
  return nullptr;
}

// Order a transfer on the RMA stream after the caller's prior work on the
// communicator's stream (the origin buffer's producers / consumers).
int order_after_stream(mpigx_comm* c) {
  if (hipEventRecord(c->rma->ev, c->stream) != hipSuccess ||
      hipStreamWaitEvent(c->rma->ws, c->rma->ev, 0) != hipSuccess) {
    (void)hipGetLastError();
    return MPIGX_ERR_INTERN;
  }
  return MPIGX_SUCCESS;
}

int pull(mpigx_win* w, void* dst, const char* src, long long bytes) {
  mpigx_comm* c = w->c;
  int rc = order_after_stream(c);
  if (rc) return rc;
  XferArgs a;
  memset(&a, 0, sizeof a);
  a.nseg = 1;
  a.coherent = rt::pull_fences();
  long long g = (bytes + (64 << 10) - 1) / (64 << 10);
  a.blk0[1] = (int)std::max(1ll, std::min(g, 256ll));
  a.dst[0] = (char*)dst;
  a.src[0] = src;
  a.bytes[0] = bytes;
  if (launch_xfer(c->rma->ws, a) != hipSuccess) {
    (void)hipGetLastError();
    return MPIGX_ERR_INTERN;
  }
  w->gets_pending = true;
  return MPIGX_SUCCESS;
}

int check_win(mpigx_win* w) {
  if (!w || !w->c) return MPIGX_ERR_WIN;
  return rt::comm_check(w->c);
}

int check_target(mpigx_win* w, int t) {
  if (t == MPIGX_PROC_NULL) return -1;  // no-op
  if (t < 0 || t >= w->c->n) return MPIGX_ERR_RANK;
  return MPIGX_SUCCESS;
}

// Common argument checks of the data-moving calls: predefined types only,
// origin and target describing the same bytes.
int check_xfer(int ocount, int otype, int tcount, int ttype, int* esize) {
  if (ocount < 0 || tcount < 0) return MPIGX_ERR_COUNT;
  const int os = rt::dtype_size(otype), ts = rt::dtype_size(ttype);
  if (os < 0 || ts < 0) return MPIGX_ERR_TYPE;
  if ((long long)os * ocount != (long long)ts * tcount) return MPIGX_ERR_TYPE;
  *esize = os;
  return MPIGX_SUCCESS;
}

struct WinBlob {
  int ok;
  int du;
  long long size;
  unsigned long long id, raw;
  long long off;
  hipIpcMemHandle_t h;
  unsigned long long sid, sraw;
  long long soff;
  hipIpcMemHandle_t sh;
};
static_assert(sizeof(WinBlob) <= 256, "control-plane blob");

int free_local(mpigx_win* w) {
  mpigx_comm* c = w->c;
  for (char* p : w->pinned) rt::unpin(c, p);
  if (w->shared_alloc) (void)hipFree(w->shared_alloc);
  if (c->rma) {
    c->rma->used &= ~(1u << w->slot);
    auto& v = c->rma->wins;
    v.erase(std::remove(v.begin(), v.end(), w), v.end());
  }
  delete w;
  return MPIGX_SUCCESS;
}

// Collective window setup shared by create / allocate_shared / create_dynamic.
int win_setup(mpigx_comm* c, int flavor, char* base, long long size, int disp_unit, mpigx_win** out) {
  int rc = rt::comm_check(c);
  if (rc) return rc;
  if (size < 0) return MPIGX_ERR_SIZE;
  if (disp_unit <= 0) return MPIGX_ERR_DISP;
  RmaState* R;
  rc = state_of(c, &R);
  if (rc) return rc;
  int slot = -1;
  for (int s = 0; s < kMaxWins; ++s)
    if (!(R->used & (1u << s))) {
      slot = s;
      break;
    }
  if (slot < 0) return MPIGX_ERR_NO_MEM;  // identical on every rank: windows are collective
  mpigx_win* w = new mpigx_win();
  w->c = c;
  w->slot = slot;
  w->flavor = flavor;
  w->base = base;
  w->size = size;
  w->disp_unit = disp_unit;
  R->used |= 1u << slot;
  R->wins.push_back(w);
  // reset my rows of the slot (nobody else touches them until the exchange)
  WinShm* S = wshm(w);
  S->lock[c->rank].store(0, std::memory_order_relaxed);
  for (int t = 0; t < kMaxRanks; ++t)
    for (int k = 0; k < kRmaSlots; ++k) {
      S->box[c->rank][t].slot[k].posted.store(0, std::memory_order_relaxed);
      S->box[c->rank][t].slot[k].done.store(0, std::memory_order_relaxed);
      S->box[c->rank][t].slot[k].err = 0;
    }
  for (int k = 0; k < kMaxAttach; ++k) S->dyn[c->rank][k].gen.store(0, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_seq_cst);

  const int n = c->n;
  const bool first = R->scratch == nullptr;  // identical on every rank (windows are collective)
  WinBlob mine;
  memset(&mine, 0, sizeof mine);
  mine.ok = 1;
  mine.du = disp_unit;
  mine.size = flavor == MPIGX_WIN_FLAVOR_DYNAMIC ? 0 : size;
  mine.raw = (unsigned long long)(uintptr_t)base;
  if (first) {
    const long long sb = env_ll("MPIGX_RMA_SCRATCH", 4ll << 20);
    R->slot_bytes = std::max(256ll, (sb / n) & ~255ll);
    if (hipMalloc(&R->scratch, R->slot_bytes * n) != hipSuccess) {
      (void)hipGetLastError();
      R->scratch = nullptr;
      mine.ok = 0;
    }
    mine.sraw = (unsigned long long)(uintptr_t)R->scratch;
    if (n > 1 && mine.ok && !rt::export_buf(c, R->scratch, &mine.sid, &mine.soff, &mine.sh)) mine.ok = 0;
  }
  if (n > 1 && mine.ok && mine.size > 0 && !rt::export_buf(c, base, &mine.id, &mine.off, &mine.h)) mine.ok = 0;
  WinBlob all[kMaxRanks];
  rc = rt::host_allgather(c, &mine, sizeof mine, all);
  if (rc) {
    free_local(w);
    return rc;
  }
  w->ready = true;  // every rank's reset happened before its contribution
  int ok = 1;
  for (int q = 0; q < n; ++q) ok &= all[q].ok;
  for (int q = 0; q < n && ok; ++q) {
    w->peer_du[q] = all[q].du;
    w->peer_size[q] = all[q].size;
    if (same_process(c, q)) {
      w->peer_base[q] = (char*)(uintptr_t)all[q].raw;
      if (first) R->peer_scratch[q] = (char*)(uintptr_t)all[q].sraw;
      continue;
    }
    if (all[q].size > 0) {
      char* b = rt::import_pinned(c, q, all[q].id, all[q].h);
      if (!b) {
        ok = 0;
        break;
      }
      w->pinned.push_back(b);
      w->peer_base[q] = b + all[q].off;
    }
    if (first) {
      char* s = rt::import_pinned(c, q, all[q].sid, all[q].sh);
      if (!s) {
        ok = 0;
        break;
      }
      R->pinned.push_back(s);
      R->peer_scratch[q] = s + all[q].soff;
    }
  }
  w->scratch = R->scratch;
  w->slot_bytes = R->slot_bytes;
  for (int q = 0; q < n; ++q) w->peer_scratch[q] = R->peer_scratch[q];
  int oks[kMaxRanks];
  rc = rt::host_allgather(c, &ok, sizeof ok, oks);
  if (!rc)
    for (int q = 0; q < n; ++q)
      if (!oks[q]) rc = MPIGX_ERR_INTERN;
  if (rc) {
    free_local(w);
    return rc;
  }
  *out = w;
  return MPIGX_SUCCESS;
}

int lock_word_acquire(mpigx_win* w, int type, int t) {
  std::atomic<int>& L = wshm(w)->lock[t];
  Deadline d(w->c);
  for (;;) {
    int v = L.load(std::memory_order_acquire);
    if (type == MPIGX_LOCK_EXCLUSIVE) {
      if (v == 0 && L.compare_exchange_weak(v, -1, std::memory_order_acq_rel)) return MPIGX_SUCCESS;
    } else if (v >= 0 && L.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel)) {
      return MPIGX_SUCCESS;
    }
    int rc = spin_progress(w, d);
    if (rc) return rc;
  }
}

}  // namespace

namespace mpigx {
namespace rt {
void rma_progress(mpigx_comm* c) {
  if (!c->rma) return;
  for (size_t i = 0; i < c->rma->wins.size(); ++i) apply_incoming(c->rma->wins[i]);
}
void rma_sync(mpigx_comm* c) {
  if (c->rma) (void)hipStreamSynchronize(c->rma->ws);
}
void rma_destroy(mpigx_comm* c) {
  RmaState* R = c->rma;
  if (!R) return;
  (void)hipStreamSynchronize(R->ws);
  while (!R->wins.empty()) free_local(R->wins.back());
  for (char* p : R->pinned) rt::unpin(c, p);
  if (R->scratch) (void)hipFree(R->scratch);
  (void)hipEventDestroy(R->ev);
  (void)hipStreamDestroy(R->ws);
  free(R->local);
  delete R;
  c->rma = nullptr;
}
}  // namespace rt
}  // namespace mpigx

// ===========================================================================
// C ABI
// ===========================================================================
extern "C" {

int mpigx_win_create(void* base, long long size, int disp_unit, mpigx_comm_t c, mpigx_win_t* win) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!win) return MPIGX_ERR_ARG;
  if (size > 0 && !base) return MPIGX_ERR_BASE;
  return win_setup(c, MPIGX_WIN_FLAVOR_CREATE, (char*)base, size, disp_unit, win);
}

int mpigx_win_create_dynamic(mpigx_comm_t c, mpigx_win_t* win) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!win) return MPIGX_ERR_ARG;
  return win_setup(c, MPIGX_WIN_FLAVOR_DYNAMIC, nullptr, 0, 1, win);
}

int mpigx_win_allocate_shared(long long size, int disp_unit, mpigx_comm_t c, void* baseptr, mpigx_win_t* win) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!win || !baseptr) return MPIGX_ERR_ARG;
  int rc = rt::comm_check(c);
  if (rc) return rc;
  if (size < 0) return MPIGX_ERR_SIZE;
  // uncached HBM: peers load/store it directly (shared-memory window), so
  // no GPU may hold it in a non-coherent cache
  char* p = nullptr;
  int ok = 1;
  if (size > 0) {
    if (hipExtMallocWithFlags((void**)&p, (size_t)size, hipDeviceMallocUncached) != hipSuccess ||
        hipMemset(p, 0, (size_t)size) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
      (void)hipGetLastError();
      ok = 0;
    }
  }
  int oks[kMaxRanks];
  rc = rt::host_allgather(c, &ok, sizeof ok, oks);
  for (int q = 0; !rc && q < c->n; ++q)
    if (!oks[q]) rc = MPIGX_ERR_NO_MEM;
  if (!rc) rc = win_setup(c, MPIGX_WIN_FLAVOR_SHARED, p, size, disp_unit, win);
  if (rc) {
    if (p) (void)hipFree(p);
    return rc;
  }
  (*win)->shared_alloc = p;
  *(void**)baseptr = p;
  return MPIGX_SUCCESS;
}

int mpigx_win_shared_query(mpigx_win_t w, int rank, long long* size, int* disp_unit, void* baseptr) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  int rc = check_win(w);
  if (rc) return rc;
  if (w->flavor != MPIGX_WIN_FLAVOR_SHARED) return MPIGX_ERR_RMA_FLAVOR;
  if (rank == MPIGX_PROC_NULL) {
    rank = -1;
    for (int q = 0; q < w->c->n; ++q)
      if (w->peer_size[q] > 0) {
        rank = q;
        break;
      }
    if (rank < 0) {
      if (size) *size = 0;
      if (disp_unit) *disp_unit = 0;
      if (baseptr) *(void**)baseptr = nullptr;
      return MPIGX_SUCCESS;
    }
  }
  if (rank < 0 || rank >= w->c->n) return MPIGX_ERR_RANK;
  if (size) *size = w->peer_size[rank];
  if (disp_unit) *disp_unit = w->peer_du[rank];
  if (baseptr) *(void**)baseptr = w->peer_base[rank];
  return MPIGX_SUCCESS;
}

int mpigx_win_get_flavor(mpigx_win_t w, int* flavor) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!w) return MPIGX_ERR_WIN;
  if (flavor) *flavor = w->flavor;
  return MPIGX_SUCCESS;
}

int mpigx_win_free(mpigx_win_t* pw) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!pw) return MPIGX_ERR_ARG;
  mpigx_win* w = *pw;
  int rc = check_win(w);
  if (rc) return rc;
  mpigx_comm* c = w->c;
  for (int t = 0; t < c->n; ++t) {
    const int r = flush_target(w, t);
    if (r && !rc) rc = r;
  }
  const int g = sync_gets(w);
  if (g && !rc) rc = g;
  // nobody may still target or read this window: barrier (with progress)
  int dummy = 0, all[kMaxRanks];
  const int b = rt::host_allgather(c, &dummy, sizeof dummy, all);
  if (b && !rc) rc = b;
  rt::rma_progress(c);
  (void)hipStreamSynchronize(c->rma->ws);
  if (!rc) rc = take_err(w);
  free_local(w);
  *pw = nullptr;
  return rc;
}

int mpigx_win_attach(mpigx_win_t w, void* base, long long size) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  int rc = check_win(w);
  if (rc) return rc;
  if (w->flavor != MPIGX_WIN_FLAVOR_DYNAMIC) return MPIGX_ERR_RMA_FLAVOR;
  if (size < 0) return MPIGX_ERR_SIZE;
  if (size == 0) return MPIGX_SUCCESS;
  if (!base) return MPIGX_ERR_BASE;
  WinShm* S = wshm(w);
  int idx = -1;
  for (int k = 0; k < kMaxAttach; ++k)
    if (S->dyn[w->c->rank][k].gen.load(std::memory_order_relaxed) % 2 == 0) {
      bool used = false;
      for (auto& a : w->attached) used |= a.idx == k;
      if (!used) {
        idx = k;
        break;
      }
    }
  if (idx < 0) return MPIGX_ERR_RMA_ATTACH;
  DynRegion& r = S->dyn[w->c->rank][idx];
  unsigned long long id = 0;
  long long off = 0;
  hipIpcMemHandle_t h;
  memset(&h, 0, sizeof h);
  if (w->c->n > 1 && !rt::export_buf(w->c, base, &id, &off, &h)) return MPIGX_ERR_BUFFER;
  const uint64_t g = r.gen.load(std::memory_order_relaxed);
  r.gen.store(g + 1, std::memory_order_release);  // odd: being written
  r.addr = (unsigned long long)(uintptr_t)base;
  r.size = (unsigned long long)size;
  r.buf_id = id;
  r.off = off;
  r.h = h;
  r.gen.store(g + 2, std::memory_order_release);
  w->attached.push_back({(char*)base, size, idx});
  return MPIGX_SUCCESS;
}

int mpigx_win_detach(mpigx_win_t w, const void* base) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  int rc = check_win(w);
  if (rc) return rc;
  if (w->flavor != MPIGX_WIN_FLAVOR_DYNAMIC) return MPIGX_ERR_RMA_FLAVOR;
  for (size_t i = 0; i < w->attached.size(); ++i)
    if (w->attached[i].base == base) {
      DynRegion& r = wshm(w)->dyn[w->c->rank][w->attached[i].idx];
      const uint64_t g = r.gen.load(std::memory_order_relaxed);
      r.gen.store(g + 1, std::memory_order_release);  // odd = not visible
      r.size = 0;
      r.gen.store(g + 2, std::memory_order_release);
      w->attached.erase(w->attached.begin() + i);
      return MPIGX_SUCCESS;
    }
  return MPIGX_ERR_RMA_ATTACH;
}

int mpigx_win_fence(int assert_, mpigx_win_t w) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  (void)assert_;
  int rc = check_win(w);
  if (rc) return rc;
  mpigx_comm* c = w->c;
  for (int t = 0; t < c->n && !rc; ++t) rc = flush_target(w, t);
  if (!rc) rc = sync_gets(w);
  if (!rc) rc = sync_stream(c);  // my local window accesses of the epoch
  int dummy = 0, all[kMaxRanks];
  // everyone's envelopes to me are applied before they arrive here
  const int b = rt::host_allgather(c, &dummy, sizeof dummy, all);
  if (!rc) rc = b;
  if (!rc) rc = take_err(w);
  return rc;
}

int mpigx_win_lock(int lock_type, int rank, int assert_, mpigx_win_t w) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  int rc = check_win(w);
  if (rc) return rc;
  // MPICH 3.3.2 reports a bad lock type as MPI_ERR_OTHER ("**locktype")
  if (lock_type != MPIGX_LOCK_EXCLUSIVE && lock_type != MPIGX_LOCK_SHARED) return MPIGX_ERR_OTHER;
  rc = check_target(w, rank);
  if (rc < 0) return MPIGX_SUCCESS;
  if (rc) return rc;
  if (w->lock_held[rank]) return MPIGX_ERR_RMA_SYNC;
  if (assert_ & MPIGX_MODE_NOCHECK) {
    w->lock_held[rank] = 3;
    return MPIGX_SUCCESS;
  }
  rc = lock_word_acquire(w, lock_type, rank);
  if (rc) return rc;
  w->lock_held[rank] = lock_type == MPIGX_LOCK_EXCLUSIVE ? 2 : 1;
  return MPIGX_SUCCESS;
}

int mpigx_win_unlock(int rank, mpigx_win_t w) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  int rc = check_win(w);
  if (rc) return rc;
  rc = check_target(w, rank);
  if (rc < 0) return MPIGX_SUCCESS;
  if (rc) return rc;
  const int held = w->lock_held[rank];
  if (!held) return MPIGX_ERR_RMA_SYNC;
  rc = flush_target(w, rank);
  const int g = sync_gets(w);
  if (!rc) rc = g;
  if (rank == w->c->rank) {
    const int s = sync_stream(w->c);  // local accesses of the epoch are complete
    if (!rc) rc = s;
  }
  std::atomic<int>& L = wshm(w)->lock[rank];
  if (held == 2) L.store(0, std::memory_order_release);
  else if (held == 1) L.fetch_sub(1, std::memory_order_acq_rel);
  w->lock_held[rank] = 0;
  if (!rc) rc = take_err(w);
  return rc;
}

int mpigx_win_flush(int rank, mpigx_win_t w) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  int rc = check_win(w);
  if (rc) return rc;
  rc = check_target(w, rank);
  if (rc < 0) return MPIGX_SUCCESS;
  if (rc) return rc;
  rc = flush_target(w, rank);
  const int g = sync_gets(w);
  if (!rc) rc = g;
  if (!rc) rc = take_err(w);
  return rc;
}

int mpigx_win_sync(mpigx_win_t w) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  int rc = check_win(w);
  if (rc) return rc;
  rt::progress_all(w->c);
  rc = sync_stream(w->c);
  const int g = sync_gets(w);
  return rc ? rc : g;
}

int mpigx_get(void* origin_addr, int origin_count, int origin_datatype, int target_rank, long long target_disp,
              int target_count, int target_datatype, mpigx_win_t w) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  int rc = check_win(w);
  if (rc) return rc;
  int es;
  rc = check_xfer(origin_count, origin_datatype, target_count, target_datatype, &es);
  if (rc) return rc;
  rc = check_target(w, target_rank);
  if (rc < 0) return MPIGX_SUCCESS;
  if (rc) return rc;
  const long long bytes = (long long)origin_count * es;
  if (bytes == 0) return MPIGX_SUCCESS;
  if (!origin_addr) return MPIGX_ERR_BUFFER;
  const char* src = remote_target(w, target_rank, target_disp, bytes);
  if (!src) return MPIGX_ERR_RMA_RANGE;
  return pull(w, origin_addr, src, bytes);
}

int mpigx_put(const void* origin_addr, int origin_count, int origin_datatype, int target_rank,
              long long target_disp, int target_count, int target_datatype, mpigx_win_t w) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  int rc = check_win(w);
  if (rc) return rc;
  int es;
  rc = check_xfer(origin_count, origin_datatype, target_count, target_datatype, &es);
  if (rc) return rc;
  rc = check_target(w, target_rank);
  if (rc < 0) return MPIGX_SUCCESS;
  if (rc) return rc;
  const long long bytes = (long long)origin_count * es;
  if (bytes == 0) return MPIGX_SUCCESS;
  if (!origin_addr) return MPIGX_ERR_BUFFER;
  const long long tdisp = w->flavor == MPIGX_WIN_FLAVOR_DYNAMIC ? target_disp : target_disp * w->peer_du[target_rank];
  if (w->flavor != MPIGX_WIN_FLAVOR_DYNAMIC && (target_disp < 0 || tdisp + bytes > w->peer_size[target_rank]))
    return MPIGX_ERR_RMA_RANGE;
  rc = sync_stream(w->c);  // the origin buffer is final when the call is made
  if (rc) return rc;
  return post(w, target_rank, RK_PUT, 0, 0, tdisp, bytes, origin_addr, 0, nullptr);
}

static int acc_common(const void* origin, int ocount, int otype, void* result, int rcount, int rtype, int t,
                      long long tdisp_el, int tcount, int ttype, int op, mpigx_win* w, bool fetch) {
  int rc = check_win(w);
  if (rc) return rc;
  if (ocount < 0 || tcount < 0 || rcount < 0) return MPIGX_ERR_COUNT;
  int rep, es, oc;
  rc = rt::acc_check(ttype, op, &rep, &es, &oc);
  if (rc) return rc;
  if (oc != O_NOOP && (otype != ttype || ocount != tcount)) return MPIGX_ERR_TYPE;
  if (fetch && (rtype != ttype || rcount != tcount)) return MPIGX_ERR_TYPE;
  rc = check_target(w, t);
  if (rc < 0) return MPIGX_SUCCESS;
  if (rc) return rc;
  const long long count = tcount;
  if (count == 0) return MPIGX_SUCCESS;
  if ((oc != O_NOOP && !origin) || (fetch && !result)) return MPIGX_ERR_BUFFER;
  const bool dyn = w->flavor == MPIGX_WIN_FLAVOR_DYNAMIC;
  const long long tdisp = dyn ? tdisp_el : tdisp_el * w->peer_du[t];
  if (!dyn && (tdisp_el < 0 || tdisp + count * es > w->peer_size[t])) return MPIGX_ERR_RMA_RANGE;
  rc = sync_stream(w->c);
  if (rc) return rc;
  if (!fetch) return post(w, t, RK_ACC, oc, rep, tdisp, count, origin, 0, nullptr);
  // Get_accumulate: chunks of one scratch slot; each chunk is applied by the
  // target (old values -> its scratch slot for me), then pulled back.
  const long long per = std::max(1ll, w->slot_bytes / es);
  const long long my_off = w->slot_bytes * w->c->rank;
  for (long long k = 0; k < count; k += per) {
    const long long m = std::min(per, count - k);
    uint64_t seq;
    rc = post(w, t, RK_GACC, oc, rep, tdisp + k * es, m, oc == O_NOOP ? nullptr : (const char*)origin + k * es,
              my_off, &seq);
    if (rc) return rc;
    rc = wait_done(w, t, seq);
    if (rc) return rc;
    rc = pull(w, (char*)result + k * es, w->peer_scratch[t] + my_off, m * es);
    if (rc) return rc;
    rc = sync_gets(w);  // the slot is reused by my next chunk
    if (rc) return rc;
  }
  return MPIGX_SUCCESS;
}

int mpigx_accumulate(const void* origin_addr, int origin_count, int origin_datatype, int target_rank,
                     long long target_disp, int target_count, int target_datatype, int op, mpigx_win_t win) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (op == MPIGX_NO_OP) return MPIGX_ERR_OP;  // MPI_NO_OP only fetches: MPICH rejects it here
  return acc_common(origin_addr, origin_count, origin_datatype, nullptr, target_count, target_datatype, target_rank,
                    target_disp, target_count, target_datatype, op, win, false);
}

int mpigx_get_accumulate(const void* origin_addr, int origin_count, int origin_datatype, void* result_addr,
                         int result_count, int result_datatype, int target_rank, long long target_disp,
                         int target_count, int target_datatype, int op, mpigx_win_t win) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  return acc_common(origin_addr, origin_count, origin_datatype, result_addr, result_count, result_datatype,
                    target_rank, target_disp, target_count, target_datatype, op, win, true);
}

int mpigx_fetch_and_op(const void* origin_addr, void* result_addr, int datatype, int target_rank,
                       long long target_disp, int op, mpigx_win_t win) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  return acc_common(origin_addr, 1, datatype, result_addr, 1, datatype, target_rank, target_disp, 1, datatype, op,
                    win, true);
}

}  // extern "C"
