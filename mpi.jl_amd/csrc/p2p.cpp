// p2p.cpp — point-to-point on device buffers, the
// MPI_Send / Isend / Recv / Irecv / Sendrecv / Probe / Wait* / Test* / Cancel
// family that src/pointtopoint.jl ccalls (:107-681).
//
// Protocol (rendezvous, pull):
//   sender   Isend: the comm's stream is synchronised (the buffer is ready),
//            the allocation holding the buffer is exported (hipIpc handle
//            cached per HIP buffer id, shared with the zero-copy Allreduce)
//            and an envelope {tag, bytes, buffer id, offset, handle} is
//            published in slot seq % 32 of the shm mailbox [me][dest].
//   receiver progress: envelopes are drained per source in sequence order
//            (MPI's non-overtaking rule) and matched against posted
//            receives in post order (ANY_SOURCE / ANY_TAG wildcards);
//            unmatched ones wait in the unexpected queue for a later
//            Irecv / Probe.  A match imports the sender's allocation once
//            and queues a pull; every pull matched in one progress pass is
//            moved by ONE xfer_kernel launch on the comm's transfer stream
//            (ordered after the receive buffer's prior work on the comm's
//            stream by an event).  When the launch's event completes the
//            receiver stores seq + 1 into the envelope's `done` word, which
//            completes the send request and frees the slot.
// Progress runs inside every p2p call and inside the host spin loops of
// blocking collectives, so a rank blocked in a collective still
// acknowledges transfers a peer waits on (the transfer stream is separate
// from the collective's stream).
//
// Request handles and statuses are MPICH's: `int` handles (REQUEST_NULL =
// 0x2c000000) and the 20-byte MPI_Status.  Semantics pinned against MPICH
// 3.3.2 (tests/golden/gen_p2p_golden.*): empty status for null requests,
// MPI_UNDEFINED index/outcount when every request is null, truncation =
// MPI_ERR_TRUNCATE with count = capacity, Waitall/Waitsome report per-request
// errors with MPI_ERR_IN_STATUS, single-completion calls leave MPI_ERROR
// untouched, send requests leave their status untouched.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <vector>

#include "launch.hpp"
#include "runtime.hpp"

using namespace mpigx;

namespace {

enum Kind { K_SEND = 1, K_RECV = 2 };
enum State { S_QUEUED = 0, S_POSTED, S_XFER, S_DONE };

constexpr int kReqTag = 0x6c000000;
constexpr int kReqMask = 0x00ffffff;
constexpr long long kXferBytesPerBlock = 64 << 10;
constexpr int kXferMaxBlocksPerSeg = 128;

struct Msg {
  int src = 0;
  uint64_t seq = 0;
  P2PEnvelope* env = nullptr;
  int tag = 0;
  long long bytes = 0;
  unsigned long long buf_id = 0, raw = 0;
  long long off = 0;
  hipIpcMemHandle_t h;
};

struct Req {
  int kind = 0;
  mpigx_comm* c = nullptr;
  int state = S_QUEUED;
  int peer = 0, tag = 0;
  const char* sbuf = nullptr;
  char* rbuf = nullptr;
  long long bytes = 0;  // send: message size; recv: capacity
  // send side
  P2PEnvelope* env = nullptr;
  uint64_t seq = 0;
  unsigned long long buf_id = 0;
  long long off = 0;
  hipIpcMemHandle_t h;
  // receive side
  hipEvent_t ready = nullptr;    // recv buffer's prior work on the comm stream
  hipEvent_t done_ev = nullptr;  // the pull's completion on the transfer stream
  Msg msg;
  const char* xsrc = nullptr;
  long long xlen = 0;
  bool has_status = false;  // recv (or PROC_NULL recv): status below is valid
  mpigx_status_t st;
  bool cancelled = false;
  bool detached = false;  // MPI_Request_free'd before completion
  int err = MPIGX_SUCCESS;
  // derived datatypes (types.cpp): the send side travels packed from a pooled
  // temporary; a non-contiguous receive is unpacked straight from the peer
  char* pack_tmp = nullptr;
  long long pack_cap = 0;
  int rtype = 0;          // receive: derived type to unpack into (0: contiguous bytes)
  long long rcount = 0;
};

std::vector<Req*> g_reqs;  // handle & kReqMask -> request
std::vector<int> g_free;

int new_handle(Req* r) {
  int i;
  if (!g_free.empty()) {
    i = g_free.back();
    g_free.pop_back();
    g_reqs[i] = r;
  } else {
    i = (int)g_reqs.size();
    g_reqs.push_back(r);
  }
  return kReqTag | i;
}

Req* lookup(int h) {
  if ((h & ~kReqMask) != kReqTag) return nullptr;
  const int i = h & kReqMask;
  if (i >= (int)g_reqs.size()) return nullptr;
  return g_reqs[i];
}

void set_empty(mpigx_status_t* s) {  // MPIR_Status_set_empty (MPI_ERROR untouched)
  if (!s || s == MPIGX_STATUS_IGNORE) return;
  s->count_lo = 0;
  s->count_hi_and_cancelled = 0;
  s->MPI_SOURCE = MPIGX_ANY_SOURCE;
  s->MPI_TAG = MPIGX_ANY_TAG;
}

void set_status(mpigx_status_t* st, long long bytes, int src, int tag, bool cancelled) {
  st->count_lo = (int)(bytes & 0x7fffffff);
  st->count_hi_and_cancelled = (int)(((bytes >> 31) << 1) | (cancelled ? 1 : 0));
  st->MPI_SOURCE = src;
  st->MPI_TAG = tag;
}

}  // namespace

namespace mpigx {
struct P2PState {
  hipStream_t xs = nullptr;
  uint64_t sseq[kMaxRanks] = {};
  uint64_t rseq[kMaxRanks] = {};
  std::deque<Req*> sendq[kMaxRanks];
  std::vector<Req*> posted;       // unmatched receives, post order
  std::deque<Msg> unexpected;     // unmatched envelopes, arrival order
  std::vector<Req*> inflight;     // pulls launched, not yet complete
  std::vector<Req*> batch;        // pulls matched, not yet launched
  std::vector<Req*> detached;     // freed by the user, still in flight
  std::vector<hipEvent_t> evpool;
  std::vector<std::pair<long long, char*>> packpool;  // free send-pack temporaries (hipMalloc, IPC-exportable)
  P2PMailbox* local = nullptr;    // single-rank communicator (no shm block)
};
}  // namespace mpigx

namespace {

P2PMailbox* box(mpigx_comm* c, int s, int d) { return c->shm ? &c->shm->box[s][d] : c->p2p->local; }

int state_of(mpigx_comm* c, P2PState** out) {
  if (!c->p2p) {
    P2PState* P = new P2PState();
    if (hipStreamCreateWithFlags(&P->xs, hipStreamNonBlocking) != hipSuccess) {
      (void)hipGetLastError();
      delete P;
      return MPIGX_ERR_INTERN;
    }
    if (!c->shm) P->local = new P2PMailbox();
    c->p2p = P;
  }
  *out = c->p2p;
  return MPIGX_SUCCESS;
}

hipEvent_t get_event(P2PState* P) {
  if (!P->evpool.empty()) {
    hipEvent_t e = P->evpool.back();
    P->evpool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return e;
}

void put_event(P2PState* P, hipEvent_t& e) {
  if (e) P->evpool.push_back(e);
  e = nullptr;
}

// max_cap > 0: only a temporary no larger than that (one the runtime can
// IPC-map, runtime.hpp ipc_alloc_max)
char* pack_get(P2PState* P, long long bytes, long long* cap, long long max_cap = 0) {
  size_t best = P->packpool.size();
  for (size_t i = 0; i < P->packpool.size(); ++i)
    if (P->packpool[i].first >= bytes && (max_cap <= 0 || P->packpool[i].first <= max_cap) &&
        (best == P->packpool.size() || P->packpool[i].first < P->packpool[best].first))
      best = i;
  if (best < P->packpool.size()) {
    char* p = P->packpool[best].second;
    *cap = P->packpool[best].first;
    P->packpool.erase(P->packpool.begin() + best);
    return p;
  }
  const long long c = (bytes + (1 << 20) - 1) & ~((1ll << 20) - 1);
  char* p = nullptr;
  if (hipMalloc(&p, c) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  *cap = c;
  return p;
}

// A completed send's temporary goes back to the pool (its exported handle and
// the receiver's import stay valid for the next message using it).
void pack_put(Req* r) {
  if (r->pack_tmp && r->c && r->c->p2p) r->c->p2p->packpool.push_back({r->pack_cap, r->pack_tmp});
  r->pack_tmp = nullptr;
}

void release(Req* r, int* handle) {
  pack_put(r);
  if (r->c && r->c->p2p) {
    put_event(r->c->p2p, r->ready);
    put_event(r->c->p2p, r->done_ev);
  }
  const int i = *handle & kReqMask;
  g_reqs[i] = nullptr;
  g_free.push_back(i);
  delete r;
  *handle = MPIGX_REQUEST_NULL;
}

void ack(Req* r) { r->msg.env->done.store(r->msg.seq + 1, std::memory_order_release); }

bool matches(const Req* r, const Msg& m) {
  return (r->peer == MPIGX_ANY_SOURCE || r->peer == m.src) && (r->tag == MPIGX_ANY_TAG || r->tag == m.tag);
}

// A receive matched message m: status, truncation, source pointer; the bytes
// move in the next flush.
void start_recv(mpigx_comm* c, Req* r, const Msg& m) {
  r->msg = m;
  const long long n = m.bytes < r->bytes ? m.bytes : r->bytes;
  if (m.bytes > r->bytes) r->err = MPIGX_ERR_TRUNCATE;
  r->has_status = true;
  set_status(&r->st, n, m.src, m.tag, false);
  if (n == 0) {
    ack(r);
    r->state = S_DONE;
    return;
  }
  const char* src;
  if (m.src == c->rank) {
    src = (const char*)(uintptr_t)m.raw;
  } else {
    char* base = rt::import_buf(c, m.src, m.buf_id, m.h);
    if (!base) {
      r->err = MPIGX_ERR_INTERN;
      ack(r);
      r->state = S_DONE;
      return;
    }
    src = base + m.off;
  }
  r->xsrc = src;
  r->xlen = n;
  r->state = S_XFER;
  c->p2p->batch.push_back(r);
}

void fail_pull(P2PState* P, Req* r) {
  r->err = MPIGX_ERR_INTERN;
  ack(r);
  r->state = S_DONE;
  put_event(P, r->done_ev);
}

// One xfer_kernel launch per <= kMaxXfer matched messages.
void flush(mpigx_comm* c) {
  P2PState* P = c->p2p;
  // non-contiguous receives: one unpack kernel each, reading the peer's
  // packed bytes over xGMI and scattering them into the typed buffer
  for (size_t k = 0; k < P->batch.size();) {
    Req* r = P->batch[k];
    if (!r->rtype) {
      ++k;
      continue;
    }
    P->batch.erase(P->batch.begin() + k);
    bool ok = !r->ready || hipStreamWaitEvent(P->xs, r->ready, 0) == hipSuccess;
    ok = ok && rt::type_pack(r->rtype, r->rbuf, r->rcount, (void*)r->xsrc, r->xlen, 1, c->device, P->xs) == 0;
    r->done_ev = ok ? get_event(P) : nullptr;
    if (!ok || !r->done_ev || hipEventRecord(r->done_ev, P->xs) != hipSuccess) {
      (void)hipGetLastError();
      fail_pull(P, r);
      continue;
    }
    P->inflight.push_back(r);
  }
  size_t i = 0;
  while (i < P->batch.size()) {
    const size_t m = std::min(P->batch.size() - i, (size_t)kMaxXfer);
    XferArgs a;
    memset(&a, 0, sizeof a);
    a.nseg = (int)m;
    a.coherent = rt::pull_fences();
    bool ok = true;
    for (size_t j = 0; j < m; ++j) {
      Req* r = P->batch[i + j];
      long long g = (r->xlen + kXferBytesPerBlock - 1) / kXferBytesPerBlock;
      g = g < 1 ? 1 : (g > kXferMaxBlocksPerSeg ? kXferMaxBlocksPerSeg : g);
      a.blk0[j + 1] = a.blk0[j] + (int)g;
      a.dst[j] = r->rbuf;
      a.src[j] = r->xsrc;
      a.bytes[j] = r->xlen;
      if (r->ready && hipStreamWaitEvent(P->xs, r->ready, 0) != hipSuccess) ok = false;
    }
    if (ok && launch_xfer(P->xs, a) != hipSuccess) ok = false;
    for (size_t j = 0; j < m; ++j) {
      Req* r = P->batch[i + j];
      r->done_ev = ok ? get_event(P) : nullptr;
      if (!ok || !r->done_ev || hipEventRecord(r->done_ev, P->xs) != hipSuccess) {
        (void)hipGetLastError();
        fail_pull(P, r);
        continue;
      }
      P->inflight.push_back(r);
    }
    i += m;
  }
  P->batch.clear();
}

void post_sends(mpigx_comm* c) {
  P2PState* P = c->p2p;
  for (int d = 0; d < c->n; ++d) {
    while (!P->sendq[d].empty()) {
      Req* r = P->sendq[d].front();
      const uint64_t seq = P->sseq[d];
      P2PEnvelope* e = &box(c, c->rank, d)->slot[seq % kP2PSlots];
      if (e->done.load(std::memory_order_acquire) != e->posted.load(std::memory_order_relaxed)) break;
      e->tag = r->tag;
      e->bytes = r->bytes;
      e->buf_id = r->buf_id;
      e->off = r->off;
      e->raw = (unsigned long long)(uintptr_t)r->sbuf;
      e->h = r->h;
      e->posted.store(seq + 1, std::memory_order_release);
      r->env = e;
      r->seq = seq;
      r->state = S_POSTED;
      P->sseq[d] = seq + 1;
      P->sendq[d].pop_front();
    }
  }
}

void drain(mpigx_comm* c) {
  P2PState* P = c->p2p;
  for (int s = 0; s < c->n; ++s) {
    for (;;) {
      P2PEnvelope* e = &box(c, s, c->rank)->slot[P->rseq[s] % kP2PSlots];
      if (e->posted.load(std::memory_order_acquire) != P->rseq[s] + 1) break;
      Msg m;
      m.src = s;
      m.seq = P->rseq[s];
      m.env = e;
      m.tag = e->tag;
      m.bytes = e->bytes;
      m.buf_id = e->buf_id;
      m.raw = e->raw;
      m.off = e->off;
      m.h = e->h;
      P->rseq[s] += 1;
      bool matched = false;
      for (size_t i = 0; i < P->posted.size(); ++i)
        if (matches(P->posted[i], m)) {
          Req* r = P->posted[i];
          P->posted.erase(P->posted.begin() + i);
          start_recv(c, r, m);
          matched = true;
          break;
        }
      if (!matched) P->unexpected.push_back(m);
    }
  }
}

void reap(mpigx_comm* c) {
  P2PState* P = c->p2p;
  for (size_t i = 0; i < P->inflight.size();) {
    Req* r = P->inflight[i];
    const hipError_t q = hipEventQuery(r->done_ev);
    if (q == hipErrorNotReady) {
      ++i;
      continue;
    }
    if (q != hipSuccess) {
      (void)hipGetLastError();
      r->err = MPIGX_ERR_INTERN;
    }
    ack(r);
    r->state = S_DONE;
    put_event(P, r->done_ev);
    P->inflight.erase(P->inflight.begin() + i);
  }
}

bool complete(Req* r) {
  if (r->state == S_DONE) return true;
  // `done` only grows per slot (the slot is reused for seq + 32 only after
  // seq was acknowledged), so >= still sees our ack after a reuse
  if (r->kind == K_SEND && r->state == S_POSTED &&
      r->env->done.load(std::memory_order_acquire) >= r->seq + 1) {
    r->state = S_DONE;
    pack_put(r);
    return true;
  }
  return false;
}

void progress(mpigx_comm* c) {
  if (c->rma && !c->in_progress) rt::rma_progress(c);  // waits here serve RMA targets too
  if (!c->p2p) return;
  post_sends(c);
  drain(c);
  flush(c);
  reap(c);
  P2PState* P = c->p2p;
  for (size_t i = 0; i < P->detached.size();) {
    Req* r = P->detached[i];
    if (complete(r)) {  // detached requests already left the handle table
      put_event(P, r->ready);
      put_event(P, r->done_ev);
      delete r;
      P->detached.erase(P->detached.begin() + i);
    } else {
      ++i;
    }
  }
}

int check_common(mpigx_comm* c, const void* buf, int count, int datatype, rt::TypeDesc* d) {
  int rc = rt::comm_check(c);
  if (rc) return rc;
  if (count < 0) return MPIGX_ERR_COUNT;
  if (rt::type_info(datatype, d)) return MPIGX_ERR_TYPE;
  if (!buf && count > 0 && d->size > 0) return MPIGX_ERR_BUFFER;
  return MPIGX_SUCCESS;
}

double limit_s(mpigx_comm* c) { return c->timeout_ticks / 1e8; }

// Fill a completed request's status (recv only; send statuses stay as they are).
void fill(const Req* r, mpigx_status_t* s, bool write_error) {
  if (!s || s == MPIGX_STATUS_IGNORE) return;
  if (r->has_status) {
    const int e = s->MPI_ERROR;
    *s = r->st;
    s->MPI_ERROR = e;
  }
  if (write_error) s->MPI_ERROR = r->err;
}

// Progress every communicator referenced by the non-null requests.
void progress_reqs(int count, const mpigx_request_t* reqs) {
  mpigx_comm* last = nullptr;
  for (int i = 0; i < count; ++i) {
    Req* r = lookup(reqs[i]);
    if (r && r->c != last) {
      progress(r->c);
      last = r->c;
    }
  }
}

// Waiting: MPI waits forever; a dead peer would hang the caller, so waits give
// up after the communicator's timeout (MPIGX_TIMEOUT_MS) with MPI_ERR_OTHER.
// How long a blocking point-to-point call waits (round 5): as long as its
// peers live, as MPI's Wait / Recv do (pointtopoint.jl) — the same rule as
// the collectives' late-rank waits.  It gives up only when a peer of one of
// its communicators is gone or its communicator failed (rt::peer_dead,
// checked every 0.25 s); past MPIGX_TIMEOUT_MS it says once on stderr that it
// is still waiting.
struct Deadline {
  static constexpr int kMax = 4;
  mpigx_comm* comms[kMax] = {};
  int nc = 0;
  double t0, lim, next;
  unsigned spins = 0;
  bool noted = false;
  explicit Deadline(double l) : t0(rt::wall()), lim(l), next(t0 + 0.25) {}
  void add(mpigx_comm* c) {
    for (int i = 0; i < nc; ++i)
      if (comms[i] == c) return;
    if (c && nc < kMax) comms[nc++] = c;
  }
  bool expired() {
    if ((++spins & 1023) != 0) return false;
    const double t = rt::wall();
    if (t < next) return false;
    next = t + 0.25;
    for (int i = 0; i < nc; ++i)
      if (rt::peer_dead(comms[i])) return true;
    if (!noted && t - t0 > lim) {
      noted = true;
      fprintf(stderr, "mpigx: a point-to-point wait has lasted %.0f s; still waiting for the peer\n", t - t0);
    }
    return false;
  }
};

double limit_of(int count, const mpigx_request_t* reqs) {
  double l = 60.0;
  for (int i = 0; i < count; ++i)
    if (Req* r = lookup(reqs[i])) l = std::max(l, limit_s(r->c));
  return l;
}
// the communicators of a request set, for Deadline (caller holds big_lock)
void comms_of(Deadline& d, int count, const mpigx_request_t* reqs) {
  for (int i = 0; i < count; ++i)
    if (Req* r = lookup(reqs[i])) d.add(r->c);
}

int validate_reqs(int count, const mpigx_request_t* reqs) {
  if (count < 0) return MPIGX_ERR_COUNT;
  if (count > 0 && !reqs) return MPIGX_ERR_REQUEST;
  for (int i = 0; i < count; ++i)
    if (reqs[i] != MPIGX_REQUEST_NULL && !lookup(reqs[i])) return MPIGX_ERR_REQUEST;
  return MPIGX_SUCCESS;
}

}  // namespace

namespace mpigx {
namespace rt {
void p2p_progress(mpigx_comm* c) { progress(c); }

void p2p_sync(mpigx_comm* c) {
  if (c->p2p) (void)hipStreamSynchronize(c->p2p->xs);
}

void p2p_destroy(mpigx_comm* c) {
  P2PState* P = c->p2p;
  if (!P) return;
  (void)hipStreamSynchronize(P->xs);
  // requests of this communicator become invalid
  for (size_t i = 0; i < g_reqs.size(); ++i)
    if (g_reqs[i] && g_reqs[i]->c == c) {
      int h = kReqTag | (int)i;
      release(g_reqs[i], &h);
    }
  for (Req* r : P->detached) {
    put_event(P, r->ready);
    put_event(P, r->done_ev);
    delete r;
  }
  for (hipEvent_t e : P->evpool) (void)hipEventDestroy(e);
  for (auto& b : P->packpool) (void)hipFree(b.second);
  (void)hipStreamDestroy(P->xs);
  delete P->local;
  delete P;
  c->p2p = nullptr;
}
}  // namespace rt
}  // namespace mpigx

// ===========================================================================
// C ABI (include/mpigx.h, point-to-point section)
// ===========================================================================
extern "C" {

int mpigx_isend(const void* buf, int count, int datatype, int dest, int tag, mpigx_comm_t c,
                mpigx_request_t* request) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!request) return MPIGX_ERR_ARG;
  rt::TypeDesc td;
  int rc = check_common(c, buf, count, datatype, &td);
  if (rc) return rc;
  if (dest != MPIGX_PROC_NULL && (dest < 0 || dest >= c->n)) return MPIGX_ERR_RANK;
  if (tag < 0 || tag > MPIGX_TAG_UB) return MPIGX_ERR_TAG;
  P2PState* P;
  if ((rc = state_of(c, &P))) return rc;
  Req* r = new Req();
  r->kind = K_SEND;
  r->c = c;
  r->peer = dest;
  r->tag = tag;
  r->sbuf = (const char*)buf;
  r->bytes = (long long)count * td.size;
  if (dest == MPIGX_PROC_NULL) {
    r->state = S_DONE;
    *request = new_handle(r);
    return MPIGX_SUCCESS;
  }
  if (r->bytes > 0) {
    if (!td.contig) {  // derived, non-contiguous: pack on device into a pooled temporary
      r->pack_tmp = pack_get(P, r->bytes, &r->pack_cap, c->ipc_alloc_max);
      if (!r->pack_tmp) {
        delete r;
        return MPIGX_ERR_NO_MEM;
      }
      if ((rc = rt::type_pack(datatype, buf, count, r->pack_tmp, r->bytes, 0, c->device, c->stream))) {
        P->packpool.push_back({r->pack_cap, r->pack_tmp});
        delete r;
        return rc;
      }
      r->sbuf = r->pack_tmp;
    }
    // the receiver reads the buffer asynchronously: it must hold its final
    // contents now (prior producers on the comm's stream have finished)
    if (hipStreamSynchronize(c->stream) != hipSuccess) {
      (void)hipGetLastError();
      delete r;
      return MPIGX_ERR_INTERN;
    }
    if (dest != c->rank && !rt::export_buf(c, r->sbuf, &r->buf_id, &r->off, &r->h)) {
      // a contiguous message in an allocation the runtime cannot IPC-map
      // (runtime.hpp ipc_alloc_max): staged in a pooled temporary of its own
      bool ok = false;
      const long long rounded = (r->bytes + (1 << 20) - 1) & ~((1ll << 20) - 1);  // pack_get's allocation
      if (!r->pack_tmp && (c->ipc_alloc_max <= 0 || rounded <= c->ipc_alloc_max)) {
        r->pack_tmp = pack_get(P, r->bytes, &r->pack_cap, c->ipc_alloc_max);
        if (r->pack_tmp && hipMemcpyAsync(r->pack_tmp, buf, r->bytes, hipMemcpyDeviceToDevice, c->stream) == hipSuccess &&
            hipStreamSynchronize(c->stream) == hipSuccess) {
          r->sbuf = r->pack_tmp;
          ok = rt::export_buf(c, r->sbuf, &r->buf_id, &r->off, &r->h);
        }
        (void)hipGetLastError();
      }
      if (!ok) {
        pack_put(r);
        delete r;
        return MPIGX_ERR_BUFFER;  // not a device allocation that can be IPC-exported
      }
    }
  }
  P->sendq[dest].push_back(r);
  *request = new_handle(r);
  progress(c);
  return MPIGX_SUCCESS;
}

int mpigx_irecv(void* buf, int count, int datatype, int source, int tag, mpigx_comm_t c,
                mpigx_request_t* request) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!request) return MPIGX_ERR_ARG;
  rt::TypeDesc td;
  int rc = check_common(c, buf, count, datatype, &td);
  if (rc) return rc;
  if (source != MPIGX_PROC_NULL && source != MPIGX_ANY_SOURCE && (source < 0 || source >= c->n))
    return MPIGX_ERR_RANK;
  if (tag != MPIGX_ANY_TAG && (tag < 0 || tag > MPIGX_TAG_UB)) return MPIGX_ERR_TAG;
  P2PState* P;
  if ((rc = state_of(c, &P))) return rc;
  Req* r = new Req();
  r->kind = K_RECV;
  r->c = c;
  r->peer = source;
  r->tag = tag;
  r->rbuf = (char*)buf;
  r->bytes = (long long)count * td.size;
  if (!td.contig) {
    r->rtype = datatype;
    r->rcount = count;
  }
  if (source == MPIGX_PROC_NULL) {
    r->has_status = true;
    set_status(&r->st, 0, MPIGX_PROC_NULL, MPIGX_ANY_TAG, false);
    r->state = S_DONE;
    *request = new_handle(r);
    return MPIGX_SUCCESS;
  }
  if (r->bytes > 0) {
    r->ready = get_event(P);
    if (!r->ready || hipEventRecord(r->ready, c->stream) != hipSuccess) {
      (void)hipGetLastError();
      put_event(P, r->ready);
      delete r;
      return MPIGX_ERR_INTERN;
    }
  }
  r->state = S_POSTED;
  // earlier-posted receives get the messages that already arrived first
  post_sends(c);
  drain(c);
  bool matched = false;
  for (auto it = P->unexpected.begin(); it != P->unexpected.end(); ++it)
    if (matches(r, *it)) {
      const Msg m = *it;
      P->unexpected.erase(it);
      start_recv(c, r, m);
      matched = true;
      break;
    }
  if (!matched) P->posted.push_back(r);
  *request = new_handle(r);
  flush(c);
  reap(c);
  return MPIGX_SUCCESS;
}

int mpigx_test(mpigx_request_t* request, int* flag, mpigx_status_t* status) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!request || !flag) return MPIGX_ERR_ARG;
  if (*request == MPIGX_REQUEST_NULL) {
    *flag = 1;
    set_empty(status);
    return MPIGX_SUCCESS;
  }
  Req* r = lookup(*request);
  if (!r) return MPIGX_ERR_REQUEST;
  progress(r->c);
  if (!complete(r)) {
    *flag = 0;
    return MPIGX_SUCCESS;
  }
  *flag = 1;
  fill(r, status, false);
  const int rc = r->err;
  release(r, request);
  return rc;
}

int mpigx_wait(mpigx_request_t* request, mpigx_status_t* status) {
  if (!request) return MPIGX_ERR_ARG;
  double lim;
  {  // the request table under the lock; the wait itself polls without it
    std::lock_guard<rt::BigLock> big(rt::big_lock());
    if (*request != MPIGX_REQUEST_NULL && !lookup(*request)) return MPIGX_ERR_REQUEST;
    lim = limit_of(1, request);
  }
  Deadline dl(lim);
  {
    std::lock_guard<rt::BigLock> big(rt::big_lock());
    comms_of(dl, 1, request);
  }
  for (;;) {
    int flag = 0;
    const int rc = mpigx_test(request, &flag, status);
    if (flag) return rc;
    if (dl.expired()) return MPIGX_ERR_OTHER;
  }
}

int mpigx_testall(int count, mpigx_request_t* requests, int* flag, mpigx_status_t* statuses) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!flag) return MPIGX_ERR_ARG;
  int rc = validate_reqs(count, requests);
  if (rc) return rc;
  progress_reqs(count, requests);
  for (int i = 0; i < count; ++i) {
    Req* r = lookup(requests[i]);
    if (r && !complete(r)) {
      *flag = 0;
      return MPIGX_SUCCESS;
    }
  }
  *flag = 1;
  const bool ign = statuses == MPIGX_STATUS_IGNORE || !statuses;
  bool any_err = false;
  for (int i = 0; i < count; ++i) {
    Req* r = lookup(requests[i]);
    mpigx_status_t* s = ign ? nullptr : &statuses[i];
    if (!r) {
      set_empty(s);
      if (s) s->MPI_ERROR = MPIGX_SUCCESS;
      continue;
    }
    fill(r, s, true);
    any_err |= r->err != MPIGX_SUCCESS;
    release(r, &requests[i]);
  }
  return any_err ? MPIGX_ERR_IN_STATUS : MPIGX_SUCCESS;
}

int mpigx_waitall(int count, mpigx_request_t* requests, mpigx_status_t* statuses) {
  int rc;
  double lim;
  {
    std::lock_guard<rt::BigLock> big(rt::big_lock());
    if ((rc = validate_reqs(count, requests))) return rc;
    lim = limit_of(count, requests);
  }
  Deadline dl(lim);
  {
    std::lock_guard<rt::BigLock> big(rt::big_lock());
    comms_of(dl, count, requests);
  }
  for (;;) {
    int flag = 0;
    rc = mpigx_testall(count, requests, &flag, statuses);
    if (flag) return rc;
    if (dl.expired()) return MPIGX_ERR_OTHER;
  }
}

int mpigx_testany(int count, mpigx_request_t* requests, int* index, int* flag, mpigx_status_t* status) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!index || !flag) return MPIGX_ERR_ARG;
  int rc = validate_reqs(count, requests);
  if (rc) return rc;
  bool any = false;
  for (int i = 0; i < count; ++i) any |= requests[i] != MPIGX_REQUEST_NULL;
  *index = MPIGX_UNDEFINED;
  if (!any) {
    *flag = 1;
    set_empty(status);
    return MPIGX_SUCCESS;
  }
  progress_reqs(count, requests);
  for (int i = 0; i < count; ++i) {
    Req* r = lookup(requests[i]);
    if (r && complete(r)) {
      *flag = 1;
      *index = i;
      fill(r, status, false);
      rc = r->err;
      release(r, &requests[i]);
      return rc;
    }
  }
  *flag = 0;
  return MPIGX_SUCCESS;
}

int mpigx_waitany(int count, mpigx_request_t* requests, int* index, mpigx_status_t* status) {
  if (!index) return MPIGX_ERR_ARG;
  int rc;
  double lim;
  {
    std::lock_guard<rt::BigLock> big(rt::big_lock());
    if ((rc = validate_reqs(count, requests))) return rc;
    lim = limit_of(count, requests);
  }
  Deadline dl(lim);
  {
    std::lock_guard<rt::BigLock> big(rt::big_lock());
    comms_of(dl, count, requests);
  }
  for (;;) {
    int flag = 0;
    rc = mpigx_testany(count, requests, index, &flag, status);
    if (flag) return rc;
    if (dl.expired()) return MPIGX_ERR_OTHER;
  }
}

int mpigx_testsome(int incount, mpigx_request_t* requests, int* outcount, int* indices,
                   mpigx_status_t* statuses) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!outcount) return MPIGX_ERR_ARG;
  int rc = validate_reqs(incount, requests);
  if (rc) return rc;
  bool any = false;
  for (int i = 0; i < incount; ++i) any |= requests[i] != MPIGX_REQUEST_NULL;
  if (!any) {
    *outcount = MPIGX_UNDEFINED;
    return MPIGX_SUCCESS;
  }
  progress_reqs(incount, requests);
  const bool ign = statuses == MPIGX_STATUS_IGNORE || !statuses;
  int k = 0;
  bool any_err = false;
  for (int i = 0; i < incount; ++i) {
    Req* r = lookup(requests[i]);
    if (!r || !complete(r)) continue;
    if (indices) indices[k] = i;
    fill(r, ign ? nullptr : &statuses[k], true);
    any_err |= r->err != MPIGX_SUCCESS;
    release(r, &requests[i]);
    ++k;
  }
  *outcount = k;
  return any_err ? MPIGX_ERR_IN_STATUS : MPIGX_SUCCESS;
}

int mpigx_waitsome(int incount, mpigx_request_t* requests, int* outcount, int* indices,
                   mpigx_status_t* statuses) {
  if (!outcount) return MPIGX_ERR_ARG;
  int rc;
  double lim;
  {
    std::lock_guard<rt::BigLock> big(rt::big_lock());
    if ((rc = validate_reqs(incount, requests))) return rc;
    lim = limit_of(incount, requests);
  }
  Deadline dl(lim);
  {
    std::lock_guard<rt::BigLock> big(rt::big_lock());
    comms_of(dl, incount, requests);
  }
  for (;;) {
    rc = mpigx_testsome(incount, requests, outcount, indices, statuses);
    if (*outcount != 0) return rc;
    if (dl.expired()) return MPIGX_ERR_OTHER;
  }
}

int mpigx_cancel(mpigx_request_t* request) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!request) return MPIGX_ERR_ARG;
  Req* r = lookup(*request);
  if (!r) return MPIGX_ERR_REQUEST;
  P2PState* P = r->c->p2p;
  if (r->kind == K_RECV && r->state == S_POSTED) {
    auto it = std::find(P->posted.begin(), P->posted.end(), r);
    if (it != P->posted.end()) {
      P->posted.erase(it);
      r->cancelled = true;
      r->has_status = true;
      set_status(&r->st, 0, MPIGX_ANY_SOURCE, MPIGX_ANY_TAG, true);
      r->state = S_DONE;
    }
  } else if (r->kind == K_SEND && r->state == S_QUEUED) {
    for (auto& q : P->sendq) {
      auto it = std::find(q.begin(), q.end(), r);
      if (it != q.end()) {
        q.erase(it);
        r->cancelled = true;
        r->has_status = true;
        set_status(&r->st, 0, MPIGX_ANY_SOURCE, MPIGX_ANY_TAG, true);
        r->state = S_DONE;
        break;
      }
    }
  }
  return MPIGX_SUCCESS;  // a request that already matched completes normally
}

int mpigx_request_free(mpigx_request_t* request) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  if (!request) return MPIGX_ERR_ARG;
  Req* r = lookup(*request);
  if (!r) return MPIGX_ERR_REQUEST;
  if (r->c) progress(r->c);
  if (complete(r)) {
    release(r, request);
    return MPIGX_SUCCESS;
  }
  // still in flight: the communicator's progress retires it
  const int i = *request & kReqMask;
  g_reqs[i] = nullptr;
  g_free.push_back(i);
  r->detached = true;
  r->c->p2p->detached.push_back(r);
  *request = MPIGX_REQUEST_NULL;
  return MPIGX_SUCCESS;
}

int mpigx_send(const void* buf, int count, int datatype, int dest, int tag, mpigx_comm_t c) {
  mpigx_request_t r = MPIGX_REQUEST_NULL;
  int rc = mpigx_isend(buf, count, datatype, dest, tag, c, &r);
  if (rc) return rc;
  return mpigx_wait(&r, MPIGX_STATUS_IGNORE);
}

int mpigx_recv(void* buf, int count, int datatype, int source, int tag, mpigx_comm_t c,
               mpigx_status_t* status) {
  mpigx_request_t r = MPIGX_REQUEST_NULL;
  int rc = mpigx_irecv(buf, count, datatype, source, tag, c, &r);
  if (rc) return rc;
  return mpigx_wait(&r, status);
}

int mpigx_sendrecv(const void* sendbuf, int sendcount, int sendtype, int dest, int sendtag, void* recvbuf,
                   int recvcount, int recvtype, int source, int recvtag, mpigx_comm_t c,
                   mpigx_status_t* status) {
  mpigx_request_t rq[2] = {MPIGX_REQUEST_NULL, MPIGX_REQUEST_NULL};
  int rc = mpigx_irecv(recvbuf, recvcount, recvtype, source, recvtag, c, &rq[1]);
  if (rc) return rc;
  rc = mpigx_isend(sendbuf, sendcount, sendtype, dest, sendtag, c, &rq[0]);
  if (rc) {
    (void)mpigx_cancel(&rq[1]);
    (void)mpigx_wait(&rq[1], MPIGX_STATUS_IGNORE);
    return rc;
  }
  const int rs = mpigx_wait(&rq[0], MPIGX_STATUS_IGNORE);
  const int rr = mpigx_wait(&rq[1], status);
  return rr ? rr : rs;
}

int mpigx_iprobe(int source, int tag, mpigx_comm_t c, int* flag, mpigx_status_t* status) {
  std::lock_guard<rt::BigLock> big(rt::big_lock());  // THREAD_MULTIPLE (runtime.hpp)
  int rc = rt::comm_check(c);
  if (rc) return rc;
  if (!flag) return MPIGX_ERR_ARG;
  if (source != MPIGX_PROC_NULL && source != MPIGX_ANY_SOURCE && (source < 0 || source >= c->n))
    return MPIGX_ERR_RANK;
  if (tag != MPIGX_ANY_TAG && (tag < 0 || tag > MPIGX_TAG_UB)) return MPIGX_ERR_TAG;
  const bool want = status && status != MPIGX_STATUS_IGNORE;
  if (source == MPIGX_PROC_NULL) {
    *flag = 1;
    if (want) set_status(status, 0, MPIGX_PROC_NULL, MPIGX_ANY_TAG, false);
    return MPIGX_SUCCESS;
  }
  P2PState* P;
  if ((rc = state_of(c, &P))) return rc;
  progress(c);
  Req probe;
  probe.peer = source;
  probe.tag = tag;
  for (const Msg& m : P->unexpected)
    if (matches(&probe, m)) {
      *flag = 1;
      if (want) set_status(status, m.bytes, m.src, m.tag, false);
      return MPIGX_SUCCESS;
    }
  *flag = 0;
  return MPIGX_SUCCESS;
}

int mpigx_probe(int source, int tag, mpigx_comm_t c, mpigx_status_t* status) {
  int rc = rt::comm_check(c);
  if (rc) return rc;
  Deadline dl(limit_s(c));
  dl.add(c);
  for (;;) {
    int flag = 0;
    rc = mpigx_iprobe(source, tag, c, &flag, status);
    if (rc || flag) return rc;
    if (dl.expired()) return MPIGX_ERR_OTHER;
  }
}

int mpigx_get_count(const mpigx_status_t* status, int datatype, int* count) {
  if (!status || !count) return MPIGX_ERR_ARG;
  mpigx::rt::TypeDesc td;
  if (mpigx::rt::type_info(datatype, &td)) return MPIGX_ERR_TYPE;
  const long long es = td.size;
  const long long bytes =
      ((long long)(status->count_hi_and_cancelled >> 1) << 31) | (long long)(status->count_lo & 0x7fffffff);
  if (es == 0 || bytes % es != 0 || bytes / es > 0x7fffffff)
    *count = MPIGX_UNDEFINED;
  else
    *count = (int)(bytes / es);
  return MPIGX_SUCCESS;
}

int mpigx_test_cancelled(const mpigx_status_t* status, int* flag) {
  if (!status || !flag) return MPIGX_ERR_ARG;
  *flag = status->count_hi_and_cancelled & 1;
  return MPIGX_SUCCESS;
}

}  // extern "C"
