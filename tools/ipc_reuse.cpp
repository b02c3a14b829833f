// ipc_reuse.cpp — what identifies an allocation for the zero-copy export and
// import caches (mpigx.cpp zc_export / lreg, zc_import / imports): after
// hipFree + hipMalloc, does HIP hand out the same base address, the same HIP
// buffer id, the same IPC handle?  And on the importing side: does a peer's
// mapping of the freed allocation still reach the old memory, the new one, or
// neither?
//
// Part 1 (one process): base / buffer id / handle reuse, hipIpcGetMemHandle
// cost.  Part 2 (two processes, forked before any HIP call, handles passed
// over a pipe): the owner exports buffer A (pattern 0xA1), the peer imports
// it; the owner frees A and allocates B of the same size (pattern 0xB2); the
// peer compares B's handle with A's, reads through its old mapping and opens
// B's handle.  Prints one JSON line.
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/ipc_reuse.cpp -o tools/ipc_reuse
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

static double now_us() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

struct Info {
  void* base;
  size_t size;
  unsigned long long id;
  hipIpcMemHandle_t h;
};

static int info(void* p, Info* o) {
  CK(hipMemGetAddressRange(&o->base, &o->size, (hipDeviceptr_t)p));
  CK(hipPointerGetAttribute(&o->id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p));
  CK(hipIpcGetMemHandle(&o->h, o->base));
  return 0;
}

static bool full_write(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t k = write(fd, c, n);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}
static bool full_read(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t k = read(fd, c, n);
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

struct Msg {
  Info a, b;
  int same_base, same_id;
};
struct Result {
  int ok;
  int handle_equal;        // B's handle byte-identical to A's
  unsigned old_map_word;   // first word read through the peer's mapping of A after the owner freed it
  unsigned new_map_word;   // first word read through the mapping opened from B's handle
  int new_map_same_va;     // opening B's handle returned the VA of A's mapping
  int close_then_read_ok;  // after closing A's mapping, B's still reads (only when the VAs differ)
};

// peer process: import A, then look at B
static int peer(int rfd, int wfd, size_t s) {
  Result res;
  memset(&res, 0, sizeof res);
  CK(hipSetDevice(0));
  Msg m;
  if (!full_read(rfd, &m, sizeof m)) return 1;
  void* pa = nullptr;
  CK(hipIpcOpenMemHandle(&pa, m.a.h, hipIpcMemLazyEnablePeerAccess));
  unsigned w = 0;
  CK(hipMemcpy(&w, pa, 4, hipMemcpyDeviceToHost));
  const int ack = w == 0xA1A1A1A1u;
  if (!full_write(wfd, &ack, sizeof ack)) return 1;
  if (!full_read(rfd, &m, sizeof m)) return 1;  // owner freed A, allocated and filled B
  res.handle_equal = memcmp(&m.a.h, &m.b.h, sizeof m.a.h) == 0;
  CK(hipMemcpy(&res.old_map_word, pa, 4, hipMemcpyDeviceToHost));
  void* pb = nullptr;
  CK(hipIpcOpenMemHandle(&pb, m.b.h, hipIpcMemLazyEnablePeerAccess));
  CK(hipMemcpy(&res.new_map_word, pb, 4, hipMemcpyDeviceToHost));
  res.new_map_same_va = pa == pb;
  if (pa != pb) {
    CK(hipIpcCloseMemHandle(pa));
    unsigned x = 0;
    res.close_then_read_ok = hipMemcpy(&x, pb, 4, hipMemcpyDeviceToHost) == hipSuccess && x == 0xB2B2B2B2u;
    CK(hipIpcCloseMemHandle(pb));
  } else {
    CK(hipIpcCloseMemHandle(pb));
  }
  (void)s;
  res.ok = 1;
  if (!full_write(wfd, &res, sizeof res)) return 1;
  return 0;
}

int main() {
  // ---- part 2 first: fork before this process touches HIP ----
  const size_t s2 = 64ull << 20;
  int p2c[2], c2p[2];
  if (pipe(p2c) || pipe(c2p)) return 1;
  const pid_t pid = fork();
  if (pid == 0) {
    close(p2c[1]);
    close(c2p[0]);
    _exit(peer(p2c[0], c2p[1], s2));
  }
  close(p2c[0]);
  close(c2p[1]);
  CK(hipSetDevice(0));
  Msg m;
  memset(&m, 0, sizeof m);
  void* A = nullptr;
  CK(hipMalloc(&A, s2));
  CK(hipMemset(A, 0xA1, s2));
  CK(hipDeviceSynchronize());
  if (info(A, &m.a)) return 1;
  if (!full_write(p2c[1], &m, sizeof m)) return 1;
  int ack = 0;
  if (!full_read(c2p[0], &ack, sizeof ack)) return 1;
  CK(hipFree(A));
  void* B = nullptr;
  CK(hipMalloc(&B, s2));
  CK(hipMemset(B, 0xB2, s2));
  CK(hipDeviceSynchronize());
  if (info(B, &m.b)) return 1;
  m.same_base = m.a.base == m.b.base;
  m.same_id = m.a.id == m.b.id;
  if (!full_write(p2c[1], &m, sizeof m)) return 1;
  Result res;
  memset(&res, 0, sizeof res);
  const bool got = full_read(c2p[0], &res, sizeof res);
  int st = 0;
  waitpid(pid, &st, 0);
  CK(hipFree(B));

  // ---- part 1 ----
  const size_t sizes[] = {64ull << 20, 512ull << 20, 2ull << 20};
  int same_base = 0, same_id = 0, same_base_id = 0, same_handle_when_base_id = 0, trials = 0;
  int same_base_bigger = 0, same_id_bigger = 0, trials_bigger = 0;
  // repeated handle of one live allocation: identical bytes?  cost?
  void* a = nullptr;
  CK(hipMalloc(&a, 64 << 20));
  Info ia, ib;
  if (info(a, &ia)) return 1;
  int repeat_equal = 1;
  const int reps = 200;
  const double t0 = now_us();
  for (int i = 0; i < reps; ++i) {
    hipIpcMemHandle_t h;
    CK(hipIpcGetMemHandle(&h, ia.base));
    repeat_equal &= memcmp(&h, &ia.h, sizeof h) == 0;
  }
  const double get_handle_us = (now_us() - t0) / reps;
  CK(hipFree(a));
  for (size_t s : sizes) {
    for (int k = 0; k < 20; ++k) {
      void* p = nullptr;
      CK(hipMalloc(&p, s));
      if (info(p, &ia)) return 1;
      CK(hipFree(p));
      void* q = nullptr;
      CK(hipMalloc(&q, s));  // same size right after the free
      if (info(q, &ib)) return 1;
      ++trials;
      same_base += ia.base == ib.base;
      same_id += ia.id == ib.id;
      if (ia.base == ib.base && ia.id == ib.id) {
        ++same_base_id;
        same_handle_when_base_id += memcmp(&ia.h, &ib.h, sizeof ia.h) == 0;
      }
      CK(hipFree(q));
      void* r = nullptr;  // a larger allocation after a free
      CK(hipMalloc(&p, s));
      if (info(p, &ia)) return 1;
      CK(hipFree(p));
      CK(hipMalloc(&r, 2 * s));
      if (info(r, &ib)) return 1;
      ++trials_bigger;
      same_base_bigger += ia.base == ib.base;
      same_id_bigger += ia.id == ib.id;
      CK(hipFree(r));
    }
  }
  printf("{\"tool\": \"ipc_reuse\", \"get_handle_us\": %.2f, \"repeat_handle_identical\": %s, "
         "\"trials_same_size\": %d, \"same_base\": %d, \"same_buffer_id\": %d, \"same_base_and_id\": %d, "
         "\"same_handle_when_base_and_id\": %d, \"trials_bigger\": %d, \"same_base_bigger\": %d, "
         "\"same_id_bigger\": %d, \"xproc\": {\"peer_ok\": %d, \"peer_exit\": %d, \"same_base\": %d, "
         "\"same_id\": %d, \"handle_equal\": %d, \"old_map_word\": \"%08x\", \"new_map_word\": \"%08x\", "
         "\"new_map_same_va\": %d, \"close_old_then_read_new_ok\": %d}}\n",
         get_handle_us, repeat_equal ? "true" : "false", trials, same_base, same_id, same_base_id,
         same_handle_when_base_id, trials_bigger, same_base_bigger, same_id_bigger, got ? res.ok : 0,
         WIFEXITED(st) ? WEXITSTATUS(st) : -1, m.same_base, m.same_id, res.handle_equal, res.old_map_word,
         res.new_map_word, res.new_map_same_va, res.close_then_read_ok);
  return 0;
}
