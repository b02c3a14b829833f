// ipc_reuse.cpp — what identifies an allocation for the zero-copy export
// cache (mpigx.cpp zc_export / lreg): after hipFree + hipMalloc, does HIP hand
// out the same base address, the same HIP buffer id, the same IPC handle?
// And what does hipIpcGetMemHandle cost per call (the cache exists to avoid
// it)?  One process, one GPU; prints one JSON line.
//
// Build: hipcc --offload-arch=gfx950 -O2 tools/ipc_reuse.cpp -o tools/ipc_reuse
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

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

int main() {
  CK(hipSetDevice(0));
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
         "\"same_id_bigger\": %d}\n",
         get_handle_us, repeat_equal ? "true" : "false", trials, same_base, same_id, same_base_id,
         same_handle_when_base_id, trials_bigger, same_base_bigger, same_id_bigger);
  return 0;
}
