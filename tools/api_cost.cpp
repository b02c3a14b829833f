// Host cost of the HIP runtime calls on the zero-copy registration path
// (mpigx.cpp zc_export): hipMemGetAddressRange, hipPointerGetAttribute
// (BUFFER_ID), hipIpcGetMemHandle, on a torch-like sub-allocation.  Also
// whether a freed-and-reallocated buffer keeps its base / buffer id / handle.
// Tooling only: hipcc -O2 tools/api_cost.cpp -o tools/api_cost
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

static double now() {
  timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main() {
  char* p = nullptr;
  if (hipMalloc(&p, 64 << 20) != hipSuccess) return 1;
  char* q = p + (3 << 20);
  const int N = 2000;
  void* base;
  size_t size;
  unsigned long long id = 0;
  hipIpcMemHandle_t h;
  double t0 = now();
  for (int i = 0; i < N; ++i) (void)hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)q);
  double t1 = now();
  for (int i = 0; i < N; ++i) (void)hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)q);
  double t2 = now();
  for (int i = 0; i < N; ++i) (void)hipIpcGetMemHandle(&h, base);
  double t3 = now();
  hipPointerAttribute_t attr;
  for (int i = 0; i < N; ++i) (void)hipPointerGetAttributes(&attr, q);
  double t4 = now();
  printf("{\"hipMemGetAddressRange_us\": %.3f, \"hipPointerGetAttribute_BUFFER_ID_us\": %.3f, "
         "\"hipIpcGetMemHandle_us\": %.3f, \"hipPointerGetAttributes_us\": %.3f",
         (t1 - t0) / N * 1e6, (t2 - t1) / N * 1e6, (t3 - t2) / N * 1e6, (t4 - t3) / N * 1e6);
  // free + realloc of the same size: same base? same id? same handle?
  hipIpcMemHandle_t h0 = h;
  unsigned long long id0 = id;
  (void)hipFree(p);
  char* p2 = nullptr;
  (void)hipMalloc(&p2, 64 << 20);
  unsigned long long id2 = 0;
  hipIpcMemHandle_t h2;
  (void)hipPointerGetAttribute(&id2, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)p2);
  (void)hipIpcGetMemHandle(&h2, p2);
  printf(", \"realloc_same_base\": %s, \"realloc_same_id\": %s, \"realloc_same_handle\": %s}\n",
         p2 == p ? "true" : "false", id2 == id0 ? "true" : "false", memcmp(&h0, &h2, sizeof h) ? "false" : "true");
  return 0;
}
