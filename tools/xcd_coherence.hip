// Cross-L2 visibility probe for the remote-store variants (push / pull-push
// two-shot, zero-copy Reduce): on the 1-GPU box a rank's block b and its
// peer's block b run on the same XCD (workgroup b -> XCD b % 8 in every
// dispatch), so the same-device tests never exercise a reader whose L2 holds a
// stale copy of a line another L2 (or, on 8 GPUs, another GPU) has rewritten.
// This probe does exactly that inside one device: a writer block on one XCD
// and a reader block on another share a coarse-grained (hipMalloc) buffer X.
//
// Per round k: the reader loads X (its XCD's L2 now holds the lines), flags
// R = k+1; the writer waits for R, stores X = k+1, s_waitcnt + release fence
// (system scope, as rank_barrier's publisher), flags W = k+1; the reader waits
// for W, applies the acquire variant under test, loads X again and counts the
// elements that are not k+1 (stale).
//
// Variants: acquire {system, agent, none, L1 only} x reader loads {plain, nontemporal
// (ld16)} x reader XCD {other, same}. The "none" rows are the control: a stale
// count there shows the probe can see stale lines at all; "L1 only"
// (buffer_inv sc0) drops the CU's vector L1 but not the L2, so a stale count
// there on the other XCD is a stale L2 line that the agent / system acquire
// (buffer_inv sc1 / sc0 sc1) removes. A final pass checks
// kernel boundaries: read kernel (XCD 1), write kernel (XCD 0), read kernel
// (XCD 1) with no fences in any kernel.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/xcd_coherence tools/xcd_coherence.hip
//   timeout -k 10 60 tools/xcd_coherence  > one JSON line
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define GP(T, p) ((__attribute__((address_space(1))) T*)(p))

constexpr int kWords = 4096;          // 16 KiB buffer
constexpr int kThreads = 256;
constexpr uint64_t kTimeout = 50000000;  // 0.5 s of the 100 MHz clock per wait

enum { ACQ_SYSTEM = 0, ACQ_AGENT = 1, ACQ_NONE = 2, ACQ_L1 = 3 };

__device__ __forceinline__ unsigned xcc_id() {
  // HW_REG_XCC_ID (hwreg 20), bits [3:0]
  return __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));
}

__device__ __forceinline__ bool wait_flag(unsigned* f, unsigned v) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < v) {
    __builtin_amdgcn_s_sleep(1);
    if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeout) return false;
  }
  return true;
}

template <bool NT>
__device__ __forceinline__ unsigned read_count(const unsigned* x, unsigned want) {
  unsigned bad = 0;
  for (int i = threadIdx.x; i < kWords / 4; i += blockDim.x) {
    u32x4 v = NT ? __builtin_nontemporal_load(GP(const u32x4, x) + i) : GP(const u32x4, x)[i];
    bad += (v.x != want) + (v.y != want) + (v.z != want) + (v.w != want);
  }
  return bad;
}

// flags[0] = R, flags[1] = W, flags[2] = abort
template <bool NT>
__global__ __launch_bounds__(kThreads) void probe(unsigned* x, unsigned* flags, unsigned* out, int reader_blk,
                                                  int acq, int rounds) {
  __shared__ unsigned s_ok, s_bad;
  const int b = blockIdx.x;
  if (b != 0 && b != reader_blk) return;
  if (threadIdx.x == 0) out[2 + (b == 0 ? 0 : 1)] = xcc_id();
  for (int k = 0; k < rounds; ++k) {
    if (b == reader_blk) {
      // 1. load X (old values) so this XCD's L2 holds the lines
      unsigned c = read_count<NT>(x, (unsigned)k);
      if (threadIdx.x == 0) s_bad = 0;
      __syncthreads();
      atomicAdd(&s_bad, c);  // LDS: consumes the loaded values
      __syncthreads();
      if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(out + 1, s_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // pre-read mismatches
        __hip_atomic_store(flags + 0, (unsigned)(k + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s_ok = wait_flag(flags + 1, k + 1);
        if (s_ok) {
          if (acq == ACQ_SYSTEM) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
          else if (acq == ACQ_AGENT) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          else if (acq == ACQ_L1) asm volatile("buffer_inv sc0\n\ts_waitcnt vmcnt(0)" ::: "memory");  // CU L1 only
        }
      }
      __syncthreads();
      if (!s_ok) {
        if (threadIdx.x == 0) flags[2] = 1;
        return;
      }
      // 2. load X again: every element must be k+1
      c = read_count<NT>(x, (unsigned)(k + 1));
      if (threadIdx.x == 0) s_bad = 0;
      __syncthreads();
      atomicAdd(&s_bad, c);
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_add(out + 0, s_bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
    } else {
      if (threadIdx.x == 0) s_ok = wait_flag(flags + 0, k + 1);
      __syncthreads();
      if (!s_ok) {
        if (threadIdx.x == 0) flags[2] = 1;
        return;
      }
      for (int i = threadIdx.x; i < kWords / 4; i += blockDim.x) {
        u32x4 v = {(unsigned)(k + 1), (unsigned)(k + 1), (unsigned)(k + 1), (unsigned)(k + 1)};
        GP(u32x4, x)[i] = v;
      }
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(flags + 1, (unsigned)(k + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __syncthreads();
    }
  }
}

// kernel-boundary pass: one role per launch, no fences
template <bool NT>
__global__ __launch_bounds__(kThreads) void kb_read(const unsigned* x, unsigned* out, int blk, unsigned want) {
  __shared__ unsigned s_bad;
  if (blockIdx.x != blk) return;
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  atomicAdd(&s_bad, read_count<NT>(x, want));
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] += s_bad;
    out[1] = xcc_id();
  }
}
__global__ __launch_bounds__(kThreads) void kb_write(unsigned* x, int blk, unsigned v, unsigned* out) {
  if (blockIdx.x != blk) return;
  for (int i = threadIdx.x; i < kWords; i += blockDim.x) x[i] = v;
  if (threadIdx.x == 0) out[2] = xcc_id();
}

int main() {
  const int rounds = 200;
  unsigned *x, *flags, *out;
  CK(hipMalloc(&x, kWords * 4));
  CK(hipExtMallocWithFlags((void**)&flags, 64, hipDeviceMallocUncached));
  CK(hipMalloc(&out, 64));
  printf("{");
  const char* acq_name[] = {"system", "agent", "none", "l1only"};
  bool first = true;
  for (int nt = 0; nt < 2; ++nt)
    for (int rb : {1, 8})
      for (int acq = 0; acq < 4; ++acq) {
        CK(hipMemset(x, 0, kWords * 4));
        CK(hipMemset(flags, 0, 64));
        CK(hipMemset(out, 0, 64));
        CK(hipDeviceSynchronize());
        if (nt)
          hipLaunchKernelGGL(probe<true>, dim3(16), dim3(kThreads), 0, 0, x, flags, out, rb, acq, rounds);
        else
          hipLaunchKernelGGL(probe<false>, dim3(16), dim3(kThreads), 0, 0, x, flags, out, rb, acq, rounds);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        unsigned h[4], f[3];
        CK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
        CK(hipMemcpy(f, flags, 12, hipMemcpyDeviceToHost));
        printf("%s\"%s_%s_reader_blk%d\": {\"stale_words\": %u, \"checked_words\": %d, \"pre_read_mismatch\": %u, "
               "\"writer_xcc\": %u, \"reader_xcc\": %u, \"timeout\": %u}",
               first ? "" : ", ", nt ? "nt" : "plain", acq_name[acq], rb, h[0], rounds * kWords, h[1], h[2], h[3],
               f[2]);
        first = false;
      }
  // kernel boundaries
  for (int nt = 0; nt < 2; ++nt) {
    CK(hipMemset(x, 0, kWords * 4));
    CK(hipMemset(out, 0, 64));
    CK(hipDeviceSynchronize());
    for (int k = 0; k < rounds; ++k) {
      if (nt) hipLaunchKernelGGL(kb_read<true>, dim3(16), dim3(kThreads), 0, 0, x, out + 4, 1, (unsigned)k);
      else hipLaunchKernelGGL(kb_read<false>, dim3(16), dim3(kThreads), 0, 0, x, out + 4, 1, (unsigned)k);
      hipLaunchKernelGGL(kb_write, dim3(16), dim3(kThreads), 0, 0, x, 0, (unsigned)(k + 1), out + 4);
    }
    if (nt) hipLaunchKernelGGL(kb_read<true>, dim3(16), dim3(kThreads), 0, 0, x, out + 4, 1, (unsigned)rounds);
    else hipLaunchKernelGGL(kb_read<false>, dim3(16), dim3(kThreads), 0, 0, x, out + 4, 1, (unsigned)rounds);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    unsigned h[8];
    CK(hipMemcpy(h, out, 32, hipMemcpyDeviceToHost));
    printf(", \"kernel_boundary_%s\": {\"stale_words\": %u, \"checked_words\": %d, \"reader_xcc\": %u, "
           "\"writer_xcc\": %u}",
           nt ? "nt" : "plain", h[4], (rounds + 1) * kWords, h[5], h[6]);
  }
  printf("}\n");
  return 0;
}
