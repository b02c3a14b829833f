// types.cpp — derived datatypes on device buffers:
// the MPI_Type_* constructors MPI.jl's Types module ccalls
// (src/datatypes.jl:62-318) and the pack / unpack kernels that let
// non-contiguous buffers (strided and dense SubArrays, buffers.jl:104-117;
// padded isbits structs, datatypes.jl:269-316) travel through the engine.
//
// Representation.  A committed type is its typemap for ONE instance,
// flattened in typemap order (MPI's pack order, not address order) into
// "runs": {off, len, n, stride} = n blocks of len bytes at off + i*stride.
// Adjacent runs merge when they continue each other, so a vector / a 2-D
// subarray is one run and a k-D subarray prod(subsizes[..k-2]) runs.  Instance
// j of a count lives at j*extent.  lb / extent / true bounds follow MPICH
// 3.3.2 (struct upper bounds padded to the largest component alignment).
//
// Kernel.  pack_kernel<W> maps packed byte p (W-byte units, W = the largest
// power of two <= 16 dividing every offset, length, stride, the extent and
// both base pointers) to its typed address: instance = p / size, run by a
// binary search over the per-instance prefix of packed bytes, block and byte
// inside the run by division.  HBM gather/scatter; used (a) on the sender to
// pack into a contiguous temporary, (b) on the receiver fused with the pull
// over xGMI (contiguous remote source -> typed local destination).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "handles.hpp"
#include "launch.hpp"
#include "runtime.hpp"

using namespace mpigx;

namespace {

constexpr size_t kMaxRuns = 1u << 22;

struct DType {
  bool live = true;
  bool committed = false;
  bool sticky = false;  // resized: bounds are explicit, no alignment padding
  long long lb = 0, ub = 0;
  long long tlb = 0, tub = 0;  // true bounds (data bytes)
  long long size = 0;
  int align = 1;
  int basic = 0;  // the one predefined type every byte belongs to, 0 = mixed
  std::vector<TypeRun> runs;
  struct Dev {
    int device;
    TypeRun* runs;
    long long* pfx;
  };
  std::vector<Dev> devs;
};

std::mutex g_mu;
// derived types live in libmpigx's own handle space (handles.hpp): an MPICH
// derived-type handle (0x8c000000 | k) never resolves here
Registry<DType, HS_DATATYPE> g_types;

DType* lookup(int h) {
  DType* t = g_types.get(h);
  return t && t->live ? t : nullptr;
}

int new_handle(DType* t) { return g_types.add(t); }

int basic_align(int handle, int size) {
  if (handle == MPIGX_C_FLOAT_COMPLEX) return 4;
  if (handle == MPIGX_C_DOUBLE_COMPLEX) return 8;
  return size >= 8 ? 8 : size;
}

// Flattened view of any handle (predefined: one contiguous block).
bool flat_of(int h, DType* out, bool need_commit = false) {
  if (const DType* d = lookup(h)) {
    if (need_commit && !d->committed) return false;
    *out = *d;
    out->devs.clear();
    return true;
  }
  const int s = rt::dtype_size(h);
  if (s < 0) return false;
  *out = DType();
  out->lb = 0;
  out->ub = s;
  out->tlb = 0;
  out->tub = s;
  out->size = s;
  out->align = basic_align(h, s);
  out->basic = h;
  out->committed = true;
  if (s > 0) out->runs.push_back({0, s, 1, s});
  return true;
}

TypeRun norm(TypeRun r) {
  if (r.n > 1 && r.stride == r.len) return {r.off, r.len * r.n, 1, r.len * r.n};
  if (r.n == 1) r.stride = r.len;
  return r;
}

void append(std::vector<TypeRun>& v, TypeRun r) {
  if (r.len <= 0 || r.n <= 0) return;
  r = norm(r);
  if (!v.empty()) {
    TypeRun& l = v.back();
    if (l.n == 1 && r.n == 1 && l.off + l.len == r.off) {  // contiguous blocks
      l.len += r.len;
      l.stride = l.len;
      return;
    }
    if (l.len == r.len) {  // r continues l's progression
      const long long s = l.n == 1 ? r.off - l.off : l.stride;
      if (s != 0 && r.off == l.off + l.n * s && (r.n == 1 || r.stride == s)) {
        l.n += r.n;
        l.stride = s;
        l = norm(l);
        return;
      }
    }
  }
  v.push_back(r);
}

// count copies of f, copy j shifted by j*stride (typemap order).
bool replicate(const DType& f, long long count, long long stride, DType* out) {
  *out = DType();
  out->align = f.align;
  out->basic = f.basic;
  out->size = f.size * count;
  if (count <= 0 || f.size == 0) {
    out->lb = out->ub = out->tlb = out->tub = 0;
    if (count > 0) {
      out->lb = f.lb + std::min(0ll, (count - 1) * stride);
      out->ub = f.ub + std::max(0ll, (count - 1) * stride);
    }
    return true;
  }
  out->lb = f.lb + std::min(0ll, (count - 1) * stride);
  out->ub = f.ub + std::max(0ll, (count - 1) * stride);
  out->tlb = f.tlb + std::min(0ll, (count - 1) * stride);
  out->tub = f.tub + std::max(0ll, (count - 1) * stride);
  if (f.runs.size() == 1) {
    const TypeRun r = f.runs[0];
    if (r.n == 1) {
      append(out->runs, {r.off, r.len, count, stride});
      return true;
    }
    if (stride == r.n * r.stride) {
      append(out->runs, {r.off, r.len, r.n * count, r.stride});
      return true;
    }
  }
  if ((size_t)count * f.runs.size() > kMaxRuns) return false;
  for (long long j = 0; j < count; ++j)
    for (const TypeRun& r : f.runs) {
      append(out->runs, {r.off + j * stride, r.len, r.n, r.stride});
      if (out->runs.size() > kMaxRuns) return false;
    }
  return true;
}

void shift(DType* t, long long d) {
  for (auto& r : t->runs) r.off += d;
  t->lb += d;
  t->ub += d;
  t->tlb += d;
  t->tub += d;
}

int finish_new(DType* t, int* out) {
  if (!out) {
    delete t;
    return MPIGX_ERR_ARG;
  }
  *out = new_handle(t);
  return MPIGX_SUCCESS;
}

// Device copy of the runs + per-instance packed-byte prefix.
int device_runs(DType* t, int device, const TypeRun** runs, const long long** pfx) {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& d : t->devs)
    if (d.device == device) {
      *runs = d.runs;
      *pfx = d.pfx;
      return MPIGX_SUCCESS;
    }
  const size_t nr = t->runs.size();
  std::vector<long long> p(nr + 1, 0);
  for (size_t i = 0; i < nr; ++i) p[i + 1] = p[i] + t->runs[i].len * t->runs[i].n;
  DType::Dev d{device, nullptr, nullptr};
  if (hipMalloc(&d.runs, std::max<size_t>(1, nr) * sizeof(TypeRun)) != hipSuccess ||
      hipMalloc(&d.pfx, (nr + 1) * sizeof(long long)) != hipSuccess ||
      (nr && hipMemcpy(d.runs, t->runs.data(), nr * sizeof(TypeRun), hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(d.pfx, p.data(), (nr + 1) * sizeof(long long), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipGetLastError();
    return MPIGX_ERR_INTERN;
  }
  t->devs.push_back(d);
  *runs = d.runs;
  *pfx = d.pfx;
  return MPIGX_SUCCESS;
}

int unit_of(const DType& t, const void* a, const void* b, long long bytes) {
  unsigned long long g = (unsigned long long)(t.ub - t.lb) | (unsigned long long)t.size |
                         (unsigned long long)(uintptr_t)a | (unsigned long long)(uintptr_t)b |
                         (unsigned long long)bytes | 16ull;
  for (const auto& r : t.runs) g |= (unsigned long long)r.off | (unsigned long long)r.len |
                                   (r.n > 1 ? (unsigned long long)r.stride : 0ull);
  return (int)(g & (~g + 1));  // lowest set bit, <= 16
}

}  // namespace

// ---------------------------------------------------------------------------
// runtime services (runtime.hpp)
// ---------------------------------------------------------------------------
namespace mpigx {
namespace rt {

int type_info(int h, TypeDesc* d) {
  if (const DType* t = lookup(h)) {
    if (!t->committed) return MPIGX_ERR_TYPE;
    d->size = t->size;
    d->extent = t->ub - t->lb;
    d->basic = t->basic;
    d->derived = true;
    d->contig = t->size == 0 || (t->lb == 0 && t->runs.size() == 1 && t->runs[0].n == 1 && t->runs[0].off == 0 &&
                                 t->runs[0].len == t->size && d->extent == t->size);
    return MPIGX_SUCCESS;
  }
  const int s = dtype_size(h);
  if (s < 0) return MPIGX_ERR_TYPE;
  d->size = s;
  d->extent = s;
  d->basic = h;
  d->derived = false;
  d->contig = true;
  return MPIGX_SUCCESS;
}

int type_pack(int h, const void* typed, long long count, void* contig, long long bytes, int unpack, int device,
              hipStream_t s) {
  DType* t = lookup(h);
  if (!t || !t->committed) return MPIGX_ERR_TYPE;
  if (bytes > count * t->size) bytes = count * t->size;
  if (bytes <= 0) return MPIGX_SUCCESS;
  PackArgs a;
  memset(&a, 0, sizeof a);
  int rc = device_runs(t, device, &a.runs, &a.pfx);
  if (rc) return rc;
  a.nruns = (int)t->runs.size();
  a.w = unit_of(*t, typed, contig, bytes);
  a.unpack = unpack;
  a.coherent = pull_fences();
  a.size = t->size;
  a.extent = t->ub - t->lb;
  a.units = bytes / a.w;
  // typemap displacements are relative to the buffer pointer
  a.typed = (char*)typed;
  a.contig = (char*)contig;
  return launch_pack(s, a) == hipSuccess ? MPIGX_SUCCESS : MPIGX_ERR_INTERN;
}

}  // namespace rt
}  // namespace mpigx

// ===========================================================================
// C ABI (include/mpigx.h, derived datatypes)
// ===========================================================================
extern "C" {

int mpigx_type_contiguous(int count, int oldtype, int* newtype) {
  if (count < 0) return MPIGX_ERR_COUNT;
  DType f;
  if (!flat_of(oldtype, &f)) return MPIGX_ERR_TYPE;
  DType* t = new DType();
  if (!replicate(f, count, f.ub - f.lb, t)) {
    delete t;
    return MPIGX_ERR_NO_MEM;
  }
  return finish_new(t, newtype);
}

static int hvector(int count, int blocklength, long long stride_bytes, int oldtype, int* newtype) {
  if (count < 0 || blocklength < 0) return MPIGX_ERR_COUNT;
  DType f, blk;
  if (!flat_of(oldtype, &f)) return MPIGX_ERR_TYPE;
  if (!replicate(f, blocklength, f.ub - f.lb, &blk)) return MPIGX_ERR_NO_MEM;
  DType* t = new DType();
  if (!replicate(blk, count, stride_bytes, t)) {
    delete t;
    return MPIGX_ERR_NO_MEM;
  }
  return finish_new(t, newtype);
}

int mpigx_type_vector(int count, int blocklength, int stride, int oldtype, int* newtype) {
  DType f;
  if (!flat_of(oldtype, &f)) return MPIGX_ERR_TYPE;
  return hvector(count, blocklength, (long long)stride * (f.ub - f.lb), oldtype, newtype);
}

int mpigx_type_create_hvector(int count, int blocklength, long long stride, int oldtype, int* newtype) {
  return hvector(count, blocklength, stride, oldtype, newtype);
}

int mpigx_type_create_subarray(int ndims, const int* sizes, const int* subsizes, const int* starts, int order,
                               int oldtype, int* newtype) {
  if (ndims <= 0 || !sizes || !subsizes || !starts) return MPIGX_ERR_ARG;
  if (order != MPIGX_ORDER_C && order != MPIGX_ORDER_FORTRAN) return MPIGX_ERR_ARG;
  for (int d = 0; d < ndims; ++d)
    if (sizes[d] <= 0 || subsizes[d] <= 0 || starts[d] < 0 || subsizes[d] + starts[d] > sizes[d])
      return MPIGX_ERR_ARG;
  DType f;
  if (!flat_of(oldtype, &f)) return MPIGX_ERR_TYPE;
  const long long ext = f.ub - f.lb;
  // dimension order from fastest to slowest varying
  std::vector<int> dims(ndims);
  for (int i = 0; i < ndims; ++i) dims[i] = order == MPIGX_ORDER_C ? ndims - 1 - i : i;
  DType cur = f;
  long long stride = ext, disp = 0;
  for (int i = 0; i < ndims; ++i) {
    const int d = dims[i];
    DType nxt;
    if (!replicate(cur, subsizes[d], stride, &nxt)) return MPIGX_ERR_NO_MEM;
    disp += (long long)starts[d] * stride;
    stride *= sizes[d];
    cur = nxt;
  }
  shift(&cur, disp);
  DType* t = new DType(cur);
  // MPI: a subarray has lb 0 and the extent of the full array
  t->lb = 0;
  t->ub = stride;
  t->sticky = true;
  return finish_new(t, newtype);
}

int mpigx_type_create_struct(int count, const int* blocklengths, const long long* displacements, const int* types,
                             int* newtype) {
  if (count < 0) return MPIGX_ERR_COUNT;
  if (count > 0 && (!blocklengths || !displacements || !types)) return MPIGX_ERR_ARG;
  DType* t = new DType();
  bool first = true, sticky = false;
  int basic = 0;
  bool mixed = false;
  for (int i = 0; i < count; ++i) {
    DType f, rep;
    if (!flat_of(types[i], &f)) {
      delete t;
      return MPIGX_ERR_TYPE;
    }
    if (blocklengths[i] < 0) {
      delete t;
      return MPIGX_ERR_COUNT;
    }
    if (blocklengths[i] == 0) continue;
    if (!replicate(f, blocklengths[i], f.ub - f.lb, &rep)) {
      delete t;
      return MPIGX_ERR_NO_MEM;
    }
    shift(&rep, displacements[i]);
    sticky |= f.sticky;
    t->align = std::max(t->align, f.align);
    if (rep.size > 0) {
      if (basic == 0 && !mixed) basic = f.basic;
      else if (f.basic != basic) mixed = true;
    }
    for (const auto& r : rep.runs) {
      append(t->runs, r);
      if (t->runs.size() > kMaxRuns) {
        delete t;
        return MPIGX_ERR_NO_MEM;
      }
    }
    if (first) {
      t->lb = rep.lb;
      t->ub = rep.ub;
      t->tlb = rep.tlb;
      t->tub = rep.tub;
      first = false;
    } else {
      t->lb = std::min(t->lb, rep.lb);
      t->ub = std::max(t->ub, rep.ub);
      if (rep.size > 0) {
        t->tlb = t->size > 0 ? std::min(t->tlb, rep.tlb) : rep.tlb;
        t->tub = t->size > 0 ? std::max(t->tub, rep.tub) : rep.tub;
      }
    }
    t->size += rep.size;
  }
  t->basic = mixed ? 0 : basic;
  if (!sticky && t->align > 1) {  // MPICH: pad the upper bound to the alignment (epsilon)
    const long long e = t->ub - t->lb, a = t->align;
    t->ub = t->lb + (e + a - 1) / a * a;
  }
  t->sticky = sticky;
  return finish_new(t, newtype);
}

int mpigx_type_create_resized(int oldtype, long long lb, long long extent, int* newtype) {
  DType f;
  if (!flat_of(oldtype, &f)) return MPIGX_ERR_TYPE;
  DType* t = new DType(f);
  t->devs.clear();
  t->committed = false;
  t->lb = lb;
  t->ub = lb + extent;
  t->sticky = true;
  return finish_new(t, newtype);
}

int mpigx_type_commit(int* datatype) {
  if (!datatype) return MPIGX_ERR_ARG;
  if (rt::dtype_size(*datatype) >= 0) return MPIGX_SUCCESS;  // predefined
  DType* t = lookup(*datatype);
  if (!t) return MPIGX_ERR_TYPE;
  t->committed = true;
  return MPIGX_SUCCESS;
}

int mpigx_type_free(int* datatype) {
  if (!datatype) return MPIGX_ERR_ARG;
  DType* t = lookup(*datatype);
  if (!t) return MPIGX_ERR_TYPE;  // predefined types cannot be freed
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& d : t->devs) {
    (void)hipFree(d.runs);
    (void)hipFree(d.pfx);
  }
  g_types.remove(*datatype);
  delete t;
  *datatype = 0x0c000000;  // MPI_DATATYPE_NULL
  return MPIGX_SUCCESS;
}

int mpigx_type_get_extent(int datatype, long long* lb, long long* extent) {
  DType f;
  if (!flat_of(datatype, &f)) return MPIGX_ERR_TYPE;
  if (lb) *lb = f.lb;
  if (extent) *extent = f.ub - f.lb;
  return MPIGX_SUCCESS;
}

int mpigx_type_get_true_extent(int datatype, long long* true_lb, long long* true_extent) {
  DType f;
  if (!flat_of(datatype, &f)) return MPIGX_ERR_TYPE;
  if (true_lb) *true_lb = f.tlb;
  if (true_extent) *true_extent = f.tub - f.tlb;
  return MPIGX_SUCCESS;
}

int mpigx_type_size_x(int datatype, long long* size) {
  DType f;
  if (!flat_of(datatype, &f)) return MPIGX_ERR_TYPE;
  if (size) *size = f.size;
  return MPIGX_SUCCESS;
}

int mpigx_pack_size(int incount, int datatype, long long* size) {
  if (incount < 0) return MPIGX_ERR_COUNT;
  DType f;
  if (!flat_of(datatype, &f)) return MPIGX_ERR_TYPE;
  if (size) *size = f.size * incount;
  return MPIGX_SUCCESS;
}

static int pack_common(int datatype, void* typed, int count, void* contig, long long room, long long* position,
                       int unpack, void* stream) {
  if (count < 0) return MPIGX_ERR_COUNT;
  if (!position) return MPIGX_ERR_ARG;
  rt::TypeDesc d;
  int rc = rt::type_info(datatype, &d);
  if (rc) return rc;
  const long long bytes = d.size * count;
  if (*position < 0 || *position + bytes > room) return MPIGX_ERR_TRUNCATE;
  if (bytes == 0) return MPIGX_SUCCESS;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return MPIGX_ERR_INTERN;
  hipStream_t s = (hipStream_t)stream;
  char* c = (char*)contig + *position;
  if (!d.derived || d.contig) {
    if ((unpack ? hipMemcpyAsync(typed, c, bytes, hipMemcpyDeviceToDevice, s)
                : hipMemcpyAsync(c, typed, bytes, hipMemcpyDeviceToDevice, s)) != hipSuccess) {
      (void)hipGetLastError();
      return MPIGX_ERR_INTERN;
    }
  } else {
    rc = rt::type_pack(datatype, typed, count, c, bytes, unpack, dev, s);
    if (rc) return rc;
  }
  if (hipStreamSynchronize(s) != hipSuccess) {
    (void)hipGetLastError();
    return MPIGX_ERR_INTERN;
  }
  *position += bytes;
  return MPIGX_SUCCESS;
}

int mpigx_pack(const void* inbuf, int incount, int datatype, void* outbuf, long long outsize, long long* position,
               void* stream) {
  return pack_common(datatype, (void*)inbuf, incount, outbuf, outsize, position, 0, stream);
}

int mpigx_unpack(const void* inbuf, long long insize, long long* position, void* outbuf, int outcount, int datatype,
                 void* stream) {
  return pack_common(datatype, outbuf, outcount, (void*)inbuf, insize, position, 1, stream);
}

}  // extern "C"
