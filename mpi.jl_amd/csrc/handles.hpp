// handles.hpp — handle spaces of the objects libmpigx creates itself (user
// ops, derived datatypes) that can never alias a handle libmpi issues.
//
// MPI.jl passes MPICH handle values through its ccalls unchanged (ops and
// datatypes are Cint, deps/consts_mpich.jl:30-72), and a Julia program may hold
// handles from BOTH libraries: MPI.Op(f, T) calls MPI_Op_create in libmpi
// (src/operators.jl:72-88) while a ROCBuffer call goes to libmpigx.  MPICH
// encodes a handle as kind (bits 31-30) | object type (29-26) | payload; the
// only kind-00 ("invalid") handles it ever issues are the *_NULL constants,
// whose payload is zero (MPI_OP_NULL = 0x18000000, MPI_DATATYPE_NULL =
// 0x0c000000, ...).  libmpigx handles are therefore
//     0x3c000000 | sub << 24 | generation << 16 | (slot + 1)
// kind 00, type 0xF, non-zero payload: outside everything MPICH (or an ABI
// following it) hands out.  `sub` separates the object classes; the 8-bit
// generation of a slot is bumped when it is freed, so a stale handle of a
// reused slot is rejected instead of resolving to the new object.  A handle
// that does not resolve is an error (MPI_ERR_OP / MPI_ERR_TYPE) — never some
// other object.
#pragma once
#include <stdint.h>

#include <mutex>
#include <vector>

namespace mpigx {

constexpr int kHandleTag = 0x3c000000;
constexpr int kHandleTagMask = (int)0xfc000000u;
enum HandleSub : int { HS_OP = 0, HS_DATATYPE = 1 };

template <class Obj, int SUB>
class Registry {
 public:
  // Registers o; returns its handle (0 if the 65535 slots are exhausted).
  int add(Obj* o) {
    std::lock_guard<std::mutex> g(mu_);
    size_t i = 0;
    while (i < slot_.size() && slot_[i]) ++i;
    if (i == slot_.size()) {
      if (i >= 0xffff) return 0;
      slot_.push_back(nullptr);
      gen_.push_back(0);
    }
    slot_[i] = o;
    return kHandleTag | (SUB << 24) | ((int)gen_[i] << 16) | (int)(i + 1);
  }
  // The object of handle h, or nullptr (foreign, stale or freed handle).
  Obj* get(int h) const {
    size_t i;
    if (!index_of(h, &i)) return nullptr;
    std::lock_guard<std::mutex> g(mu_);
    return i < slot_.size() && gen_[i] == (uint8_t)(h >> 16) ? slot_[i] : nullptr;
  }
  // Unregisters h and returns its object (nullptr if h does not resolve).
  Obj* remove(int h) {
    size_t i;
    if (!index_of(h, &i)) return nullptr;
    std::lock_guard<std::mutex> g(mu_);
    if (i >= slot_.size() || gen_[i] != (uint8_t)(h >> 16) || !slot_[i]) return nullptr;
    Obj* o = slot_[i];
    slot_[i] = nullptr;
    ++gen_[i];
    return o;
  }
  static bool ours(int h) { return (h & kHandleTagMask) == kHandleTag && ((h >> 24) & 3) == SUB && (h & 0xffff); }

 private:
  static bool index_of(int h, size_t* i) {
    if (!ours(h)) return false;
    *i = (size_t)(h & 0xffff) - 1;
    return true;
  }
  mutable std::mutex mu_;
  std::vector<Obj*> slot_;
  std::vector<uint8_t> gen_;
};

}  // namespace mpigx
