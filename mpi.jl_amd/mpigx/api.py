"""MPI.jl's collective API surface: device buffers -> libmpigx, host -> libmpi.

This is the host-side mirror of the reference's plugin point.  Julia is absent
from this image, so the MPI.jl wrappers that north_star keeps (src/comm.jl,
src/buffers.jl, src/datatypes.jl, src/operators.jl, src/collective.jl) are
restated in Python with the same names (`!` becomes a trailing `_`), the same
argument meaning, defaults and error behaviour:

* argument checks are the reference's `@assert_minlength` / `@assert`
  (buffers.jl:25-31) and raise ``AssertionError``;
* non-zero return codes raise :class:`MPIError` like ``@mpichk``
  (error.jl:5-8);
* IN_PLACE, ``nothing``-recvbuf on non-roots, count defaults and the
  allocating/scalar forms follow collective.jl line by line (cited per
  function).

Dispatch is the one MPI.jl performs with CuArrays (src/cuda.jl): device
buffers (torch tensors on a ROCm device — the ``ROCBuffer`` role of SURVEY.md
§7 step 7) go to ``mpigx_<coll>`` in libmpigx.so; host numpy arrays keep going
to ``MPI_<Coll>`` in libmpi (hostmpi.py).  Both receive the *same* argument
list — that identity is the drop-in boundary.  The Julia glue that does the
same for MPI.jl is mpi.jl_amd/julia/MPIGX.jl.
"""
from __future__ import annotations

import ctypes
import operator
import os
import time

import numpy as np

from . import consts as C
from . import hostmpi
from ._lib import UniqueId, lib

IN_PLACE = object()  # MPI_IN_PLACE sentinel (consts_mpich.jl:105)
_IN_PLACE_PTR = ctypes.c_void_p(-1 & ((1 << 64) - 1))


class MPIError(Exception):
    """error.jl:1-19: an MPI error code with its error string."""

    def __init__(self, code: int):
        self.code = code
        super().__init__(f"MPIError({code}): {error_string(code)}")


def error_string(code: int) -> str:
    buf = ctypes.create_string_buffer(512)
    n = ctypes.c_int(0)
    lib().mpigx_error_string(code, buf, ctypes.byref(n))
    return buf.value.decode()


def _check(rc: int):
    if rc != C.MPI_SUCCESS:
        raise MPIError(rc)


def Error_class(code: int) -> int:
    """MPI_Error_class.  libmpigx returns classes already (and a class is
    its own code); host libmpi codes are decoded by libmpi."""
    if _state["host"]:
        out = ctypes.c_int()
        hostmpi.lib().MPI_Error_class(int(code), ctypes.byref(out))
        return out.value
    return int(code)


# ---------------------------------------------------------------------------
# Datatype (src/datatypes.jl:16-60, 269-292)
# ---------------------------------------------------------------------------
class Datatype:
    """`val`: the handle libmpigx takes (MPICH's predefined values; derived
    types: libmpigx's own, types.cpp); `host_val`: the host libmpi handle of a
    derived type (same value for predefined types)."""
    __slots__ = ("val", "name", "host_val")

    def __init__(self, T, name=None, host_val=None):
        if isinstance(T, Datatype):
            self.val, self.name, self.host_val = T.val, T.name, T.host_val
            return
        if isinstance(T, int) and name is not None:
            self.val, self.name, self.host_val = T, name, host_val
            return
        dt = _datatype_of(T)
        self.val, self.name, self.host_val = dt.val, dt.name, dt.host_val

    @property
    def host(self):
        """Handle for host libmpi."""
        return self.val if self.host_val is None else self.host_val

    def __eq__(self, o):
        return isinstance(o, Datatype) and o.val == self.val

    def __hash__(self):
        return hash(self.val)

    def __repr__(self):
        return f"MPI.Datatype({self.name})"


def _mk(name, val):
    return Datatype(val, name)


INT8_T, UINT8_T = _mk("INT8_T", C.MPI_INT8_T), _mk("UINT8_T", C.MPI_UINT8_T)
INT16_T, UINT16_T = _mk("INT16_T", C.MPI_INT16_T), _mk("UINT16_T", C.MPI_UINT16_T)
INT32_T, UINT32_T = _mk("INT32_T", C.MPI_INT32_T), _mk("UINT32_T", C.MPI_UINT32_T)
INT64_T, UINT64_T = _mk("INT64_T", C.MPI_INT64_T), _mk("UINT64_T", C.MPI_UINT64_T)
BYTE, CHAR, WCHAR = _mk("BYTE", C.MPI_BYTE), _mk("CHAR", C.MPI_CHAR), _mk("WCHAR", C.MPI_WCHAR)
FLOAT, DOUBLE = _mk("FLOAT", C.MPI_FLOAT), _mk("DOUBLE", C.MPI_DOUBLE)
C_FLOAT_COMPLEX, C_DOUBLE_COMPLEX = _mk("C_FLOAT_COMPLEX", C.MPI_C_FLOAT_COMPLEX), _mk(
    "C_DOUBLE_COMPLEX", C.MPI_C_DOUBLE_COMPLEX)
BFLOAT16 = _mk("BFLOAT16", C.MPIGX_BFLOAT16)
_BY_VAL = {d.val: d for d in (INT8_T, UINT8_T, INT16_T, UINT16_T, INT32_T, UINT32_T, INT64_T, UINT64_T, BYTE,
                              CHAR, WCHAR, FLOAT, DOUBLE, C_FLOAT_COMPLEX, C_DOUBLE_COMPLEX, BFLOAT16)}


def _torch():
    import torch
    return torch


def _datatype_of(T) -> Datatype:
    """Datatype(T) for torch / numpy dtypes and Python scalar types
    (datatypes.jl:29-60).  Unnamed 1/2/4/8-byte primitives go by size to
    UINT8/16/32/64_T exactly as datatypes.jl:281-284 does (so float16 and bool
    are integer bit patterns, as in the reference); torch.bfloat16 gets the
    BFLOAT16 extension."""
    if T is int:
        return INT64_T
    if T is float:
        return DOUBLE
    if T is complex:
        return C_DOUBLE_COMPLEX
    if T is bool:
        return UINT8_T
    if isinstance(T, np.dtype) or (isinstance(T, type) and issubclass(T, np.generic)):
        if np.dtype(T).fields is not None or np.dtype(T).kind == "V":
            from .types import struct_datatype  # isbits structs / primitive types (datatypes.jl:269-316)
            return struct_datatype(np.dtype(T))
        h = hostmpi.HANDLE_OF_NP.get(np.dtype(T))
        if h is None:
            raise TypeError(f"no MPI datatype for {T!r}")
        return _BY_VAL[h]
    torch = _torch()
    table = {
        torch.int8: INT8_T, torch.uint8: UINT8_T, torch.int16: INT16_T, torch.int32: INT32_T,
        torch.int64: INT64_T, torch.float32: FLOAT, torch.float64: DOUBLE,
        torch.complex64: C_FLOAT_COMPLEX, torch.complex128: C_DOUBLE_COMPLEX,
        torch.bfloat16: BFLOAT16, torch.float16: UINT16_T, torch.bool: UINT8_T,
    }
    for nm, dt in (("uint16", UINT16_T), ("uint32", UINT32_T), ("uint64", UINT64_T)):
        if hasattr(torch, nm):
            table[getattr(torch, nm)] = dt
    if T in table:
        return table[T]
    raise TypeError(f"no MPI datatype for {T!r}")


_INTEGER = ("int8", "uint8", "int16", "uint16", "int32", "uint32", "int64", "uint64")
_FLOAT = ("float32", "float64", "bfloat16")
_COMPLEX = ("complex64", "complex128")


def _kind(T) -> str:
    if isinstance(T, np.dtype):
        T = T.name
    name = str(T).replace("torch.", "")
    if T is int or name in _INTEGER:
        return "int"
    if T is float or name in _FLOAT:
        return "float"
    if T is complex or name in _COMPLEX:
        return "complex"
    return "other"


# ---------------------------------------------------------------------------
# Op (src/operators.jl)
# ---------------------------------------------------------------------------
class Op:
    """Built-in op handle, or a user function (OpWrapper, operators.jl:56-88).

    `fptr` mirrors MPI.jl's `Op.fptr` (operators.jl:20, :77-79): the
    MPI_User_function of an op created in libmpi (`libmpi_op`); a device-buffer
    call re-registers it with libmpigx (`_op_val`)."""
    __slots__ = ("val", "name", "fn", "iscommutative", "fptr")

    def __init__(self, f, T=None, iscommutative=False, *, _val=None, _name=None, _fptr=None):
        self.fptr = _fptr
        if _val is not None:
            self.val, self.name, self.fn = _val, _name, None
            self.iscommutative = True if _fptr is None else bool(iscommutative)
            return
        if isinstance(f, Op):
            self.val, self.name, self.fn, self.iscommutative = f.val, f.name, f.fn, f.iscommutative
            self.fptr = f.fptr
            return
        b = _builtin_for(f, T)
        if b is not None:
            self.val, self.name, self.fn, self.iscommutative = b.val, b.name, None, True
        else:
            # user-defined: inout[i] = f(in[i], inout[i]) (operators.jl:60-69)
            self.val, self.name, self.fn, self.iscommutative = None, getattr(f, "__name__", "user"), f, iscommutative

    def __repr__(self):
        return f"MPI.Op({self.name})"


def _op(name, val):
    return Op(None, _val=val, _name=name)


def libmpi_op(handle, fptr, iscommutative=False, name="libmpi"):
    """An op as MPI.jl's `MPI.Op(f, T)` holds it (operators.jl:72-88): the
    handle libmpi's MPI_Op_create returned and the MPI_User_function pointer
    (a ctypes USER_FN object or a raw address) it was created from."""
    return Op(None, None, iscommutative, _val=int(handle), _name=name, _fptr=fptr)


OP_NULL = _op("OP_NULL", C.MPI_OP_NULL)
BAND, BOR, BXOR = _op("BAND", C.MPI_BAND), _op("BOR", C.MPI_BOR), _op("BXOR", C.MPI_BXOR)
LAND, LOR, LXOR = _op("LAND", C.MPI_LAND), _op("LOR", C.MPI_LOR), _op("LXOR", C.MPI_LXOR)
MAX, MIN = _op("MAX", C.MPI_MAX), _op("MIN", C.MPI_MIN)
PROD, SUM = _op("PROD", C.MPI_PROD), _op("SUM", C.MPI_SUM)
REPLACE, NO_OP = _op("REPLACE", C.MPI_REPLACE), _op("NO_OP", C.MPI_NO_OP)


def _builtin_for(f, T):
    """operators.jl:39-45: min/max/+/* for numbers, &,|,xor for integers."""
    k = _kind(T) if T is not None else "any"
    num = k in ("int", "float", "any")
    if f is min and num:
        return MIN
    if f is max and num:
        return MAX
    if f is operator.add and (num or k == "complex"):
        return SUM
    if f is operator.mul and (num or k == "complex"):
        return PROD
    if k in ("int", "any"):
        if f is operator.and_:
            return BAND
        if f is operator.or_:
            return BOR
        if f is operator.xor:
            return BXOR
    return None


def _as_op(op, T) -> Op:
    if isinstance(op, Op):
        return op
    return Op(op, T)


# ---------------------------------------------------------------------------
# Buffer (src/buffers.jl:78-127)
# ---------------------------------------------------------------------------
class Buffer:
    """MPI.Buffer(data, count, datatype): array + count + Datatype."""
    __slots__ = ("data", "count", "datatype")

    def __init__(self, data, count=None, datatype=None):
        if isinstance(data, Buffer):
            self.data, self.count, self.datatype = data.data, data.count, data.datatype
            return
        if count is None and datatype is None and _noncontiguous(data):
            # buffers.jl:104-117: strided / dense sub-arrays become one
            # element of a vector / subarray datatype
            from .types import view_buffer
            self.data, self.count, self.datatype = view_buffer(data)
            return
        self.data = data
        self.count = int(count if count is not None else _len(data))
        self.datatype = Datatype(datatype if datatype is not None else data.dtype)


def _unwrap(buf):
    return buf.data if isinstance(buf, Buffer) else buf


def _is_host(buf):
    return isinstance(_unwrap(buf), np.ndarray)


def _noncontiguous(a):
    if isinstance(a, np.ndarray):
        return not a.flags.c_contiguous
    return hasattr(a, "is_contiguous") and not a.is_contiguous()


def _ptr(buf):
    if buf is None:
        return None
    if buf is IN_PLACE:
        return _IN_PLACE_PTR
    if isinstance(buf, Buffer) and _noncontiguous(buf.data):  # typed by its datatype
        d = buf.data
        return ctypes.c_void_p(d.ctypes.data if isinstance(d, np.ndarray) else d.data_ptr())
    b = _unwrap(buf)
    if isinstance(b, np.ndarray):
        if not b.flags.c_contiguous:
            raise ValueError("non-contiguous buffers need derived datatypes (out of scope)")
        return ctypes.c_void_p(b.ctypes.data)
    if not getattr(b, "is_cuda", False):
        raise TypeError("buffers must be numpy arrays (host, libmpi) or ROCm tensors (device, libmpigx)")
    if not b.is_contiguous():
        raise ValueError("non-contiguous device buffers need derived datatypes (SURVEY.md §8f, out of scope)")
    return ctypes.c_void_p(b.data_ptr())


def _len(buf):
    if isinstance(buf, Buffer):
        return buf.count
    return buf.size if isinstance(buf, np.ndarray) else buf.numel()


def _eltype(buf):
    if isinstance(buf, Buffer):
        return buf.datatype
    return Datatype(buf.dtype)


def _assert_minlength(buf, count):
    """buffers.jl:25-31: only array buffers are checked (not MPI.Buffer)."""
    if buf is not None and buf is not IN_PLACE and not isinstance(buf, Buffer):
        assert _len(buf) >= count, f"buffer length {_len(buf)} < count {count}"


def _is_array(x):
    return isinstance(x, (np.ndarray, Buffer)) or hasattr(x, "numel")


def _empty_like(buf, count=None):
    b = _unwrap(buf)
    if isinstance(b, np.ndarray):
        return np.empty(b.shape if count is None else (count,), dtype=b.dtype)
    torch = _torch()
    return torch.empty_like(b) if count is None else torch.empty(count, dtype=b.dtype, device=b.device)


def _dtype(buf):
    return getattr(_unwrap(buf), "dtype", None)


# ---------------------------------------------------------------------------
# Comm (src/comm.jl) + environment (src/environment.jl)
# ---------------------------------------------------------------------------
class Comm:
    """`val` = libmpigx communicator (device buffers), `host` = libmpi MPI_Comm
    handle (host buffers); either may be None."""
    __slots__ = ("val", "host", "_rank", "_size", "device")

    def __init__(self, handle, rank, size, device, host=None):
        self.val, self._rank, self._size, self.device, self.host = handle, rank, size, device, host

    def __repr__(self):
        return f"MPI.Comm(rank={self._rank}, size={self._size}, device={self.device})"


COMM_WORLD = None
_state = {"init": False, "final": False, "pg_owned": False, "host": False}


def _env_int(*names, default=None):
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            return int(v)
    return default


def _bootstrap_id(rank, size, host_comm=None):
    """Distribute rank 0's mpigx unique id: host MPI_Bcast when libmpi is up
    (what the Julia glue does), else torch.distributed (gloo)."""
    uid = UniqueId()
    if rank == 0:
        _check(lib().mpigx_get_unique_id(ctypes.byref(uid)))
    if size == 1:
        return uid
    raw = ctypes.string_at(ctypes.addressof(uid), 128)
    if host_comm is not None:
        raw = hostmpi.bcast_bytes(raw, 0, host_comm)
    else:
        import torch.distributed as dist
        if not dist.is_initialized():
            dist.init_process_group("gloo", rank=rank, world_size=size)
            _state["pg_owned"] = True
        obj = [raw if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        raw = obj[0]
    ctypes.memmove(ctypes.addressof(uid), bytes(raw), 128)
    return uid


def Init(threadlevel=None):
    """environment.jl:80: Init binds this rank to its GPU and builds COMM_WORLD.

    Rank/size come from the launcher (hydra/mpiexec PMI_RANK/PMI_SIZE, which
    also brings up host libmpi, or torchrun RANK/WORLD_SIZE/LOCAL_RANK);
    device = MPIGX_DEVICE or the node-local rank mod visible devices
    (comm.jl:107 Comm_split_type(SHARED)).  Without a ROCm device (or with
    MPIGX_HOST_ONLY=1) only the host (libmpi) side exists.
    """
    global COMM_WORLD
    if _state["init"]:
        raise AssertionError("MPI.Init called twice")
    host = None
    if hostmpi.available():
        rank, size = hostmpi.init()
        host = C.MPI_COMM_WORLD
        _state["host"] = True
    else:
        rank = _env_int("RANK", "PMI_RANK", "OMPI_COMM_WORLD_RANK", default=0)
        size = _env_int("WORLD_SIZE", "PMI_SIZE", "OMPI_COMM_WORLD_SIZE", default=1)
    local = _env_int("LOCAL_RANK", "MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", default=rank)
    ndev = 0
    if os.environ.get("MPIGX_HOST_ONLY") != "1":
        ndev = _torch().cuda.device_count()
    handle, device = None, None
    if ndev > 0:
        device = _env_int("MPIGX_DEVICE", default=local % ndev)
        _torch().cuda.set_device(device)
        uid = _bootstrap_id(rank, size, host)
        h = ctypes.c_void_p()
        _check(lib().mpigx_comm_init_rank(ctypes.byref(h), size, ctypes.byref(uid), rank, device))
        handle = h
    elif host is None:
        raise RuntimeError("mpigx: no ROCm device and no host libmpi (start under mpiexec for host buffers)")
    COMM_WORLD = Comm(handle, rank, size, device, host)
    _state["init"] = True
    return COMM_WORLD


# environment.jl:111-116 ThreadLevel (MPICH values)
THREAD_SINGLE, THREAD_FUNNELED, THREAD_SERIALIZED, THREAD_MULTIPLE = 0, 1, 2, 3


def Init_thread(required):
    """environment.jl:142-162: Init, then the provided thread level — the
    engine's (mpigx_query_thread: THREAD_MULTIPLE) and, under mpiexec, host
    libmpi's, whichever is lower; a warning when it is below `required`."""
    Init()
    p = ctypes.c_int(THREAD_SINGLE)
    if COMM_WORLD is not None and COMM_WORLD.val:
        _check(lib().mpigx_query_thread(ctypes.byref(p)))
    else:
        p.value = THREAD_MULTIPLE
    provided = min(p.value, hostmpi.query_thread()) if _state["host"] and hasattr(hostmpi, "query_thread") \
        else p.value
    if provided < required:
        import warnings
        warnings.warn(f"Thread level requested = {required}, provided = {provided}")
    _state["thread"] = provided
    return provided


def Query_thread():
    """environment.jl:174-180"""
    return _state.get("thread", THREAD_SINGLE)


def Is_thread_main():
    """environment.jl:190-196: the thread that initialized MPI."""
    import threading
    return threading.current_thread() is threading.main_thread()


def Initialized():
    return _state["init"]


def Finalized():
    return _state["final"]


def Finalize():
    global COMM_WORLD
    if COMM_WORLD is not None and COMM_WORLD.val:
        _check(lib().mpigx_comm_free(COMM_WORLD.val))
    COMM_WORLD = None
    if _state["pg_owned"]:
        import torch.distributed as dist
        dist.destroy_process_group()
        _state["pg_owned"] = False
    if _state["host"]:
        hostmpi.finalize()
    _state["final"] = True


def Wtime():
    return time.perf_counter()


def has_rocm():
    """has_cuda() analogue (environment.jl:308-323): device buffers supported.
    JULIA_MPI_HAS_ROCM=true/false overrides, as JULIA_MPI_HAS_CUDA does there."""
    flag = os.environ.get("JULIA_MPI_HAS_ROCM")
    if flag is not None:
        return flag.strip().lower() in ("true", "1", "yes")
    try:
        lib()
        return _torch().cuda.is_available()
    except Exception:
        return False


def Comm_rank(comm: Comm) -> int:
    return comm._rank


def Comm_size(comm: Comm) -> int:
    return comm._size


def Comm_dup(comm: Comm) -> Comm:
    """comm.jl:78: a new communicator over the same ranks (own arenas/epochs).
    The unique id is broadcast over `comm` itself (host libmpi, or the engine)."""
    uid = UniqueId()
    if comm._rank == 0:
        _check(lib().mpigx_get_unique_id(ctypes.byref(uid)))
    raw = ctypes.string_at(ctypes.addressof(uid), 128)
    if comm.host is not None:
        raw = hostmpi.bcast_bytes(raw, 0, comm.host)
    elif comm.val:
        torch = _torch()
        t = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(f"cuda:{comm.device}")
        Bcast_(t, 0, comm)
        raw = bytes(t.cpu().numpy().tobytes())
    ctypes.memmove(ctypes.addressof(uid), raw, 128)
    h = None
    if comm.val:
        h = ctypes.c_void_p()
        _check(lib().mpigx_comm_init_rank(ctypes.byref(h), comm._size, ctypes.byref(uid), comm._rank, comm.device))
    return Comm(h, comm._rank, comm._size, comm.device, comm.host)


def Comm_split(comm: Comm, color, key) -> Comm:
    """comm.jl:92-105: color None (`nothing`) = MPI_UNDEFINED -> COMM_NULL (None)."""
    col = C.MPI_UNDEFINED if color is None else int(color)
    host = None
    if comm.host is not None:
        hc = ctypes.c_int(0)
        _check(hostmpi.lib().MPI_Comm_split(comm.host, col, int(key), ctypes.byref(hc)))
        host = hc.value if hc.value != C.MPI_COMM_NULL else None
    h = None
    rank = size = None
    if comm.val:
        hv = ctypes.c_void_p()
        _check(lib().mpigx_comm_split(comm.val, col, int(key), ctypes.byref(hv)))
        if hv.value:
            h = hv
            r, s = ctypes.c_int(), ctypes.c_int()
            lib().mpigx_comm_rank(h, ctypes.byref(r))
            lib().mpigx_comm_size(h, ctypes.byref(s))
            rank, size = r.value, s.value
    if host is not None and rank is None:
        r, s = ctypes.c_int(), ctypes.c_int()
        hostmpi.lib().MPI_Comm_rank(host, ctypes.byref(r))
        hostmpi.lib().MPI_Comm_size(host, ctypes.byref(s))
        rank, size = r.value, s.value
    if h is None and host is None:
        return None
    return Comm(h, rank, size, comm.device, host)


def Comm_split_type(comm: Comm, split_type, key, info=None) -> Comm:
    """comm.jl:107: COMM_TYPE_SHARED on one node is every rank."""
    if split_type != C.MPI_COMM_TYPE_SHARED:
        raise MPIError(C.MPI_ERR_ARG)
    return Comm_dup(comm)


def free(comm: Comm):
    if comm is not None and comm.val:
        _check(lib().mpigx_comm_free(comm.val))
        comm.val = None


def set_reduce_order(comm: Comm, order: int):
    """mpigx extension: MPIGX_ORDER_MPICH (default) or MPIGX_ORDER_LINEAR."""
    _check(lib().mpigx_comm_set_reduce_order(comm.val, order))


# Path-selecting knobs (include/mpigx.h MPIGX_KNOB_*): read once per
# communicator from the environment at init and checked to agree on every
# rank; set_knob changes one collectively (every rank, same value).
KNOBS = {"ALGO": 0, "BCAST": 1, "RING_CHANNELS": 2, "MAX_BLOCKS": 3, "ONESHOT_MAX": 4, "ZC_MIN": 5,
         "BCAST_SAG_MIN": 6, "ZC_REQUIRE": 7, "BYTES_PER_BLOCK": 8, "LL_AUTO": 9, "AR_TUNE": 10,
         "ZC_OPTIMISTIC": 11, "SYNC_SPIN": 12, "STAGING_BYTES": 13, "LL_MAX": 14, "AR_SLICES": 15,
         "SCAN_PP": 16, "SHARE_HEADROOM": 17, "SHARED_GATE": 18, "PEER_MEM": 19, "CONCURRENT_COMMS": 20}
ALGOS = {None: 0, "": 0, "auto": 0, "ll": 1, "ll2": 2, "oneshot": 3, "twoshot": 4, "push": 5, "ring": 6,
         "pull": 7, "pull_generic": 8, "pullpush": 9}
BCAST_MODES = {None: 0, "": 0, "auto": 0, "direct": 1, "sag": 2, "relay": 3}


def _knob_id(knob):
    return KNOBS[knob.upper()] if isinstance(knob, str) else int(knob)


def set_knob(comm: Comm, knob, value):
    """mpigx extension, COLLECTIVE: every rank calls it with the same knob and
    value (names as the MPIGX_* environment variables without the prefix;
    ALGO / BCAST also take the environment's names, e.g. "ring", "sag", or
    None for the default).  Differing values -> MPIError(MPI_ERR_ARG) on every
    rank and nothing changes."""
    k = _knob_id(knob)
    if k == KNOBS["ALGO"] and (value is None or isinstance(value, str)):
        value = ALGOS[value]
    elif k == KNOBS["BCAST"] and (value is None or isinstance(value, str)):
        value = BCAST_MODES[value]
    _check(lib().mpigx_comm_set_knob(comm.val, k, int(value)))


def get_knob(comm: Comm, knob) -> int:
    v = ctypes.c_longlong(0)
    _check(lib().mpigx_comm_get_knob(comm.val, _knob_id(knob), ctypes.byref(v)))
    return v.value


def peer_memory(comm: Comm):
    """(rw_mask, same_device_mask): bit q of rw_mask = rank q writes my
    ordinary-memory signal array / LL area (same-GPU protocol); clear = the
    uncached, cross-GPU protocol (every peer under MPIGX_PEER_MEM=xdev)."""
    rw, sd = ctypes.c_uint(0), ctypes.c_uint(0)
    _check(lib().mpigx_comm_diag_peer_mem(comm.val, ctypes.byref(rw), ctypes.byref(sd)))
    return rw.value, sd.value


def device_share(comm: Comm):
    """(ranks on the most-loaded GPU, grid cap of the spinning kernels)."""
    r, cap = ctypes.c_int(0), ctypes.c_int(0)
    _check(lib().mpigx_comm_device_share(comm.val, ctypes.byref(r), ctypes.byref(cap)))
    return r.value, cap.value


def _stream(comm):
    torch = _torch()
    s = torch.cuda.current_stream(comm.device).cuda_stream
    lib().mpigx_comm_set_stream(comm.val, ctypes.c_void_p(s))


class InexactError(ValueError):
    """Julia's InexactError: a ccall argument declared `Cint` that does not
    fit (e.g. a count of 2^31 elements, collective.jl:698-700) fails in
    `convert(Cint, x)` before any MPI call is made."""


def _cint(x) -> int:
    """`count` as MPI.jl passes it: Julia's `convert(Cint, count)`
    (collective.jl:698-700 `ccall(..., Cint, ...)`) — InexactError, and no
    call, when it does not fit (ctypes would wrap it to a negative count)."""
    x = int(x)
    if not -(1 << 31) <= x < (1 << 31):
        raise InexactError(f"InexactError: trunc(Int32, {x})")
    return x


def _call(coll, buf, comm, *args):
    """One ccall: `MPI_<coll>` in libmpi for host buffers, `mpigx_<coll>` in
    libmpigx for device buffers — the same argument list either way."""
    if _is_host(buf):
        if comm.host is None:
            raise TypeError("host buffers need host libmpi (start the ranks with mpiexec)")
        from .types import _host_args  # derived datatypes have their own host handles
        rc = getattr(hostmpi.lib(), "MPI_" + coll)(*_host_args(args), comm.host)
    else:
        if not comm.val:
            raise TypeError("device buffers need a ROCm device")
        _stream(comm)
        rc = getattr(lib(), "mpigx_" + coll.lower())(*args, comm.val)
    _check(rc)


_ENGINE_TAG, _ENGINE_MASK = 0x3C000000, 0xFC000000  # csrc/handles.hpp: libmpigx's own handle space
_LIBMPI_OPS = {}  # id(Op) -> (Op, engine handle, function object)


def _engine_user_op(opx):
    """A libmpi user op (handle + MPI_User_function) on device buffers: the
    same function registered with libmpigx once (mpigx_op_create takes the
    MPI_User_function ABI), as the Julia glue's engine_op does."""
    from ._lib import USER_FN
    hit = _LIBMPI_OPS.get(id(opx))
    if hit is not None and hit[0] is opx:
        return hit[1]
    f = opx.fptr if isinstance(opx.fptr, USER_FN) else USER_FN(int(opx.fptr))
    commute = int(bool(opx.iscommutative))
    if hostmpi.available():  # the reference asks libmpi (MPI_Op_commutative)
        c = ctypes.c_int(0)
        if hostmpi.lib().MPI_Op_commutative(ctypes.c_int(opx.val), ctypes.byref(c)) == 0:
            commute = c.value
    h = ctypes.c_int(0)
    _check(lib().mpigx_op_create(f, commute, ctypes.byref(h)))
    _LIBMPI_OPS[id(opx)] = (opx, h.value, f)
    return h.value


def _op_val(opx, buf):
    """Built-in handle, or an MPI_Op_create'd user function: libmpi's for host
    buffers, libmpigx's device-callback op for device buffers.  A libmpi op
    carrying its function pointer (libmpi_op) is re-registered with libmpigx
    for device buffers; a foreign handle without one goes through unchanged
    and libmpigx rejects it (MPI_ERR_OP)."""
    if opx.val is not None:
        if (opx.fptr is not None and not _is_host(buf) and buf is not IN_PLACE
                and (opx.val & _ENGINE_MASK) != _ENGINE_TAG):
            return _engine_user_op(opx)
        return opx.val
    if _is_host(buf):
        return hostmpi.user_op(opx.fn, _unwrap(buf).dtype, opx.iscommutative)
    return _device_user_op(opx, buf)


_DEV_OPS = {}  # (function, torch dtype, commute) -> (op handle, ctypes callback)


def _device_user_op(opx, buf):
    """operators.jl:56-88 on device: `inout[i] = f(in[i], inout[i])` as torch
    ops on the device pointers libmpigx hands the callback (enqueued on the
    communicator's stream, which is torch's current stream)."""
    from ._lib import DEVICE_FN
    from .rma import _dlpack_wrap
    b = _unwrap(buf)
    tdt, dev = b.dtype, b.device.index
    key = (opx.fn, tdt, bool(opx.iscommutative))
    if key in _DEV_OPS:
        return _DEV_OPS[key][0]
    fn = opx.fn

    def cb(inp, inout, n, dt, stream):
        sz = ctypes.c_longlong(0)  # bytes per element of the (maybe derived) datatype
        lib().mpigx_type_size_x(dt, ctypes.byref(sz))
        a = _dlpack_wrap(inp, np.dtype(np.uint8), (n * sz.value,), dev).view(tdt)
        y = _dlpack_wrap(inout, np.dtype(np.uint8), (n * sz.value,), dev).view(tdt)
        y.copy_(fn(a, y))

    f = DEVICE_FN(cb)
    h = ctypes.c_int(0)
    _check(lib().mpigx_op_create_device(f, int(bool(opx.iscommutative)), ctypes.byref(h)))
    _DEV_OPS[key] = (h.value, f)
    return h.value


# ---------------------------------------------------------------------------
# collectives (src/collective.jl)
# ---------------------------------------------------------------------------
def Barrier(comm: Comm):
    """collective.jl:15-19 (device engine barrier when a device exists)."""
    if comm.val:
        _stream(comm)
        _check(lib().mpigx_barrier(comm.val))
    if comm.host is not None:
        _check(hostmpi.lib().MPI_Barrier(comm.host))


def Bcast_(buf, *args):
    """Bcast!(buf[, count], root, comm) — collective.jl:29-42."""
    if len(args) == 3:
        count, root, comm = args
    else:
        root, comm = args
        count = _len(buf)
    _call("Bcast", buf, comm, _ptr(buf), _cint(count), _eltype(buf).val, int(root))
    return buf


def _side(buf, count, T):
    """(count, datatype handle) one side of a collective passes: an explicit
    MPI.Buffer carries its own (count, datatype) — e.g. a strided view's
    vector type — otherwise the wrapper's count and element type."""
    if isinstance(buf, Buffer):
        return int(buf.count), buf.datatype.val
    return _cint(count), T.val


def Allgather_(*args):
    """Allgather!(sendbuf, recvbuf, count, comm) / Allgather!(sendrecvbuf, count, comm)
    — collective.jl:295-311."""
    if len(args) == 3:
        sendbuf, (recvbuf, count, comm) = IN_PLACE, args
    else:
        sendbuf, recvbuf, count, comm = args
    assert recvbuf is not None
    _assert_minlength(recvbuf, count * Comm_size(comm))
    _assert_minlength(sendbuf, count)
    T = _eltype(recvbuf)
    _call("Allgather", recvbuf, comm, _ptr(sendbuf), *_side(sendbuf, count, T), _ptr(recvbuf),
          *_side(recvbuf, count, T))
    return recvbuf


def Allgather(*args):
    """Allgather(sendbuf[, count], comm) / Allgather(obj, comm) — collective.jl:327-335."""
    if len(args) == 3:
        sendbuf, count, comm = args
        return Allgather_(sendbuf, _empty_like(sendbuf, Comm_size(comm) * count), count, comm)
    sendbuf, comm = args
    if _is_array(sendbuf):
        return Allgather(sendbuf, _len(sendbuf), comm)
    ref = _scalar_ref(sendbuf, comm)
    out = _empty_like(ref, Comm_size(comm))
    Allgather_(ref, out, 1, comm)
    return (out if isinstance(out, np.ndarray) else out.cpu().numpy()).tolist()


def Alltoall_(*args):
    """Alltoall!(sendbuf, recvbuf, count, comm) — collective.jl:489-501.
    The in-place 3-argument form (:503-505 references an undefined `recvbuf`
    in the reference) is implemented as evidently intended."""
    if len(args) == 3:
        sendbuf, (recvbuf, count, comm) = IN_PLACE, args
    else:
        sendbuf, recvbuf, count, comm = args
    buflength = count * Comm_size(comm)
    _assert_minlength(recvbuf, buflength)
    _assert_minlength(sendbuf, buflength)
    if sendbuf is not IN_PLACE and not isinstance(sendbuf, Buffer):
        assert _eltype(sendbuf) == _eltype(recvbuf)
    T = _eltype(recvbuf)
    _call("Alltoall", recvbuf, comm, _ptr(sendbuf), *_side(sendbuf, count, T), _ptr(recvbuf),
          *_side(recvbuf, count, T))
    return recvbuf


def Alltoall(sendbuf, count, comm):
    """collective.jl:529-532."""
    return Alltoall_(sendbuf, _empty_like(sendbuf, Comm_size(comm) * count), count, comm)


# ---------------------------------------------------------------------------
# v-collectives and rooted variants (collective.jl:90-578)
# ---------------------------------------------------------------------------
def _cints(xs):
    xs = [int(x) for x in xs]
    return (ctypes.c_int * max(1, len(xs)))(*xs)


def _disps(counts):
    """accumulate(+, counts) - counts (collective.jl:169, :365, :425, :551)."""
    d, acc = [], 0
    for c in counts:
        d.append(acc)
        acc += int(c)
    return d


def Scatter_(sendbuf, recvbuf, *args):
    """Scatter!(sendbuf, recvbuf[, count], root, comm) — collective.jl:90-112.
    `recvbuf = None` at the root means MPI_IN_PLACE."""
    if len(args) == 2:
        root, comm = args
        count = _len(recvbuf)
    else:
        count, root, comm = args
    isroot = Comm_rank(comm) == root
    if isroot:
        assert sendbuf is not None
        _assert_minlength(sendbuf, count * Comm_size(comm))
        if recvbuf is None:
            recvbuf = IN_PLACE
    _assert_minlength(recvbuf, count)
    T = _eltype(sendbuf) if recvbuf is IN_PLACE else _eltype(recvbuf)
    data = sendbuf if recvbuf is IN_PLACE or recvbuf is None else recvbuf
    _call("Scatter", data, comm, _ptr(sendbuf), *_side(sendbuf, count, T), _ptr(recvbuf), *_side(recvbuf, count, T),
          int(root))
    return recvbuf


def Scatter(sendbuf, count, root, comm):
    """collective.jl:127-129."""
    return Scatter_(sendbuf, _empty_like(sendbuf, count), count, root, comm)


def Scatterv_(sendbuf, recvbuf, counts, root, comm):
    """Scatterv!(sendbuf, recvbuf, counts, root, comm) — collective.jl:156-175."""
    rank = Comm_rank(comm)
    if rank == root:
        assert sendbuf is not None
        _assert_minlength(sendbuf, sum(counts))
    if recvbuf is None:
        recvbuf = IN_PLACE
    _assert_minlength(recvbuf, counts[rank])
    T = _eltype(sendbuf) if recvbuf is IN_PLACE else _eltype(recvbuf)
    data = sendbuf if recvbuf is IN_PLACE else recvbuf
    _call("Scatterv", data, comm, _ptr(sendbuf), _cints(counts), _cints(_disps(counts)), T.val, _ptr(recvbuf),
          _cint(counts[rank]), T.val, int(root))
    return recvbuf


def Scatterv(sendbuf, counts, root, comm):
    """collective.jl:193-196."""
    return Scatterv_(sendbuf, _empty_like(sendbuf, counts[Comm_rank(comm)]), counts, root, comm)


def Gather_(sendbuf, recvbuf, *args):
    """Gather!(sendbuf, recvbuf[, count=length(sendbuf)], root, comm) — collective.jl:230-251.
    `sendbuf = None` at the root means MPI_IN_PLACE; returns recvbuf at root, None elsewhere."""
    if len(args) == 2:
        root, comm = args
        count = _len(sendbuf)
    else:
        count, root, comm = args
    isroot = Comm_rank(comm) == root
    if isroot:
        assert recvbuf is not None
        _assert_minlength(recvbuf, count * Comm_size(comm))
        if sendbuf is None:
            sendbuf = IN_PLACE
    _assert_minlength(sendbuf, count)
    T = _eltype(recvbuf) if sendbuf is IN_PLACE else _eltype(sendbuf)
    data = recvbuf if sendbuf is IN_PLACE else sendbuf
    _call("Gather", data, comm, _ptr(sendbuf), *_side(sendbuf, count, T), _ptr(recvbuf), *_side(recvbuf, count, T),
          int(root))
    return recvbuf if isroot else None


def Gather(*args):
    """Gather(sendbuf[, count], root, comm) / Gather(obj, root, comm) — collective.jl:267-275."""
    if len(args) == 4:
        sendbuf, count, root, comm = args
        recv = _empty_like(sendbuf, Comm_size(comm) * count) if Comm_rank(comm) == root else None
        return Gather_(sendbuf, recv, count, root, comm)
    sendbuf, root, comm = args
    if _is_array(sendbuf):
        return Gather(sendbuf, _len(sendbuf), root, comm)
    ref = _scalar_ref(sendbuf, comm)
    recv = _empty_like(ref, Comm_size(comm)) if Comm_rank(comm) == root else None
    out = Gather_(ref, recv, 1, root, comm)
    return None if out is None else (out if isinstance(out, np.ndarray) else out.cpu().numpy()).tolist()


def Gatherv_(sendbuf, recvbuf, counts, root, comm):
    """Gatherv!(sendbuf, recvbuf, counts, root, comm) — collective.jl:363-382."""
    rank = Comm_rank(comm)
    isroot = rank == root
    if isroot:
        assert recvbuf is not None
        _assert_minlength(recvbuf, sum(counts))
        if sendbuf is None:
            sendbuf = IN_PLACE
    _assert_minlength(sendbuf, counts[rank])
    T = _eltype(recvbuf) if sendbuf is IN_PLACE else _eltype(sendbuf)
    data = recvbuf if sendbuf is IN_PLACE else sendbuf
    _call("Gatherv", data, comm, _ptr(sendbuf), _cint(counts[rank]), T.val, _ptr(recvbuf), _cints(counts),
          _cints(_disps(counts)), T.val, int(root))
    return recvbuf if isroot else None


def Gatherv(sendbuf, counts, root, comm):
    """collective.jl:401-403."""
    recv = _empty_like(sendbuf, sum(counts)) if Comm_rank(comm) == root else None
    return Gatherv_(sendbuf, recv, counts, root, comm)


def Allgatherv_(*args):
    """Allgatherv!(sendbuf, recvbuf, counts, comm) / Allgatherv!(sendrecvbuf, counts, comm)
    — collective.jl:424-442."""
    if len(args) == 3:
        sendbuf, (recvbuf, counts, comm) = IN_PLACE, args
    else:
        sendbuf, recvbuf, counts, comm = args
    sendcnt = counts[Comm_rank(comm)]
    assert recvbuf is not None
    _assert_minlength(recvbuf, sum(counts))
    _assert_minlength(sendbuf, sendcnt)
    T = _eltype(recvbuf)
    _call("Allgatherv", recvbuf, comm, _ptr(sendbuf), _cint(sendcnt), T.val, _ptr(recvbuf), _cints(counts),
          _cints(_disps(counts)), T.val)
    return recvbuf


def Allgatherv(sendbuf, counts, comm):
    """collective.jl:458-461."""
    return Allgatherv_(sendbuf, _empty_like(sendbuf, sum(counts)), counts, comm)


def Alltoallv_(sendbuf, recvbuf, scounts, rcounts, comm):
    """Alltoallv!(sendbuf, recvbuf, scounts, rcounts, comm) — collective.jl:545-559."""
    _assert_minlength(sendbuf, sum(scounts))
    _assert_minlength(recvbuf, sum(rcounts))
    assert _eltype(sendbuf) == _eltype(recvbuf)
    T = _eltype(sendbuf)
    _call("Alltoallv", recvbuf, comm, _ptr(sendbuf), _cints(scounts), _cints(_disps(scounts)), T.val,
          _ptr(recvbuf), _cints(rcounts), _cints(_disps(rcounts)), T.val)
    return recvbuf


def Alltoallv(sendbuf, scounts, rcounts, comm):
    """collective.jl:574-578."""
    return Alltoallv_(sendbuf, _empty_like(sendbuf, sum(rcounts)), scounts, rcounts, comm)


def _scalar_ref(obj, comm):
    """`Ref(object)` of the scalar forms: a 1-element host array when host
    libmpi is up (as in MPI.jl), else a 1-element device tensor."""
    if isinstance(obj, (bool, np.bool_)):
        npdt = np.uint8
    elif isinstance(obj, (int, np.integer)):
        npdt = np.int64 if isinstance(obj, int) else obj.dtype
    elif isinstance(obj, (float, np.floating)):
        npdt = np.float64 if isinstance(obj, float) else obj.dtype
    elif isinstance(obj, (complex, np.complexfloating)):
        npdt = np.complex128 if isinstance(obj, complex) else obj.dtype
    else:
        raise TypeError(f"unsupported scalar {obj!r}")
    a = np.array([obj], dtype=npdt)
    if comm.host is not None:
        return a
    return _torch().from_numpy(a).to(f"cuda:{comm.device}")


def _item(x):
    return x[0].item() if isinstance(x, np.ndarray) else x.item()


def Reduce_(*args):
    """Reduce!(sendbuf, recvbuf, count, op, root, comm)          collective.jl:605
    Reduce!(sendbuf, recvbuf, op, root, comm)                     :626
    Reduce!(buf, op, root, comm)  (IN_PLACE at root)              :632"""
    if len(args) == 4:
        buf, op, root, comm = args
        if Comm_rank(comm) == root:
            return Reduce_(IN_PLACE, buf, _len(buf), op, root, comm)
        return Reduce_(buf, None, _len(buf), op, root, comm)
    if len(args) == 5:
        sendbuf, recvbuf, op, root, comm = args
        return Reduce_(sendbuf, recvbuf, _len(sendbuf), op, root, comm)
    sendbuf, recvbuf, count, op, root, comm = args
    isroot = Comm_rank(comm) == root
    _assert_minlength(sendbuf, count)
    if isroot:
        assert recvbuf is not None
        _assert_minlength(recvbuf, count)
    data = recvbuf if sendbuf is IN_PLACE else sendbuf
    T = _eltype(data)
    opx = _as_op(op, _dtype(data))
    _call("Reduce", data, comm, _ptr(sendbuf), _ptr(recvbuf), _cint(count), T.val, _op_val(opx, data), int(root))
    return recvbuf


def Reduce(sendbuf, op, root, comm):
    """collective.jl:657-666: allocating; `nothing` (None) on non-roots."""
    if _is_array(sendbuf):
        recv = _empty_like(sendbuf) if Comm_rank(comm) == root else None
        return Reduce_(sendbuf, recv, _len(sendbuf), op, root, comm)
    ref = _scalar_ref(sendbuf, comm)
    if Comm_rank(comm) == root:
        out = _empty_like(ref)
        Reduce_(ref, out, 1, op, root, comm)
        return _item(out)
    Reduce_(ref, None, 1, op, root, comm)
    return None


def Allreduce_(*args):
    """Allreduce!(sendbuf, recvbuf, count, op, comm)   collective.jl:691-701
    Allreduce!(sendbuf, recvbuf, op, comm)              :707 (count = length(recvbuf))
    Allreduce!(buf, op, comm)  (IN_PLACE)               :712"""
    if len(args) == 3:
        buf, op, comm = args
        return Allreduce_(IN_PLACE, buf, _len(buf), op, comm)
    if len(args) == 4:
        sendbuf, recvbuf, op, comm = args
        return Allreduce_(sendbuf, recvbuf, _len(recvbuf), op, comm)
    sendbuf, recvbuf, count, op, comm = args
    _assert_minlength(sendbuf, count)
    _assert_minlength(recvbuf, count)
    if sendbuf is not IN_PLACE:
        assert _eltype(sendbuf) == _eltype(recvbuf)
    T = _eltype(recvbuf)
    opx = _as_op(op, _dtype(recvbuf))
    _call("Allreduce", recvbuf, comm, _ptr(sendbuf), _ptr(recvbuf), _cint(count), T.val, _op_val(opx, recvbuf))
    return recvbuf


def Allreduce(sendbuf, op, comm):
    """collective.jl:733-738: allocating (`similar`) or scalar (`Ref`) form."""
    if _is_array(sendbuf):
        return Allreduce_(sendbuf, _empty_like(sendbuf), _len(sendbuf), op, comm)
    ref = _scalar_ref(sendbuf, comm)
    out = _empty_like(ref)
    Allreduce_(ref, out, 1, op, comm)
    return _item(out)


def _scan_dispatch(args):
    """Scan!/Exscan!(sendbuf, recvbuf, count, op, comm) | (sendbuf, recvbuf, op, comm)
    | in-place (buf, count, op, comm) | (buf, op, comm).  (collective.jl:760-783 /
    :834-857 — the reference's in-place forms use an undefined `sendbuf`; here
    they are the evident IN_PLACE calls.)"""
    if len(args) == 3:
        buf, op, comm = args
        return IN_PLACE, buf, _len(buf), op, comm
    if len(args) == 4:
        a, b, c, comm = args
        if isinstance(b, int) and not _is_array(b):  # (buf, count, op, comm)
            return IN_PLACE, a, b, c, comm
        return a, b, _len(a), c, comm
    return args


def _scan_common(args, exclusive):
    sendbuf, recvbuf, count, op, comm = _scan_dispatch(args)
    T = _eltype(recvbuf)
    opx = _as_op(op, _dtype(recvbuf))
    _call("Exscan" if exclusive else "Scan", recvbuf, comm, _ptr(sendbuf), _ptr(recvbuf), _cint(count), T.val,
          _op_val(opx, recvbuf))
    return recvbuf


def Scan_(*args):
    """Inclusive prefix reduction over ranks 0..r — collective.jl:760-783."""
    return _scan_common(args, False)


def Exscan_(*args):
    """Exclusive prefix reduction; rank 0's recvbuf untouched — collective.jl:834-857."""
    return _scan_common(args, True)


def Scan(sendbuf, op, comm):
    """collective.jl:803-808."""
    if _is_array(sendbuf):
        return Scan_(sendbuf, _empty_like(sendbuf), op, comm)
    ref = _scalar_ref(sendbuf, comm)
    out = _empty_like(ref)
    Scan_(ref, out, 1, op, comm)
    return _item(out)


def Exscan(sendbuf, op, comm):
    """collective.jl:877-882 (rank 0's result is undefined: its buffer is untouched)."""
    if _is_array(sendbuf):
        return Exscan_(sendbuf, _empty_like(sendbuf), op, comm)
    ref = _scalar_ref(sendbuf, comm)
    out = np.zeros_like(ref) if isinstance(ref, np.ndarray) else _torch().zeros_like(ref)
    Exscan_(ref, out, 1, op, comm)
    return _item(out)


# ---------------------------------------------------------------------------
# local op (config 2): the built-in MPI.Op set on device buffers
# ---------------------------------------------------------------------------
def Reduce_local_(inbuf, inoutbuf, count, op):
    """MPI_Reduce_local (mpi.h:1357): inoutbuf = op(inoutbuf, inbuf)."""
    T = _eltype(inoutbuf)
    opx = _as_op(op, _dtype(inoutbuf))
    _check(lib().mpigx_reduce_local(_ptr(inbuf), _ptr(inoutbuf), _cint(count), T.val, opx.val))
    return inoutbuf


def reduce_local_multi(inputs, out, op, order=C.MPIGX_ORDER_MPICH, stream=None, count=None):
    """out = fold(inputs) as an len(inputs)-rank Allreduce would (asynchronous,
    on `stream` (torch stream or raw handle; default: current stream))."""
    torch = _torch()
    n = len(inputs)
    arr = (ctypes.c_void_p * n)(*[t.data_ptr() for t in inputs])
    if stream is None:
        stream = torch.cuda.current_stream(out.device).cuda_stream
    elif hasattr(stream, "cuda_stream"):
        stream = stream.cuda_stream
    T = _eltype(out)
    opx = _as_op(op, out.dtype)
    cnt = out.numel() if count is None else count
    _check(lib().mpigx_reduce_local_multi(arr, n, ctypes.c_void_p(out.data_ptr()), cnt, T.val, opx.val, order,
                                          ctypes.c_void_p(stream)))
    return out
