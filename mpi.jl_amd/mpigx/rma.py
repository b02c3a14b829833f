"""MPI.jl's one-sided API (src/onesided.jl) over libmpigx / libmpi.

Same split as the collectives and point-to-point: a window over a torch tensor
on a ROCm device goes to ``mpigx_win_*`` (rma.cpp: Get pulled by the origin
over xGMI, Put / Accumulate applied by the target to its own HBM), a window
over a numpy array goes to ``MPI_Win_*`` of the process's libmpi.  Names and
argument meaning follow onesided.jl (``Win_create(base, comm)``,
``Get(origin, count, target_rank, target_disp, win)``, ...).

Scalar ``Ref`` operands of the reference (``Fetch_and_op(Ref(x), Ref(y), ...)``,
``Get(Ref(addr), r, win)``) are 1-element numpy arrays here.  With a device
window they are staged through device tensors; results land in the host array
when the operation completes (Get: at the next flush / unlock / fence, as MPI
specifies; Fetch_and_op / Get_accumulate: on return, since the engine
completes them synchronously).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import consts as C
from . import hostmpi
from ._lib import lib
from .api import MPIError, _as_op, _check, _is_host, _stream, _torch, _unwrap

__all__ = ["Win", "WIN_NULL", "LockType", "LOCK_EXCLUSIVE", "LOCK_SHARED", "MODE_NOCHECK", "Win_create",
           "Win_create_dynamic", "Win_allocate_shared", "Win_shared_query", "Win_attach", "Win_detach",
           "Win_fence", "Win_flush", "Win_sync", "Win_lock", "Win_unlock", "Get", "Put", "Fetch_and_op",
           "Accumulate", "Get_accumulate", "Get_address", "unsafe_wrap", "win_free"]

MPI_INFO_NULL = 0x1c000000
MPI_WIN_NULL = 0x20000000
MODE_NOCHECK = 1024


class LockType:
    __slots__ = ("val",)

    def __init__(self, val):
        self.val = val


LOCK_EXCLUSIVE = LockType(234)
LOCK_SHARED = LockType(235)


class Win:
    """MPI.Win (onesided.jl:1-3).  `val`: libmpigx window handle (device) or
    MPICH MPI_Win int (host); `backend` 'dev' / 'host'."""
    __slots__ = ("val", "backend", "comm", "base", "device", "_deferred", "__weakref__")

    def __init__(self, val=None, backend=None, comm=None, base=None):
        self.val, self.backend, self.comm, self.base = val, backend, comm, base
        self.device = comm.device if comm is not None else None
        self._deferred = []  # (device tmp, host array) copies owed at the next completion

    def __repr__(self):
        return f"MPI.Win({self.backend})"


WIN_NULL = Win()


def _host(win):
    return win.backend == "host"


def _hcheck(rc):
    if rc:
        raise MPIError(rc)


def _aint(x):
    return ctypes.c_longlong(int(x))


def _hptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def _dptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _dtype_val(x):
    from .api import Datatype
    return Datatype(_unwrap(x).dtype).val


def _nbytes(x):
    x = _unwrap(x)
    return x.nbytes if isinstance(x, np.ndarray) else x.numel() * x.element_size()


# ---------------------------------------------------------------------------
# window creation (onesided.jl:24-108)
# ---------------------------------------------------------------------------
def Win_create(base, comm, **infokws):
    """onesided.jl:24-34: collective; disp_unit = sizeof(eltype)."""
    b = _unwrap(base)
    if isinstance(b, np.ndarray):
        w = ctypes.c_int(0)
        _hcheck(hostmpi.lib().MPI_Win_create(_hptr(b), _aint(b.nbytes), b.itemsize, MPI_INFO_NULL, comm.host,
                                             ctypes.byref(w)))
        hostmpi.lib().MPI_Win_set_errhandler(w, hostmpi.MPI_ERRORS_RETURN)
        return Win(w.value, "host", comm, b)
    if not b.is_contiguous():
        raise ValueError("window base must be contiguous")
    h = ctypes.c_void_p()
    _stream(comm)
    _check(lib().mpigx_win_create(_dptr(b), b.numel() * b.element_size(), b.element_size(), comm.val,
                                  ctypes.byref(h)))
    return Win(h, "dev", comm, b)


def Win_create_dynamic(comm, **kwargs):
    """onesided.jl:47-56.  Device when the communicator has a device."""
    if comm.val:
        h = ctypes.c_void_p()
        _stream(comm)
        _check(lib().mpigx_win_create_dynamic(comm.val, ctypes.byref(h)))
        return Win(h, "dev", comm)
    w = ctypes.c_int(0)
    _hcheck(hostmpi.lib().MPI_Win_create_dynamic(MPI_INFO_NULL, comm.host, ctypes.byref(w)))
    hostmpi.lib().MPI_Win_set_errhandler(w, hostmpi.MPI_ERRORS_RETURN)
    return Win(w.value, "host", comm)


def Win_allocate_shared(T, length, comm, device=None, **kwargs):
    """onesided.jl:72-83: returns (win, ptr).  `device` (default: the comm's
    device exists) selects engine-owned HBM; else libmpi shared memory."""
    npdt = np.dtype(T)
    size = int(length) * npdt.itemsize
    use_dev = bool(comm.val) if device is None else device
    out = ctypes.c_void_p()
    if use_dev:
        h = ctypes.c_void_p()
        _stream(comm)
        _check(lib().mpigx_win_allocate_shared(size, npdt.itemsize, comm.val, ctypes.byref(out), ctypes.byref(h)))
        return Win(h, "dev", comm), (out.value or 0)
    w = ctypes.c_int(0)
    _hcheck(hostmpi.lib().MPI_Win_allocate_shared(_aint(size), npdt.itemsize, MPI_INFO_NULL, comm.host,
                                                  ctypes.byref(out), ctypes.byref(w)))
    hostmpi.lib().MPI_Win_set_errhandler(w, hostmpi.MPI_ERRORS_RETURN)
    return Win(w.value, "host", comm), (out.value or 0)


def Win_shared_query(win, owner_rank):
    """onesided.jl:98-108: (length in bytes, disp_unit, base pointer)."""
    size = ctypes.c_longlong(0)
    du = ctypes.c_int(0)
    p = ctypes.c_void_p()
    if _host(win):
        _hcheck(hostmpi.lib().MPI_Win_shared_query(win.val, owner_rank, ctypes.byref(size), ctypes.byref(du),
                                                   ctypes.byref(p)))
    else:
        _check(lib().mpigx_win_shared_query(win.val, owner_rank, ctypes.byref(size), ctypes.byref(du),
                                            ctypes.byref(p)))
    return size.value, du.value, (p.value or 0)


def unsafe_wrap(ptr, T, shape, win=None, device=None):
    """Julia's `unsafe_wrap(Array, ptr, dims)`: a numpy view of host memory,
    or (device window) a torch tensor over device memory via DLPack."""
    npdt = np.dtype(T)
    shape = (shape,) if isinstance(shape, int) else tuple(shape)
    nel = int(np.prod(shape))
    if win is None or _host(win):
        buf = (ctypes.c_char * (nel * npdt.itemsize)).from_address(ptr)
        return np.frombuffer(buf, dtype=npdt).reshape(shape, order="F")
    dev = win.device if device is None else device
    return _dlpack_wrap(ptr, npdt, shape, dev)


# --- DLPack capsule over a raw ROCm pointer (no torch allocation) ----------
class _DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class _DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class _DLTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("device", _DLDevice), ("ndim", ctypes.c_int32),
                ("dtype", _DLDataType), ("shape", ctypes.POINTER(ctypes.c_int64)),
                ("strides", ctypes.POINTER(ctypes.c_int64)), ("byte_offset", ctypes.c_uint64)]


class _DLManagedTensor(ctypes.Structure):
    pass


_DELETER = ctypes.CFUNCTYPE(None, ctypes.POINTER(_DLManagedTensor))
_DLManagedTensor._fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", ctypes.c_void_p), ("deleter", _DELETER)]
_KEEP = {}


@_DELETER
def _dl_deleter(p):
    _KEEP.pop(ctypes.addressof(p.contents), None)


def _dlpack_wrap(ptr, npdt, shape, device):
    torch = _torch()
    code = {"i": 0, "u": 1, "f": 2, "c": 5, "b": 6}[npdt.kind]
    ndim = len(shape)
    shp = (ctypes.c_int64 * ndim)(*shape)
    # column-major like Julia arrays
    st, acc = [], 1
    for s in shape:
        st.append(acc)
        acc *= s
    strides = (ctypes.c_int64 * ndim)(*st)
    mt = _DLManagedTensor()
    mt.dl_tensor = _DLTensor(ctypes.c_void_p(ptr), _DLDevice(10, device), ndim,  # kDLROCM = 10
                             _DLDataType(code, npdt.itemsize * 8, 1), shp, strides, 0)
    mt.manager_ctx = None
    mt.deleter = _dl_deleter
    _KEEP[ctypes.addressof(mt)] = (mt, shp, strides)
    ctypes.pythonapi.PyCapsule_New.restype = ctypes.py_object
    ctypes.pythonapi.PyCapsule_New.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
    cap = ctypes.pythonapi.PyCapsule_New(ctypes.addressof(mt), b"dltensor", None)
    return torch.utils.dlpack.from_dlpack(cap)


def win_free(win):
    """MPI.free(win) (onesided.jl:85-92)."""
    if win.val is None:
        return
    if _host(win):
        w = ctypes.c_int(win.val)
        _hcheck(hostmpi.lib().MPI_Win_free(ctypes.byref(w)))
    else:
        _complete(win)
        h = ctypes.c_void_p(win.val.value if isinstance(win.val, ctypes.c_void_p) else win.val)
        _stream(win.comm)
        _check(lib().mpigx_win_free(ctypes.byref(h)))
    win.val = None


def Win_attach(win, base):
    """onesided.jl:110-115."""
    if _host(win):
        _hcheck(hostmpi.lib().MPI_Win_attach(win.val, _hptr(base), _aint(base.nbytes)))
    else:
        _check(lib().mpigx_win_attach(win.val, _dptr(base), base.numel() * base.element_size()))


def Win_detach(win, base):
    """onesided.jl:117-122."""
    if _host(win):
        _hcheck(hostmpi.lib().MPI_Win_detach(win.val, _hptr(base)))
    else:
        _check(lib().mpigx_win_detach(win.val, _dptr(base)))


def Get_address(buf):
    """MPI_Get_address: the absolute address (device pointer for device
    buffers), used as target_disp of dynamic windows."""
    b = _unwrap(buf)
    if isinstance(b, np.ndarray):
        return int(b.ctypes.data)
    return int(b.data_ptr())


# ---------------------------------------------------------------------------
# synchronisation (onesided.jl:124-148)
# ---------------------------------------------------------------------------
def _complete(win):
    """Host copies owed by Gets into host arrays (device window)."""
    if win._deferred:
        _torch().cuda.synchronize(win.device)
        for tmp, host in win._deferred:
            host.reshape(-1)[:] = tmp.cpu().numpy().reshape(-1)
        win._deferred.clear()


def _dev_call(win, fn, *args):
    _stream(win.comm)
    _check(getattr(lib(), fn)(*args))


def Win_fence(assert_, win):
    if _host(win):
        _hcheck(hostmpi.lib().MPI_Win_fence(int(assert_), win.val))
        return
    _dev_call(win, "mpigx_win_fence", int(assert_), win.val)
    _complete(win)


def Win_flush(rank, win):
    if _host(win):
        _hcheck(hostmpi.lib().MPI_Win_flush(int(rank), win.val))
        return
    _dev_call(win, "mpigx_win_flush", int(rank), win.val)
    _complete(win)


def Win_sync(win):
    if _host(win):
        _hcheck(hostmpi.lib().MPI_Win_sync(win.val))
        return
    _dev_call(win, "mpigx_win_sync", win.val)
    _complete(win)


def Win_lock(lock_type, rank, assert_, win):
    lt = lock_type.val if isinstance(lock_type, LockType) else int(lock_type)
    if _host(win):
        _hcheck(hostmpi.lib().MPI_Win_lock(lt, int(rank), int(assert_), win.val))
        return
    _dev_call(win, "mpigx_win_lock", lt, int(rank), int(assert_), win.val)


def Win_unlock(rank, win):
    if _host(win):
        _hcheck(hostmpi.lib().MPI_Win_unlock(int(rank), win.val))
        return
    _dev_call(win, "mpigx_win_unlock", int(rank), win.val)
    _complete(win)


# ---------------------------------------------------------------------------
# data movement (onesided.jl:150-219)
# ---------------------------------------------------------------------------
def _to_dev(win, x):
    """Device operand for a device window (numpy scalars/arrays are staged)."""
    b = _unwrap(x)
    if isinstance(b, np.ndarray):
        return _torch().from_numpy(np.ascontiguousarray(b).reshape(-1).copy()).to(f"cuda:{win.device}")
    return b


def _count_of(x):
    b = _unwrap(x)
    return b.size if isinstance(b, np.ndarray) else b.numel()


def Get(origin_buffer, *args):
    """Get(origin, count, target_rank, target_disp, win) (onesided.jl:150-159)
    or Get(origin, target_rank, win) (:160-166: count = length, disp 0)."""
    if len(args) == 2:
        count, (target_rank, win), target_disp = _count_of(origin_buffer), args, 0
    else:
        count, target_rank, target_disp, win = args
    dt = _dtype_val(origin_buffer)
    if _host(win):
        o = _unwrap(origin_buffer)
        _hcheck(hostmpi.lib().MPI_Get(_hptr(o), int(count), dt, int(target_rank), _aint(target_disp), int(count), dt,
                                      win.val))
        return
    b = _unwrap(origin_buffer)
    dst = _to_dev(win, b)
    _dev_call(win, "mpigx_get", _dptr(dst), int(count), dt, int(target_rank), ctypes.c_longlong(int(target_disp)),
              int(count), dt, win.val)
    if isinstance(b, np.ndarray):
        win._deferred.append((dst, b))


def Put(origin_buffer, *args):
    """Put(origin, count, target_rank, target_disp, win) (onesided.jl:168-177)
    or Put(origin, target_rank, win) (:178-184)."""
    if len(args) == 2:
        count, (target_rank, win), target_disp = _count_of(origin_buffer), args, 0
    else:
        count, target_rank, target_disp, win = args
    dt = _dtype_val(origin_buffer)
    if _host(win):
        o = _unwrap(origin_buffer)
        _hcheck(hostmpi.lib().MPI_Put(_hptr(o), int(count), dt, int(target_rank), _aint(target_disp), int(count), dt,
                                      win.val))
        return
    src = _to_dev(win, origin_buffer)
    _dev_call(win, "mpigx_put", _dptr(src), int(count), dt, int(target_rank), ctypes.c_longlong(int(target_disp)),
              int(count), dt, win.val)


def _opval(op, x):
    o = _as_op(op, _unwrap(x).dtype)
    if o.val is None:
        raise MPIError(C.MPI_ERR_OP)  # RMA takes predefined ops only (MPI-3 §11.3.4)
    return o.val


def Fetch_and_op(sourceval, returnval, target_rank, target_disp, op, win):
    """onesided.jl:186-195."""
    assert _unwrap(sourceval).dtype == _unwrap(returnval).dtype
    dt = _dtype_val(sourceval)
    opv = _opval(op, sourceval)
    if _host(win):
        _hcheck(hostmpi.lib().MPI_Fetch_and_op(_hptr(_unwrap(sourceval)), _hptr(_unwrap(returnval)), dt,
                                               int(target_rank), _aint(target_disp), opv, win.val))
        return
    src = _to_dev(win, sourceval)
    rb = _unwrap(returnval)
    res = _to_dev(win, rb)
    _dev_call(win, "mpigx_fetch_and_op", _dptr(src), _dptr(res), dt, int(target_rank),
              ctypes.c_longlong(int(target_disp)), opv, win.val)
    if isinstance(rb, np.ndarray):
        rb.reshape(-1)[:] = res.cpu().numpy()


def Accumulate(origin_buffer, count, target_rank, target_disp, op, win):
    """onesided.jl:197-206."""
    dt = _dtype_val(origin_buffer)
    opv = _opval(op, origin_buffer)
    if _host(win):
        _hcheck(hostmpi.lib().MPI_Accumulate(_hptr(_unwrap(origin_buffer)), int(count), dt, int(target_rank),
                                             _aint(target_disp), int(count), dt, opv, win.val))
        return
    src = _to_dev(win, origin_buffer)
    _dev_call(win, "mpigx_accumulate", _dptr(src), int(count), dt, int(target_rank),
              ctypes.c_longlong(int(target_disp)), int(count), dt, opv, win.val)


def Get_accumulate(origin_buffer, result_buffer, count, target_rank, target_disp, op, win):
    """onesided.jl:208-219."""
    assert _unwrap(origin_buffer).dtype == _unwrap(result_buffer).dtype
    dt = _dtype_val(origin_buffer)
    opv = _opval(op, origin_buffer)
    if _host(win):
        _hcheck(hostmpi.lib().MPI_Get_accumulate(_hptr(_unwrap(origin_buffer)), int(count), dt,
                                                 _hptr(_unwrap(result_buffer)), int(count), dt, int(target_rank),
                                                 _aint(target_disp), int(count), dt, opv, win.val))
        return
    src = _to_dev(win, origin_buffer)
    rb = _unwrap(result_buffer)
    res = _to_dev(win, rb)
    _dev_call(win, "mpigx_get_accumulate", _dptr(src), int(count), dt, _dptr(res), int(count), dt, int(target_rank),
              ctypes.c_longlong(int(target_disp)), int(count), dt, opv, win.val)
    if isinstance(rb, np.ndarray):
        rb.reshape(-1)[:] = res.cpu().numpy()
