"""Host buffers: the untouched libmpi path of MPI.jl.

MPI.jl sends host `Array`s to libmpi (src/collective.jl ccalls) and only
device buffers to the engine.  The Python mirror keeps that split: numpy
arrays and host scalars go to the process's libmpi — MPICH 3.3.2 from
/opt/conda when the rank was started by `mpiexec` — through ctypes, with the
same handle values, IN_PLACE sentinel and user-function callback
(src/operators.jl:56-88 OpWrapper, `inout[i] = f(in[i], inout[i])`).
This is the reference's own host path, not a fallback for device buffers:
torch device tensors never come here.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import consts as C

MPI_ERRORS_RETURN = 0x54000001  # MPICH handle
_IN_PLACE = ctypes.c_void_p(-1 & ((1 << 64) - 1))
_USER_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                            ctypes.POINTER(ctypes.c_int))

NP_OF_HANDLE = {
    C.MPI_INT8_T: np.int8, C.MPI_UINT8_T: np.uint8, C.MPI_INT16_T: np.int16, C.MPI_UINT16_T: np.uint16,
    C.MPI_INT32_T: np.int32, C.MPI_UINT32_T: np.uint32, C.MPI_INT64_T: np.int64, C.MPI_UINT64_T: np.uint64,
    C.MPI_FLOAT: np.float32, C.MPI_DOUBLE: np.float64, C.MPI_C_FLOAT_COMPLEX: np.complex64,
    C.MPI_C_DOUBLE_COMPLEX: np.complex128, C.MPI_CHAR: np.int8, C.MPI_BYTE: np.uint8,
}
HANDLE_OF_NP = {
    np.dtype(np.int8): C.MPI_INT8_T, np.dtype(np.uint8): C.MPI_UINT8_T, np.dtype(np.int16): C.MPI_INT16_T,
    np.dtype(np.uint16): C.MPI_UINT16_T, np.dtype(np.int32): C.MPI_INT32_T, np.dtype(np.uint32): C.MPI_UINT32_T,
    np.dtype(np.int64): C.MPI_INT64_T, np.dtype(np.uint64): C.MPI_UINT64_T, np.dtype(np.float32): C.MPI_FLOAT,
    np.dtype(np.float64): C.MPI_DOUBLE, np.dtype(np.complex64): C.MPI_C_FLOAT_COMPLEX,
    np.dtype(np.complex128): C.MPI_C_DOUBLE_COMPLEX, np.dtype(np.bool_): C.MPI_UINT8_T,
    np.dtype(np.float16): C.MPI_UINT16_T,  # by size, datatypes.jl:281-284
}

_lib = None
_ops = []  # keep user-op callbacks alive


def available() -> bool:
    """A libmpi to use: started under mpiexec (PMI env) and the library exists."""
    return ("PMI_RANK" in os.environ or "PMI_SIZE" in os.environ) and os.path.exists(_path())


def _path():
    return os.environ.get("MPIGX_HOST_LIBMPI", "/opt/conda/lib/libmpi.so.12")


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(_path(), mode=ctypes.RTLD_GLOBAL)
    return _lib


def init():
    L = lib()
    flag = ctypes.c_int(0)
    L.MPI_Initialized(ctypes.byref(flag))
    if not flag.value:
        rc = L.MPI_Init(None, None)
        if rc:
            raise RuntimeError(f"MPI_Init failed: {rc}")
    L.MPI_Comm_set_errhandler(C.MPI_COMM_WORLD, MPI_ERRORS_RETURN)
    r, s = ctypes.c_int(), ctypes.c_int()
    L.MPI_Comm_rank(C.MPI_COMM_WORLD, ctypes.byref(r))
    L.MPI_Comm_size(C.MPI_COMM_WORLD, ctypes.byref(s))
    return r.value, s.value


def finalize():
    if _lib is not None:
        for op in _ops:
            _lib.MPI_Op_free(ctypes.byref(op[0]))
        _ops.clear()
        _lib.MPI_Finalize()


def ptr(a):
    if a is None:
        return None
    if a is _IN_PLACE:
        return _IN_PLACE
    return ctypes.c_void_p(a.ctypes.data)


def dtype_handle(a):
    return HANDLE_OF_NP[np.dtype(a.dtype)]


def user_op(fn, npdt, commute=False):
    """MPI_Op_create over a Python function (operators.jl:72-88)."""
    def cb(invec, inoutvec, plen, pdt):
        sz = ctypes.c_int(0)  # bytes per element of the (maybe derived) datatype
        lib().MPI_Type_size(pdt[0], ctypes.byref(sz))
        nb = plen[0] * sz.value
        a = np.ctypeslib.as_array((ctypes.c_char * nb).from_address(invec)).view(npdt)
        b = np.ctypeslib.as_array((ctypes.c_char * nb).from_address(inoutvec)).view(npdt)
        b[:] = np.asarray(fn(a, b), dtype=npdt)

    f = _USER_FN(cb)
    h = ctypes.c_int(0)
    rc = lib().MPI_Op_create(f, int(bool(commute)), ctypes.byref(h))
    if rc:
        raise RuntimeError(f"MPI_Op_create: {rc}")
    _ops.append((h, f))
    return h.value


def bcast_bytes(raw: bytes, root: int, comm: int) -> bytes:
    buf = ctypes.create_string_buffer(raw, len(raw))
    rc = lib().MPI_Bcast(buf, len(raw), C.MPI_BYTE, root, comm)
    if rc:
        raise RuntimeError(f"MPI_Bcast: {rc}")
    return buf.raw
