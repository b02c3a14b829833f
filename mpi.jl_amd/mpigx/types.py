"""MPI.jl's `MPI.Types` module (src/datatypes.jl:62-318) and the derived
datatypes behind `Buffer(::SubArray)` (src/buffers.jl:98-117).

Every constructor makes the type twice when both sides exist: in libmpigx
(``mpigx_type_*``, types.cpp — device buffers; needs no GPU to build) and in
the host libmpi (``MPI_Type_*`` — numpy buffers), so one `Datatype` object
works with either kind of buffer, like MPI.jl's does with its one libmpi.
Names follow the reference (``commit!`` -> ``commit_``).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import consts as C
from . import hostmpi
from ._lib import lib
from .api import Datatype, MPIError, _check, _state

__all__ = ["Types"]

_HOST_OF = {}  # libmpigx derived handle -> host libmpi handle

MPI_ORDER_C, MPI_ORDER_FORTRAN = 56, 57


def host_handle(v):
    """Host libmpi handle for a libmpigx datatype handle (identity for predefined)."""
    return _HOST_OF.get(v, v)


def _hcheck(rc):
    if rc:
        raise MPIError(rc)


def _make(name, dev_call, host_call):
    dv = ctypes.c_int(0)
    _check(dev_call(ctypes.byref(dv)))
    hv = None
    if _state["host"]:
        h = ctypes.c_int(0)
        _hcheck(host_call(ctypes.byref(h)))
        hv = h.value
        _HOST_OF[dv.value] = hv
    return Datatype(dv.value, name, host_val=hv)


def _ints(xs):
    xs = [int(x) for x in xs]
    return (ctypes.c_int * max(1, len(xs)))(*xs)


class Types:
    """MPI.Types (datatypes.jl:62-318)."""

    @staticmethod
    def extent(dt):
        """(lb, extent) in bytes (datatypes.jl:75-84)."""
        lb, ex = ctypes.c_longlong(0), ctypes.c_longlong(0)
        _check(lib().mpigx_type_get_extent(Datatype(dt).val, ctypes.byref(lb), ctypes.byref(ex)))
        return lb.value, ex.value

    @staticmethod
    def host_extent(dt):
        """The same query answered by host libmpi (for parity checks)."""
        lb, ex = ctypes.c_long(0), ctypes.c_long(0)
        _hcheck(hostmpi.lib().MPI_Type_get_extent(Datatype(dt).host, ctypes.byref(lb), ctypes.byref(ex)))
        return lb.value, ex.value

    @staticmethod
    def size(dt):
        s = ctypes.c_longlong(0)
        _check(lib().mpigx_type_size_x(Datatype(dt).val, ctypes.byref(s)))
        return s.value

    @staticmethod
    def create_contiguous(count, oldtype):
        """datatypes.jl:97-106."""
        o = Datatype(oldtype)
        return _make(f"contiguous({count},{o.name})",
                     lambda p: lib().mpigx_type_contiguous(int(count), o.val, p),
                     lambda p: hostmpi.lib().MPI_Type_contiguous(int(count), o.host, p))

    @staticmethod
    def create_vector(count, blocklength, stride, oldtype):
        """datatypes.jl:135-145."""
        o = Datatype(oldtype)
        return _make(f"vector({count},{blocklength},{stride},{o.name})",
                     lambda p: lib().mpigx_type_vector(int(count), int(blocklength), int(stride), o.val, p),
                     lambda p: hostmpi.lib().MPI_Type_vector(int(count), int(blocklength), int(stride), o.host, p))

    @staticmethod
    def create_hvector(count, blocklength, stride_bytes, oldtype):
        """MPI_Type_create_hvector (byte stride): general strided views."""
        o = Datatype(oldtype)
        return _make(f"hvector({count},{blocklength},{stride_bytes},{o.name})",
                     lambda p: lib().mpigx_type_create_hvector(int(count), int(blocklength), int(stride_bytes), o.val,
                                                               p),
                     lambda p: hostmpi.lib().MPI_Type_create_hvector(int(count), int(blocklength),
                                                                     ctypes.c_long(int(stride_bytes)), o.host, p))

    @staticmethod
    def create_subarray(sizes, subsizes, offset, oldtype, rowmajor=False):
        """datatypes.jl:163-185 (column-major unless rowmajor)."""
        assert len(sizes) == len(subsizes) == len(offset)
        o = Datatype(oldtype)
        nd = len(sizes)
        order = MPI_ORDER_C if rowmajor else MPI_ORDER_FORTRAN
        a, b, c = _ints(sizes), _ints(subsizes), _ints(offset)
        return _make(f"subarray({list(sizes)},{list(subsizes)},{list(offset)},{o.name})",
                     lambda p: lib().mpigx_type_create_subarray(nd, a, b, c, order, o.val, p),
                     lambda p: hostmpi.lib().MPI_Type_create_subarray(nd, a, b, c, order, o.host, p))

    @staticmethod
    def create_struct(blocklengths, displacements, types):
        """datatypes.jl:197-213."""
        assert len(blocklengths) == len(displacements) == len(types)
        n = len(blocklengths)
        ts = [Datatype(t) for t in types]
        bl = _ints(blocklengths)
        dl = (ctypes.c_longlong * max(1, n))(*[int(d) for d in displacements])
        dv = _ints([t.val for t in ts])
        hv = _ints([t.host for t in ts])
        return _make(f"struct({list(blocklengths)},{list(displacements)})",
                     lambda p: lib().mpigx_type_create_struct(n, bl, dl, dv, p),
                     lambda p: hostmpi.lib().MPI_Type_create_struct(n, bl, dl, hv, p))

    @staticmethod
    def create_resized(oldtype, lb, extent):
        """datatypes.jl:235-245."""
        o = Datatype(oldtype)
        return _make(f"resized({o.name},{lb},{extent})",
                     lambda p: lib().mpigx_type_create_resized(o.val, int(lb), int(extent), p),
                     lambda p: hostmpi.lib().MPI_Type_create_resized(o.host, ctypes.c_long(int(lb)),
                                                                    ctypes.c_long(int(extent)), p))

    @staticmethod
    def commit_(dt):
        """commit! (datatypes.jl:256-261)."""
        v = ctypes.c_int(dt.val)
        _check(lib().mpigx_type_commit(ctypes.byref(v)))
        if dt.host_val is not None:
            h = ctypes.c_int(dt.host_val)
            _hcheck(hostmpi.lib().MPI_Type_commit(ctypes.byref(h)))
        return dt


# ---------------------------------------------------------------------------
# Datatype(T) for isbits structs and primitive types (datatypes.jl:263-316)
# ---------------------------------------------------------------------------
_STRUCT_CACHE = {}
_BY_SIZE = None


def _basic_by_size():
    from .api import UINT8_T, UINT16_T, UINT32_T, UINT64_T
    return ((8, UINT64_T), (4, UINT32_T), (2, UINT16_T), (1, UINT8_T))


def struct_datatype(npdt, commit=True):
    """numpy structured dtype (a Julia isbits struct: fields in declaration
    order at their offsets; consecutive fields of the same type merge into one
    block) or a void dtype 'V<n>' (a Julia primitive type: by size, split into
    8/4/2/1-byte blocks) -> a derived Datatype, as datatypes.jl:269-316."""
    key = (npdt, commit)
    if key in _STRUCT_CACHE:
        return _STRUCT_CACHE[key]
    bl, disp, types = [], [], []
    if npdt.fields is None:
        szrem = sz = npdt.itemsize
        d = 0
        for i, base in _basic_by_size():
            if sz == i:
                return base
            blk, szrem = divmod(szrem, i)
            if blk:
                bl.append(blk)
                disp.append(d)
                types.append(base)
                d += i * blk
    else:
        prev = None
        for name in npdt.names:
            F, off = npdt.fields[name][0], npdt.fields[name][1]
            if F.itemsize == 0:
                continue
            if prev is not None and F == prev:
                bl[-1] += 1
            else:
                bl.append(1)
                disp.append(off)
                if F.fields is not None or F.kind == "V":
                    types.append(struct_datatype(F, commit=False))
                else:
                    types.append(Datatype(F))
                prev = F
    dt = Types.create_struct(bl, disp, types)
    if commit:
        Types.commit_(dt)
    _STRUCT_CACHE[key] = dt
    return dt


# ---------------------------------------------------------------------------
# Buffer(view) (buffers.jl:98-117)
# ---------------------------------------------------------------------------
def _subarray_of(shape, strides, offset, total):
    """Dense sub-block view (element strides of a C-contiguous parent, unit
    inner stride) -> (parent sizes, starts), or None.  The parent's shape is
    recovered from the strides (numpy / torch keep only the storage owner)."""
    nd = len(shape)
    if strides[-1] != 1 or any(s <= 0 for s in strides):
        return None
    sizes = [0] * nd
    for d in range(1, nd):
        if strides[d - 1] % strides[d]:
            return None
        sizes[d] = strides[d - 1] // strides[d]
    starts, rem = [], offset
    for st in strides:
        q, rem = divmod(rem, st)
        starts.append(q)
    sizes[0] = max(starts[0] + shape[0], total // strides[0])
    if rem or any(starts[d] + shape[d] > sizes[d] for d in range(nd)):
        return None
    return sizes, starts


def view_buffer(a):
    """(data, count, datatype) for a non-contiguous numpy / torch view:
    a 1-D strided view is one element of vector(len, 1, stride) at the view
    (buffers.jl:104-109); an N-D dense sub-block is one element of a
    row-major subarray of its parent at the parent's base (buffers.jl:110-117;
    numpy / torch are row-major where Julia is column-major); anything else
    (stepped N-D slices) nests hvectors over the view's strides."""
    elt = Datatype(a.dtype)
    if isinstance(a, np.ndarray):
        item = a.itemsize
        shape, strides = a.shape, [s // item for s in a.strides]
        owner = a
        while isinstance(owner.base, np.ndarray):
            owner = owner.base
        offset = (a.ctypes.data - owner.ctypes.data) // item
        total = owner.nbytes // item
        base = owner
    else:
        item = a.element_size()
        shape, strides = tuple(a.shape), list(a.stride())
        offset = a.storage_offset()
        total = a.untyped_storage().nbytes() // item
        base = None
    if len(shape) == 1:
        return a, 1, Types.commit_(Types.create_vector(shape[0], 1, strides[0], elt))
    sub = _subarray_of(shape, strides, offset, total)
    if sub is not None:
        if base is None:  # the storage's first element, as a flat tensor
            base = a.as_strided((total,), (1,), 0)
        dt = Types.commit_(Types.create_subarray(sub[0], shape, sub[1], elt, rowmajor=True))
        return base, 1, dt
    dt = elt  # general strided view: innermost dimension first
    for n_, st in zip(reversed(shape), reversed(strides)):
        dt = Types.create_hvector(n_, 1, st * item, dt)
    return a, 1, Types.commit_(dt)


def _host_args(args):
    return tuple(_HOST_OF.get(x, x) if isinstance(x, int) and not isinstance(x, bool) else x for x in args)


C.MPI_ORDER_C, C.MPI_ORDER_FORTRAN = MPI_ORDER_C, MPI_ORDER_FORTRAN
