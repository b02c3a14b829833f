"""Derived datatypes, host side (no GPU): libmpigx's MPI_Type_* constructors
(types.cpp) must give the lb / extent / true extent / size MPICH 3.3.2 gives
for every type of tests/spmd/types_cases.py (tests/golden/types_golden.json,
recorded by tests/golden/gen_types_golden.py), including the reference's
test_datatype.jl expectations extent == cld(sizeof(T), align) * align."""
import json
import os
import sys

import numpy as np
import pytest

import mpigx as MPI

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "spmd"))
from types_cases import BOUNDARY, BOUNDARY2, NTUPLE3, build  # noqa: E402


def gold():
    with open(os.path.join(HERE, "golden", "types_golden.json")) as f:
        return {t["name"]: t for t in json.load(f)["types"]}


def test_type_bounds_match_mpich():
    g = gold()
    built = build(MPI)
    assert len(built) == len(g)
    import ctypes
    for name, dt in built:
        lb, ex = MPI.Types.extent(dt)
        tl, te = ctypes.c_longlong(), ctypes.c_longlong()
        assert MPI.lib().mpigx_type_get_true_extent(dt.val, ctypes.byref(tl), ctypes.byref(te)) == 0
        got = (lb, ex, tl.value, te.value, MPI.Types.size(dt))
        want = tuple(g[name][k] for k in ("lb", "extent", "true_lb", "true_extent", "size"))
        assert got == want, (name, got, want)


@pytest.mark.parametrize("T,al", [(BOUNDARY, 8), (BOUNDARY2, 8), (NTUPLE3, 1)])
def test_reference_extent_rule(T, al):
    """test_datatype.jl: MPI.Types.extent(MPI.Datatype(T)) == (0, cld(sz, al) * al)."""
    sz = T.itemsize
    assert MPI.Types.extent(MPI.Datatype(T)) == (0, -(-sz // al) * al)


def test_view_buffers_follow_buffers_jl():
    """buffers.jl:104-117: strided 1-D view -> vector(len, 1, stride); dense
    N-D sub-block -> subarray of the parent, count 1."""
    X = np.arange(16.0).reshape(4, 4)
    b = MPI.Buffer(X[:, 1])  # strided column (row-major parent)
    assert b.count == 1 and MPI.Types.size(b.datatype) == 4 * 8
    assert MPI.Types.extent(b.datatype) == (0, (3 * 4 + 1) * 8)
    b = MPI.Buffer(X[1:3, 2:4])
    assert b.count == 1 and b.data.ctypes.data == X.ctypes.data and MPI.Types.size(b.datatype) == 4 * 8
    assert MPI.Types.extent(b.datatype) == (0, 16 * 8)
    b = MPI.Buffer(X[0, :])  # contiguous view: a plain buffer
    assert b.count == 4 and b.datatype == MPI.Datatype(np.float64)


def test_invalid_constructor_arguments():
    import ctypes
    out = ctypes.c_int()
    L = MPI.lib()
    assert L.mpigx_type_contiguous(-1, MPI.Datatype(np.int32).val, ctypes.byref(out)) == MPI.consts.MPI_ERR_COUNT
    assert L.mpigx_type_contiguous(2, 12345, ctypes.byref(out)) == MPI.consts.MPI_ERR_TYPE
    sizes = (ctypes.c_int * 2)(4, 4)
    sub = (ctypes.c_int * 2)(2, 5)
    st = (ctypes.c_int * 2)(0, 0)
    assert L.mpigx_type_create_subarray(2, sizes, sub, st, 56, MPI.Datatype(np.int32).val,
                                        ctypes.byref(out)) == MPI.consts.MPI_ERR_ARG
