"""CPU restatement of MPICH 3.3.2's one-sided accumulate semantics — TEST
INFRASTRUCTURE ONLY (tests/ import it as the checker; libmpigx never does).

src/onesided.jl:186-219 ccalls MPI_Accumulate / MPI_Get_accumulate /
MPI_Fetch_and_op; the arithmetic happens in libmpi (MPICH 3.3.2, the library
MPI.jl's default MPICH_jll ships, Project.toml:10).  MPICH applies the origin
data to the target with its MPIR op loops, the window being ``inout`` and the
origin ``in`` (the user-function signature ``(invec, inoutvec)``), so
MAX keeps the window value only when it is strictly greater (NaN and tie
roles follow from that).  REPLACE stores the origin, NO_OP leaves the window
(fetch only); Get_accumulate / Fetch_and_op return the window's previous
contents.  Pinned by tests/golden/rma_golden.json, recorded from MPICH itself
(tests/golden/make_rma_golden.sh), in tests/test_rma_oracle.py.
"""
from __future__ import annotations

import numpy as np

from . import mpich_model as M

NP_TO_MPI = {
    np.dtype(np.int8): "INT8_T", np.dtype(np.uint8): "UINT8_T", np.dtype(np.int16): "INT16_T",
    np.dtype(np.uint16): "UINT16_T", np.dtype(np.int32): "INT32_T", np.dtype(np.uint32): "UINT32_T",
    np.dtype(np.int64): "INT64_T", np.dtype(np.uint64): "UINT64_T", np.dtype(np.float32): "FLOAT",
    np.dtype(np.float64): "DOUBLE", np.dtype(np.complex64): "C_FLOAT_COMPLEX",
    np.dtype(np.complex128): "C_DOUBLE_COMPLEX",
}


def valid(opname: str, dtname: str) -> bool:
    """RMA accepts the collective (op, type) matrix plus REPLACE / NO_OP."""
    return opname in ("REPLACE", "NO_OP") or M.op_valid(dtname, opname) == M.MPI_SUCCESS


def accumulate(window: np.ndarray, origin: np.ndarray, opname: str):
    """MPI_Get_accumulate on one target range: (new window, old window)."""
    old = window.copy()
    if opname == "REPLACE":
        return origin.astype(window.dtype, copy=True), old
    if opname == "NO_OP":
        return old.copy(), old
    return M.apply_op(opname, NP_TO_MPI[window.dtype], window, origin), old
