"""CPU-only checks of the drop-in boundary (no GPU calls):

* libmpigx.so loads and exports every function include/mpigx.h declares;
* handle/error constants in the header are MPICH's (deps/consts_mpich.jl,
  mpi.h:782-809) and agree with the Python mirror and the oracle;
* host-side validation (mpigx_op_valid / mpigx_type_size) reproduces MPICH's
  op x type matrix recorded in tests/golden/op_type_matrix.json.
"""
import ctypes
import os
import re

import pytest

import mpigx
from golden_io import op_type_matrix
from mpigx import consts as C
from oracle import mpich_model as M


def header_text():
    with open(mpigx.HEADER_PATH) as f:
        return f.read()


def declared_functions(path=None):
    """Functions of the MPI-facing header and the diagnostic one together
    (or of one header, `path`)."""
    paths = [path] if path else [mpigx.HEADER_PATH, mpigx.DIAG_HEADER_PATH]
    out = set()
    for p in paths:
        with open(p) as f:
            txt = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
        out |= set(re.findall(r"^\s*int\s+(mpigx_\w+)\s*\(", txt, flags=re.M))
    return sorted(out)


def test_diagnostics_live_outside_the_mpi_facing_header():
    """the diagnostic exports (phase stamps, slot and
    mapping checks, tuner statistics, probes) are declared in
    include/mpigx_diag.h, not in the MPI-facing include/mpigx.h."""
    public = declared_functions(mpigx.HEADER_PATH)
    diag = declared_functions(mpigx.DIAG_HEADER_PATH)
    assert not set(public) & set(diag)
    assert not [f for f in public if "_diag_" in f or (f.startswith("mpigx_comm_") and f.endswith(
        ("_stats", "_stamps", "_probe")))], public
    assert {"mpigx_comm_diag_slots", "mpigx_comm_diag_state", "mpigx_comm_diag_mapcheck",
            "mpigx_comm_set_stamps"} <= set(diag)


def header_defines():
    return {k: int(v) for k, v in re.findall(r"#define\s+(MPIGX_\w+)\s+(-?\d+)\s*$", header_text(), flags=re.M)}


def test_library_exports_every_declared_symbol():
    L = mpigx.lib()
    fns = declared_functions()
    assert len(fns) >= 25
    missing = [f for f in fns if not hasattr(L, f)]
    assert not missing, missing
    # and the Python binding declares prototypes for all of them
    from mpigx._lib import PROTOTYPES
    assert sorted(PROTOTYPES) == fns


def test_constants_match_mpich():
    d = header_defines()
    for name, (handle, _, kind) in M.DTYPES.items():
        assert d[f"MPIGX_{name}"] == handle, name
        assert getattr(C, f"MPI_{name}" if name != "BFLOAT16" else "MPIGX_BFLOAT16") == handle
    for name, handle in M.OPS.items():
        assert d[f"MPIGX_{name}"] == handle == getattr(C, f"MPI_{name}")
    for cls in ("SUCCESS", "ERR_BUFFER", "ERR_COUNT", "ERR_TYPE", "ERR_COMM", "ERR_ROOT", "ERR_OP", "ERR_ARG",
                "ERR_OTHER", "ERR_INTERN"):
        assert d[f"MPIGX_{cls}"] == getattr(C, f"MPI_{cls}")


def test_op_type_matrix_host_validation():
    L = mpigx.lib()
    m = op_type_matrix()
    for key, cls in m.items():
        dt, op = key.split("/")
        assert L.mpigx_op_valid(M.DTYPES[dt][0], M.OPS[op]) == cls, key
    # bf16 extension: like FLOAT
    for op in M.OPS:
        assert L.mpigx_op_valid(C.MPIGX_BFLOAT16, M.OPS[op]) == M.op_valid("BFLOAT16", op)
    assert L.mpigx_op_valid(12345, C.MPI_SUM) == C.MPI_ERR_TYPE
    assert L.mpigx_op_valid(C.MPI_FLOAT, 777) == C.MPI_ERR_OP


def test_type_sizes():
    L = mpigx.lib()
    sz = ctypes.c_int()
    for name, (handle, npdt, _) in M.DTYPES.items():
        assert L.mpigx_type_size(handle, ctypes.byref(sz)) == 0
        import numpy as np
        assert sz.value == np.dtype(npdt).itemsize, name
    assert L.mpigx_type_size(1, ctypes.byref(sz)) == C.MPI_ERR_TYPE


def test_error_strings_and_null_comm():
    assert "Invalid MPI_Op" in mpigx.error_string(C.MPI_ERR_OP)
    L = mpigx.lib()
    # a NULL communicator is rejected before any device work
    assert L.mpigx_allreduce(None, None, 1, C.MPI_FLOAT, C.MPI_SUM, None) == C.MPI_ERR_COMM
    assert L.mpigx_barrier(None) == C.MPI_ERR_COMM
    uid = mpigx._lib.UniqueId()
    assert L.mpigx_get_unique_id(ctypes.byref(uid)) == 0
    raw = ctypes.string_at(ctypes.addressof(uid), 128)
    assert raw.startswith(b"/mpigx-")


def test_python_mirror_op_mapping():
    """operators.jl:39-45: Julia functions -> built-in ops; others are user ops."""
    import operator

    import torch
    assert mpigx.Op(operator.add, torch.float32).val == C.MPI_SUM
    assert mpigx.Op(operator.mul, torch.complex64).val == C.MPI_PROD
    assert mpigx.Op(max, torch.int32).val == C.MPI_MAX
    assert mpigx.Op(min, float).val == C.MPI_MIN
    assert mpigx.Op(operator.and_, torch.int64).val == C.MPI_BAND
    assert mpigx.Op(operator.xor, torch.uint8).val == C.MPI_BXOR
    # & on floats is not a built-in (operators.jl:43-45 restricts to integers)
    assert mpigx.Op(operator.and_, torch.float32).val is None
    u = mpigx.Op(lambda x, y: 2 * x + y - x, torch.int64)
    assert u.val is None and u.fn is not None


def test_python_mirror_datatypes():
    """datatypes.jl:29-60 + the by-size mapping of other primitives (:281-284)."""
    import torch
    D = mpigx.Datatype
    assert D(torch.float32).val == C.MPI_FLOAT
    assert D(torch.float64).val == C.MPI_DOUBLE
    assert D(torch.int64).val == C.MPI_INT64_T
    assert D(torch.complex128).val == C.MPI_C_DOUBLE_COMPLEX
    assert D(torch.bfloat16).val == C.MPIGX_BFLOAT16
    assert D(torch.float16).val == C.MPI_UINT16_T
    assert D(torch.bool).val == C.MPI_UINT8_T
    assert D(int).val == C.MPI_INT64_T
    with pytest.raises(TypeError):
        D(str)


def test_own_handles_never_alias_mpich():
    """User ops and derived datatypes live in libmpigx's own handle space
    (csrc/handles.hpp).  An op or type MPI.jl created in libmpi (MPICH user op
    0x98000000 | k, derived type 0x8c000000 | k) must be rejected with
    MPI_ERR_OP / MPI_ERR_TYPE, never resolve to a libmpigx object; a freed
    handle is rejected even after its slot is reused."""
    L = mpigx.lib()
    FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                          ctypes.POINTER(ctypes.c_int))
    fn = FN(lambda a, b, n, t: None)
    ops = []
    for _ in range(3):
        op = ctypes.c_int()
        assert L.mpigx_op_create(fn, 0, ctypes.byref(op)) == 0
        ops.append(op.value)
    for h in ops:
        assert h & 0xFC000000 == 0x3C000000 and h & 0xFFFF, hex(h)
        com = ctypes.c_int(7)
        assert L.mpigx_op_commutative(h, ctypes.byref(com)) == 0 and com.value == 0
    com = ctypes.c_int()
    for k in range(4):  # MPICH direct / indirect user-op handles
        for foreign in (0x98000000 | k, 0xD8000000 | k):
            foreign = ctypes.c_int(foreign - (1 << 32)).value
            assert L.mpigx_op_commutative(foreign, ctypes.byref(com)) == C.MPI_ERR_OP
            f = ctypes.c_int(foreign)
            assert L.mpigx_op_free(ctypes.byref(f)) == C.MPI_ERR_OP
    # free, then reuse the slot: the old handle stays invalid
    old = ctypes.c_int(ops[0])
    assert L.mpigx_op_free(ctypes.byref(old)) == 0 and old.value == 0x18000000  # MPI_OP_NULL
    assert L.mpigx_op_commutative(ops[0], ctypes.byref(com)) == C.MPI_ERR_OP
    again = ctypes.c_int()
    assert L.mpigx_op_create(fn, 1, ctypes.byref(again)) == 0
    assert again.value != ops[0] and again.value & 0xFFFF == ops[0] & 0xFFFF  # same slot, new generation
    assert L.mpigx_op_commutative(ops[0], ctypes.byref(com)) == C.MPI_ERR_OP
    for h in (again.value, ops[1], ops[2]):
        x = ctypes.c_int(h)
        assert L.mpigx_op_free(ctypes.byref(x)) == 0
    # derived datatypes
    t = ctypes.c_int()
    assert L.mpigx_type_contiguous(4, C.MPI_FLOAT, ctypes.byref(t)) == 0
    assert t.value & 0xFC000000 == 0x3C000000 and t.value & 0xFFFF
    assert L.mpigx_type_commit(ctypes.byref(t)) == 0
    sz = ctypes.c_int()
    assert L.mpigx_type_size(t.value, ctypes.byref(sz)) == 0 and sz.value == 16
    for k in range(4):
        foreign = ctypes.c_int(0x8C000000 | k).value
        assert L.mpigx_type_size(foreign, ctypes.byref(sz)) == C.MPI_ERR_TYPE
    # user ops and datatypes are different handle classes
    assert L.mpigx_op_commutative(t.value, ctypes.byref(com)) == C.MPI_ERR_OP
    freed = t.value
    assert L.mpigx_type_free(ctypes.byref(t)) == 0
    assert L.mpigx_type_size(freed, ctypes.byref(sz)) == C.MPI_ERR_TYPE


def test_knob_constants_match_the_python_mirror():
    """include/mpigx.h MPIGX_KNOB_* / MPIGX_ALGO_* == mpigx.KNOBS / mpigx.ALGOS."""
    txt = re.sub(r"/\*.*?\*/", "", header_text(), flags=re.S)
    d = {k: int(v) for k, v in re.findall(r"#define\s+(MPIGX_\w+)\s+(-?\d+)\s*$", txt, flags=re.M)}
    knobs = {k[len("MPIGX_KNOB_"):]: v for k, v in d.items() if k.startswith("MPIGX_KNOB_") and k != "MPIGX_KNOB_COUNT"}
    assert knobs == mpigx.KNOBS
    assert d["MPIGX_KNOB_COUNT"] == len(knobs)
    algos = {k[len("MPIGX_ALGO_"):].lower(): v for k, v in d.items() if k.startswith("MPIGX_ALGO_")}
    assert {("auto" if k == "auto" else k): v for k, v in algos.items()} == \
        {k: v for k, v in mpigx.ALGOS.items() if k}


def test_libmpi_op_carries_its_function():
    """MPI.jl's Op(val, fptr) (operators.jl:20, :77-79): the mirror keeps both,
    and copies keep the function (the engine re-registers it, api._op_val)."""
    from mpigx._lib import USER_FN
    f = USER_FN(lambda a, b, n, t: None)
    op = mpigx.libmpi_op(0x98000001, f, iscommutative=True)
    assert op.val == 0x98000001 and op.fptr is f and op.iscommutative
    assert mpigx.Op(op).fptr is f
    assert mpigx.SUM.fptr is None


def test_count_is_a_cint():
    """collective.jl:698-700 passes `count` as Cint: 2^31 - 1 goes through,
    2^31 is Julia's InexactError before any call (no silent wrap to a
    negative count in ctypes).  Handles are not counts: MPICH op handles
    such as 0x98000042 go through ctypes' int wrap as before."""
    from mpigx import api
    assert api._cint((1 << 31) - 1) == (1 << 31) - 1
    assert api._cint(-(1 << 31)) == -(1 << 31)
    for bad in (1 << 31, -(1 << 31) - 1, 1 << 40):
        with pytest.raises(api.InexactError):
            api._cint(bad)


def test_comm_world_is_live():
    """MPI.COMM_WORLD is the communicator Init() / Init_thread() built (MPI.jl's
    MPI.COMM_WORLD), not a copy of the pre-Init placeholder."""
    from mpigx import api
    saved = api.COMM_WORLD
    try:
        api.COMM_WORLD = "built-by-Init"
        assert mpigx.COMM_WORLD == "built-by-Init"
    finally:
        api.COMM_WORLD = saved
    assert mpigx.THREAD_SINGLE < mpigx.THREAD_FUNNELED < mpigx.THREAD_SERIALIZED < mpigx.THREAD_MULTIPLE == 3
    v = ctypes.c_int(-1)
    assert mpigx.lib().mpigx_query_thread(ctypes.byref(v)) == 0 and v.value == 3


def test_knob_env_names_follow_the_header_and_are_documented():
    """mpigx.cpp kKnobEnv[k] is the environment variable of MPIGX_KNOB_* index k
    (init reads it, and names it when ranks disagree), and INTEGRATION.md's
    knob table documents every one of them."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "mpi.jl_amd", "csrc", "mpigx.cpp")).read()
    m = re.search(r"kKnobEnv\[MPIGX_KNOB_COUNT\]\s*=\s*\{(.*?)\};", src, flags=re.S)
    assert m, "kKnobEnv table not found"
    env = re.findall(r'"(MPIGX_\w+)"', m.group(1))
    by_index = {v: k for k, v in mpigx.KNOBS.items()}
    assert env == ["MPIGX_" + by_index[i] for i in range(len(by_index))]
    doc = open(os.path.join(root, "INTEGRATION.md")).read()
    assert [e for e in env if f"| `{e}` |" not in doc] == []
