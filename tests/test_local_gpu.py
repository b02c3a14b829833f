"""Config 2 parity: the device MPI.Op kernels (mpigx_reduce_local_multi /
mpigx_reduce_local) against the MPICH-pinned oracle, bit for bit.

The fold of n buffers must equal what an n-rank MPICH Allreduce returns
(binomial regime <= 2 KiB, Rabenseifner regime above, operand roles
included), or the rank-ordered left fold in LINEAR order.
"""
import ctypes

import numpy as np
import pytest

from gen_inputs import make, valid_pairs
from golden_io import same_bits
from oracle import mpich_model as M

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

REPRESENTATIVE = ["INT8_T", "UINT8_T", "INT16_T", "UINT16_T", "INT32_T", "UINT32_T", "INT64_T", "UINT64_T",
                  "BYTE", "CHAR", "LONG", "FLOAT", "DOUBLE", "C_FLOAT_COMPLEX", "C_DOUBLE_COMPLEX", "BFLOAT16"]


@pytest.fixture(scope="module")
def L():
    import mpigx
    assert torch.cuda.is_available()
    return mpigx.lib()


def dev(a, pad=0):
    """numpy -> device uint8 tensor (optionally starting `pad` bytes into an allocation)."""
    raw = np.frombuffer(a.tobytes(), dtype=np.uint8)
    t = torch.empty(raw.size + pad + 16, dtype=torch.uint8, device="cuda")
    v = t[pad:pad + raw.size]
    v.copy_(torch.from_numpy(raw.copy()))
    return v


def host(t, like, count):
    return t.cpu().numpy().view(like.dtype)[:count]


def run_multi(L, ins, dtname, opname, order, pad=0):
    count = ins[0].size
    h = M.DTYPES[dtname][0]
    dins = [dev(x, pad) for x in ins]
    out = dev(np.zeros_like(ins[0]), pad)
    ptrs = (ctypes.c_void_p * len(ins))(*[t.data_ptr() for t in dins])
    rc = L.mpigx_reduce_local_multi(ptrs, len(ins), ctypes.c_void_p(out.data_ptr()), count, h, M.OPS[opname],
                                    order, None)
    assert rc == 0
    torch.cuda.synchronize()
    return host(out, ins[0], count)


def expected(ins, dtname, opname, order):
    if order == 1:
        return M.fold_linear(ins, dtname, opname)
    return M.allreduce(ins, dtname, opname)[0]


@pytest.mark.parametrize("dtname,opname", valid_pairs(REPRESENTATIVE))
def test_all_ops_types(L, dtname, opname):
    """(~1 s) Every valid (op, type) pair of the local fold, bit-exact against the MPICH-pinned oracle."""
    for n, count, seed in ((8, 1037, 1), (3, 517, 2), (5, 4099, 3), (2, 64, 4)):
        ins = make(dtname, opname, n, count, seed, edge=True)
        for order in (0, 1):
            got = run_multi(L, ins, dtname, opname, order)
            assert same_bits(got, expected(ins, dtname, opname, order), dtname == "BFLOAT16"), (n, count, order)


@pytest.mark.parametrize("n", [1, 2, 4, 6, 7, 8, 9, 12, 13, 15, 16])
def test_rank_counts(L, n):
    """(~1 s) The local fold at 1..16 inputs against the oracle's association."""
    for dtname, opname in (("FLOAT", "SUM"), ("FLOAT", "MAX"), ("INT64_T", "BXOR"), ("DOUBLE", "MIN")):
        for count in (7, 300, 20011):
            ins = make(dtname, opname, n, count, 10 + n, edge=True)
            for order in (0, 1):
                got = run_multi(L, ins, dtname, opname, order)
                assert same_bits(got, expected(ins, dtname, opname, order), dtname == "BFLOAT16"), (dtname, opname, n, count, order)


def test_full_shape_multi_vector(L):
    """(~1 s) The 8-buffer shape (SH_FULL, U vectors per thread): sizes with whole and
    partial U-blocks, Rabenseifner block boundaries inside a vector (count/8
    not a multiple of the vector width) and ragged tails, every op family."""
    for dtname, opname in (("FLOAT", "SUM"), ("FLOAT", "MAX"), ("BFLOAT16", "SUM"), ("BFLOAT16", "MAX"),
                           ("BFLOAT16", "MIN"), ("DOUBLE", "MIN"), ("INT32_T", "BAND"), ("C_FLOAT_COMPLEX", "PROD")):
        for count in ((1 << 20) + 13, 3 * 1024 * 8 + 5, 65536):
            ins = make(dtname, opname, 8, count, 77 + count, edge=True)
            got = run_multi(L, ins, dtname, opname, 0)
            assert same_bits(got, expected(ins, dtname, opname, 0), dtname == "BFLOAT16"), (dtname, opname, count)


def test_local_u_variants(L):
    """(~6 s) The 8-buffer shape at every vectors-per-thread variant
    (common.hpp local_u, round 6): U = 1 / 2 / 4 forced through
    MPIGX_LOCAL_U on ragged sizes with Rabenseifner boundaries inside
    vectors, and the host's own choice on both sides of its threshold (f32:
    U = 1 below 1 Mi elements per input, 4 from there), bit-exact against
    the oracle."""
    import os
    try:
        for u in ("1", "2", "4"):
            os.environ["MPIGX_LOCAL_U"] = u
            for dtname, opname in (("FLOAT", "SUM"), ("BFLOAT16", "SUM"), ("DOUBLE", "MAX"), ("INT64_T", "BXOR")):
                for count in ((1 << 16) + 13, 3 * 1024 * 8 + 5):
                    ins = make(dtname, opname, 8, count, 91 + count, edge=True)
                    for order in (0, 1):  # MPICH tree / rank-ordered LINEAR
                        got = run_multi(L, ins, dtname, opname, order)
                        assert same_bits(got, expected(ins, dtname, opname, order), dtname == "BFLOAT16"), \
                            (u, dtname, count, order)
    finally:
        os.environ.pop("MPIGX_LOCAL_U", None)
    for dtname, opname, count in (("FLOAT", "SUM", (1 << 20) - 13), ("FLOAT", "MAX", (1 << 20) + 5),
                                  ("DOUBLE", "SUM", (1 << 19) + 3), ("INT32_T", "BOR", (4 << 20) + 7)):
        ins = make(dtname, opname, 8, count, 5 + count, edge=True)
        got = run_multi(L, ins, dtname, opname, 0)
        assert same_bits(got, expected(ins, dtname, opname, 0)), (dtname, opname, count)


def test_output_aliases_an_input(L):
    """(~2 s) The output written over one of the inputs (MPI_Reduce_local's
    inoutbuf; the in-place variants bench.py reports): every leaf of an
    element is loaded before its result is stored, so the result equals the
    out-of-place fold bit for bit — at both vectors-per-thread choices, with
    ragged tails and Rabenseifner boundaries inside vectors, tree and linear
    order."""
    for dtname, opname, count in (("FLOAT", "SUM", (1 << 20) + 13), ("FLOAT", "MAX", 3 * 1024 * 8 + 5),
                                  ("BFLOAT16", "SUM", (4 << 20) + 3), ("INT64_T", "BXOR", (1 << 19) + 7)):
        ins = make(dtname, opname, 8, count, 17 + count, edge=True)
        h = M.DTYPES[dtname][0]
        for order in (0, 1):
            for k in (0, 7):
                dins = [dev(x) for x in ins]
                ptrs = (ctypes.c_void_p * 8)(*[t.data_ptr() for t in dins])
                rc = L.mpigx_reduce_local_multi(ptrs, 8, ctypes.c_void_p(dins[k].data_ptr()), count, h, M.OPS[opname],
                                                order, None)
                assert rc == 0
                torch.cuda.synchronize()
                got = host(dins[k], ins[0], count)
                assert same_bits(got, expected(ins, dtname, opname, order), dtname == "BFLOAT16"), \
                    (dtname, opname, count, order, k)


def test_bf16_random_bit_patterns(L):
    """(~1 s) bf16 definition (fp32 compute, RNE to bf16 after every op, NaN quiet) on
    uniformly random 16-bit patterns — NaN payloads, infinities, denormals,
    rounding ties — through the packed pair ops (v_pk_add/mul_f32 +
    v_cvt_pk_bf16_f32) against the oracle's software rounding."""
    rng = np.random.default_rng(5)
    for n in (8, 5):
        for opname in ("SUM", "PROD", "MAX", "MIN"):
            ins = [rng.integers(0, 1 << 16, size=(1 << 18) + 3, dtype=np.uint16) for _ in range(n)]
            got = run_multi(L, ins, "BFLOAT16", opname, 0)
            assert same_bits(got, expected(ins, "BFLOAT16", opname, 0), True), (n, opname)


def test_unaligned_and_empty(L):
    """(~1 s) Unaligned inputs / output and empty counts through the local fold."""
    ins = make("FLOAT", "SUM", 8, 1001, 7)
    for pad in (1, 4, 8, 12):
        got = run_multi(L, ins, "FLOAT", "SUM", 0, pad=pad)
        assert same_bits(got, expected(ins, "FLOAT", "SUM", 0)), pad
    empty = [np.zeros(0, np.float32)] * 4
    ptrs = (ctypes.c_void_p * 4)(*([0] * 4))
    assert L.mpigx_reduce_local_multi(ptrs, 4, None, 0, M.DTYPES["FLOAT"][0], M.OPS["SUM"], 0, None) == 0


def test_invalid_pairs_rejected(L):
    """(~1 s) (op, type) pairs MPICH rejects return MPI_ERR_OP before any launch."""
    t = torch.zeros(16, dtype=torch.uint8, device="cuda")
    ptrs = (ctypes.c_void_p * 2)(t.data_ptr(), t.data_ptr())
    for dtname, opname, code in (("FLOAT", "BAND", 9), ("C_FLOAT_COMPLEX", "MAX", 9), ("BYTE", "SUM", 9),
                                 ("WCHAR", "SUM", 9)):
        rc = L.mpigx_reduce_local_multi(ptrs, 2, ctypes.c_void_p(t.data_ptr()), 4, M.DTYPES[dtname][0],
                                        M.OPS[opname], 0, None)
        assert rc == code
    assert L.mpigx_reduce_local_multi(ptrs, 2, ctypes.c_void_p(t.data_ptr()), 4, 12345, M.OPS["SUM"], 0,
                                      None) == 3


def test_reduce_local_matches_mpich_fixtures(L):
    """(~1 s) MPI_Reduce_local golden vectors (MPICH 3.3.2) through mpigx_reduce_local."""
    from golden_io import load, typed
    cases, arr = load()
    bad = []
    for c in cases:
        if c["coll"] != "reduce_local":
            continue
        dt = M.DTYPES[c["dtype"]][1]
        a, b = typed(arr[c["id"] + ".in"], dt)
        exp = typed(arr[c["id"] + ".out"], dt)[0]
        din, dio = dev(a), dev(b)
        rc = L.mpigx_reduce_local(ctypes.c_void_p(din.data_ptr()), ctypes.c_void_p(dio.data_ptr()), c["count"],
                                  M.DTYPES[c["dtype"]][0], M.OPS[c["op"]])
        assert rc == 0
        if not same_bits(host(dio, b, c["count"]), exp):
            bad.append(c["id"])
    assert not bad, bad


def test_full_size_property(L):
    """(~1 s) Config 2 at full size (8 x 256 MiB f32): SUM of (k+1)*ones in bf16-exact
    integers is exact, and linearity across two calls holds."""
    n, count = 8, 64 << 20
    ins = [torch.full((count,), float(k + 1), device="cuda") for k in range(n)]
    out = torch.empty(count, device="cuda")
    import mpigx
    mpigx.reduce_local_multi(ins, out, mpigx.SUM)
    torch.cuda.synchronize()
    assert torch.all(out == 36.0)
    mpigx.reduce_local_multi(ins, out, mpigx.MAX)
    torch.cuda.synchronize()
    assert torch.all(out == 8.0)
