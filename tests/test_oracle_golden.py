"""Pins the CPU oracle (oracle/mpich_model.py) to MPICH 3.3.2 itself.

Every case in tests/golden/mpich_golden.npz was recorded by
tests/golden/gen_mpich_golden.c calling MPICH 3.3.2 with the argument shapes of
MPI.jl's ccall sites (src/collective.jl:34,:304,:498,:615,:698,:765,:839) at
n = 1..8 ranks; the oracle must reproduce every rank's output bit for bit
(NaN payloads excepted).
"""
import collections

import numpy as np
import pytest

from golden_io import load, op_type_matrix, same_bits, typed
from oracle import mpich_model as M

CASES, ARR = load()


def oracle_outputs(c, ins):
    coll, op, dt = c["coll"], c["op"], c["dtype"]
    if coll == "reduce_local":
        return [M.reduce_local(ins[0], ins[1], dt, op)], None
    if coll == "allreduce":
        return M.allreduce(ins, dt, op), None
    if coll == "reduce":
        return [M.reduce(ins, dt, op, c["root"])], [c["root"]]
    if coll == "scan":
        return M.scan(ins, dt, op), None
    if coll == "exscan":
        return M.exscan(ins, dt, op)[1:], list(range(1, c["n"]))
    if coll == "bcast":
        return M.bcast(ins, c["root"]), None
    if coll == "allgather":
        return M.allgather(ins), None
    if coll == "alltoall":
        return M.alltoall(ins, c["count"]), None
    raise KeyError(coll)


VCOLLS = ("gather", "gatherv", "scatter", "scatterv", "allgatherv", "alltoallv")


def v_expected(c, ins):
    """rank -> expected output prefix for a v-collective golden case."""
    n, seed, base, root = c["n"], c["seed"], c["count"], c["root"]
    K = [[M.vcnt(seed, a, b, base) for b in range(16)] for a in range(16)]
    coll = c["coll"]
    if coll == "gather":
        return {root: M.gather(ins, base, root)}
    if coll == "gatherv":
        return {root: M.gatherv(ins, [K[p][0] for p in range(n)])}
    if coll == "scatter":
        return dict(enumerate(M.scatter(ins[root], base, n)))
    if coll == "scatterv":
        return dict(enumerate(M.scatterv(ins[root], [K[p][1] for p in range(n)])))
    if coll == "allgatherv":
        return dict(enumerate(M.allgatherv(ins, [K[p][2] for p in range(n)])))
    return dict(enumerate(M.alltoallv(ins, [[K[p][q] for q in range(n)] for p in range(n)])))


GROUPS = collections.defaultdict(list)
for _c in CASES:
    if _c["coll"] not in VCOLLS:
        GROUPS[(_c["coll"], _c["n"])].append(_c)


@pytest.mark.parametrize("coll", VCOLLS)
def test_oracle_matches_mpich_vcollectives(coll):
    bad, tot = [], 0
    for c in CASES:
        if c["coll"] != coll:
            continue
        dt = M.DTYPES[c["dtype"]][1]
        ins = typed(ARR[c["id"] + ".in"], dt)
        outs = ARR[c["id"] + ".out"]
        for r, e in v_expected(c, ins).items():
            tot += 1
            got = np.ascontiguousarray(outs[r][: e.nbytes]).view(dt)
            if not (same_bits(got, e) and (outs[r][e.nbytes:] == 0xCD).all()):
                bad.append((c["id"], r))
    assert tot > 0 and not bad, bad[:10]


@pytest.mark.parametrize("key", sorted(GROUPS), ids=lambda k: f"{k[0]}-n{k[1]}")
def test_oracle_matches_mpich(key):
    bad = []
    for c in GROUPS[key]:
        dt = M.DTYPES[c["dtype"]][1]
        ins = typed(ARR[c["id"] + ".in"], dt)
        outs = typed(ARR[c["id"] + ".out"], dt)
        got, ranks = oracle_outputs(c, ins)
        exp = [outs[r] for r in ranks] if ranks is not None else (outs if c["coll"] != "reduce_local" else [outs[0]])
        if not all(same_bits(g, e) for g, e in zip(got, exp)):
            bad.append(c["id"])
    assert not bad, f"oracle differs from MPICH on {bad[:10]}"


def test_exscan_rank0_untouched():
    """MPICH leaves rank 0's Exscan recvbuf untouched (collective.jl:834 doc)."""
    for c in CASES:
        if c["coll"] == "exscan":
            raw = ARR[c["id"] + ".out"][0]
            assert (raw == 0xCD).all(), c["id"]


def test_op_type_matrix_matches_oracle():
    m = op_type_matrix()
    for key, cls in m.items():
        dt, op = key.split("/")
        assert M.op_valid(dt, op) == cls, key


def test_fixture_coverage():
    colls = {c["coll"] for c in CASES}
    assert colls == {"reduce_local", "allreduce", "reduce", "scan", "exscan", "bcast", "allgather", "alltoall",
                     *VCOLLS}
    assert {c["n"] for c in CASES if c["coll"] == "allreduce"} == {2, 3, 4, 5, 6, 8}
    # the Rabenseifner regime (> 2048 B) is exercised for f32 and f64
    assert any(c["count"] * 4 > 2048 and c["dtype"] == "FLOAT" and c["coll"] == "allreduce" for c in CASES)


def test_bf16_rounding_definition():
    """bf16 has no MPICH counterpart (parity unpinned): check the RNE helper."""
    f = np.array([1.0, 1.00390625, 1.01171875, -2.5, np.inf, np.nan], dtype=np.float32)
    b = M.f32_to_bf16(f)
    back = M.bf16_to_f32(b)
    assert back[0] == 1.0 and back[1] == 1.0 and back[2] == 1.015625 and back[3] == -2.5
    assert np.isinf(back[4]) and np.isnan(back[5])
