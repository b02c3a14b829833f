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


def _ring_step_simulation(inputs, dtname, opname, nch, round_elems):
    """The ring schedule of csrc/kernels.hpp ring_body played out message by
    message (per ring, per step: position p folds chunk p-s-1 with the left
    neighbour's partial as inout, then the allgather hands final chunks right)."""
    n = len(inputs)
    count = inputs[0].shape[0]
    vec = max(1, 16 // np.dtype(M.DTYPES[dtname][1]).itemsize)
    strides = M.ring_strides(n, nch)
    recv = [np.empty_like(inputs[0]) for _ in range(n)]
    for off in range(0, count, round_elems):
        cnt = min(round_elems, count - off)
        part = -(-(-(-cnt // len(strides))) // (n * vec)) * (n * vec)
        chunk = part // n
        for k, st in enumerate(strides):
            p0, p1 = min(k * part, cnt), min(k * part + part, cnt)
            rank_at = [(i * st) % n for i in range(n)]

            def sl(c):
                lo = min(p0 + c * chunk, p1)
                return slice(off + lo, off + min(lo + chunk, p1))
            stage = [dict() for _ in range(n)]
            for s in range(n - 1):
                new = [dict() for _ in range(n)]
                for pos in range(n):
                    q, left = rank_at[pos], rank_at[(pos - 1) % n]
                    c = (pos - s - 1) % n
                    acc = inputs[left][sl(c)] if s == 0 else stage[left][c]
                    val = M.apply_op(opname, dtname, acc, inputs[q][sl(c)])
                    if s == n - 2:
                        recv[q][sl(c)] = val
                    else:
                        new[q][c] = val
                stage = new
            for t in range(n - 1):
                snap = [x.copy() for x in recv]
                for pos in range(n):
                    q, left = rank_at[pos], rank_at[(pos - 1) % n]
                    c = (pos - t) % n
                    recv[q][sl(c)] = snap[left][sl(c)]
    return recv


@pytest.mark.parametrize("n", [2, 3, 5, 8])
def test_ring_oracle_matches_step_simulation(n):
    """oracle fold_ring (the association the ring kernel is checked against on
    the GPU) equals the ring schedule simulated step by step, on every rank;
    integer results equal MPICH's; float SUM stays within sum_tolerance of
    MPICH's pairwise tree."""
    rng = np.random.default_rng(n)
    for dt, op, count in (("FLOAT", "SUM", 1000), ("FLOAT", "MAX", 333), ("INT32_T", "SUM", 517),
                          ("BFLOAT16", "SUM", 999), ("DOUBLE", "SUM", 64)):
        if dt == "BFLOAT16":
            ins = [M.f32_to_bf16(rng.uniform(-1, 1, count).astype(np.float32)) for _ in range(n)]
        elif dt == "INT32_T":
            ins = [rng.integers(-2**31, 2**31, count, dtype=np.int64).astype(np.int32) for _ in range(n)]
        else:
            ins = [rng.uniform(-1, 1, count).astype(M.DTYPES[dt][1]) for _ in range(n)]
        for nch in (1, 2, 4):
            for rnd in (count, 16 * n * 4):
                sim = _ring_step_simulation(ins, dt, op, nch, rnd)
                exp = M.fold_ring(ins, dt, op, nch, rnd)
                for q in range(n):
                    assert same_bits(sim[q], exp, dt == "BFLOAT16"), (dt, op, nch, rnd, q)
        mp = M.allreduce(ins, dt, op)[0]
        if dt == "INT32_T":
            assert np.array_equal(M.fold_ring(ins, dt, op), mp)
        if dt in ("FLOAT", "DOUBLE") and op == "SUM":
            err = np.abs(M.fold_ring(ins, dt, op).astype(np.float64) - mp.astype(np.float64))
            assert (err <= M.sum_tolerance(ins, dt)).all()


def test_ring_strides():
    assert M.ring_strides(8, 4) == [1, 7, 3, 5]
    assert M.ring_strides(2, 4) == [1]
    assert M.ring_strides(6, 4) == [1, 5]
    for n in range(2, 17):
        for st in M.ring_strides(n, 4):
            assert sorted((i * st) % n for i in range(n)) == list(range(n))


# ---------------------------------------------------------------------------
# Large counts: MPICH 3.3.2 recorded at 4,194,307
# (Allreduce / Reduce: f32 SUM, f64 SUM, f32 MAX with +-0 / inf / NaN /
# denormal edges) and 1,048,579 elements (Int64 Scan / Exscan BOR, f64 Scan
# SUM) at n = 5 and 8 (tests/golden/make_large_golden.sh).  The fixture holds
# sampled output spans — prefix, tail and +-64 elements around every
# Rabenseifner block boundary — and the inputs are regenerated from their
# splitmix64 seeds (gen_inputs.splitmix_input), so the headline-size regime
# is pinned by MPICH itself, not by extrapolation from 1,100 elements.
# ---------------------------------------------------------------------------
def _large():
    import json
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(here, "mpich_large_manifest.json")) as f:
        cases = json.load(f)
    return cases, np.load(os.path.join(here, "mpich_large.npz"))


LARGE, LARGE_ARR = _large()


@pytest.mark.parametrize("case", LARGE, ids=[c["id"] for c in LARGE])
def test_oracle_matches_mpich_large_counts(case):
    from gen_inputs import splitmix_input
    n, dt, op = case["n"], case["dtype"], case["op"]
    ins = [splitmix_input(case["kind"], case["seed"], q, case["count"], bool(case["edge"])) for q in range(n)]
    coll = case["coll"]
    if coll == "allreduce":
        outs = {0: M.fold_rsag(ins, dt, op)}
        assert case["count"] * ins[0].itemsize > 2048  # the Rabenseifner regime (what fold_rsag restates)
    elif coll == "reduce":
        outs = {case["root"]: M.reduce(ins, dt, op, case["root"])}
    elif coll == "scan":
        outs = dict(enumerate(M.scan(ins, dt, op)))
    else:
        outs = {q: v for q, v in enumerate(M.exscan(ins, dt, op)) if q > 0}
    checked = 0
    for q, full in outs.items():
        got = LARGE_ARR[f"{case['id']}.r{q}"].view(full.dtype)
        exp = np.concatenate([full[lo:hi] for lo, hi in case["spans"]])
        assert same_bits(exp, got), (case["id"], q)
        checked += 1
    assert checked == len(outs)
    if coll == "exscan":  # rank 0's recvbuf untouched (0xCD sentinel), as in collective.jl's Exscan!
        assert (LARGE_ARR[f"{case['id']}.r0"] == 0xCD).all()


def test_large_fixture_coverage():
    kinds = {(c["coll"], c["n"]) for c in LARGE}
    for coll in ("allreduce", "reduce", "scan", "exscan"):
        for n in (5, 8):
            assert (coll, n) in kinds
    assert max(c["count"] for c in LARGE) >= 4_194_304
