"""The one-sided oracle (oracle/rma_model.py) against MPICH 3.3.2's own
records (tests/golden/rma_golden.json, made by tests/golden/make_rma_golden.sh
from tests/spmd/rma_worker.py on host arrays): every valid accumulate /
get_accumulate record of the 12-type x 12-op matrix at n = 2, 3, 4 is
recomputed from the same operands and must match bit for bit, and the fixed
scenario records (test_onesided.jl, fetch chains, multi-origin sums) hold
the values the reference's tests assert."""
import json
import os
import sys

import numpy as np
import pytest

from oracle import rma_model as R

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "spmd"))
from rma_cases import K, operands  # noqa: E402


def gold():
    with open(os.path.join(HERE, "golden", "rma_golden.json")) as f:
        return json.load(f)["runs"]


def bits(a):
    a = np.asarray(a)
    if a.dtype.kind in "fc":
        u = {2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize if a.dtype.kind == "f" else
                                                       a.dtype.itemsize // 2]
        return [format(int(v), "x") for v in a.view(u).reshape(-1)]
    return [int(v) for v in a.reshape(-1)]


@pytest.mark.parametrize("n", [2, 3, 4])
def test_accumulate_matrix_matches_mpich(n):
    runs = gold()[str(n)]
    checked = 0
    for r in range(n):
        src = (r - 1) % n
        for x in runs[r]:
            if x["case"] != "acc":
                continue
            dt = np.dtype(x["dt"])
            salt = 2 if x["fetch"] else 1
            v = R.valid(x["op"], R.NP_TO_MPI[dt])
            assert v == (not x.get("invalid", False)), x
            if not v:
                continue
            init = operands(dt, x["op"], 100 + r, salt + 10 * src)
            org = operands(dt, x["op"], src, salt)
            if x["op"] == "NO_OP" and not x["fetch"]:
                assert x["rc"] == 9 and x["win"] == bits(init)  # MPICH rejects NO_OP in MPI_Accumulate
                continue
            assert x["rc"] == 0
            new, _ = R.accumulate(init, org, x["op"])
            assert x["win"] == bits(new), (r, x["dt"], x["op"], x["fetch"])
            if x["fetch"]:
                # my result buffer holds what MY target ((r+1) % n) had in my range before my op
                t = (r + 1) % n
                _, old_t = R.accumulate(operands(dt, x["op"], 100 + t, salt + 10 * r), operands(dt, x["op"], r, salt),
                                        x["op"])
                assert x["res"] == bits(old_t)
            checked += 1
    assert checked >= n * 150


@pytest.mark.parametrize("n", [2, 3, 4])
def test_reference_scenarios_hold(n):
    runs = gold()[str(n)]
    by = [{x["case"]: x for x in recs} for recs in runs]
    # test_onesided.jl assertions
    for r in range(n):
        assert by[r]["fence_get"]["received"] == [(r + 1) % n] * n
        assert by[r]["dynamic_result"]["value"] == r + 5
        assert by[r]["shared_cols"] == {"case": "shared_cols", "c0": True, "c1": True}
    assert by[0]["lock_put"]["buf"] == list(range(n))
    assert by[0]["get_accumulate"]["result"] == [3] * n
    assert by[1]["after_gacc"]["buf"] == [5] * n
    assert by[0]["after_acc"]["buf"] == [0] * n
    assert by[0]["dynamic_fetch_and_op"]["received"] == list(range(n))
    # multi-origin integer accumulates are order-independent
    assert by[0]["multi_origin"]["win"][:4] == [n * (n + 1) // 2] * 2 + [(1 << n) - 1] * 2
    assert by[0]["shared_lock_acc"]["win"][:2] == [n * (n + 1)] * 2
