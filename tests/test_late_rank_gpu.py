"""A rank that reaches a collective late or never, ranks sharing one GPU
(tests/spmd/late_worker.py): a late rank is waited for (MPI semantics, past
MPIGX_TIMEOUT_MS, exact results); a vanished one fails the waiting ranks'
call within seconds instead of hanging them."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_TIMEOUT_MS": "2000"}
WORKER = os.path.join(ROOT, "tests", "spmd", "late_worker.py")


def _results(outs):
    return [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"scenario"' in l]


@pytest.mark.parametrize("n", [2, 4])
def test_late_rank_is_waited_for(n):
    rcs, outs = launch(WORKER, n, timeout=240, extra_env=ENV, args=("late",))
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-2000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    res = _results(outs)
    assert len(res) == n and all(not x["fails"] for x in res), res
    early = [x["late_call_s"] for x in res if x["rank"] != n - 1]
    assert min(early) >= 2.0 * 2.0, res  # they waited past their 2 s timeout


def test_vanished_rank_fails_the_call():
    n = 3
    rcs, outs = launch(WORKER, n, timeout=240, extra_env=ENV, args=("gone",))
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-2000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    res = _results(outs)
    assert len(res) == n - 1, msg
    assert all(not x["fails"] and x["gone_call_s"] < 30 for x in res), res
    assert all(rc == 0 for rc in rcs[: n - 1]), msg
