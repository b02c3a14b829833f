"""Communicator agreement guards (tests/spmd/knob_worker.py): path-selecting
knobs compared at init and changed only collectively, the ranks-per-device
guard and grid cap, agreement on zero-copy import failures, and
the LL flag generation wrap."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_TIMEOUT_MS": "20000"}
W = os.path.join(ROOT, "tests", "spmd", "knob_worker.py")


def _run(n, scenario, **env):
    rcs, outs = launch(W, n, timeout=300, extra_env=dict(ENV, MPIGX_TEST_SCENARIO=scenario, **env))
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    res = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"nfail"' in l]
    assert len(res) == n and all(x["nfail"] == 0 for x in res), res
    return res


@pytest.mark.parametrize("scenario", ["mismatch_init", "bad_name"])
def test_knob_mismatch_fails_at_init(scenario):
    """(~7 s) Path-selecting knobs that differ between ranks fail comm init on every rank."""
    extra = {"MPIGX_ALGO": "warp"} if scenario == "bad_name" else {}
    res = _run(2, scenario, **extra)
    assert all(x["code"] == 12 for x in res), res


def test_set_knob_is_collective():
    """(~4 s) mpigx_comm_set_knob changes a path-selecting knob collectively; results stay exact across the change."""
    _run(2, "set_knob")


@pytest.mark.parametrize("n", [2, 4])
def test_device_share_and_grid_cap(n):
    """(~8 s) Ranks sharing a device are counted and the spinning kernels' grids capped for residency."""
    res = _run(n, "share")
    print(res[0])


def test_device_share_limit():
    """(~3 s) More ranks per device than MPIGX_MAX_RANKS_PER_DEVICE fail init with MPI_ERR_OTHER."""
    res = _run(2, "share_limit", MPIGX_MAX_RANKS_PER_DEVICE="1")
    assert all(x["code"] == 15 for x in res), res


def test_zero_copy_import_failure_agreed():
    """(~4 s) A failed peer import is agreed by every rank, which all take the staged path: exact results."""
    _run(2, "import_fail")


@pytest.mark.parametrize("base", [(1 << 31) - 12, (1 << 31) - 36])
def test_ll_flag_generation_wrap(base):
    """(~6 s) LL flags across the 2^31 epoch generation boundary (area cleared, no stale flag accepted)."""
    _run(2, "ll_wrap", MPIGX_EPOCH_BASE=str(base))
