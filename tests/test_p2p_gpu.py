"""Point-to-point on device buffers: the scenario script
(tests/spmd/p2p_worker.py — the reference's test_sendrecv.jl, test_test.jl and
test_wait.jl plus matching-order, wildcard, cancel, truncation, PROC_NULL,
probe, mailbox-wrap and error cases) on ROCm tensors must reproduce the
records MPICH 3.3.2 produced on host arrays (tests/golden/p2p_golden.json)
exactly, at 2, 3 and 4 ranks sharing the box's GPU through hipIpc; and the
random-traffic worker checks payloads against the MPI matching model
(oracle/p2p_model.py) at up to 8 MiB per message."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_MAX_BLOCKS": "16", "MPIGX_TIMEOUT_MS": "30000",
       "MPIGX_STAGING_BYTES": str(64 << 20), "MPIGX_TEST_ARRAYTYPE": "ROCArray"}


def _records(outs):
    recs = {}
    for o in outs:
        for line in o.splitlines():
            if line.startswith("{") and '"records"' in line:
                d = json.loads(line)
                recs[d["rank"]] = d
    return recs


@pytest.mark.parametrize("n", [2, 3, 4])
def test_p2p_scenarios_device_match_mpich(n):
    """(~11 s) MPICH-recorded point-to-point scenarios reproduced on device at n = 2, 3, 4."""
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "p2p_worker.py"), n, timeout=600, extra_env=ENV)
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    recs = _records(outs)
    with open(os.path.join(ROOT, "tests", "golden", "p2p_golden.json")) as f:
        gold = json.load(f)["runs"][str(n)]
    for r in range(n):
        assert recs[r]["device"] is True
        assert recs[r]["failed"] is None, recs[r]["failed"]
        for got, want in zip(recs[r]["records"], gold[r]):
            assert got == want, (r, got, want)
        assert len(recs[r]["records"]) == len(gold[r])


@pytest.mark.parametrize("n,seed,maxb", [(2, 7, 8 << 20), (4, 11, 2 << 20), (3, 5, 1 << 16)])
def test_p2p_random_traffic_device(n, seed, maxb):
    """(~13 s) Random point-to-point traffic against the matching model (oracle/p2p_model.py)."""
    env = dict(ENV, P2P_SEED=str(seed), P2P_MAXB=str(maxb))
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "p2p_random_worker.py"), n, timeout=600, extra_env=env)
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    lines = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"checks"' in l]
    assert len(lines) == n and all(d["nbad"] == 0 and d["failed"] is None for d in lines), lines
