"""One-sided communication on device buffers: the
scenario script tests/spmd/rma_worker.py — the reference's test_onesided.jl
and test_shared_win.jl restated, the 12-type x 12-op Accumulate /
Get_accumulate matrix (NaN, +-0, ties, wraparound), Fetch_and_op chains,
multi-origin and shared-lock accumulates, chunked large Get_accumulate and
error classes — on ROCm tensors must reproduce the records MPICH 3.3.2
produced on host arrays (tests/golden/rma_golden.json) exactly, at 2, 3 and
4 ranks sharing the box's GPU through hipIpc.  Engine-only checks (erroneous
(op, type) pairs rejected with MPI_ERR_OP, window untouched) must all hold."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_MAX_BLOCKS": "16", "MPIGX_TIMEOUT_MS": "30000",
       "MPIGX_STAGING_BYTES": str(32 << 20), "MPIGX_TEST_ARRAYTYPE": "ROCArray"}


@pytest.mark.parametrize("n", [2, 3, 4])
def test_rma_scenarios_device_match_mpich(n, tmp_path):
    """(~15 s) test_onesided.jl / test_shared_win.jl restated and the Accumulate matrix: MPICH-recorded records reproduced at n = 2, 3, 4."""
    env = dict(ENV, RMA_OUT=str(tmp_path / "rma"))
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "rma_worker.py"), n, timeout=600, extra_env=env)
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    recs = {}
    for r in range(n):
        p = tmp_path / f"rma.{r}"
        if p.exists():
            recs[r] = json.loads(p.read_text())
    assert all(rc == 0 for rc in rcs), msg + "\n" + "\n".join(str(recs.get(r, {}).get("failed")) for r in range(n))
    with open(os.path.join(ROOT, "tests", "golden", "rma_golden.json")) as f:
        gold = json.load(f)["runs"][str(n)]
    for r in range(n):
        assert recs[r]["device"] is True
        assert recs[r]["failed"] is None, recs[r]["failed"]
        bad = [c for c in recs[r]["dev_checks"] if not c["ok"]]
        assert not bad, bad
        # 3 bitwise ops x 2 floats + 8 ops x 2 complex, Accumulate and Get_accumulate each; + BAND on f64
        assert len(recs[r]["dev_checks"]) == 45
        for got, want in zip(recs[r]["records"], gold[r]):
            assert got == want, (r, got, want)
        assert len(recs[r]["records"]) == len(gold[r])
