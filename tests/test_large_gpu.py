"""MPICH-recorded large-count fixtures through the HIP path (VERDICT r03 item
4): n = 5 and 8 ranks on the test box's GPU run every fixture case of their
rank count through every Allreduce / Reduce / Scan / Exscan algorithm and
compare the recorded output spans bit for bit (tests/spmd/large_worker.py).
The CPU-side pin of the same fixture against the oracle is
test_oracle_golden.py::test_oracle_matches_mpich_large_counts."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_TIMEOUT_MS": "60000"}


@pytest.mark.parametrize("n", [5, 8])
def test_mpich_large_fixtures_on_device(n):
    """(~11 s) MPICH-recorded 4,194,307 / 1,048,579-element collectives (mpich_large.npz) reproduced on device at n = 5, 8."""
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "large_worker.py"), n, timeout=600, extra_env=ENV)
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    res = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"nfail"' in l]
    assert len(res) == n and all(x["nfail"] == 0 for x in res), res
    assert all(x["cases"] == 9 and x["checked"] > 0 for x in res), res
