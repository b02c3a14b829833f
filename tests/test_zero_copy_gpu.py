"""Zero-copy protocol on device buffers (tests/spmd/zc_worker.py): cached
views with no host exchange in the steady state, abort-and-retry when any
rank's buffers change, lockstep alternation, IN_PLACE and Alltoall — all
results exact."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_MAX_BLOCKS": "16", "MPIGX_TIMEOUT_MS": "30000",
       "MPIGX_STAGING_BYTES": str(64 << 20)}


@pytest.mark.parametrize("n", [2, 4])
def test_zero_copy_views(n):
    """(~8 s) Optimistic launches on cached zero-copy views, re-registration after a buffer change, exact results."""
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "zc_worker.py"), n, timeout=600, extra_env=ENV)
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    res = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"nfail"' in l]
    assert len(res) == n and all(x["nfail"] == 0 for x in res), res
    print(json.dumps(res[0]["host_cost"]))
