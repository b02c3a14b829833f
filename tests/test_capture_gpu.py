"""mpigx calls refuse a stream under HIP-graph capture (tests/spmd/capture_worker.py)."""
import json
import os

import pytest

from spmd_launch import launch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [2])
def test_capture_is_refused(n):
    """(~3 s) A call on a stream under HIP-graph capture is refused with MPI_ERR_OTHER before anything is enqueued; the capture and the communicator stay usable."""
    env = {"MPIGX_DEVICE": "0", "MPIGX_TIMEOUT_MS": "30000"}
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "capture_worker.py"), n, timeout=300, extra_env=env)
    summ = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"checks"' in l]
    assert all(rc == 0 for rc in rcs), "\n".join(o[-2000:] for o in outs)
    assert len(summ) == n and all(s["nfail"] == 0 for s in summ), summ
