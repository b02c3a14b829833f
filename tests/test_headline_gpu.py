"""Parity at BASELINE's headline sizes on the default (size-selected,
zero-copy) paths — 256 MiB Allreduce, 512 MiB Bcast/Allgather/Alltoall,
64 Mi-element integer Scan/Exscan/Reduce (tests/spmd/headline_worker.py) — at
n = 2, 4 and 8 ranks sharing the one GPU of the test box, on the PRODUCTION
grid: no MPIGX_MAX_BLOCKS, so the collective kernels run the default 256-block
grid wherever the ranks-per-device residency cap allows it (n = 8 is capped
so that 8 grids fit the device).  The 256 MiB Allreduce is checked on the
whole buffer; at every n every algorithm also runs at 16 MiB and 1 MiB on
whole buffers, and one 1 GiB Allreduce is sampled."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_TIMEOUT_MS": "60000"}


@pytest.mark.parametrize("n", [2, 4, 8])
def test_headline_sizes(n):
    """(~15 s) The 256 MiB default Allreduce path (whole buffer) and every algorithm at 16 MiB / 1 MiB on the production grid, bit-exact against the oracle."""
    env = dict(ENV, MPIGX_HEADLINE_EXTRA="1")
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "headline_worker.py"), n, timeout=900, extra_env=env)
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    res = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"nfail"' in l]
    assert len(res) == n and all(x["nfail"] == 0 for x in res), res
