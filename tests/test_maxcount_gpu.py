"""The largest message MPI.jl can hand the engine: `count` is a Cint
(collective.jl:698-700), so 2^31 - 1 elements, through Allreduce (default
zero-copy path with the tuner's calls, in place, staged rounds; int8 and
8 GiB f32), Reduce, Scan / Exscan, Bcast, Allgather (n·count elements in
recvbuf) and Alltoall, plus the local MPI.Op kernel over 8 inputs — exact
against results recomputed on the device (tests/spmd/maxcount_worker.py).
Any 32-bit element or byte offset left in a kernel or in the host's
partition arithmetic shows here and nowhere else."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_TIMEOUT_MS": os.environ.get("MPIGX_TIMEOUT_MS", "60000")}


@pytest.mark.parametrize("n", [2, 3])
def test_max_count(n):
    """(~12 s) Every collective at MPI.jl's largest count (2^31 - 1 elements)."""
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "maxcount_worker.py"), n, timeout=600, extra_env=ENV)
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    res = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"nfail"' in l]
    assert len(res) == n and all(x["nfail"] == 0 for x in res), res
