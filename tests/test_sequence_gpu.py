"""The 8-rank Scan! / Exscan! / Reduce! sequence on a FRESH communicator
(tools/scan_repro.py): 64 Mi Int32 / Int64 elements, BAND / BOR / MAX, the
Reduce! root allocating its recvbuf right before the first zero-copy Reduce.
This is the sequence that stalled in round 3 (the root's entry-barrier word
never reached rank 0); the headline test reaches Reduce!
only after Allreduce! / Bcast! / Allgather! / Alltoall! on the same
communicator.  Every result is checked exactly (integer ops), every call has
per-block stamps on."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_TIMEOUT_MS": "30000"}


@pytest.mark.parametrize("n,cfg", [(8, "same"), (8, "xdev")])
def test_scan_exscan_reduce_sequence_fresh_comm(n, cfg):
    """(~8 s) cfg xdev: the one-rank-per-GPU signalling, no host gate (the early
    ranks' kernels wait on the device while their peers run torch work)."""
    env = dict(ENV, MPIGX_PEER_MEM="xdev", MPIGX_SHARED_GATE="0") if cfg == "xdev" else ENV
    rcs, outs = launch(os.path.join(ROOT, "tools", "scan_repro.py"), n, timeout=600, extra_env=env)
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-2500:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    res = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"nbad"' in l]
    assert len(res) == n and all(x["nbad"] == 0 for x in res), res
