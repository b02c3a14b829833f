"""A rank that reaches a collective late or never (tests/spmd/late_worker.py):
a late rank is waited for (MPI semantics, collective.jl:698-700: past
MPIGX_TIMEOUT_MS, exact results); a vanished one, or one whose communicator
failed, fails the waiting ranks' call within seconds instead of hanging them.

Two configurations: `gate` — ranks sharing the GPU meet on the host first
(shared_gate, the test-box default); `xdev` — no gate and the cross-GPU
signalling (MPIGX_PEER_MEM=xdev), i.e. what a rank on its own GPU runs: the
early ranks' KERNELS wait, their hosts watch the peers and cancel the wait
only for a dead or broken peer (mpigx.cpp finish, PeerView.cancel; VERDICT
r04 item 2)."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_TIMEOUT_MS": "2000"}
XDEV = dict(ENV, MPIGX_SHARED_GATE="0", MPIGX_PEER_MEM="xdev")
CONFIGS = {"gate": ENV, "xdev": XDEV}
WORKER = os.path.join(ROOT, "tests", "spmd", "late_worker.py")


def _results(outs):
    return [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"scenario"' in l]


# every case waits 2.5 x the 2 s timeout for the late rank: four cover the
# protocols (host gate; one-rank-per-GPU blocking, stream-ordered, and a
# rank late on its own stream), the rest are `slow`
SLOW = pytest.mark.slow
@pytest.mark.parametrize("cfg,n,scenario", [("gate", 2, "late"), pytest.param("gate", 4, "late", marks=SLOW),
                                             ("xdev", 2, "late"),
                                             pytest.param("xdev", 2, "late_small", marks=SLOW),
                                             pytest.param("xdev", 3, "late", marks=SLOW),
                                             pytest.param("xdev", 2, "late_vx", marks=SLOW),
                                             pytest.param("xdev", 2, "late_so", marks=SLOW),
                                             ("xdev", 2, "late_so_small"),
                                             pytest.param("gate", 3, "late_so_small", marks=SLOW),
                                             pytest.param("xdev", 2, "late_p2p", marks=SLOW),
                                             ("xdev", 2, "late_stream")])
def test_late_rank_is_waited_for(cfg, n, scenario):
    """(~32 s) A rank 2.5 x MPIGX_TIMEOUT_MS late — on its host, or on its
    GPU behind earlier stream work (late_stream) — is waited
    for: exact results, no error."""
    rcs, outs = launch(WORKER, n, timeout=240, extra_env=CONFIGS[cfg], args=(scenario,))
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-2000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    res = _results(outs)
    assert len(res) == n and all(not x["fails"] for x in res), res
    early = [x["late_call_s"] for x in res if x["rank"] != n - 1]
    # they waited past their 2 s timeout (late_stream: the late rank's GPU
    # work is sized by a calibrated torch.cuda._sleep, so only "well past")
    assert min(early) >= (1.5 if scenario == "late_stream" else 2.0) * 2.0, res


@pytest.mark.parametrize("cfg,scenario", [("gate", "gone"), pytest.param("xdev", "gone", marks=SLOW),
                                          ("xdev", "gone_so"), pytest.param("xdev", "gone_p2p", marks=SLOW)])
def test_vanished_rank_fails_the_call(cfg, scenario):
    """(~8 s) A rank that exits without finalizing fails its peers' next call within seconds."""
    n = 3
    rcs, outs = launch(WORKER, n, timeout=240, extra_env=CONFIGS[cfg], args=(scenario,))
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-2000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    res = _results(outs)
    assert len(res) == n - 1, msg
    assert all(not x["fails"] and x["gone_call_s"] < 30 for x in res), res
    assert all(rc == 0 for rc in rcs[: n - 1]), msg


@pytest.mark.parametrize("cfg", ["gate", "xdev"])
def test_broken_peer_fails_the_call(cfg):
    """(~7 s) ADVICE r04: a rank whose communicator already failed never reaches the
    gate or launches; its peers learn it from the shm block (ShmRank.broken)
    and fail within seconds instead of waiting for it."""
    n = 3
    rcs, outs = launch(WORKER, n, timeout=240, extra_env=CONFIGS[cfg], args=("broken",))
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-2000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    res = _results(outs)
    assert len(res) == n, msg
    assert all(not x["fails"] for x in res), res
    assert all(x["broken_call_s"] < 30 for x in res if x["rank"] != n - 1), res
    assert all(rc == 0 for rc in rcs), msg
