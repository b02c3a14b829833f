"""The one-rank-per-GPU signalling protocol, executed on the 1-GPU test box
(VERDICT r04 "what's missing" 1).

Ranks on different GPUs store their barrier words and LL lines into each
other's UNCACHED signal arrays / LL areas (hipDeviceMallocUncached, imported
through `sig_h` / `ll_h`), and no host gate holds them back: each rank's
`rw_mask` holds its own bit only (DESIGN §3 "one memory type per writer /
reader pair").  On one GPU every peer is same-device, so by default every
pair takes the ordinary-memory arrays and the gate instead.
`MPIGX_PEER_MEM=xdev` (an agreed, init-only knob) makes comm_init treat
every peer as if on another GPU; with `MPIGX_SHARED_GATE=0` that is the code
a rank bound to its own GPU runs, except for the device share (grid caps),
which stays.  Each worker reports the protocol it actually ran
(`mpigx_comm_diag_peer_mem`) and these tests check it before the parity
results: the MPICH golden fixtures (staged, LL and zero-copy paths), the
headline sizes on whole buffers, the MPICH large-count fixtures and the
zero-copy view protocol — at n = 8 too, the rank count of the driver's
8-GPU node.

The reference call behind all of it is MPI.Allreduce! and friends,
/root/reference/src/collective.jl:698-700 (and :605-618, :29-37, :295-307,
:489-501, :760-768, :834-842), as they run on 8 GPUs."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

XDEV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_TIMEOUT_MS": "30000",
        "MPIGX_PEER_MEM": "xdev", "MPIGX_SHARED_GATE": "0"}
GOLDEN_ENV = dict(XDEV, MPIGX_MAX_BLOCKS="16", MPIGX_STAGING_BYTES=str(64 << 20))


def _run(worker, n, env, timeout=900):
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", worker), n, timeout=timeout, extra_env=env)
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    res = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"nfail"' in l]
    return rcs, res, msg


def _check_protocol(res, n):
    """Every rank ran the cross-GPU protocol: own bit only in rw_mask, while
    every peer is on the same device."""
    full = (1 << n) - 1
    for x in res:
        rw, same = x["peer_mem"]
        assert rw == 1 << x["rank"], x
        assert same == full, x


@pytest.mark.parametrize("n", [2, 3, 4, 8])
def test_golden_collectives_xdev(n):
    """(~23 s) Every MPICH golden case (Allreduce / Reduce / Bcast / Allgather /
    Alltoall / Scan / Exscan / v-collectives, LL step and tuner cases)."""
    rcs, res, msg = _run("golden_worker.py", n, GOLDEN_ENV)
    assert all(rc == 0 for rc in rcs), msg
    assert len(res) == n, msg
    _check_protocol(res, n)
    assert all(x["nfail"] == 0 and x["checks"] > 200 for x in res), res


@pytest.mark.parametrize("n", [2, 4, 8])
def test_golden_collectives_zero_copy_xdev(n):
    """(~23 s) The zero-copy paths (pull, push, pull-push, ring, zero-copy Reduce /
    Scan / Bcast relay) at every fixture size."""
    env = dict(GOLDEN_ENV, MPIGX_ZC_MIN="1", MPIGX_ZC_REQUIRE="1")
    rcs, res, msg = _run("golden_worker.py", n, env)
    assert all(rc == 0 for rc in rcs), msg
    assert len(res) == n, msg
    _check_protocol(res, n)
    assert all(x["nfail"] == 0 and x["checks"] > 200 for x in res), res


@pytest.mark.parametrize("n", [2, 4, 8])
def test_headline_sizes_xdev(n):
    """(~17 s) 256 MiB Allreduce (whole buffer), 512 MiB Bcast / Allgather /
    Alltoall, 64 Mi-element Scan / Exscan / Reduce, every algorithm at 16 MiB
    and 1 MiB, on the production grid."""
    rcs, res, msg = _run("headline_worker.py", n, dict(XDEV, MPIGX_HEADLINE_EXTRA="1"))
    assert all(rc == 0 for rc in rcs), msg
    assert len(res) == n, msg
    _check_protocol(res, n)
    assert all(x["nfail"] == 0 for x in res), res


def test_mpich_large_fixtures_xdev():
    """(~5 s) MPICH 4,194,307-element Allreduce / Reduce and 1,048,579-element Scan /
    Exscan fixtures at n = 5 through every algorithm; the host gate stays on
    here (5 ranks on one GPU run torch compares between the calls)."""
    env = dict(XDEV, MPIGX_SHARED_GATE="1", MPIGX_TIMEOUT_MS="60000")
    rcs, res, msg = _run("large_worker.py", 5, env, timeout=600)
    assert all(rc == 0 for rc in rcs), msg
    assert len(res) == 5, msg
    _check_protocol(res, 5)
    assert all(x["nfail"] == 0 for x in res), res


def test_zero_copy_views_xdev():
    """(~3 s) Optimistic launches on cached views, a rank alone switching buffers
    (the abort verdict through the completion word), import agreement."""
    env = dict(XDEV, MPIGX_MAX_BLOCKS="16", MPIGX_STAGING_BYTES=str(64 << 20))
    rcs, res, msg = _run("zc_worker.py", 2, env, timeout=600)
    assert all(rc == 0 for rc in rcs), msg
    assert len(res) == 2, msg
    _check_protocol(res, 2)
    assert all(x["nfail"] == 0 for x in res), res


@pytest.mark.parametrize("worker", ["headline_worker.py", "golden_worker.py"])
def test_production_grid_xdev(worker):
    """(~9 s) Two ranks, the cross-GPU signalling AND the production grid: without
    the shared-GPU residency headroom (MPIGX_SHARE_HEADROOM=0) every
    collective kernel of a 2-rank communicator gets 256 blocks, as on a GPU of
    its own (bench r05p: pull / push / pull-push phases report 256 blocks),
    so the per-block barrier slots of blocks 128-255 run the uncached
    protocol too.  Headline sizes on whole buffers; the MPICH fixtures through
    the zero-copy paths."""
    env = dict(XDEV, MPIGX_SHARE_HEADROOM="0")
    if worker == "headline_worker.py":
        env["MPIGX_HEADLINE_EXTRA"] = "1"
    else:
        env.update(MPIGX_ZC_MIN="1", MPIGX_ZC_REQUIRE="1", MPIGX_STAGING_BYTES=str(64 << 20))
    rcs, res, msg = _run(worker, 2, env)
    assert all(rc == 0 for rc in rcs), msg
    assert len(res) == 2, msg
    _check_protocol(res, 2)
    assert all(x["nfail"] == 0 for x in res), res
