"""MPI.jl's collective test scripts (tests/spmd/ref_tests.py) in device mode —
the equivalent of JULIA_MPI_TEST_ARRAYTYPE=CuArray (test_allreduce.jl:4-9):
every buffer is a ROCm tensor and goes through libmpigx."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,cfg", [(2, "same"), (4, "same"), (3, "xdev"), (8, "xdev")])
def test_reference_suite_device(n, cfg):
    """cfg xdev: the one-rank-per-GPU signalling (MPIGX_PEER_MEM=xdev, no host
    gate; tests/test_xdev_gpu.py), at n = 8 the driver node's rank count."""
    env = {"MPIGX_TEST_ARRAYTYPE": "ROCArray", "MPIGX_DEVICE": "0", "MPIGX_MAX_BLOCKS": "16",
           "MPIGX_TIMEOUT_MS": "30000", "MPIGX_STAGING_BYTES": str(16 << 20)}
    if cfg == "xdev":
        env.update(MPIGX_PEER_MEM="xdev", MPIGX_SHARED_GATE="0")
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "ref_tests.py"), n, timeout=600, extra_env=env)
    summ = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"checks"' in l]
    assert all(rc == 0 for rc in rcs), "\n".join(o[-2000:] for o in outs)
    assert len(summ) == n and all(s["nfail"] == 0 and s["device"] for s in summ), summ


@pytest.mark.parametrize("n", [2, 3])
def test_reference_threads_device(n):
    """test/test_threads.jl in device mode (tests/spmd/threads_worker.py):
    Init_thread(THREAD_MULTIPLE), threaded Irecv! / Isend of one-element
    device views, Waitall on the main thread."""
    # the worker runs collectives of three communicators at once: their
    # spinning kernels must fit on the GPU together (MPIGX_CONCURRENT_COMMS)
    env = {"MPIGX_DEVICE": "0", "MPIGX_TIMEOUT_MS": "30000", "MPIGX_CONCURRENT_COMMS": "4"}
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "threads_worker.py"), n, timeout=300, extra_env=env)
    summ = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"checks"' in l]
    assert all(rc == 0 for rc in rcs), "\n".join(o[-2000:] for o in outs)
    assert len(summ) == n and all(s["nfail"] == 0 and s["provided"] == 3 for s in summ), summ


def test_concurrent_comms_stuck_is_an_error():
    """VERDICT r05 item 2 (~30 s): the threads worker's three-communicator
    case at n = 3 on one GPU with MPIGX_CONCURRENT_COMMS left at 1, where the
    three grids need not fit on the GPU together (round 5: stalled without
    end).  A launch stuck behind the other communicators' kernels now ends
    its call with MPI_ERR_OTHER within about MPIGX_TIMEOUT_MS (mpigx.cpp
    stuck_peer), naming MPIGX_CONCURRENT_COMMS; every thread of every rank
    comes back, and every result that is returned is exact."""
    env = {"MPIGX_DEVICE": "0", "MPIGX_TIMEOUT_MS": "5000", "MPIGX_CONCURRENT_COMMS": "1",
           "THREADS_MODE": "stuck"}
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "threads_worker.py"), 3, timeout=240, extra_env=env)
    summ = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"checks"' in l]
    stuck = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"stuck_results"' in l]
    assert all(rc == 0 for rc in rcs), "\n".join(o[-2000:] for o in outs)
    assert len(summ) == 3 and all(s["nfail"] == 0 for s in summ), summ
    print("stuck-mode results:", stuck)
    if any(s["errors"] for s in stuck):  # a stall happened: the engine said why
        assert any("MPIGX_CONCURRENT_COMMS" in o for o in outs), "\n".join(o[-2000:] for o in outs)
