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
    """(~15 s) cfg xdev: the one-rank-per-GPU signalling (MPIGX_PEER_MEM=xdev, no host
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
    """(~8 s) test/test_threads.jl in device mode (tests/spmd/threads_worker.py):
    Init_thread(THREAD_MULTIPLE), threaded Irecv! / Isend of one-element
    device views, Waitall on the main thread."""
    # the worker runs collectives of three communicators at once: their
    # spinning kernels must fit on the GPU together (MPIGX_CONCURRENT_COMMS)
    # ... and every stream of a rank its own hardware queue: HIP maps streams
    # onto GPU_MAX_HW_QUEUES queues (4 by default), and two communicators'
    # kernels sharing one queue wait for each other in queue order —
    # differently on each rank (r06b: a deadlock the stuck-peer rule turned
    # into MPI_ERR_OTHER after 30 s; INTEGRATION.md "Threads")
    env = {"MPIGX_DEVICE": "0", "MPIGX_TIMEOUT_MS": "30000", "MPIGX_CONCURRENT_COMMS": "4",
           "GPU_MAX_HW_QUEUES": "16"}
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "threads_worker.py"), n, timeout=300, extra_env=env)
    summ = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"checks"' in l]
    assert all(rc == 0 for rc in rcs), "\n".join(o[-2000:] for o in outs)
    assert len(summ) == n and all(s["nfail"] == 0 and s["provided"] == 3 for s in summ), summ


@pytest.mark.parametrize("k,mode", [(1, "stuck"), (3, "stuck"), (1, "stuck_so")])
def test_concurrent_comms_beyond_residency(k, mode):
    """(~16 s) VERDICT r05 item 2: three communicators' 64 MiB Allreduce! at
    once from three threads per rank, n = 3 on one GPU, no host gate (the
    one-rank-per-GPU protocol), grids at their residency caps, rank 0 first
    (tests/spmd/threads_worker.py stuck_case).  k = 1: the grids cannot all
    be resident, which waited forever in round 5; now every call of every
    rank ends with MPI_ERR_OTHER within about MPIGX_TIMEOUT_MS and stderr
    names MPIGX_CONCURRENT_COMMS.  k = 3 (the knob at the number of
    communicators): exact.  stuck_so: the same three communicators with
    stream-ordered launches at k = 1 (the ranks launch together after each
    zero-copy view agreement): every thread comes back, exact or with the
    named MPI_ERR_OTHER from the process-wide watcher."""
    env = {"MPIGX_DEVICE": "0", "MPIGX_TIMEOUT_MS": "3000", "MPIGX_CONCURRENT_COMMS": str(k),
           "MPIGX_MAX_BLOCKS": "4096", "MPIGX_SHARED_GATE": "0", "MPIGX_PEER_MEM": "xdev",
           "THREADS_MODE": mode, "GPU_MAX_HW_QUEUES": "16"}
    # the pull-push two-shot with ticket-dealt slices ends in ONE whole-launch
    # barrier (rank_barrier_grid): every block of every rank must be resident
    # at once, so grids that cannot all fit deadlock for certain when rank 0's
    # are resident first (blocking mode).  With per-block barriers only (the
    # tuner's other choices) blocks pair by index and the residency headroom
    # often lets them trickle through (r06h: k = 1 completed).  Stream-ordered,
    # the zero-copy view is agreed on the host before each launch, so the
    # ranks launch together and which grids win the slots is up to the GPU
    env.update(MPIGX_ALGO="pullpush", MPIGX_AR_SLICES="4")
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "threads_worker.py"), 3, timeout=240, extra_env=env)
    msg = "\n".join(o[-3000:] for o in outs)
    summ = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"checks"' in l]
    stuck = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"stuck_results"' in l]
    assert all(rc == 0 for rc in rcs), msg
    assert len(summ) == 3 and all(s["nfail"] == 0 for s in summ), summ
    assert len(stuck) == 3, msg
    if mode == "stuck_so":
        # every thread comes back: exact, or the named MPI_ERR_OTHER from the
        # process-wide watcher (stuck peer, or every rank in a launch that
        # other communicators' grids keep from completing)
        assert all(r is True or r == "MPIError 15" for s in stuck for r in s["stuck_results"]), stuck
        if any(s["errors"] for s in stuck):
            assert "MPIGX_CONCURRENT_COMMS" in msg, msg
    elif k == 1:
        assert all(s["errors"] >= 1 for s in stuck), stuck
        assert all(t < 3.0 * 3 + 10 for s in stuck for t in s["call_s"]), stuck
        assert "MPIGX_CONCURRENT_COMMS" in msg, msg
    else:
        assert all(r is True for s in stuck for r in s["stuck_results"]), stuck
