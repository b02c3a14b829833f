"""SPMD worker: an mpigx call issued while its stream is being captured into
a HIP graph (torch.cuda.graph) is refused with MPI_ERR_OTHER before anything
is enqueued (mpigx.cpp check_comm): a replay would repeat the launch's epoch
and argument block, which the peers never expect again.  The capture and the
communicator both stay usable: after the refused call (blocking and
stream-ordered) the same Allreduce! outside the capture is exact.  Launched
by tests/test_capture_gpu.py."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))

import torch  # noqa: E402

import mpigx as MPI  # noqa: E402

FAIL = []
NCHECK = [0]


def check(cond, what):
    NCHECK[0] += 1
    if not bool(cond):
        FAIL.append(what)


def main():
    MPI.Init()
    comm = MPI.COMM_WORLD
    rank, size = MPI.Comm_rank(comm), MPI.Comm_size(comm)
    want = float(sum(q + 1 for q in range(size)))
    x = torch.full((4096,), float(rank + 1), device="cuda")
    check(bool((MPI.Allreduce(x, MPI.SUM, comm) == want).all()), "before capture")
    for blocking in (1, 0):
        MPI.api._check(MPI.lib().mpigx_comm_set_blocking(comm.val, blocking))
        y = torch.empty_like(x)
        torch.cuda.synchronize()
        g, s = torch.cuda.CUDAGraph(), torch.cuda.Stream()
        code = None
        try:
            with torch.cuda.graph(g, stream=s):
                MPI.Allreduce_(x, y, MPI.SUM, comm)
        except MPI.MPIError as e:
            code = e.code
        except Exception as e:  # noqa: BLE001 - the capture itself must not fail
            FAIL.append(f"blocking={blocking}: {type(e).__name__}: {e}")
        check(code == 15, f"blocking={blocking}: refused with MPI_ERR_OTHER (got {code})")
        torch.cuda.synchronize()
        y.zero_()
        MPI.Allreduce_(x, y, MPI.SUM, comm)
        torch.cuda.synchronize()
        check(bool((y == want).all()), f"blocking={blocking}: exact after the refused capture")
    MPI.api._check(MPI.lib().mpigx_comm_set_blocking(comm.val, 1))
    MPI.Barrier(comm)
    MPI.Finalize()
    print(json.dumps({"rank": rank, "checks": NCHECK[0], "failures": FAIL[:10], "nfail": len(FAIL)}), flush=True)
    sys.exit(1 if FAIL else 0)


if __name__ == "__main__":
    main()
