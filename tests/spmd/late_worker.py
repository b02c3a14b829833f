"""SPMD worker: a rank that reaches a collective late, or never (ranks
sharing one GPU, so every launch goes through the host gate, mpigx.cpp
shared_gate).

* late — the last rank sleeps on the host for 2.5 x MPIGX_TIMEOUT_MS before
  a 16 MiB zero-copy Allreduce; the others are already in it.  MPI semantics:
  the call waits for it and every rank gets the exact sum (the gate holds the
  early ranks on the host, so no device barrier times out).  A second call
  right after must be exact too.
* gone — after one good call the last rank exits without finalizing; the
  others' next Allreduce must fail (MPIError) within seconds instead of
  waiting for ever.
Launched by tests/test_late_rank_gpu.py.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "mpi.jl_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import mpigx as MPI  # noqa: E402


def main():
    scenario = sys.argv[1]
    comm = MPI.Init()
    r, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
    timeout_s = int(os.environ["MPIGX_TIMEOUT_MS"]) / 1000.0
    count = (16 << 20) // 4
    send = torch.full((count,), float(r + 1), device="cuda")
    recv = torch.empty(count, device="cuda")
    want = float(n * (n + 1) // 2)
    out = {"rank": r, "n": n, "scenario": scenario}
    fails = []

    MPI.Allreduce_(send, recv, MPI.SUM, comm)
    if not bool((recv == want).all()):
        fails.append("first call")
    if scenario == "late":
        if r == n - 1:
            time.sleep(2.5 * timeout_s)
        recv.fill_(-1)
        t0 = time.time()
        MPI.Allreduce_(send, recv, MPI.SUM, comm)
        out["late_call_s"] = round(time.time() - t0, 3)
        if not bool((recv == want).all()):
            fails.append("late call")
        recv.fill_(-1)
        MPI.Allreduce_(send, recv, MPI.SUM, comm)
        if not bool((recv == want).all()):
            fails.append("call after")
        MPI.Barrier(comm)
        MPI.Finalize()
    elif scenario == "gone":
        if r == n - 1:
            sys.stdout.flush()
            os._exit(0)
        t0 = time.time()
        try:
            MPI.Allreduce_(send, recv, MPI.SUM, comm)
            fails.append("no error with a vanished peer")
        except MPI.MPIError as e:
            out["error"] = str(e)
        out["gone_call_s"] = round(time.time() - t0, 3)
        torch.cuda.synchronize()
        out["fails"] = fails
        print(json.dumps(out), flush=True)
        os._exit(1 if fails else 0)  # no Finalize: a peer is gone
    out["fails"] = fails
    print(json.dumps(out), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
