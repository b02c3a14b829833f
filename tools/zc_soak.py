#!/usr/bin/env python3
"""Diagnostic SPMD worker (launch: REPRO_SCRIPT=tools/zc_soak.py
tools/scan_repro_launch.py N): the remote-store zero-copy kernels in a loop —
Allreduce! of 64 MiB f32 with the pull-push, pull and push two-shots forced,
Reduce! (MAX, Int32, 64 MiB) and Bcast! (128 MiB) to and from a rotating
root — SOAK_REPS times, every result checked exactly (integer-valued floats,
so any association gives the same sum).  Prints {"rank", "nbad"}."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))

import torch  # noqa: E402

import mpigx as MPI  # noqa: E402


def main():
    comm = MPI.Init()
    r, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
    reps = int(os.environ.get("SOAK_REPS", 50))
    cnt = 16 << 20
    x = torch.full((cnt,), float(r + 1), device="cuda")
    y = torch.empty_like(x)
    want = float(n * (n + 1) // 2)
    xi = torch.full((cnt,), r, dtype=torch.int32, device="cuda")
    b = torch.empty(32 << 20, device="cuda")
    nbad = 0
    for it in range(reps):
        for algo in ("pullpush", "pull", "push"):
            MPI.set_knob(comm, "ALGO", algo)
            y.zero_()
            MPI.Allreduce_(x, y, MPI.SUM, comm)
            nbad += int(not bool((y == want).all()))
        MPI.set_knob(comm, "ALGO", None)
        root = it % n
        out = torch.zeros_like(xi) if r == root else None
        MPI.Reduce_(xi, out, MPI.MAX, root, comm)
        if r == root:
            nbad += int(not bool((out == n - 1).all()))
        b.fill_(float(it) if r == root else -1.0)
        MPI.Bcast_(b, root, comm)
        nbad += int(not bool((b == float(it)).all()))
        if it % 10 == 0:
            print(f"r{r} it {it} t={time.time():.3f}", file=sys.stderr, flush=True)
    MPI.Barrier(comm)
    MPI.Finalize()
    print(json.dumps({"rank": r, "n": n, "reps": reps, "nbad": nbad}), flush=True)
    sys.exit(1 if nbad else 0)


if __name__ == "__main__":
    main()
