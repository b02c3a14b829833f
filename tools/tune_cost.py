#!/usr/bin/env python3
"""Host cost of the measured algorithm choices: for each
size class, the wall time of the first calls on a fresh communicator (the
tuner's sampling calls: HIP event sync after each + one host exchange per
class) against the same calls on a communicator with MPIGX_AR_TUNE off.

    torchrun-style env (RANK, WORLD_SIZE, MASTER_*):  python3 tools/tune_cost.py

Rank 0 prints one JSON line: per size, the static per-call time, the first
`calls` tuned calls' total, and the extra cost of tuning that class.
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import mpigx as MPI  # noqa: E402


def main():
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    world = MPI.Init()
    calls = 12
    out = {"n": n, "calls": calls, "sizes": {}}
    for nb in (8 << 10, 64 << 10, 1 << 20, 4 << 20, 64 << 20):
        x = torch.rand(nb // 4, device="cuda")
        y = torch.empty_like(x)

        def run(comm, k):
            ts = []
            for _ in range(k):
                dist.barrier()
                t0 = time.perf_counter()
                MPI.Allreduce_(x, y, MPI.SUM, comm)
                ts.append(time.perf_counter() - t0)
            return ts

        static = MPI.Comm_dup(world)
        MPI.set_knob(static, "AR_TUNE", 0)
        run(static, 3)
        st = run(static, calls)
        tuned = MPI.Comm_dup(world)  # a fresh communicator: this size class is undecided
        tt = run(tuned, calls)
        per = sorted(st)[len(st) // 2]
        rec = torch.tensor([per, sum(tt), sum(tt[:2]), max(tt)], dtype=torch.float64)
        dist.all_reduce(rec, op=dist.ReduceOp.MAX)
        per, tot, first2, mx = rec.tolist()
        out["sizes"][f"{nb >> 10}KiB"] = {
            "static_us_per_call": round(per * 1e6, 1),
            "tuned_first_calls_total_us": round(tot * 1e6, 1),
            "tuning_extra_us": round((tot - calls * per) * 1e6, 1),
            "slowest_tuned_call_us": round(mx * 1e6, 1)}
        MPI.free(static)
        MPI.free(tuned)
    if rank == 0:
        print(json.dumps(out), flush=True)
    MPI.Finalize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
