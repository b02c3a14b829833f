#!/usr/bin/env python3
"""One rank of a collective profile (tools/coll_prof.py starts n of these,
each under its own rocprofv3 when asked).

    RANK=r WORLD_SIZE=n MASTER_ADDR=127.0.0.1 MASTER_PORT=p \
        python3 tools/coll_rank.py --mib 256 --algo pull --iters 20

Blocking MPI.Allreduce!(SUM) f32 of `mib` MiB per rank through the algorithm
`algo` (the MPIGX_ALGO names; "auto" = the engine's own choice), `warmup`
untimed calls, `iters` timed calls (HIP events around each call on the comm
stream, max over ranks), then one call with the per-block phase timestamps on
(mpigx_comm_set_stamps).  Rank 0 prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import mpigx as MPI  # noqa: E402

PHASES = ("entry_barrier", "reduce_scatter", "mid_barrier", "allgather", "exit_barrier")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--algo", default="pull")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--slices", type=int, default=None, help="MPIGX_AR_SLICES knob (pull-push two-shot)")
    args = ap.parse_args()
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=n)
    comm = MPI.Init()
    if args.algo != "auto":
        MPI.set_knob(comm, "ALGO", args.algo)
    if args.slices is not None:
        MPI.set_knob(comm, "AR_SLICES", args.slices)
    dev = torch.device("cuda:0")
    count = (args.mib << 20) // 4
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    send = torch.rand(count, device=dev, generator=g) * 2 - 1
    recv = torch.empty_like(send)
    stream = torch.cuda.current_stream(dev)
    for _ in range(args.warmup):
        MPI.Allreduce_(send, recv, MPI.SUM, comm)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.iters)]
    dist.barrier()
    t0 = time.perf_counter()
    for a, b in ev:
        a.record(stream)
        MPI.Allreduce_(send, recv, MPI.SUM, comm)
        b.record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.iters
    dev_ms = sorted(a.elapsed_time(b) for a, b in ev)
    # one stamped call
    st = torch.zeros(1024 * 8, dtype=torch.int64, device=dev)
    MPI.lib().mpigx_comm_set_stamps(comm.val, ctypes.c_void_p(st.data_ptr()))
    MPI.Allreduce_(send, recv, MPI.SUM, comm)
    torch.cuda.synchronize()
    MPI.lib().mpigx_comm_set_stamps(comm.val, None)
    t = st.view(1024, 8)[:, :6].cpu().numpy().astype(np.int64)
    t = t[t[:, 0] > 0]
    phases = {}
    if t.size:
        d = np.diff(t, axis=1) / 100.0
        phases = {nm: round(float(np.median(d[:, k])), 2) for k, nm in enumerate(PHASES)}
        phases.update({nm + "_max": round(float(d[:, k].max()), 2) for k, nm in enumerate(PHASES)})
        phases["span_us"] = round(float(t[:, 5].max() - t[:, 0].min()) / 100.0, 2)
        phases["blocks"] = int(t.shape[0])
    mx = torch.tensor([wall, dev_ms[len(dev_ms) // 2], dev_ms[0]], dtype=torch.float64)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    allp = [None] * n
    dist.all_gather_object(allp, phases)
    ranks_share, cap = MPI.device_share(comm)
    if rank == 0:
        S = args.mib << 20
        print(json.dumps({
            "n": n, "mib": args.mib, "algo": args.algo, "iters": args.iters,
            "wall_ms": round(mx[0].item() * 1e3, 4), "device_ms_median": round(mx[1].item(), 4),
            "device_ms_min": round(mx[2].item(), 4),
            "busbw_GBps_device_median": round(S / (mx[1].item() / 1e3) * 2 * (n - 1) / n / 1e9, 1),
            "max_blocks": MPI.get_knob(comm, "MAX_BLOCKS"), "grid_cap": cap, "ranks_per_device": ranks_share,
            "phases_us_per_rank": allp}), flush=True)
    MPI.Finalize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
