"""Point-to-point measurements on device buffers (run as >= 2 ranks).

* ping-pong latency: rank 0 Send -> rank 1 Recv -> rank 1 Send -> rank 0 Recv,
  half round trip per size (the MPI "latency" convention);
* Sendrecv ring bandwidth: every rank sends S bytes to r+1 and receives S
  bytes from r-1 in one call; reports per-rank S / t and the xfer_kernel copy
  rate (2 S HBM bytes per rank: read the peer's buffer, write mine).

Prints one JSON line on rank 0.  Example (one GPU, 2 ranks sharing it):
  MPIGX_DEVICE=0 python -m torch.distributed.run --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29600 tools/p2p_bench.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))
import torch  # noqa: E402

import mpigx as MPI  # noqa: E402

comm = MPI.Init()
r, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
dev = f"cuda:{comm.device}"
res = {"n": n}
sizes = [int(v) for v in os.environ.get("P2P_SIZES", "8,4096,65536,1048576,16777216,268435456").split(",")]
for nb in sizes:
    x = torch.full((max(nb // 4, 1),), float(r), device=dev)
    y = torch.empty_like(x)
    it = 200 if nb <= (1 << 20) else (20 if nb <= (64 << 20) else 5)
    # ping-pong between 0 and 1
    def pingpong():
        if r == 0:
            MPI.Send(x, 1, 1, comm)
            MPI.Recv_(y, 1, 2, comm)
        elif r == 1:
            MPI.Recv_(y, 0, 1, comm)
            MPI.Send(x, 0, 2, comm)
    for _ in range(3):
        pingpong()
    MPI.Barrier(comm)
    t0 = time.perf_counter()
    for _ in range(it):
        pingpong()
    dt = (time.perf_counter() - t0) / it / 2
    res[f"{nb}B_latency_us"] = round(dt * 1e6, 2)
    # ring Sendrecv
    for _ in range(2):
        MPI.Sendrecv_(x, (r + 1) % n, 3, y, (r - 1) % n, 3, comm)
    MPI.Barrier(comm)
    t0 = time.perf_counter()
    for _ in range(it):
        MPI.Sendrecv_(x, (r + 1) % n, 3, y, (r - 1) % n, 3, comm)
    dt = (time.perf_counter() - t0) / it
    res[f"{nb}B_sendrecv_us"] = round(dt * 1e6, 2)
    res[f"{nb}B_sendrecv_GBps_per_rank"] = round(x.numel() * 4 / dt / 1e9, 2)
    assert float(y[0]) == float((r - 1) % n)
if r == 0:
    print(json.dumps(res), flush=True)
MPI.Finalize()
