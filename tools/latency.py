"""Small-message latency breakdown of mpigx_allreduce (run as N ranks)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import mpigx as MPI  # noqa: E402

comm = MPI.Init()
L = MPI.lib()
r = MPI.Comm_rank(comm)
res = {}
SIZES = [int(v) for v in os.environ.get("LAT_SIZES", "8,4096,65536,1048576,8388608").split(",")]
for nbytes in SIZES:
    x = torch.ones(nbytes // 4, device="cuda")
    y = torch.empty_like(x)
    px, py = ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr())
    for mode in ("api", "raw", "raw_nonblocking"):
        if mode == "raw_nonblocking":
            L.mpigx_comm_set_blocking(comm.val, 0)
        for _ in range(20):
            if mode == "api":
                MPI.Allreduce_(x, y, MPI.SUM, comm)
            else:
                L.mpigx_allreduce(px, py, nbytes // 4, MPI.FLOAT.val, MPI.SUM.val, comm.val)
        torch.cuda.synchronize()
        MPI.Barrier(comm)
        t0 = time.perf_counter()
        it = 200 if nbytes <= (8 << 20) else 20
        for _ in range(it):
            if mode == "api":
                MPI.Allreduce_(x, y, MPI.SUM, comm)
            else:
                L.mpigx_allreduce(px, py, nbytes // 4, MPI.FLOAT.val, MPI.SUM.val, comm.val)
        L.mpigx_comm_synchronize(comm.val)
        dt = (time.perf_counter() - t0) / it
        L.mpigx_comm_set_blocking(comm.val, 1)
        res[f"{nbytes}B_{mode}_us"] = round(dt * 1e6, 2)
# empty-kernel + sync floor
s = torch.cuda.current_stream()
t0 = time.perf_counter()
for _ in range(200):
    torch.cuda._sleep(1)
    s.synchronize()
res["launch+sync_floor_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 2)
if r == 0:
    print(json.dumps(res), flush=True)
MPI.Finalize()
