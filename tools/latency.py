"""Per-call latency of mpigx_allreduce through the raw C ABI and the MPI.jl
mirror (run as N ranks): blocking wall time, device time of the same calls
(HIP events on the comm's stream) and their difference — the host cost per
call (argument checks, zero-copy view resolution, launch, completion wait).
Also the zero-copy view counters (optimistic hits vs host exchanges)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))
import torch  # noqa: E402

import mpigx as MPI  # noqa: E402

comm = MPI.Init()
L = MPI.lib()
r = MPI.Comm_rank(comm)
res = {}
SIZES = [int(v) for v in os.environ.get("LAT_SIZES", "8,65536,1048576,16777216,67108864").split(",")]
s = torch.cuda.current_stream()


def stats():
    h, x = ctypes.c_ulonglong(), ctypes.c_ulonglong()
    L.mpigx_comm_zc_stats(comm.val, ctypes.byref(h), ctypes.byref(x))
    return h.value, x.value


for nbytes in SIZES:
    x = torch.ones(nbytes // 4, device="cuda")
    y = torch.empty_like(x)
    px, py = ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr())
    for mode in ("api", "raw", "raw_nonblocking"):
        if mode == "raw_nonblocking":
            L.mpigx_comm_set_blocking(comm.val, 0)

        def call():
            if mode == "api":
                MPI.Allreduce_(x, y, MPI.SUM, comm)
            else:
                assert L.mpigx_allreduce(px, py, nbytes // 4, MPI.FLOAT.val, MPI.SUM.val, comm.val) == 0
        for _ in range(20):
            call()
        torch.cuda.synchronize()
        MPI.Barrier(comm)
        h0, x0 = stats()
        it = 200 if nbytes <= (8 << 20) else 30
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(it)]
        pre = []
        t0 = time.perf_counter()
        for a, b in ev:
            a.record(s)
            call()
            b.record(s)
            p_ = ctypes.c_double()
            L.mpigx_comm_host_stats(comm.val, ctypes.byref(p_))
            pre.append(p_.value)
        L.mpigx_comm_synchronize(comm.val)
        dt = (time.perf_counter() - t0) / it
        torch.cuda.synchronize()
        dev = sum(a.elapsed_time(b) for a, b in ev) / it / 1e3
        h1, x1 = stats()
        L.mpigx_comm_set_blocking(comm.val, 1)
        key = f"{nbytes}B_{mode}"
        pre.sort()
        res[key] = {"wall_us": round(dt * 1e6, 2), "device_us": round(dev * 1e6, 2),
                    "prelaunch_us_median": round(pre[len(pre) // 2], 2)}
        if mode != "raw_nonblocking":
            res[key]["host_us"] = round((dt - dev) * 1e6, 2)
        if nbytes >= (16 << 20):
            res[key]["zc_hits"] = h1 - h0
            res[key]["zc_exchanges"] = x1 - x0
# empty-kernel + sync floor
t0 = time.perf_counter()
for _ in range(200):
    torch.cuda._sleep(1)
    s.synchronize()
res["launch+sync_floor_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 2)
if r == 0:
    print(json.dumps(res), flush=True)
MPI.Finalize()
