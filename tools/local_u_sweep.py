"""Config-2 fold (8 inputs, f32 SUM) kernel time per size for U = 1 / 2 / 4
16-B vectors per thread (MPIGX_LOCAL_U forces one; unset = the product rule,
common.hpp local_u) — the measurement behind the size rule (VERDICT r05
item 4).  HIP events on the launch stream over 50 back-to-back launches.
Each size also replays the launches from one captured HIP graph (us_graph),
which takes the host's per-launch cost out: below ~4 MiB the eager loop is
bound by the host issuing launches, not by the kernel.  Prints one JSON
line.  Run on the GPU box from the repo root."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))

import torch  # noqa: E402

import mpigx as MPI  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    nbuf = 8
    sizes_mib = [0.25, 0.5, 1, 2, 4, 8, 16, 32, 64, 256]
    top = 256 << 18
    g = torch.Generator(device=dev).manual_seed(5)
    ins = [torch.rand(top, device=dev, generator=g) for _ in range(nbuf)]
    out = torch.empty(top, device=dev)
    s = torch.cuda.current_stream(dev)
    res = {}
    for u in ("1", "2", "4", "auto"):
        if u == "auto":
            os.environ.pop("MPIGX_LOCAL_U", None)
        else:
            os.environ["MPIGX_LOCAL_U"] = u
        row = {}
        for mib in sizes_mib:
            k = int(mib * (1 << 18))
            xs, o = [x[:k] for x in ins], out[:k]
            for _ in range(5):
                MPI.reduce_local_multi(xs, o, MPI.SUM, stream=s)
            reps = 50 if mib < 64 else 10
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            for _ in range(reps):
                MPI.reduce_local_multi(xs, o, MPI.SUM, stream=s)
            b.record(s)
            torch.cuda.synchronize()
            us = a.elapsed_time(b) / reps * 1e3
            # the same launches captured in one HIP graph and replayed: no
            # host launch cost between kernels (device-bound per-launch time)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(reps):
                    MPI.reduce_local_multi(xs, o, MPI.SUM)
            graph.replay()
            torch.cuda.synchronize()
            usg = 1e9
            for _ in range(3):  # best of three replays (a single replay catches box noise)
                a.record(s)
                graph.replay()
                b.record(s)
                torch.cuda.synchronize()
                usg = min(usg, a.elapsed_time(b) / reps * 1e3)
            row[f"{mib}MiB"] = {"us": round(us, 2), "GBps": round((nbuf + 1) * k * 4 / (us / 1e6) / 1e9, 1),
                                "us_graph": round(usg, 2),
                                "GBps_graph": round((nbuf + 1) * k * 4 / (usg / 1e6) / 1e9, 1)}
            del graph
        # correctness of the last (largest) size against torch's own sum order is
        # not the point here; the GPU suite checks bits.  Keep the output used.
        res[f"U={u}"] = row
    os.environ.pop("MPIGX_LOCAL_U", None)
    print(json.dumps({"tool": "local_u_sweep", "nbuf": nbuf, "dtype": "f32", "op": "SUM", "results": res}), flush=True)


if __name__ == "__main__":
    main()
