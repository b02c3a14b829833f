"""Config 2's secondary variants (8 x 256 MiB inputs) at U = 1 / 2 / 4 16-B
vectors per thread (MPIGX_LOCAL_U): which U each (type, op) should take at
full size.  U = 4 was tuned on f32 SUM (160 VGPRs, 3 waves per SIMD); the
role-sensitive MIN / MAX trees hold more registers (f32 MAX: 181 VGPRs, 2
waves per SIMD).  Kernel time per launch from HIP events over 10
back-to-back launches replayed from one captured graph.  Prints one JSON
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
    s = torch.cuda.current_stream(dev)
    nbytes = 256 << 20
    base = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(9)]
    g = torch.Generator(device=dev).manual_seed(3)
    cases = [("f32", torch.float32, "SUM"), ("f32", torch.float32, "MAX"), ("f32", torch.float32, "MIN"),
             ("bf16", torch.bfloat16, "SUM"), ("bf16", torch.bfloat16, "MAX"), ("f64", torch.float64, "SUM"),
             ("f64", torch.float64, "MAX"), ("i32", torch.int32, "BAND"), ("i32", torch.int32, "MAX"),
             ("i64", torch.int64, "SUM")]
    res = {}
    for name, dt, opn in cases:
        xs = [b.view(dt) for b in base[:8]]
        for x in xs:
            if dt.is_floating_point:
                x.copy_(torch.rand(x.numel(), device=dev, generator=g).to(dt))
            else:
                x.copy_(torch.randint(-1000, 1000, (x.numel(),), device=dev, generator=g, dtype=dt))
        o = base[8].view(dt)
        op = getattr(MPI, opn)
        row = {}
        for u in ("1", "2", "4"):
            os.environ["MPIGX_LOCAL_U"] = u
            for _ in range(2):
                MPI.reduce_local_multi(xs, o, op, stream=s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                for _ in range(10):
                    MPI.reduce_local_multi(xs, o, op)
            graph.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            best = 1e9
            for _ in range(3):
                a.record(s)
                graph.replay()
                b.record(s)
                torch.cuda.synchronize()
                best = min(best, a.elapsed_time(b) / 10 * 1e3)
            row[f"U={u}"] = {"us": round(best, 1), "GBps": round(9 * nbytes / (best / 1e6) / 1e9, 1)}
            del graph
        os.environ.pop("MPIGX_LOCAL_U", None)
        res[f"{name}_{opn}"] = row
    print(json.dumps({"tool": "local_variant_u", "bytes_per_input": nbytes, "results": res}), flush=True)


if __name__ == "__main__":
    main()
