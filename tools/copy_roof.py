#!/usr/bin/env python3
"""Copy roofline of the box (one process, one GPU): device-to-device copy
(read S + write S) through hipMemcpyAsync and through torch's copy kernel,
and a 2:1 read:write mix (torch.add), timed with HIP events over `iters` calls.  The collective
kernels' traffic is a read/write mix (pull-push two-shot 1:1, pull two-shot
1.5:1), so their HBM fraction is bounded by these rates, not by the
read-only stream.  Prints one JSON line.

    python3 tools/copy_roof.py [--mib 512] [--iters 20]
"""
import argparse
import ctypes
import json

import torch


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters / 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=512)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    S = a.mib << 20
    dev = torch.device("cuda:0")
    x = torch.rand(S // 4, device=dev)
    y = torch.empty_like(x)
    hip = ctypes.CDLL("libamdhip64.so")
    stream = torch.cuda.current_stream().cuda_stream
    out = {"mib": a.mib, "iters": a.iters}

    def memcpy():
        hip.hipMemcpyAsync(ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(x.data_ptr()), ctypes.c_size_t(S),
                           ctypes.c_int(3), ctypes.c_void_p(stream))
    t = timed(memcpy, a.iters)
    out["hipMemcpy_d2d_GBps"] = round(2 * S / t / 1e9, 1)  # read S + write S
    t = timed(lambda: y.copy_(x), a.iters)
    out["torch_copy_GBps"] = round(2 * S / t / 1e9, 1)
    z = torch.rand_like(x)
    t = timed(lambda: torch.add(x, z, out=y), a.iters)
    out["add_2r1w_GBps"] = round(3 * S / t / 1e9, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
