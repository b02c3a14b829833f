#!/usr/bin/env python3
"""Torch alone, no mpigx: how long one rank's `(x != y).nonzero()` (the
round-3 repro's compare) and other single-stream torch ops take when n
processes share one GPU, all at once or with one rank idle.  Isolates the
multi-second compare / synchronize stalls of the 8-rank same-device repro
 from the collective library.

    python3 tools/nonzero_contention.py 8      # launcher: n ranks on cuda:0
"""
import json
import os
import socket
import subprocess
import sys
import time


def worker():
    import torch
    import torch.distributed as dist
    r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=r, world_size=n)
    dev = torch.device("cuda:0")
    cnt = int(os.environ.get("NZ_COUNT", 64 << 20))
    g = torch.Generator(device=dev).manual_seed(7000 + 31 * r)
    a = torch.randint(-(1 << 31), 1 << 31, (cnt,), dtype=torch.int32, device=dev, generator=g)
    b = a.clone()
    torch.cuda.synchronize()
    res = {}

    def phase(name, fn, active):
        ts = []
        for _ in range(int(os.environ.get("NZ_ITERS", 3))):
            dist.barrier()
            t0 = time.perf_counter()
            if active:
                fn()
                torch.cuda.synchronize()
            ts.append(round(time.perf_counter() - t0, 4))
            print(json.dumps({"rank": r, "phase": name, "s": ts[-1]}), flush=True)
        res[name] = ts

    nz = lambda: (a != b).nonzero()  # noqa: E731
    phase("equal_all", lambda: torch.equal(a, b), True)
    phase("sum_item_all", lambda: int((a != b).sum().item()), True)
    phase("nonzero_alone_rank1", nz, r == 1)
    phase("cumsum_all", lambda: torch.cumsum(a, 0, dtype=torch.int64), True)
    phase("nonzero_all", nz, True)
    print(json.dumps({"rank": r, "n": n, **res}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def launch(n):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   NZ_WORKER="1", OMP_NUM_THREADS="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                                      start_new_session=True))
    t0 = time.time()
    limit = float(os.environ.get("NZ_WAIT", 240))
    while any(p.poll() is None for p in procs) and time.time() - t0 < limit:
        time.sleep(5)
        print(f"[{time.time() - t0:.0f}s] running: {[r for r, p in enumerate(procs) if p.poll() is None]}", flush=True)
    for p in procs:
        if p.poll() is None:
            os.killpg(p.pid, 9)
    rc = 0
    for r, p in enumerate(procs):
        out = p.communicate()[0]
        rc |= p.returncode != 0
        lines = [l for l in out.splitlines() if l.startswith("{")]
        print("\n".join(lines) if lines else f"rank {r} rc={p.returncode}: {out[-600:]}", flush=True)
    return rc


if __name__ == "__main__":
    if os.environ.get("NZ_WORKER"):
        worker()
    else:
        sys.exit(launch(int(sys.argv[1]) if len(sys.argv) > 1 else 8))
