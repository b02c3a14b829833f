#!/usr/bin/env python3
"""Start tools/scan_repro.py as N ranks on one GPU and print every rank's
result.  Each rank's output streams to gpurun_out/scan_repro_r<k>.log while
it runs (progress is visible; nothing waits on a pipe).

    python3 tools/scan_repro_launch.py 8 [path/to/libmpigx.so]"""
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
env0 = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000",
        "MPIGX_TIMEOUT_MS": os.environ.get("MPIGX_TIMEOUT_MS", "20000")}
if len(sys.argv) > 2:
    env0["MPIGX_LIB"] = os.path.abspath(sys.argv[2])  # another build of libmpigx.so (A/B)
s = socket.socket()
s.bind(("127.0.0.1", 0))
port = s.getsockname()[1]
s.close()
out_dir = os.path.join(ROOT, "gpurun_out")
os.makedirs(out_dir, exist_ok=True)
procs, files = [], []
for r in range(n):
    env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), OMP_NUM_THREADS="1", **env0)
    f = open(os.path.join(out_dir, f"scan_repro_r{r}.log"), "w")
    files.append(f)
    script = os.environ.get("REPRO_SCRIPT", os.path.join(ROOT, "tools", "scan_repro.py"))
    procs.append(subprocess.Popen([sys.executable, "-u", script], env=env,
                                  cwd=ROOT, stdout=f, stderr=subprocess.STDOUT, start_new_session=True))
t0 = time.time()
while any(p.poll() is None for p in procs) and time.time() - t0 < float(os.environ.get("REPRO_WAIT", 280)):
    time.sleep(5)
    print(f"[{time.time() - t0:.0f}s] running: {[r for r, p in enumerate(procs) if p.poll() is None]}", flush=True)
for p in procs:
    if p.poll() is None:
        os.killpg(p.pid, 9)
        p.wait()
for f in files:
    f.close()
for r, p in enumerate(procs):
    o = open(os.path.join(out_dir, f"scan_repro_r{r}.log")).read()
    lines = [l for l in o.splitlines() if l.startswith("{")]
    prog = [l for l in o.splitlines() if l.startswith(f"r{r} ")]
    print(f"rank {r} rc={p.returncode} last={prog[-1] if prog else None}", *(lines[-4:] if lines else [o[-800:]]),
          flush=True)
    if p.returncode and os.environ.get("MPIGX_DIAG_TRACE"):
        ev = [l for l in o.splitlines() if l.startswith("[trace") or l.startswith(f"r{r} ")]
        print("\n".join(ev[-14:]), flush=True)
sys.exit(0 if all(p.returncode == 0 for p in procs) else 1)
