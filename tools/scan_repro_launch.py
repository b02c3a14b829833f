#!/usr/bin/env python3
"""Start tools/scan_repro.py as N ranks on one GPU (tests/spmd_launch.py) and
print every rank's JSON line.   python3 tools/scan_repro_launch.py 8"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from spmd_launch import launch  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
env = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_TIMEOUT_MS": "20000"}
if len(sys.argv) > 2:
    env["MPIGX_LIB"] = os.path.abspath(sys.argv[2])  # another build of libmpigx.so (A/B)
rcs, outs = launch(os.path.join(ROOT, "tools", "scan_repro.py"), n, timeout=500, extra_env=env)
for r, (rc, o) in enumerate(zip(rcs, outs)):
    lines = [l for l in o.splitlines() if l.startswith("{")]
    prog = [l for l in o.splitlines() if l.startswith(f"r{r} ")]
    print(f"rank {r} rc={rc} last={prog[-1] if prog else None}", *(lines[-2:] if lines else [o[-1500:]]), flush=True)
    if rc and os.environ.get("MPIGX_DIAG_TRACE"):
        ev = [l for l in o.splitlines() if l.startswith("[trace") or l.startswith(f"r{r} ")]
        print("\n".join(ev[-14:]), flush=True)
sys.exit(0 if all(rc == 0 for rc in rcs) else 1)
