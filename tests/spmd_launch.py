"""Launch an SPMD script as N rank processes (the role of `mpiexec -n N` in
the reference's test/runtests.jl:28-45).  Ranks rendezvous over 127.0.0.1.

Each rank's output goes to a file as it is written: a temporary directory by
default, or `$SPMD_LIVE_DIR/<script>_<n>r_<k>/rank<r>.log` when that is set
(GPU runs point it under gpurun_out/, so a long multi-rank case shows
progress there and its per-rank logs survive a kill).  While the ranks run,
one heartbeat line per minute goes to stderr."""
import itertools
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_SEQ = itertools.count()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _logdir(script, n):
    live = os.environ.get("SPMD_LIVE_DIR")
    if not live:
        return tempfile.mkdtemp(prefix="spmd_"), True
    name = f"{os.path.splitext(os.path.basename(script))[0]}_{n}r_{os.getpid()}_{next(_SEQ)}"
    d = os.path.join(live, name)
    os.makedirs(d, exist_ok=True)
    return d, False


def launch(script, n, timeout=600, extra_env=None, args=()):
    port = free_port()
    logdir, temporary = _logdir(script, n)
    procs, files = [], []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_RANK": str(r), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "OMP_NUM_THREADS": "1", "PYTHONUNBUFFERED": "1"})
        env.update(extra_env or {})
        f = open(os.path.join(logdir, f"rank{r}.log"), "w")
        files.append(f)
        procs.append(subprocess.Popen([sys.executable, script, *args], env=env, cwd=ROOT, stdout=f,
                                      stderr=subprocess.STDOUT, start_new_session=True, text=True))
    t0 = time.time()
    beat = t0 + 60
    killed = False
    while any(p.poll() is None for p in procs):
        now = time.time()
        if now - t0 > timeout:
            for p in procs:
                if p.poll() is None:
                    os.killpg(p.pid, signal.SIGKILL)
            killed = True
            break
        if now > beat:
            beat = now + 60
            alive = [r for r, p in enumerate(procs) if p.poll() is None]
            print(f"[spmd] {os.path.basename(script)} n={n}: {now - t0:.0f} s, ranks still running {alive} "
                  f"(logs: {logdir})", file=sys.stderr, flush=True)
        time.sleep(0.2)
    for p in procs:
        p.wait()
    outs = []
    for r, f in enumerate(files):
        f.close()
        with open(f.name, errors="replace") as g:
            o = g.read()
        if killed and procs[r].returncode == -signal.SIGKILL:
            o += "\n<killed: timeout>"
        outs.append(o)
    if temporary:
        for f in files:
            os.unlink(f.name)
        os.rmdir(logdir)
    return [p.returncode for p in procs], outs
