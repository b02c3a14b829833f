"""Launch an SPMD script as N rank processes (the role of `mpiexec -n N` in
the reference's test/runtests.jl:28-45).  Ranks rendezvous over 127.0.0.1."""
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(script, n, timeout=600, extra_env=None, args=()):
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_RANK": str(r), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "OMP_NUM_THREADS": "1"})
        env.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable, script, *args], env=env, cwd=ROOT, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, start_new_session=True, text=True))
    t0 = time.time()
    outs = [None] * n
    try:
        for i, p in enumerate(procs):
            left = max(1, timeout - (time.time() - t0))
            outs[i], _ = p.communicate(timeout=left)
    except subprocess.TimeoutExpired:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGKILL)
        for i, p in enumerate(procs):
            if outs[i] is None:
                outs[i] = (p.communicate()[0] or "") + "\n<killed: timeout>"
    return [p.returncode for p in procs], outs
