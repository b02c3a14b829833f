#!/usr/bin/env python3
"""Diagnostic SPMD worker (launched by tools/scan_repro_launch.py): the
headline worker's 64 Mi-element Int32 / Int64 Scan / Exscan / Reduce
sequence at n ranks.  Per-block stamps are on for every call: when a call
fails, every rank prints its blocks' entry times (device wall clock, 100 MHz,
one clock for all ranks of a GPU) and the per-block timeout records (epoch
awaited, word last seen, the peer, when the block gave up) so that the ranks'
records line up in time.

Modes (one script since round 5; round 4's separate variant is in history at
commit 8a5ba8c):
  REPRO_COMPARE=equal    (default) torch.equal compares between the calls
  REPRO_COMPARE=nonzero  round 3's `(out != exp).nonzero()` compares: with 8
                         processes on one GPU they take tens of seconds
                         (rocPRIM look-back scans time-sliced, DESIGN §12
                         "n = 8 stall") and rank 0, which has no Exscan result
                         to compare, reaches the Reduce that much earlier
  REPRO_WATCH=1          a thread reporting, after every 4 s without progress,
                         where the rank is (mpigx_comm_diag_state)"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# REPRO_PKG: another copy of the Python mirror (A/B against an older library)
sys.path.insert(0, os.environ.get("REPRO_PKG", os.path.join(ROOT, "mpi.jl_amd")))

import torch  # noqa: E402

import mpigx as MPI  # noqa: E402


def main():
    comm = MPI.Init()
    r, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
    L = MPI.lib()
    dev = torch.device("cuda:0")
    cnt = int(os.environ.get("REPRO_COUNT", 64 << 20))
    reps = int(os.environ.get("REPRO_REPS", 1))
    st = torch.zeros(1024 * 8, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    L.mpigx_comm_set_stamps(comm.val, ctypes.c_void_p(st.data_ptr()))

    def run(what, fn):
        st.zero_()
        torch.cuda.synchronize()
        t_host = time.time()
        try:
            fn()
            torch.cuda.synchronize()
        except MPI.MPIError as e:
            torch.cuda.synchronize()
            t = st.view(1024, 8).cpu()
            started = t[:, 0] > 0
            e0 = t[started, 0]
            tmo = [(int(b), int(t[b, 6]), int(t[b, 7]) & ((1 << 56) - 1), int(t[b, 7]) >> 56, int(t[b, 2]),
                    int(t[b, 3]), int(t[b, 4]), int(t[b, 5]))
                   for b in (t[:, 6] != 0).nonzero().flatten()[:4]]
            print(json.dumps({"rank": r, "at": what, "error": str(e), "host_t": t_host,
                              "blocks_started": int(started.sum()),
                              "entry_min": int(e0.min()) if e0.numel() else None,
                              "entry_max": int(e0.max()) if e0.numel() else None,
                              "timeouts_b_ep_seen_lane_tgiveup_rmw_nt_acq": tmo}), flush=True)
            sys.exit(1)

    nonzero = os.environ.get("REPRO_COMPARE", "equal") == "nonzero"

    def same(out, exp):
        if nonzero:
            return (out != exp).nonzero().numel() == 0
        return torch.equal(out, exp)

    if os.environ.get("REPRO_WATCH") and hasattr(L, "mpigx_comm_diag_state"):
        import threading
        main_t = threading.main_thread()

        def watch():
            last = None
            while main_t.is_alive():
                time.sleep(4.0)
                st8 = (ctypes.c_ulonglong * 8)()
                L.mpigx_comm_diag_state(comm.val, st8)
                cur = tuple(st8)
                if cur == last:  # nothing moved for 4 s: say where the rank is
                    frame = sys._current_frames().get(main_t.ident)
                    where = f"{frame.f_code.co_name}:{frame.f_lineno}" if frame else "?"
                    print(json.dumps({"watch": r, "t": round(time.time(), 3), "at": where, "state": list(cur)}),
                          file=sys.stderr, flush=True)
                last = cur

        threading.Thread(target=watch, daemon=True).start()

    ops = (("BAND", MPI.BAND, torch.bitwise_and), ("BOR", MPI.BOR, torch.bitwise_or), ("MAX", MPI.MAX, torch.maximum))
    nbad = 0
    for tdt, lim in ((torch.int32, 1 << 31), (torch.int64, 1 << 62)):
        def gen(q):
            g = torch.Generator(device=dev).manual_seed(7000 + 31 * q)
            return torch.randint(-lim, lim, (cnt,), dtype=tdt, device=dev, generator=g)
        mine = gen(r)
        for rep in range(reps):
            for oname, op, fn in ops:
                pref = None
                for q in range(r + 1):
                    pref = gen(q) if pref is None else fn(pref, gen(q))
                ex = None
                for q in range(r):
                    ex = gen(q) if ex is None else fn(ex, gen(q))
                out = torch.zeros_like(mine)
                print(f"r{r} {tdt} {oname} scan t={time.time():.3f}", file=sys.stderr, flush=True)
                run(f"{tdt} {oname} scan", lambda: MPI.Scan_(mine, out, op, comm))
                nbad += int(not same(out, pref))
                out.fill_(7)
                print(f"r{r} {tdt} {oname} exscan t={time.time():.3f}", file=sys.stderr, flush=True)
                run(f"{tdt} {oname} exscan", lambda: MPI.Exscan_(mine, out, op, comm))
                nbad += int(not same(out, ex) if r > 0 else not bool((out == 7).all()))
                root = n - 1
                rout = torch.zeros_like(mine) if r == root else None
                print(f"r{r} {tdt} {oname} reduce t={time.time():.3f}", file=sys.stderr, flush=True)
                run(f"{tdt} {oname} reduce", lambda: MPI.Reduce_(mine, rout, op, root, comm))
                if r == root:
                    tot = pref
                    for q in range(r + 1, n):
                        tot = fn(tot, gen(q))
                    nbad += int(not same(rout, tot))
                del out, rout, pref, ex
        del mine
    L.mpigx_comm_set_stamps(comm.val, None)
    MPI.Barrier(comm)
    MPI.Finalize()
    print(json.dumps({"rank": r, "n": n, "nbad": nbad}), flush=True)


if __name__ == "__main__":
    main()
