#!/usr/bin/env python3
"""Diagnostic SPMD worker (launched by tools/scan_repro_launch.py): the
headline worker's 64 Mi-element Int64 Scan / Exscan / Reduce sequence at n
ranks, printing for every mismatching call where the wrong elements are
(chunk / block-slice of the pull-push partition), what they hold, the
recvbuf address and the zero-copy counters around the call."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))

import torch  # noqa: E402

import mpigx as MPI  # noqa: E402


def main():
    comm = MPI.Init()
    r, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
    L = MPI.lib()
    dev = torch.device("cuda:0")
    cnt = int(os.environ.get("REPRO_COUNT", 64 << 20))
    reps = int(os.environ.get("REPRO_REPS", 1))

    def zc():
        h, x = ctypes.c_ulonglong(0), ctypes.c_ulonglong(0)
        L.mpigx_comm_zc_stats(comm.val, ctypes.byref(h), ctypes.byref(x))
        return h.value, x.value

    log = []
    ops = (("BAND", MPI.BAND, torch.bitwise_and), ("BOR", MPI.BOR, torch.bitwise_or), ("MAX", MPI.MAX, torch.maximum))
    chunk = -(-cnt // n)
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
                for coll in ("scan", "exscan"):
                    z0 = zc()
                    print(f"r{r} {tdt} {oname} {coll} out={hex(out.data_ptr())} t={time.time():.3f}", file=sys.stderr, flush=True)
                    if coll == "scan":
                        MPI.Scan_(mine, out, op, comm)
                        exp = pref
                    else:
                        out.fill_(7)
                        MPI.Exscan_(mine, out, op, comm)
                        exp = ex
                    torch.cuda.synchronize()
                    z1 = zc()
                    if exp is None:
                        continue
                    bad = (out != exp).nonzero().flatten()
                    if bad.numel():
                        idx = bad.cpu()
                        chunks = sorted(set((idx // chunk).tolist()))
                        vals = out[bad[:4]].tolist()
                        zeros = int((out[bad] == 0).sum().item())
                        sevens = int((out[bad] == 7).sum().item())
                        log.append({"coll": coll, "dtype": str(tdt), "op": oname, "rep": rep, "bad": int(idx.numel()),
                                    "first": int(idx[0]), "last": int(idx[-1]), "chunks": chunks[:16],
                                    "zeros": zeros, "sevens": sevens, "vals": vals,
                                    "exp": exp[bad[:4]].tolist(), "out_ptr": hex(out.data_ptr()),
                                    "zc_hits": z1[0] - z0[0], "zc_exchanges": z1[1] - z0[1]})
                    else:
                        log.append({"coll": coll, "dtype": str(tdt), "op": oname, "rep": rep, "ok": True,
                                    "out_ptr": hex(out.data_ptr()), "zc_hits": z1[0] - z0[0],
                                    "zc_exchanges": z1[1] - z0[1]})
                root = n - 1
                rout = torch.zeros_like(mine) if r == root else None
                print(f"r{r} {tdt} {oname} reduce t={time.time():.3f}", file=sys.stderr, flush=True)
                st = torch.zeros(1024 * 8, dtype=torch.int64, device=dev)
                torch.cuda.synchronize()
                L.mpigx_comm_set_stamps(comm.val, ctypes.c_void_p(st.data_ptr()))
                try:
                    MPI.Reduce_(mine, rout, op, root, comm)
                    L.mpigx_comm_set_stamps(comm.val, None)
                except MPI.MPIError as e:
                    L.mpigx_comm_set_stamps(comm.val, None)
                    torch.cuda.synchronize()
                    t = st.view(1024, 8).cpu()
                    started = t[:, 0] > 0
                    blocks = int(started.sum())
                    phase = {k: int((t[:, k] > 0).sum()) for k in range(6)}
                    t0 = int(t[started, 0].min()) if blocks else 0
                    first_missing = [int(b) for b in ((t[:, 1] == 0) & started).nonzero().flatten()[:8]]
                    tmo = [(int(b), int(t[b, 6]), int(t[b, 7]) & ((1 << 56) - 1), int(t[b, 7]) >> 56)
                           for b in (t[:, 6] != 0).nonzero().flatten()[:6]]
                    print(json.dumps({"rank": r, "timeouts_block_ep_seen_lane": tmo}), flush=True)
                    print(json.dumps({"rank": r, "stamps_blocks": blocks, "stamps_phase_counts": phase,
                                      "entry_span_us": (int(t[started, 0].max()) - t0) / 100.0 if blocks else None,
                                      "blocks_stuck_at_entry": first_missing}), flush=True)
                    print(json.dumps({"rank": r, "n": n, "error": str(e), "at": [str(tdt), oname, "reduce"],
                                      "log": [x for x in log if not x.get("ok")][:12],
                                      "ptrs": [(x["coll"], x["op"], x["out_ptr"], x["zc_exchanges"]) for x in log]}),
                          flush=True)
                    sys.exit(1)
                del out, rout, pref, ex
        del mine
    MPI.Barrier(comm)
    MPI.Finalize()
    nbad = sum(1 for x in log if not x.get("ok"))
    print(json.dumps({"rank": r, "n": n, "nbad": nbad, "log": [x for x in log if not x.get("ok")][:12],
                      "ptrs": [(x["coll"], x["op"], x["out_ptr"], x["zc_exchanges"]) for x in log][:24]}), flush=True)


if __name__ == "__main__":
    main()
