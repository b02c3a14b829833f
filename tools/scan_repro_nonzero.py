#!/usr/bin/env python3
"""Diagnostic SPMD worker (launched by tools/scan_repro_launch.py with
REPRO_SCRIPT=tools/scan_repro_nonzero.py): round 3's 8-rank repro — the
64 Mi-element Int32 / Int64 Scan / Exscan / Reduce sequence with
`(out != exp).nonzero()` compares between the calls (rank 0 skips its
Exscan compare, so it reaches the Reduce early), printing for every
mismatching call where the wrong elements are, the recvbuf address and the
zero-copy counters around the call.  With 8 processes on one GPU the peers'
compares take tens of seconds (DESIGN §12 "n = 8 stall");
REPRO_WATCH=1 starts a thread that reports every 4 s of no progress where
the rank is (mpigx_comm_diag_state).  Variants: REPRO_EQUAL (torch.equal
compares), REPRO_SUM_BETWEEN, REPRO_ALLOC_BETWEEN=<MiB>, REPRO_PIN_BETWEEN,
REPRO_WARM_PINNED, REPRO_SYNC_BEFORE, REPRO_MAPCHECK, REPRO_ST_ONCE."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("REPRO_PKG", os.path.join(ROOT, "mpi.jl_amd")))

import torch  # noqa: E402

import mpigx as MPI  # noqa: E402


def main():
    import faulthandler
    faulthandler.dump_traceback_later(float(os.environ.get("REPRO_DUMP_S", 40)), exit=False)
    if os.environ.get("REPRO_WARM_PINNED"):  # pinned host memory allocated before any IPC mapping exists
        _warm = [torch.empty(4 << 20, dtype=torch.uint8, pin_memory=True) for _ in range(4)]
        (torch.arange(1 << 20, device="cuda") % 3 == 0).nonzero()
        torch.cuda.synchronize()
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
    keep_pinned = []
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
                if cur == last:  # nothing moved for 4 s: say where everything is
                    frame = sys._current_frames().get(main_t.ident)
                    where = f"{frame.f_code.co_name}:{frame.f_lineno}" if frame else "?"
                    print(json.dumps({"watch": r, "t": round(time.time(), 3), "at": where,
                                      "comm_stream_busy": cur[0], "done_word_seq": cur[1] >> 1,
                                      "done_word_abort": cur[1] & 1, "done_target": cur[2], "dcount_total": cur[3],
                                      "launch_seq": cur[4], "epoch": cur[5], "xseq": cur[6], "xseq_min_all": cur[7]}),
                          file=sys.stderr, flush=True)
                last = cur
        threading.Thread(target=watch, daemon=True).start()
    nonce = [0x5150000000000000]

    def mapcheck(tag):
        if not hasattr(L, "mpigx_comm_diag_mapcheck") or not os.environ.get("REPRO_MAPCHECK"):
            return
        nonce[0] += 1 << 8
        m = ctypes.c_uint(0)
        rc = L.mpigx_comm_diag_mapcheck(comm.val, ctypes.c_ulonglong(nonce[0]), ctypes.byref(m))
        if r == 0:
            print(json.dumps({"mapcheck": tag, "rc": rc, "stale_mask": m.value}), flush=True)
    mapcheck("init")
    ST0 = torch.zeros(1024 * 8, dtype=torch.int64, device=dev)
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
                        if os.environ.get("REPRO_SYNC_BEFORE"):
                            torch.cuda.synchronize()
                        MPI.Scan_(mine, out, op, comm)
                        exp = pref
                    else:
                        out.fill_(7)
                        if os.environ.get("REPRO_SYNC_BEFORE"):
                            torch.cuda.synchronize()
                        MPI.Exscan_(mine, out, op, comm)
                        exp = ex
                    busy = not torch.cuda.current_stream().query()
                    t_s = time.time()
                    torch.cuda.synchronize()
                    print(f"r{r} {coll} returned; stream busy={busy} sync {time.time() - t_s:.4f}s", file=sys.stderr,
                          flush=True)
                    mapcheck(f"after {coll} {oname} {tdt}")
                    z1 = zc()
                    if exp is None:
                        continue
                    t_n = time.time()
                    if os.environ.get("REPRO_EQUAL") and torch.equal(out, exp):
                        bad = torch.zeros(0, dtype=torch.int64)
                    else:
                        bad = (out != exp).nonzero().flatten()
                    print(f"r{r} compare {time.time() - t_n:.4f}s", file=sys.stderr, flush=True)
                    if os.environ.get("REPRO_ALLOC_BETWEEN"):  # a fresh device segment, kept alive
                        keep_pinned.append(torch.empty(int(os.environ["REPRO_ALLOC_BETWEEN"]) << 20,
                                                       dtype=torch.uint8, device=dev))
                        torch.cuda.synchronize()
                    if os.environ.get("REPRO_SUM_BETWEEN"):  # a device-wide reduction + D2H of a scalar
                        int((out != exp).sum().item())
                    if os.environ.get("REPRO_PIN_BETWEEN"):  # a fresh pinned host allocation, nothing else
                        keep_pinned.append(torch.empty(2 << 20, dtype=torch.uint8, pin_memory=True))
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
                torch.cuda.synchronize()
                mapcheck(f"after rout alloc {oname} {tdt}")
                print(f"r{r} {tdt} {oname} reduce t={time.time():.3f}", file=sys.stderr, flush=True)
                st = ST0 if os.environ.get("REPRO_ST_ONCE") else torch.zeros(1024 * 8, dtype=torch.int64, device=dev)
                st.zero_()
                torch.cuda.synchronize()
                mapcheck(f"before reduce {oname} {tdt}")
                L.mpigx_comm_set_stamps(comm.val, ctypes.c_void_p(st.data_ptr()))
                try:
                    MPI.Reduce_(mine, rout, op, root, comm)
                    L.mpigx_comm_set_stamps(comm.val, None)
                except MPI.MPIError as e:
                    L.mpigx_comm_set_stamps(comm.val, None)
                    torch.cuda.synchronize()
                    if hasattr(L, "mpigx_comm_diag_slots"):
                        mi, th = (ctypes.c_ulonglong * 16)(), (ctypes.c_ulonglong * 16)()
                        L.mpigx_comm_diag_slots(comm.val, 0, mi, th)
                        print(json.dumps({"rank": r, "slots_b0_from_peer_epoch": [x >> 25 for x in mi[:n]],
                                          "my_words_at_peers_epoch": [x >> 25 for x in th[:n]]}), flush=True)
                    t = st.view(1024, 8).cpu()
                    started = t[:, 0] > 0
                    blocks = int(started.sum())
                    phase = {k: int((t[:, k] > 0).sum()) for k in range(6)}
                    t0 = int(t[started, 0].min()) if blocks else 0
                    first_missing = [int(b) for b in ((t[:, 1] == 0) & started).nonzero().flatten()[:8]]
                    tmo = [(int(b), int(t[b, 6]), int(t[b, 7]) & ((1 << 56) - 1), int(t[b, 7]) >> 56,
                            int(t[b, 3]), int(t[b, 4]), int(t[b, 5]))
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
