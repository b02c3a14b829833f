"""Random point-to-point traffic checked against the MPI matching model.

Every rank builds the same seeded plan: each rank sends M messages (random
destination incl. itself, tag in [0, 4), size in [0, MAXB] bytes, dtype
u8/f32/i64) — at most 32 per (source, destination) pair so every envelope is
in the receiver's mailbox before the barrier; after the barrier every rank
posts one receive per incoming message, in a shuffled order, with the exact
tag or MPI_ANY_TAG, and waits for all.  Which message each receive gets is
predicted by oracle/p2p_model.match_unexpected_first; payloads (splitmix64
bytes keyed by message id) and status (source, tag, bytes) must agree
exactly.  Device buffers (ROCm tensors) unless MPIGX_TEST_ARRAYTYPE is unset.
"""
import json
import os
import random
import sys
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import mpigx as MPI  # noqa: E402
from oracle.p2p_model import ANY_TAG, match_unexpected_first  # noqa: E402

DEVICE = os.environ.get("MPIGX_TEST_ARRAYTYPE", "") == "ROCArray"
if DEVICE:
    import torch

SEED = int(os.environ.get("P2P_SEED", "7"))
M = int(os.environ.get("P2P_MSGS", "24"))
MAXB = int(os.environ.get("P2P_MAXB", str(1 << 20)))
DTYPES = [np.uint8, np.float32, np.int64]


def payload(mid, nbytes):
    x = (np.arange(nbytes // 8 + 1, dtype=np.uint64) + np.uint64(mid) * np.uint64(0x9E3779B97F4A7C15))
    x ^= x >> np.uint64(30)
    x *= np.uint64(0xBF58476D1CE4E5B9)
    x ^= x >> np.uint64(27)
    return x.view(np.uint8)[:nbytes].copy()


def plan(n):
    rng = random.Random(SEED * 1000 + n)
    msgs = []  # (src, dst, tag, nbytes, dtype_idx, id)
    per_pair = {}
    for s in range(n):
        for k in range(M):
            d = rng.randrange(n)
            if per_pair.get((s, d), 0) >= 32:
                continue
            per_pair[(s, d)] = per_pair.get((s, d), 0) + 1
            di = rng.randrange(len(DTYPES))
            es = np.dtype(DTYPES[di]).itemsize
            nb = rng.choice([0, es, rng.randrange(0, MAXB // es + 1) * es, (MAXB // es) * es])
            msgs.append((s, d, rng.randrange(4), nb, di, s * 10000 + k))
    recvs = {}
    for d in range(n):
        inc = [m for m in msgs if m[1] == d]
        for attempt in range(100):
            order = inc[:]
            rng.shuffle(order)
            rl = [(m[0], ANY_TAG if rng.random() < 0.3 else m[2], m[4]) for m in order]
            arrived = [(m[0], m[2], m[5]) for m in inc]  # per-source order = send order
            got = match_unexpected_first(arrived, [(s, t) for s, t, _ in rl])
            if all(g is not None for g in got):
                break
        else:
            rl = [(m[0], m[2], m[4]) for m in inc]
            got = [m[5] for m in inc]
        recvs[d] = (rl, got)
    return msgs, recvs


comm = MPI.Init()
rank, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
failed = None
checks = 0
bad = []
try:
    msgs, recvs = plan(n)
    byid = {m[5]: m for m in msgs}

    def buf_of(raw, di):
        a = raw.view(DTYPES[di]) if raw.size else np.zeros(0, DTYPES[di])
        if DEVICE:
            return torch.from_numpy(a.copy()).to(f"cuda:{comm.device}")
        return a.copy()

    sends = []
    for s, d, tag, nb, di, mid in msgs:
        if s == rank:
            sends.append(MPI.Isend(buf_of(payload(mid, nb), di), d, tag, comm))
    MPI.Barrier(comm)
    rl, expect = recvs[rank]
    rbufs, rreqs = [], []
    for (s, t, _), mid in zip(rl, expect):
        di = byid[mid][4]  # receive with the type the sender used
        cap = max([m[3] for m in msgs if m[0] == s and m[1] == rank] + [0])
        es = np.dtype(DTYPES[di]).itemsize
        b = buf_of(np.zeros((cap + es - 1) // es * es, np.uint8), di)
        rbufs.append(b)
        rreqs.append(MPI.Irecv_(b, s, t, comm))
    stats = MPI.Waitall_(sends + rreqs)[len(sends):]
    for b, st, mid in zip(rbufs, stats, expect):
        s, d, tag, nb, di, _ = byid[mid]
        checks += 1
        if (st.source, st.tag, st.count_lo) != (s, tag, nb):
            bad.append(f"status {(st.source, st.tag, st.count_lo)} != {(s, tag, nb)} for msg {mid}")
            continue
        got = (b.cpu().numpy() if DEVICE else b).view(np.uint8)[:nb]
        if not np.array_equal(got, payload(mid, nb)):
            bad.append(f"payload of msg {mid} ({nb} B) differs")
except Exception:  # noqa: BLE001
    failed = traceback.format_exc()
print(json.dumps({"rank": rank, "checks": checks, "bad": bad[:10], "nbad": len(bad), "failed": failed}), flush=True)
MPI.Finalize()
sys.exit(1 if (failed or bad) else 0)
