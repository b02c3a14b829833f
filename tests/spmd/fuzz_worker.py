"""SPMD worker: randomized parity sweep of the collectives against the
MPICH-pinned oracle (oracle/mpich_model.py).  Where the golden worker replays
the recorded MPICH cases at their sizes, this draws cases the fixtures do not
hold: every valid (op, type) pair, counts from 1 element to a few MiB around
the LL / one-shot / two-shot / zero-copy thresholds and the chunk and slice
boundaries, buffers at element offsets that break 16-B alignment, IN_PLACE,
every root, and every Allreduce algorithm (MPIGX_ALGO through the collective
knob setter; the ring only for integer types, whose results do not depend on
the association).  Every rank draws the same case list from FUZZ_SEED.

Reference calls: collective.jl:698-700 (Allreduce!), :615-617 (Reduce!),
:34 (Bcast!), :304 (Allgather!), :498 (Alltoall!), :765 (Scan!), :839
(Exscan!).  Launched by tests/test_fuzz_gpu.py."""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "mpi.jl_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpigx as MPI  # noqa: E402
from gen_inputs import make  # noqa: E402
from golden_io import same_bits  # noqa: E402
from oracle import mpich_model as M  # noqa: E402

IN_PLACE = ctypes.c_void_p(-1 & ((1 << 64) - 1))
COLLS = ("allreduce", "allreduce", "allreduce", "reduce", "scan", "exscan", "bcast", "allgather", "alltoall")
ALGOS = ("auto", "ll", "ll2", "oneshot", "twoshot", "push", "pull", "pull_generic", "pullpush", "ring")
TYPES = [t for t in M.DTYPES if M.DTYPES[t][2] != "none"]


def draw_cases(seed, n, ncases):
    rng = np.random.default_rng(seed)
    cases = []
    while len(cases) < ncases:
        coll = COLLS[rng.integers(len(COLLS))]
        dt = TYPES[rng.integers(len(TYPES))]
        es = np.dtype(M.DTYPES[dt][1]).itemsize
        if coll in ("bcast", "allgather", "alltoall"):
            op = None
        else:
            op = list(M.OPS)[rng.integers(len(M.OPS))]
            if M.op_valid(dt, op) != 0:
                continue
        # bytes around the thresholds: tiny, LL (<= 16 KiB / 256 KiB), one-shot
        # (<= 256 KiB), two-shot, zero-copy (the test lowers MPIGX_ZC_MIN),
        # with odd element counts
        band = rng.integers(5)
        nbytes = int([rng.integers(1, 64), rng.integers(64, 16 << 10), rng.integers(16 << 10, 300 << 10),
                      rng.integers(300 << 10, 2 << 20), rng.integers(2 << 20, 6 << 20)][band])
        count = max(1, nbytes // es + int(rng.integers(-3, 4)))
        if coll == "alltoall":
            count = max(1, count // n)
        algo = "auto"
        if coll in ("allreduce", "reduce"):
            algo = ALGOS[rng.integers(len(ALGOS))]
            if algo == "ring" and (coll != "allreduce" or M.DTYPES[dt][2] not in ("int", "uint", "byte")):
                algo = "auto"
        cases.append({"coll": coll, "dtype": dt, "op": op, "count": count, "algo": algo,
                      "root": int(rng.integers(n)), "inplace": bool(rng.integers(2)) and coll != "bcast",
                      "off": int(rng.choice([0, 0, 1, 3, 5])), "edge": bool(rng.integers(4) == 0),
                      "seed": int(rng.integers(1 << 30))})
    return cases


def dev_at(a, off_elems):
    """Device copy of numpy array `a` starting `off_elems` elements into its
    allocation (off > 0: not 16-B aligned for every element size < 16)."""
    raw = np.frombuffer(np.ascontiguousarray(a).tobytes(), dtype=np.uint8)
    ob = off_elems * a.itemsize
    t = torch.empty(raw.size + ob + 64, dtype=torch.uint8, device="cuda")[ob: ob + raw.size]
    if raw.size:
        t.copy_(torch.from_numpy(raw.copy()))
    return t


def vcoll_cases(comm, seed, ncases):
    """Gatherv / Scatterv / Allgatherv / Alltoallv (collective.jl:363-382,
    :156-175, :424-442, :545-559) with random per-rank counts (zeros
    included) and displacements with gaps between the blocks: the bytes in
    the gaps and past the last block must stay untouched."""
    r, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
    L, cv = MPI.lib(), comm.val
    I = ctypes.c_int * 16
    rng = np.random.default_rng(seed + 7919)
    fails, ran = [], 0
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    for k in range(ncases):
        coll = ("gatherv", "scatterv", "allgatherv", "alltoallv")[k % 4]
        dt = TYPES[rng.integers(len(TYPES))]
        npdt = M.DTYPES[dt][1]
        h = M.DTYPES[dt][0]
        es = np.dtype(npdt).itemsize
        big = rng.integers(3) == 0
        hi = int(rng.integers(1, (256 << 10) // es if big else 3000))
        C = rng.integers(0, hi, size=(n, n))
        C[rng.random((n, n)) < 0.2] = 0  # some empty blocks
        gaps = rng.integers(0, 4, size=(n, n))
        root = int(rng.integers(n))
        cseed = int(rng.integers(1 << 30))

        def displs(counts, g):
            d, acc = [], 0
            for c_, g_ in zip(counts, g):
                acc += int(g_)
                d.append(acc)
                acc += int(c_)
            return d, acc + 8  # 8 spare elements at the end

        def layout(counts, g, blocks):
            """sentinel-filled buffer with blocks[p] at displs[p]"""
            d, tot = displs(counts, g)
            buf = np.frombuffer(np.full(tot * es, 0xCD, np.uint8).tobytes(), dtype=npdt).copy()
            for p, b in enumerate(blocks):
                if b is not None:
                    buf[d[p]:d[p] + counts[p]] = b
            return buf, d

        srcs = make(dt, "SUM", n, int(C.sum()) + 1, cseed)  # rank p's data
        if coll in ("gatherv", "allgatherv"):
            cnt = [int(C[p][0]) for p in range(n)]
            mine = srcs[r][:cnt[r]]
            exp, d = layout(cnt, gaps[0], [srcs[p][:cnt[p]] for p in range(n)])
            init, _ = layout(cnt, gaps[0], [None] * n)
            recv = dev_at(init, 0)
            sb = dev_at(mine, int(rng.integers(3)))
            if coll == "gatherv":
                rc = L.mpigx_gatherv(P(sb), cnt[r], h, P(recv) if r == root else None, I(*cnt), I(*d), h, root, cv)
                want = exp if r == root else None
            else:
                rc = L.mpigx_allgatherv(P(sb), cnt[r], h, P(recv), I(*cnt), I(*d), h, cv)
                want = exp
        elif coll == "scatterv":
            cnt = [int(C[0][p]) for p in range(n)]
            o = [sum(cnt[:p]) for p in range(n)]  # block p = the root's elements o[p] .. o[p] + cnt[p]
            sendbuf, d = layout(cnt, gaps[0], [srcs[root][o[p]:o[p] + cnt[p]] for p in range(n)])
            sb = dev_at(sendbuf, 0) if r == root else None
            want = np.concatenate([srcs[root][o[r]:o[r] + cnt[r]],
                                   np.frombuffer(np.full(8 * es, 0xCD, np.uint8).tobytes(), dtype=npdt)])
            recv = dev_at(np.frombuffer(np.full((cnt[r] + 8) * es, 0xCD, np.uint8).tobytes(), dtype=npdt).copy(),
                          int(rng.integers(3)))
            rc = L.mpigx_scatterv(P(sb) if sb is not None else None, I(*cnt), I(*d), h, P(recv), cnt[r], h, root, cv)
        else:  # alltoallv: rank p sends C[p][q] elements to q
            sc = [int(C[r][q]) for q in range(n)]
            rcn = [int(C[p][r]) for p in range(n)]
            def block(p, q):  # what rank p sends rank q: its elements sum(C[p][:q]) ..
                o_ = int(C[p][:q].sum())
                return srcs[p][o_:o_ + int(C[p][q])]

            sendbuf, sd = layout(sc, gaps[r], [block(r, q) for q in range(n)])
            exp, rd = layout(rcn, gaps[(r + 1) % n], [block(p, r) for p in range(n)])
            init, _ = layout(rcn, gaps[(r + 1) % n], [None] * n)
            sb = dev_at(sendbuf, int(rng.integers(3)))
            recv = dev_at(init, 0)
            rc = L.mpigx_alltoallv(P(sb), I(*sc), I(*sd), h, P(recv), I(*rcn), I(*rd), h, cv)
            want = exp
        ran += 1
        if rc != 0:
            fails.append({"coll": coll, "k": k, "dtype": dt, "rc": int(rc)})
            continue
        if want is not None:
            got = recv.cpu().numpy().view(np.uint8)
            if not np.array_equal(got, np.ascontiguousarray(want).view(np.uint8)):
                fails.append({"coll": coll, "k": k, "dtype": dt, "counts": C.tolist()[:2], "root": root})
    return fails, ran


def local_cases(seed, ncases):
    """The local MPI.Op kernel (config 2's API, mpigx_reduce_local_multi):
    2-16 inputs, every valid (op, type), odd counts and unaligned buffers, and
    config 2's aligned 8-input shape at sizes that draw every vectors-per-
    thread variant, against the oracle's fold of the same inputs (an
    nin-rank Allreduce)."""
    rng = np.random.default_rng(seed + 104729)
    fails, ran = [], 0
    stream = torch.cuda.current_stream()
    while ran < ncases:
        dt = TYPES[rng.integers(len(TYPES))]
        op = list(M.OPS)[rng.integers(len(M.OPS))]
        if M.op_valid(dt, op) != 0:
            continue
        # one case in three: config 2's shape — 8 aligned inputs (the SH_FULL
        # vector kernel), at sizes up to 20 MiB per input so both
        # vectors-per-thread variants the host picks by size (local_u: 1 / 4)
        # are drawn; otherwise 2-16 inputs at element offsets
        full = rng.integers(3) == 0
        nin = 8 if full else int(rng.integers(2, 17))
        es = np.dtype(M.DTYPES[dt][1]).itemsize
        top = (20 << 20) if full and rng.integers(2) == 0 else (4 << 20)
        count = int(rng.integers(1, top // es if rng.integers(3) == 0 else 5000))
        ins = make(dt, op, nin, count, int(rng.integers(1 << 30)), edge=bool(rng.integers(3) == 0))
        dins = [dev_at(x, 0 if full else int(rng.integers(3))) for x in ins]
        out = dev_at(np.zeros_like(ins[0]), 0 if full else int(rng.integers(3)))
        arr = (ctypes.c_void_p * nin)(*[t.data_ptr() for t in dins])
        rc = MPI.lib().mpigx_reduce_local_multi(arr, nin, ctypes.c_void_p(out.data_ptr()), count, M.DTYPES[dt][0],
                                                M.OPS[op], 0, ctypes.c_void_p(stream.cuda_stream))
        torch.cuda.synchronize()
        ran += 1
        if rc != 0:
            fails.append({"coll": "reduce_local_multi", "dtype": dt, "op": op, "nin": nin, "rc": int(rc)})
            continue
        exp = M.allreduce(ins, dt, op)[0]
        got = out.cpu().numpy().view(M.DTYPES[dt][1])
        if not same_bits(got, exp, bf16=(dt == "BFLOAT16")):
            fails.append({"coll": "reduce_local_multi", "dtype": dt, "op": op, "nin": nin, "count": count})
    return fails, ran


def main():
    comm = MPI.Init()
    r, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
    L, cv = MPI.lib(), comm.val
    cases = draw_cases(int(os.environ.get("FUZZ_SEED", 1)), n, int(os.environ.get("FUZZ_CASES", 120)))
    fails, ran = [], 0
    algo_now = None
    for k, c in enumerate(cases):
        if c["algo"] != algo_now:
            MPI.set_knob(comm, "ALGO", c["algo"])
            algo_now = c["algo"]
        dt, op, count, root = c["dtype"], c["op"], c["count"], c["root"]
        npdt = M.DTYPES[dt][1]
        h = M.DTYPES[dt][0]
        ops = M.OPS.get(op, 0) if op else 0
        per = count * n if c["coll"] == "alltoall" else count
        ins = make(dt, op or "SUM", n, per, c["seed"], edge=c["edge"])
        x = ins[r]
        off = c["off"]
        coll = c["coll"]
        exp = None
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        if coll in ("allreduce", "scan", "exscan"):
            if c["inplace"]:
                recv = dev_at(x, off)
                send = IN_PLACE
            else:
                recv = dev_at(np.full(x.size, 0, npdt), off)
                sbuf = dev_at(x, (off + 1) % 6)  # held until the call returns
                send = P(sbuf)
            if coll == "exscan" and r == 0:
                pre = recv.clone()
            f = {"allreduce": L.mpigx_allreduce, "scan": L.mpigx_scan, "exscan": L.mpigx_exscan}[coll]
            rc = f(send, P(recv), count, h, ops, cv)
            if coll == "allreduce":  # (the ring runs integer types only: any association gives these bits)
                exp = M.allreduce(ins, dt, op)[r]
            elif coll == "scan":
                exp = M.scan(ins, dt, op)[r]
            else:
                exp = M.exscan(ins, dt, op)[r] if r > 0 else pre.cpu().numpy().view(npdt)
            got = recv
        elif coll == "reduce":
            if r == root and c["inplace"]:
                got = dev_at(x, off)
                rc = L.mpigx_reduce(IN_PLACE, P(got), count, h, ops, root, cv)
            else:
                got = dev_at(np.zeros_like(x), off) if r == root else None
                sbuf = dev_at(x, (off + 1) % 6)
                rc = L.mpigx_reduce(P(sbuf), P(got) if got is not None else None, count, h, ops, root, cv)
            exp = M.reduce(ins, dt, op, root) if r == root else None
        elif coll == "bcast":
            got = dev_at(x if r == root else np.zeros_like(x), off)
            rc = L.mpigx_bcast(P(got), count, h, root, cv)
            exp = ins[root]
        elif coll == "allgather":
            if c["inplace"]:
                full = np.zeros(count * n, dtype=npdt)
                full[r * count:(r + 1) * count] = x
                got = dev_at(full, off)
                rc = L.mpigx_allgather(IN_PLACE, 0, 0, P(got), count, h, cv)
            else:
                got = dev_at(np.zeros(count * n, dtype=npdt), off)
                sbuf = dev_at(x, (off + 1) % 6)
                rc = L.mpigx_allgather(P(sbuf), count, h, P(got), count, h, cv)
            exp = M.allgather(ins)[r]
        else:  # alltoall
            if c["inplace"]:
                got = dev_at(x, off)
                rc = L.mpigx_alltoall(IN_PLACE, 0, 0, P(got), count, h, cv)
            else:
                got = dev_at(np.zeros(count * n, dtype=npdt), off)
                sbuf = dev_at(x, (off + 1) % 6)
                rc = L.mpigx_alltoall(P(sbuf), count, h, P(got), count, h, cv)
            exp = M.alltoall(ins, count)[r]
        ran += 1
        desc = dict(c, k=k)
        if rc != 0:
            fails.append(dict(desc, rc=int(rc)))
            continue
        if exp is None:
            continue
        out = got.cpu().numpy().view(npdt)
        exp = np.asarray(exp)
        if not same_bits(out, exp, bf16=(dt == "BFLOAT16")):
            es = out.itemsize
            diff = (out.view(np.uint8).reshape(-1, es) != exp.view(np.uint8).reshape(-1, es)).any(1) \
                if out.shape == exp.shape else np.ones(1, bool)
            bad = np.nonzero(diff)[0]
            fails.append(dict(desc, first_bad=int(bad[0]) if bad.size else -1, nbad=int(bad.size)))
    MPI.set_knob(comm, "ALGO", None)
    f2, r2 = vcoll_cases(comm, int(os.environ.get("FUZZ_SEED", 1)), int(os.environ.get("FUZZ_VCASES", 40)))
    fails += f2
    ran += r2
    if r == 0:
        f3, r3 = local_cases(int(os.environ.get("FUZZ_SEED", 1)), int(os.environ.get("FUZZ_LCASES", 40)))
        fails += f3
        ran += r3
    MPI.Barrier(comm)
    MPI.Finalize()
    print(json.dumps({"rank": r, "n": n, "nfail": len(fails), "ran": ran, "fails": fails[:6]}), flush=True)


if __name__ == "__main__":
    main()
