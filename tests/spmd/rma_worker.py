"""One-sided (RMA) scenarios with deterministic, recordable outcomes.

Run as N ranks.  MPIGX_TEST_ARRAYTYPE=ROCArray puts every window and operand
on the rank's GPU (libmpigx, rma.cpp); otherwise they are numpy arrays on host
libmpi (MPICH 3.3.2 under mpiexec).  Each rank prints one JSON line {"rank",
"n", "records"}; the host run's records are the golden fixture
(tests/golden/make_rma_golden.sh -> tests/golden/rma_golden.json) that the
device run must reproduce exactly.

Scenarios (src/onesided.jl:24-219):
* onesided_ref — test/test_onesided.jl restated line by line (fence Get,
  exclusive-lock Put, local access under a self lock, Get_accumulate SUM,
  Accumulate SUM, dynamic window + Get_address + Fetch_and_op REPLACE);
* shared_win — test/test_shared_win.jl restated (Comm_split,
  Win_allocate_shared on one owner, Win_shared_query, direct stores by two
  ranks, Barrier, every rank reads);
* acc_matrix — Accumulate and Get_accumulate for every predefined op
  (+REPLACE, NO_OP) x 12 types incl. NaN / +-0 / ties / wraparound, one origin
  per target range so the result does not depend on arrival order; invalid
  (op, type) pairs record their error class;
* fetch_ops — Fetch_and_op SUM / NO_OP / REPLACE / MAX chains;
* multi_origin — every rank accumulates into the same elements of rank 0
  (SUM, BOR, MAX on integers: order-independent), shared-lock Gets;
* large — 4 MiB Put/Get and a Get_accumulate larger than the engine's scratch
  slot (chunked) checked by exact integer-valued sums;
* errors — unlock without lock, bad lock type, bad rank, invalid op.
"""
import json
import os
import sys
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

import mpigx as MPI  # noqa: E402

DEVICE = os.environ.get("MPIGX_TEST_ARRAYTYPE", "") == "ROCArray"
if DEVICE:
    import torch

REC = []
DEV_CHECKS = []  # engine-only checks: (op, type) pairs MPICH does not reject at the call (see acc_matrix)


def A(x, dtype=np.int64):
    a = np.ascontiguousarray(np.asarray(x, dtype=dtype))
    if DEVICE:
        return torch.from_numpy(a.copy()).to(f"cuda:{comm.device}")
    return a


def H(x):
    """Host numpy copy of an operand."""
    if DEVICE and not isinstance(x, np.ndarray):
        torch.cuda.synchronize()
        return x.cpu().numpy()
    return np.array(x, copy=True)


def bits(x):
    """Exact record: integers as ints, floats/complex as bit patterns."""
    a = H(x)
    if a.dtype.kind in "fc":
        u = {2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize if a.dtype.kind == "f" else
                                                       a.dtype.itemsize // 2]
        return [format(int(v), "x") for v in a.view(u).reshape(-1)]
    return [int(v) for v in a.reshape(-1)]


def setv(buf, idx, v):
    buf[idx] = v


def fill(buf, v):
    if isinstance(buf, np.ndarray):
        buf.fill(v)
    else:
        buf.fill_(v)


def rec(name, **kw):
    REC.append({"case": name, **kw})


def err_class(fn):
    try:
        fn()
    except MPI.MPIError as e:
        return MPI.Error_class(e.code)
    return 0


comm = MPI.Init()
rank, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)


def onesided_ref():
    """test/test_onesided.jl (whole file, in order)."""
    N = n
    buf = A(np.full(N, rank))
    received = A(np.full(N, -1))
    win = MPI.Win_create(buf, comm)
    MPI.Win_fence(0, win)
    MPI.Get(received, (rank + 1) % N, win)
    MPI.Win_fence(0, win)
    rec("fence_get", received=bits(received))
    # locked window
    if rank != 0:
        MPI.Win_lock(MPI.LOCK_EXCLUSIVE, 0, 0, win)
        setv(received, 0, rank)
        MPI.Put(received, 1, 0, rank, win)
        MPI.Win_unlock(0, win)
    else:
        setv(buf, 0, 0)
    MPI.Win_fence(0, win)
    if rank == 0:
        rec("lock_put", buf=bits(buf))
    MPI.Barrier(comm)
    if rank == 1:
        MPI.Win_lock(MPI.LOCK_EXCLUSIVE, 1, 0, win)
        fill(buf, 3)
        MPI.Win_unlock(1, win)
    MPI.Barrier(comm)
    if rank == 0:
        MPI.Win_lock(MPI.LOCK_EXCLUSIVE, 0, 0, win)
        fill(buf, 2)
        MPI.Win_unlock(0, win)
        MPI.Win_lock(MPI.LOCK_EXCLUSIVE, 1, 0, win)
        result = A(np.zeros(N, np.int64))
        MPI.Get_accumulate(buf, result, N, 1, 0, MPI.SUM, win)
        MPI.Win_unlock(1, win)
        rec("get_accumulate", result=bits(result))
    MPI.Barrier(comm)
    if rank == 1:
        MPI.Win_lock(MPI.LOCK_EXCLUSIVE, 1, 0, win)
        rec("after_gacc", buf=bits(buf))
        fill(buf, -2)
        MPI.Win_unlock(1, win)
        MPI.Win_lock(MPI.LOCK_EXCLUSIVE, 0, 0, win)
        MPI.Accumulate(buf, N, 0, 0, MPI.SUM, win)
        MPI.Win_unlock(0, win)
        MPI.Win_lock(MPI.LOCK_EXCLUSIVE, 1, 0, win)
        fill(buf, 1)
        MPI.Win_unlock(1, win)
    MPI.Barrier(comm)
    if rank == 0:
        MPI.Win_lock(MPI.LOCK_EXCLUSIVE, 0, 0, win)
        rec("after_acc", buf=bits(buf))
        MPI.Win_unlock(0, win)
    MPI.Barrier(comm)
    MPI.free(win)
    MPI.Barrier(comm)
    # dynamic window
    win = MPI.Win_create_dynamic(comm)
    MPI.Win_attach(win, buf)
    address_buf = A(np.zeros(1, np.int64))
    address_win = MPI.Win_create(address_buf, comm)
    MPI.Win_lock(MPI.LOCK_EXCLUSIVE, rank, 0, address_win)
    setv(address_buf, 0, MPI.Get_address(buf))
    MPI.Win_unlock(rank, address_win)
    MPI.Barrier(comm)
    if rank == 0:
        received = np.zeros(1, np.int64)
        to_send = np.zeros(1, np.int64)
        got = []
        for r in range(N):
            address = np.zeros(1, np.int64)
            MPI.Win_lock(MPI.LOCK_EXCLUSIVE, r, 0, address_win)
            MPI.Get(address, r, address_win)
            MPI.Win_flush(r, address_win)
            to_send[0] = r + 5
            MPI.Win_lock(MPI.LOCK_EXCLUSIVE, r, 0, win)
            MPI.Fetch_and_op(to_send, received, r, int(address[0]) + r * 8, MPI.REPLACE, win)
            MPI.Win_flush(r, win)
            got.append(int(received[0]))
            MPI.Win_unlock(r, win)
            MPI.Win_unlock(r, address_win)
        rec("dynamic_fetch_and_op", received=got)
    MPI.Barrier(comm)
    rec("dynamic_result", value=bits(buf)[rank])
    MPI.Barrier(comm)
    MPI.Win_detach(win, buf)
    MPI.free(win)
    MPI.free(address_win)


def shared_win():
    """test/test_shared_win.jl: owner 1 allocates a 100x2 Float32 array."""
    node_comm = MPI.Comm_split(comm, 1, rank)
    node_rank = MPI.Comm_rank(node_comm)
    owner = 1
    sz = (100, 2)
    length = int(np.prod(sz)) if node_rank == owner else 0
    win, ptr = MPI.Win_allocate_shared(np.float32, length, node_comm)
    if node_rank != owner:
        _, _, ptr = MPI.Win_shared_query(win, owner)
    arr = MPI.unsafe_wrap(ptr, np.float32, sz, win)
    if node_rank == 0:
        v = np.arange(1, 101, dtype=np.float32)
        arr[:, 0] = torch.from_numpy(v).to(arr.device) if DEVICE else v
    elif node_rank == 1:
        v = np.arange(901, 1001, dtype=np.float32)
        arr[:, 1] = torch.from_numpy(v).to(arr.device) if DEVICE else v
    MPI.Barrier(node_comm)
    h = H(arr)
    rec("shared_cols", c0=bool((h[:, 0] == np.arange(1, 101)).all()), c1=bool((h[:, 1] == np.arange(901, 1001)).all()))
    if node_rank <= 1:
        ln, elsize, base = MPI.Win_shared_query(win, owner)
        p = arr.data_ptr() if DEVICE else arr.ctypes.data
        rec("shared_query", elsize=elsize, len=ln, same_ptr=base == p)
    MPI.Barrier(node_comm)
    MPI.free(win)
    MPI.free(node_comm)


from rma_cases import K, OPS, TYPES, operands  # noqa: E402


def acc_matrix():
    t = (rank + 1) % n  # I accumulate into my right neighbour's range [rank*K, rank*K+K)
    for dt in TYPES:
        for opname in OPS:
            op = getattr(MPI, opname)
            valid = opname in ("REPLACE", "NO_OP") or MPI.lib().mpigx_op_valid(MPI.Datatype(dt).val, op.val) == 0
            for salt, fetch in ((1, False), (2, True)):
                mine = np.concatenate([operands(dt, opname, 100 + rank, salt + 10 * q) for q in range(n)])
                wbuf = A(mine, dt)
                win = MPI.Win_create(wbuf, comm)
                o = A(operands(dt, opname, rank, salt), dt)
                res = A(np.zeros(K, dt), dt)
                MPI.Win_fence(0, win)
                rc = None
                # an erroneous (op, type) pair is not issued on MPICH: 3.3.2 returns MPI_SUCCESS at the call,
                # then fails the next fence ("Invalid MPI_Op") or leaves the window undefined; the engine
                # rejects it with MPI_ERR_OP before touching anything (checked on the device only)
                if valid or DEVICE:
                    if fetch:
                        rc = err_class(lambda: MPI.Get_accumulate(o, res, K, t, rank * K, op, win))
                    else:
                        rc = err_class(lambda: MPI.Accumulate(o, K, t, rank * K, op, win))
                MPI.Win_fence(0, win)
                if not valid:
                    if DEVICE:
                        DEV_CHECKS.append({"check": f"acc {np.dtype(dt).name} {opname} fetch={fetch}",
                                           "ok": rc == 9 and bits(wbuf) == bits(mine)})
                    rec("acc", dt=np.dtype(dt).name, op=opname, fetch=fetch, invalid=True)
                    MPI.free(win)
                    continue
                src = (rank - 1) % n
                d = {"rc": rc, "win": bits(H(wbuf)[src * K:(src + 1) * K])}
                if fetch and rc == 0:
                    d["res"] = bits(res)
                rec("acc", dt=np.dtype(dt).name, op=opname, fetch=fetch, **d)
                MPI.free(win)


def fetch_ops():
    wbuf = A(np.arange(4, dtype=np.int64) * 10 + rank)
    win = MPI.Win_create(wbuf, comm)
    MPI.Win_fence(0, win)
    MPI.Win_fence(0, win)
    t = (rank + 1) % n
    res = np.zeros(1, np.int64)
    out = []
    MPI.Win_lock(MPI.LOCK_EXCLUSIVE, t, 0, win)
    for opname, val, disp in (("SUM", 7, 0), ("SUM", 5, 0), ("NO_OP", 0, 0), ("REPLACE", -4, 1), ("MAX", 100, 2),
                              ("MAX", -100, 2), ("MIN", 3, 3), ("PROD", -2, 3)):
        src = np.array([val], np.int64)  # alive until the flush completes the operation
        MPI.Fetch_and_op(src, res, t, disp, getattr(MPI, opname), win)
        MPI.Win_flush(t, win)  # the result is defined once the operation completed
        out.append(int(res[0]))
    MPI.Win_unlock(t, win)
    MPI.Win_fence(0, win)
    rec("fetch_ops", fetched=out, win=bits(wbuf))
    MPI.free(win)


def multi_origin():
    wbuf = A(np.zeros(6, np.int64))
    win = MPI.Win_create(wbuf, comm)
    # origin buffers must stay alive until the epoch completes (MPI-3 §11.3)
    o1, o2, o3 = A(np.full(2, rank + 1)), A(np.full(2, 1 << rank)), A(np.array([rank * 3 - 5, -rank]))
    MPI.Win_fence(0, win)
    MPI.Accumulate(o1, 2, 0, 0, MPI.SUM, win)
    MPI.Accumulate(o2, 2, 0, 2, MPI.BOR, win)
    MPI.Accumulate(o3, 2, 0, 4, MPI.MAX, win)
    MPI.Win_fence(0, win)
    if rank == 0:
        rec("multi_origin", win=bits(wbuf))
    MPI.Barrier(comm)
    # shared locks: everyone reads rank 0 at once
    got = A(np.zeros(6, np.int64))
    MPI.Win_lock(MPI.LOCK_SHARED, 0, 0, win)
    MPI.Get(got, 0, win)
    MPI.Win_unlock(0, win)
    rec("shared_lock_get", got=bits(got))
    MPI.Barrier(comm)  # every Get of the shared epoch is complete before anyone accumulates
    # passive-target accumulates from everyone, then a fence
    o4 = A(np.full(6, rank + 1))
    MPI.Win_lock(MPI.LOCK_SHARED, 0, 0, win)
    MPI.Accumulate(o4, 6, 0, 0, MPI.SUM, win)
    MPI.Win_unlock(0, win)
    MPI.Win_fence(0, win)
    MPI.Win_fence(0, win)
    if rank == 0:
        rec("shared_lock_acc", win=bits(wbuf))
    MPI.Barrier(comm)
    MPI.free(win)


def large():
    M = 1 << 20  # float32 elements per block (4 MiB)
    wbuf = A(np.zeros(3 * M, np.float32), np.float32)
    win = MPI.Win_create(wbuf, comm)
    t = (rank + 1) % n
    x = A((np.arange(M) % 1024 + rank).astype(np.float32), np.float32)
    MPI.Win_fence(0, win)
    MPI.Put(x, M, t, M, win)
    MPI.Win_fence(0, win)
    back = A(np.zeros(M, np.float32), np.float32)
    MPI.Get(back, M, t, M, win)
    MPI.Win_fence(0, win)
    hb = H(back)
    ok_get = bool((hb == (np.arange(M) % 1024 + rank)).all())
    # Get_accumulate over 2M elements (8 MiB, larger than the scratch slot)
    y = A(np.ones(2 * M, np.float32), np.float32)
    res = A(np.zeros(2 * M, np.float32), np.float32)
    MPI.Win_lock(MPI.LOCK_EXCLUSIVE, t, 0, win)
    MPI.Get_accumulate(y, res, 2 * M, t, M, MPI.SUM, win)
    MPI.Win_unlock(t, win)
    MPI.Win_fence(0, win)
    hr, hw = H(res), H(wbuf)
    rec("large", ok_get=ok_get, res_sum=float(hr.astype(np.float64).sum()), win_sum=float(hw.astype(np.float64).sum()),
        res_head=bits(hr[:4]), res_mid=bits(hr[M - 2:M + 2]))
    MPI.free(win)


def errors():
    wbuf = A(np.zeros(4, np.float64), np.float64)
    win = MPI.Win_create(wbuf, comm)
    e = {
        "unlock_unlocked": err_class(lambda: MPI.Win_unlock(0, win)),
        "lock_bad_rank": err_class(lambda: MPI.Win_lock(MPI.LOCK_EXCLUSIVE, n + 2, 0, win)),
        "lock_bad_type": err_class(lambda: MPI.Win_lock(MPI.LockType(7), 0, 0, win)),
    }
    MPI.Win_fence(0, win)
    ones = A(np.ones(4), np.float64)
    if DEVICE:  # erroneous on MPICH (see acc_matrix)
        rc = err_class(lambda: MPI.Accumulate(ones, 4, 0, 0, MPI.BAND, win))
        DEV_CHECKS.append({"check": "acc_band_float -> MPI_ERR_OP", "ok": rc == 9})
    e["get_bad_rank"] = err_class(lambda: MPI.Get(ones, 4, n + 1, 0, win))
    MPI.Win_fence(0, win)
    rec("errors", **e)
    MPI.free(win)


CASES = [onesided_ref, shared_win, fetch_ops, multi_origin, large, acc_matrix, errors]

failed = None
try:
    for c in CASES:
        c()
        MPI.Barrier(comm)
except Exception:  # noqa: BLE001
    failed = traceback.format_exc()
_line = json.dumps({"rank": rank, "n": n, "device": DEVICE, "records": REC, "failed": failed,
                    "dev_checks": DEV_CHECKS})
if os.environ.get("RMA_OUT"):  # one file per rank (long lines from several ranks interleave on a pipe)
    with open(f"{os.environ['RMA_OUT']}.{rank}", "w") as f:
        f.write(_line + "\n")
else:
    print(_line, flush=True)
MPI.Finalize()
sys.exit(1 if failed else 0)
