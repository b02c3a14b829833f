"""Point-to-point scenarios with deterministic, recordable outcomes.

Run as N ranks.  MPIGX_TEST_ARRAYTYPE=ROCArray puts every buffer on the rank's
GPU (libmpigx); otherwise buffers are numpy arrays on host libmpi (MPICH 3.3.2
under mpiexec).  Each rank prints one JSON line {"rank", "n", "records"}; the
host run's records are the golden fixture (tests/golden/make_p2p_golden.sh ->
tests/golden/p2p_golden.json) that the device run must reproduce exactly.

Scenarios are built so the MPI matching rules fix the outcome independently
of timing: specific sources (ANY_SOURCE only where one sender exists), tags
chosen so posted-first and unexpected-first matching agree, and barriers that
force one or the other order.  Semantics covered (pointtopoint.jl:107-681):
ring Isend/Irecv + Waitall statuses, blocking Send/Recv chains, Sendrecv
shifts on sub-views, Test/Testall/Testany/Waitany/Waitsome/Testsome incl. all
null arrays, Cancel, PROC_NULL, truncation, Get_count (incl. MPI_UNDEFINED),
Iprobe/Probe on self-sends, zero-size messages, tag matching order with
wildcards, >32 outstanding sends per peer (mailbox wrap), 1 MiB payloads,
error classes.
"""
import json
import os
import sys
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))

import numpy as np  # noqa: E402

import mpigx as MPI  # noqa: E402

DEVICE = os.environ.get("MPIGX_TEST_ARRAYTYPE", "") == "ROCArray"
if DEVICE:
    import torch

REC = []


def A(x, dtype=np.float64):
    a = np.ascontiguousarray(np.asarray(x, dtype=dtype))
    if DEVICE:
        return torch.from_numpy(a.copy()).to(f"cuda:{comm.device}")
    return a


def full(n, v, dtype=np.float64):
    return A(np.full(n, v, dtype=dtype), dtype)


def tolist(x):
    if DEVICE:
        torch.cuda.synchronize()
        return x.cpu().numpy().tolist()
    return x.tolist()


def st(s, with_src=True):
    if s is None:
        return None
    if s.count_hi_and_cancelled & 1:
        return {"cancelled": 1, "bytes": s.count_lo}
    d = {"bytes": s.count_lo, "cancelled": 0, "error": s.error}
    if with_src:
        d.update(source=s.source, tag=s.tag)
    return d


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
dst, src = (rank + 1) % n, (rank - 1) % n


def ring_waitall():
    """test_sendrecv.jl:22-43."""
    N = 32
    send_mesg = full(N, rank)
    recv_mesg = full(N, -1.0)
    rreq = MPI.Irecv_(recv_mesg, src, src + 32, comm)
    sreq = MPI.Isend(send_mesg, dst, rank + 32, comm)
    stats = MPI.Waitall_([sreq, rreq])
    rec("ring_waitall", recv=st(stats[1]), send_null=MPI.isnull(sreq), recv_null=MPI.isnull(rreq),
        data_ok=tolist(recv_mesg) == [float(src)] * N)
    done, stats2 = MPI.Testall_([sreq, rreq])
    rec("testall_after", done=done, stats=[st(s) for s in stats2])


def chain_blocking():
    """test_sendrecv.jl:45-70 (Send/Recv! on arrays, then scalars)."""
    N = 8
    send_mesg = full(N, rank)
    recv_mesg = full(N, -1.0)
    if rank == 0:
        MPI.Send(send_mesg, dst, rank + 32, comm)
        s = None
    elif rank == n - 1:
        s = MPI.Recv_(recv_mesg, src, src + 32, comm)
    else:
        s = MPI.Recv_(recv_mesg, src, src + 32, comm)
        MPI.Send(send_mesg, dst, rank + 32, comm)
    rec("chain", status=st(s), data=None if rank == 0 else tolist(recv_mesg))
    # serialized objects (MPI.send / MPI.recv)
    obj = {"from": rank, "v": [rank, rank * 2]}
    if rank == 0:
        MPI.send(obj, dst, 77, comm)
        got = None
    elif rank == n - 1:
        got, _ = MPI.recv(src, 77, comm)
    else:
        got, _ = MPI.recv(src, 77, comm)
        MPI.send(obj, dst, 77, comm)
    rec("chain_obj", got=got)


def waitsome_test():
    """test_test.jl."""
    N = 16
    send_mesg = full(N, rank)
    recv_mesg = full(N, -1.0)
    rreq = MPI.Irecv_(recv_mesg, src, src + 32, comm)
    sreq = MPI.Isend(send_mesg, dst, rank + 32, comm)
    reqs = [sreq, rreq]
    inds, stats = MPI.Waitsome_(reqs)
    ok = bool(inds)
    for i in inds:
        done, s = MPI.Test_(reqs[i - 1])
        ok &= done and s == MPI.STATUS_EMPTY
    MPI.Waitall_(reqs)
    i2, s2 = MPI.Waitsome_(reqs)
    i3, s3 = MPI.Testsome_(reqs)
    rec("waitsome", ok=ok, after_waitsome=[i2, [st(s) for s in s2]], after_testsome=[i3, [st(s) for s in s3]],
        data_ok=tolist(recv_mesg) == [float(src)] * N)


def null_arrays():
    reqs = [MPI.Request(), MPI.Request()]
    i, s = MPI.Waitany_(reqs)
    f, i2, s2 = MPI.Testany_(reqs)
    w = MPI.Waitall_(reqs)
    ok1, t = MPI.Testall_(reqs)
    s5 = MPI.Wait_(MPI.Request())
    f6, s6 = MPI.Test_(MPI.Request())
    rec("null_arrays", waitany=[i, st(s)], testany=[f, i2, st(s2)], waitall=[st(x) for x in w],
        testall=[ok1, [st(x) for x in t]], wait=st(s5), test=[f6, st(s6)])


def waitany_self():
    """test_wait.jl: sends/receives to self, Waitany! order-free accounting."""
    nsends = 2
    send_arr = [A([i + 1], np.int64) for i in range(nsends)]
    recv_arr = [A([0], np.int64) for _ in range(nsends)]
    send_reqs = [MPI.Isend(send_arr[i], rank, i + 1, comm) for i in range(nsends)]
    recv_reqs = [MPI.Irecv_(recv_arr[i], rank, i + 1, comm) for i in range(nsends)]
    send_check = [0] * nsends
    recv_check = [0] * nsends
    for _ in range(nsends):
        idx, _s = MPI.Waitany_(send_reqs)
        send_check[idx - 1] += 1
        assert MPI.isnull(send_reqs[idx - 1])
    for _ in range(nsends):
        idx, _s = MPI.Waitany_(recv_reqs)
        recv_check[idx - 1] += 1
    rec("waitany_self", send_check=send_check, recv_check=recv_check, data=[tolist(r) for r in recv_arr])


def cancel_procnull():
    buf = full(4, -1.0)
    r = MPI.Irecv_(buf, src, 999, comm)
    MPI.Cancel_(r)
    s = MPI.Wait_(r)
    rec("cancel", status=st(s), cancelled=MPI.Test_cancelled(s), null=MPI.isnull(r), buffer_none=r.buffer is None)
    s2 = MPI.Recv_(buf, MPI.PROC_NULL, 3, comm)
    MPI.Send(buf, MPI.PROC_NULL, 3, comm)
    r3 = MPI.Irecv_(buf, MPI.PROC_NULL, 3, comm)
    s3 = MPI.Wait_(r3)
    f, s4 = MPI.Iprobe(MPI.PROC_NULL, 3, comm)
    rec("procnull", recv=st(s2), irecv=st(s3), iprobe=[f, st(s4)], data=tolist(buf))


def truncation_getcount():
    MPI.Barrier(comm)
    if rank == 0:
        MPI.Send(full(8, 5.0), 1 % n, 5, comm)
    cls = None
    if rank == 1 % n:
        out = full(4, -1.0)
        cls = err_class(lambda: MPI.Recv_(out, 0, 5, comm))
    MPI.Barrier(comm)
    cnt = None
    if rank == 0:
        MPI.Send(A([1, 2, 3], np.uint8), 1 % n, 6, comm)
    if rank == 1 % n:
        out = A(np.zeros(8, np.uint8), np.uint8)
        s = MPI.Recv_(out, 0, 6, comm)
        cnt = [MPI.Get_count(s, np.float64), MPI.Get_count(s, np.uint8), MPI.Get_count(s, np.int16)]
    rec("truncation", err=cls, counts=cnt)
    MPI.Barrier(comm)


def probe_self_zero():
    r0 = MPI.Isend(full(5, rank), rank, 44, comm)
    f, s = MPI.Iprobe(rank, 44, comm)
    while not f:
        f, s = MPI.Iprobe(rank, 44, comm)
    s2 = MPI.Probe(rank, MPI.ANY_TAG, comm)
    out = full(16, -1.0)
    s3 = MPI.Recv_(out, rank, MPI.ANY_TAG, comm)
    MPI.Wait_(r0)
    f4, s4 = MPI.Iprobe(rank, MPI.ANY_TAG, comm)
    z = A(np.zeros(0))
    r5 = MPI.Isend(z, rank, 45, comm)
    s5 = MPI.Recv_(A(np.zeros(0)), rank, 45, comm)
    MPI.Wait_(r5)
    rec("probe_self", iprobe=st(s), probe=st(s2), recv=st(s3), count=MPI.Get_count(s3, np.float64),
        data=tolist(out)[:6], after=[f4, st(s4)], zero=st(s5))


def tag_order():
    """Non-overtaking + wildcard matching, unexpected-first then posted-first."""
    tags = [5, 6, 5, 7, 6]
    pattern = [7, 5, MPI.ANY_TAG, 5, 6]
    res = {}
    for mode in ("unexpected_first", "posted_first"):
        bufs = [full(3, -1.0) for _ in pattern]
        sends = []
        rreqs = []
        if mode == "unexpected_first":
            sends = [MPI.Isend(full(3, 100 * rank + k), dst, t, comm) for k, t in enumerate(tags)]
            MPI.Barrier(comm)
            rreqs = [MPI.Irecv_(b, src, t, comm) for b, t in zip(bufs, pattern)]
        else:
            rreqs = [MPI.Irecv_(b, src, t, comm) for b, t in zip(bufs, pattern)]
            MPI.Barrier(comm)
            sends = [MPI.Isend(full(3, 100 * rank + k), dst, t, comm) for k, t in enumerate(tags)]
        stats = MPI.Waitall_(rreqs + sends)
        res[mode] = {"tags": [s.tag for s in stats[:len(pattern)]], "data": [tolist(b)[0] for b in bufs]}
        MPI.Barrier(comm)
    rec("tag_order", **res)


def many_outstanding():
    """40 messages to one peer (more than the 32 mailbox slots), received in
    reverse tag order."""
    K = 40
    MPI.Barrier(comm)
    sends = [MPI.Isend(full(2, 1000 * rank + k), dst, k, comm) for k in range(K)]
    bufs = [full(2, -1.0) for _ in range(K)]
    rreqs = [MPI.Irecv_(bufs[k], src, k, comm) for k in reversed(range(K))]
    MPI.Waitall_(sends + rreqs)
    rec("many_outstanding", data=[tolist(b)[0] for b in bufs])


def sendrecv_shift():
    """test_sendrecv.jl:80-140 (Cart_shift(comm_cart, 0, -1) on a periodic
    1-D grid: dest = rank-1, source = rank+1)."""
    dest_rank, src_rank = (rank - 1) % n, (rank + 1) % n
    a = A([rank, rank, rank])
    MPI.Sendrecv_(a[0:1], dest_rank, 0, a[2:3], src_rank, 0, comm)
    r1 = tolist(a)
    a = A([rank, rank, rank])
    b = A([-1, -1, -1])
    MPI.Sendrecv_(a[0:2], dest_rank, 1, b[0:2], src_rank, 1, comm)
    r2 = tolist(b)
    a = A([rank, rank, rank])
    b = A([-1, -1, -1])
    s = MPI.Sendrecv_(a, dest_rank, 2, b, src_rank, 2, comm)
    rec("sendrecv", r1=r1, r2=r2, r3=tolist(b), status=st(s))


def big():
    N = 1 << 17  # 1 MiB of float64
    x = A(np.arange(N, dtype=np.float64) + rank * N)
    y = full(N, -1.0)
    s = MPI.Sendrecv_(x, dst, 9, y, src, 9, comm)
    yl = np.asarray(tolist(y))
    rec("big", status=st(s), ok=bool((yl == np.arange(N) + src * N).all()))


def errors():
    buf = full(2, 0.0)
    e = {
        "send_rank": err_class(lambda: MPI.Send(buf, n + 3, 0, comm)),
        "send_tag": err_class(lambda: MPI.Send(buf, 0, -3, comm)),
        "send_anysrc": err_class(lambda: MPI.Send(buf, MPI.ANY_SOURCE, 0, comm)),
        "send_anytag": err_class(lambda: MPI.Send(buf, 0, MPI.ANY_TAG, comm)),
        "send_tag_ub": err_class(lambda: MPI.Send(buf, 0, 268435456, comm)),
        "recv_rank": err_class(lambda: MPI.Recv_(buf, n + 3, 0, comm)),
        "recv_tag": err_class(lambda: MPI.Recv_(buf, 0, -5, comm)),
        "send_count": err_class(lambda: MPI.Send(MPI.Buffer(buf, -1, np.float64), 0, 0, comm)),
    }
    rec("errors", **e)


CASES = [ring_waitall, chain_blocking, waitsome_test, null_arrays, waitany_self, cancel_procnull,
         truncation_getcount, probe_self_zero, tag_order, many_outstanding, sendrecv_shift, big, errors]

failed = None
try:
    for c in CASES:
        c()
        MPI.Barrier(comm)
except Exception:  # noqa: BLE001
    failed = traceback.format_exc()
print(json.dumps({"rank": rank, "n": n, "device": DEVICE, "records": REC, "failed": failed}), flush=True)
MPI.Finalize()
sys.exit(1 if failed else 0)
