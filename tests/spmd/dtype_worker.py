"""Derived-datatype scenarios with deterministic, recordable outcomes.

Run as N ranks.  MPIGX_TEST_ARRAYTYPE=ROCArray puts every buffer on the rank's
GPU (libmpigx: types.cpp pack / unpack kernels); otherwise buffers are numpy
arrays on host libmpi (MPICH 3.3.2 under mpiexec).  Each rank writes one JSON
record list; the host run's records are the golden fixture
(tests/golden/make_dtype_golden.sh -> tests/golden/dtype_golden.json) that the
device run must reproduce exactly (tests/test_types_gpu.py).

Scenarios:
* subarray — test/test_subarray.jl restated (contiguous, strided and dense
  SubArray sends / receives around a ring; Julia's column-major 4x4 X is
  stored row-major transposed so every view touches the same bytes);
* structs — test/test_datatype.jl restated (Boundary, Boundary2, Primitive16 /
  24 / 80, packed NTuple{3,UInt8}, 0-sized Nothing) — receive buffers start
  as 0xEE so the bytes MPI must leave alone (padding) are checked too;
* collectives — Bcast / Allgather / Alltoall / Gather / Scatter with struct,
  vector and subarray datatypes; Allreduce / Reduce / Scan over a contiguous
  derived type.
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
from types_cases import BOUNDARY, BOUNDARY2, NTUPLE3  # noqa: E402

DEVICE = os.environ.get("MPIGX_TEST_ARRAYTYPE", "") == "ROCArray"
if DEVICE:
    import torch

REC = []
DEV_CHECKS = []  # engine extensions MPICH has no answer for


def dev(a):
    """Same bytes / shape on the device (torch) or host (numpy copy)."""
    a = np.ascontiguousarray(a)
    if DEVICE:
        return torch.from_numpy(a.copy()).to(f"cuda:{comm.device}")
    return a.copy()


def H(x):
    if DEVICE and not isinstance(x, np.ndarray):
        torch.cuda.synchronize()
        return x.cpu().numpy()
    return np.array(x, copy=True)


def raw(x):
    """bytes of a (device or host) array as hex"""
    return np.ascontiguousarray(H(x)).view(np.uint8).tobytes().hex()


def rec(name, **kw):
    REC.append({"case": name, **kw})


comm = MPI.Init()
rank, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
dest, src = (rank + 1) % n, (rank - 1) % n


def julia_X(r):
    """X = r .+ reshape(1.0:16.0, 4, 4) (column-major) as Xt[j, i] = X[i, j]."""
    X = r + np.arange(1.0, 17.0).reshape(4, 4, order="F")
    return np.ascontiguousarray(X.T)


def subarray():
    """test/test_subarray.jl (testsets contiguous, strided, dense subarray)."""
    # contiguous: @view(X[:,1]) -> Xt[0, :]
    X = dev(julia_X(rank))
    Y = dev(np.zeros(4))
    rs = MPI.Isend(X[0, :], dest, 0, comm)
    rr = MPI.Irecv_(Y, src, 0, comm)
    MPI.Wait_(rs)
    MPI.Wait_(rr)
    rec("contiguous_send", Y=H(Y).tolist())
    Y = dev(np.zeros(2))
    rs = MPI.Isend(Y, dest, 1, comm)
    rr = MPI.Irecv_(X[0, 2:4], src, 1, comm)  # @view(X[3:4,1])
    MPI.Wait_(rs)
    MPI.Wait_(rr)
    rec("contiguous_recv", X=H(X).tolist())
    # strided: @view(X[2,:]) -> Xt[:, 1]
    X = dev(julia_X(rank))
    Y = dev(np.zeros(4))
    rs = MPI.Isend(X[:, 1], dest, 0, comm)
    rr = MPI.Irecv_(Y, src, 0, comm)
    MPI.Wait_(rs)
    MPI.Wait_(rr)
    rec("strided_send", Y=H(Y).tolist())
    Y = dev(np.zeros(2))
    rs = MPI.Isend(Y, dest, 1, comm)
    rr = MPI.Irecv_(X[0:2, 2], src, 1, comm)  # @view(X[3,1:2])
    MPI.Wait_(rs)
    MPI.Wait_(rr)
    rec("strided_recv", X=H(X).tolist())
    # dense subarray: @view(X[2:3,3:4]) -> Xt[2:4, 1:3]
    X = dev(julia_X(rank))
    Y = dev(np.zeros((2, 2)))
    rs = MPI.Isend(X[2:4, 1:3], dest, 0, comm)
    rr = MPI.Irecv_(Y, src, 0, comm)
    MPI.Wait_(rs)
    MPI.Wait_(rr)
    rec("dense_send", Y=H(Y).tolist())
    Y = dev(np.zeros((2, 2)))
    rs = MPI.Isend(Y, dest, 1, comm)
    rr = MPI.Irecv_(X[0:2, 2:4], src, 1, comm)  # @view(X[3:4,1:2])
    MPI.Wait_(rs)
    MPI.Wait_(rr)
    rec("dense_recv", X=H(X).tolist())
    # a stepped 2-D view (general strides -> nested hvector)
    X = dev(julia_X(rank))
    Y = dev(np.zeros((2, 2)))
    st = MPI.Sendrecv_(X[0:4:2, 0:4:3], dest, 2, Y, src, 2, comm)
    rec("stepped_sendrecv", Y=H(Y).tolist(), bytes=st.count_lo)


def struct_exchange(T, count, make, tag):
    arr = np.zeros(count, dtype=T)
    for i in range(count):
        make(arr, i, rank)
    send = dev(arr.view(np.uint8))
    recv = dev(np.full(count * T.itemsize, 0xEE, np.uint8))
    dt = MPI.Datatype(T)
    rr = MPI.Irecv_(MPI.Buffer(recv, count, dt), src, tag, comm)
    rs = MPI.Isend(MPI.Buffer(send, count, dt), dest, tag, comm)
    s = MPI.Wait_(rr)
    MPI.Wait_(rs)
    return raw(recv), s.count_lo, MPI.Get_count(s, dt)


def structs():
    """test/test_datatype.jl (Boundary, Boundary2, primitive types, tuples, Nothing)."""
    def mk_b(a, i, r):
        a[i]["c"] = (r + i + 1) % 127
        a[i]["a"] = i + 1 + r
        a[i]["b"] = (i + 1) % 64
    rec("boundary", **dict(zip(("bytes", "count_lo", "count"), struct_exchange(BOUNDARY, 3, mk_b, 1))))

    def mk_b2(a, i, r):
        a[i]["a"] = (r + i + 1) % 127
        a[i]["b"]["f0"] = i + 1 + r
        a[i]["b"]["f1"] = (i + 1) % 64
    rec("boundary2", **dict(zip(("bytes", "count_lo", "count"), struct_exchange(BOUNDARY2, 3, mk_b2, 1))))

    # primitive types: Julia arrays place them at their aligned size (the MPI extent)
    for bits, nbytes in ((16, 2), (24, 3), (80, 10)):
        V = np.dtype(f"V{nbytes}")
        ext = MPI.Types.extent(MPI.Datatype(V))[1]
        L = np.dtype({"names": ["v"], "formats": [V], "offsets": [0], "itemsize": ext})
        arr = np.zeros(4, dtype=np.dtype([("v", np.uint8, (ext,))]))
        for i in range(4):
            val = (rank + i + 1).to_bytes(16, "little")[:nbytes]
            arr[i]["v"][:nbytes] = np.frombuffer(val, np.uint8)
        send = dev(arr.view(np.uint8))
        recv = dev(np.full(4 * ext, 0xEE, np.uint8))
        dt = MPI.Datatype(V)
        rr = MPI.Irecv_(MPI.Buffer(recv, 4, dt), src, 2, comm)
        rs = MPI.Isend(MPI.Buffer(send, 4, dt), dest, 2, comm)
        s = MPI.Wait_(rr)
        MPI.Wait_(rs)
        del L
        rec(f"primitive{bits}", bytes=raw(recv), count_lo=s.count_lo)

    def mk_t(a, i, r):
        a[i] = (r % 256, i + 1, 0)
    rec("ntuple3", **dict(zip(("bytes", "count_lo", "count"), struct_exchange(NTUPLE3, 8, mk_t, 1))))
    # 0-sized type: 100 elements of Nothing
    dt = MPI.Datatype(np.dtype([]))
    send, recv = dev(np.zeros(1, np.uint8)), dev(np.zeros(1, np.uint8))
    rr = MPI.Irecv_(MPI.Buffer(recv, 100, dt), src, 1, comm)
    rs = MPI.Isend(MPI.Buffer(send, 100, dt), dest, 1, comm)
    s = MPI.Wait_(rr)
    MPI.Wait_(rs)
    rec("nothing", count_lo=s.count_lo, source=s.source, tag=s.tag)


def collectives():
    dtb = MPI.Datatype(BOUNDARY)
    # Bcast of 5 Boundary structs from rank n-1
    arr = np.zeros(5, dtype=BOUNDARY)
    for i in range(5):
        arr[i] = (rank * 10 + i, rank * 1000 + i, i + 7)
    buf = dev(arr.view(np.uint8)) if rank == n - 1 else dev(np.full(5 * 24, 0xEE, np.uint8))
    MPI.Bcast_(MPI.Buffer(buf, 5, dtb), n - 1, comm)
    rec("bcast_struct", bytes=raw(buf))
    # Allgather: send a strided column (vector type), receive contiguous
    X = dev(julia_X(rank))
    out = dev(np.zeros(4 * n))
    MPI.Allgather_(MPI.Buffer(X[:, 1]), MPI.Buffer(out, 4, MPI.Datatype(np.float64)), 4, comm)
    rec("allgather_vector", out=H(out).tolist())
    # Allgather IN_PLACE with a struct type
    ag = np.zeros(2 * n, dtype=BOUNDARY)
    for i in range(2):
        ag[2 * rank + i] = (rank, rank * 100 + i, i)
    agd = dev(ag.view(np.uint8))
    MPI.Allgather_(MPI.IN_PLACE, MPI.Buffer(agd, 2, dtb), 2, comm)
    rec("allgather_inplace_struct", bytes=raw(agd))
    # Alltoall with a struct type: block j goes to rank j
    a2 = np.zeros(n, dtype=BOUNDARY)
    for j in range(n):
        a2[j] = (rank, rank * 100 + j, j)
    s2 = dev(a2.view(np.uint8))
    r2 = dev(np.full(n * 24, 0xEE, np.uint8))
    MPI.Alltoall_(MPI.Buffer(s2, 1, dtb), MPI.Buffer(r2, 1, dtb), 1, comm)
    rec("alltoall_struct", bytes=raw(r2))
    # Gather: each rank sends a dense 2x2 sub-block; root receives contiguous
    X = dev(julia_X(rank))
    g = dev(np.zeros(4 * n))
    MPI.Gather_(MPI.Buffer(X[2:4, 1:3]), MPI.Buffer(g, 4, MPI.Datatype(np.float64)), 4, 0, comm)
    if rank == 0:
        rec("gather_subarray", g=H(g).tolist())
    # Scatter: root sends contiguous blocks of 4, each rank receives into a strided column
    sc = dev(np.arange(4.0 * n) + 0.5)
    Z = dev(np.zeros((4, 4)))
    MPI.Scatter_(MPI.Buffer(sc, 4, MPI.Datatype(np.float64)), MPI.Buffer(Z[:, 2]), 4, 1, comm)
    rec("scatter_vector", Z=H(Z).tolist())
    # reductions over a contiguous derived type (4 x int32 per element): MPICH 3.3.2 rejects predefined ops
    # on derived types (MPI_ERR_OP), the engine reduces them element-wise — checked on the device only
    if DEVICE:
        c4 = MPI.Types.commit_(MPI.Types.create_contiguous(4, MPI.Datatype(np.int32)))
        x = dev(np.arange(12, dtype=np.int32) * (rank + 1))
        y = dev(np.zeros(12, np.int32))
        MPI.Allreduce_(MPI.Buffer(x, 3, c4), MPI.Buffer(y, 3, c4), MPI.SUM, comm)
        want = np.arange(12) * (n * (n + 1) // 2)
        DEV_CHECKS.append({"check": "allreduce_contig_type", "ok": H(y).tolist() == want.tolist()})
        z = dev(np.zeros(12, np.int32))
        MPI.Scan_(MPI.Buffer(x, 3, c4), MPI.Buffer(z, 3, c4), MPI.MAX, comm)
        DEV_CHECKS.append({"check": "scan_contig_type", "ok": H(z).tolist() == (np.arange(12) * (rank + 1)).tolist()})


CASES = [subarray, structs, collectives]

failed = None
try:
    for c in CASES:
        c()
        MPI.Barrier(comm)
except Exception:  # noqa: BLE001
    failed = traceback.format_exc()
_line = json.dumps({"rank": rank, "n": n, "device": DEVICE, "records": REC, "failed": failed,
                    "dev_checks": DEV_CHECKS})
with open(f"{os.environ['DT_OUT']}.{rank}", "w") as f:
    f.write(_line + "\n")
MPI.Finalize()
sys.exit(1 if failed else 0)
