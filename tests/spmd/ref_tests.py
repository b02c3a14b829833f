"""The reference's collective test scripts, restated on the Python mirror.

Each `t_*` function follows one MPI.jl test file line by line
(test/test_allreduce.jl, test_reduce.jl, test_scan.jl, test_exscan.jl,
test_bcast.jl, test_allgather.jl, test_alltoall.jl).  As in the reference,
`ArrayType` is switched by an environment variable:

  MPIGX_TEST_ARRAYTYPE=ROCArray  -> torch tensors on the rank's GPU (libmpigx)
  otherwise                      -> numpy host arrays (libmpi = MPICH 3.3.2)

The reference runs host arrays under `mpiexec -n nprocs`; so does
tests/test_reference_suite_cpu.py.  Device mode (like JULIA_MPI_TEST_ARRAYTYPE=
CuArray) is tests/test_reference_suite_gpu.py.  Deviation: the custom op
(x,y)->2x+y-x also runs in device mode here (the reference skips it for
CuArray, test_allreduce.jl:15-22) because the mirror supports user ops on
device buffers; the Double64 case of test_reduce.jl:104-118 is skipped
(DoubleFloats has no Python counterpart).
"""
import json
import operator
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

# MPIDatatype = Union{Char, Int8..UInt64, Float32, Float64, ComplexF32, ComplexF64} (buffers.jl:5-8)
TYPES = [np.int8, np.uint8, np.int16, np.uint16, np.int32, np.uint32, np.int64, np.uint64, np.float32, np.float64,
         np.complex64, np.complex128]
if DEVICE:  # torch has no uint32/uint64 arithmetic on device; they still move as raw bits
    TYPES = [t for t in TYPES]

FAIL = []
NCHECK = [0]


def check(cond, what):
    NCHECK[0] += 1
    if not bool(cond):
        FAIL.append(what)


def raises(exc, fn, what):
    NCHECK[0] += 1
    try:
        fn()
    except exc:
        return
    except Exception as e:  # noqa: BLE001
        FAIL.append(f"{what}: wrong exception {e!r}")
        return
    FAIL.append(f"{what}: no exception")


def arr(x, T=None):
    """ArrayType(x)."""
    a = np.asarray(x, dtype=T)
    if DEVICE:
        if a.dtype in (np.uint16, np.uint32, np.uint64):
            t = torch.from_numpy(a.view({2: np.int16, 4: np.int32, 8: np.int64}[a.itemsize]).copy())
            return t.cuda().view({2: torch.uint16, 4: torch.uint32, 8: torch.uint64}[a.itemsize])
        return torch.from_numpy(np.ascontiguousarray(a)).cuda()
    return np.ascontiguousarray(a)


def undef(shape, T):
    """ArrayType{T}(undef, shape)."""
    return arr(np.zeros(shape, dtype=T))


def host(x):
    if DEVICE and hasattr(x, "cpu"):
        if str(x.dtype) in ("torch.uint16", "torch.uint32", "torch.uint64"):
            isz = x.element_size()
            npdt = {2: np.uint16, 4: np.uint32, 8: np.uint64}[isz]
            return x.view({2: torch.int16, 4: torch.int32, 8: torch.int64}[isz]).cpu().numpy().view(npdt)
        return x.cpu().numpy()
    return np.asarray(x)


def eq(a, b):
    a, b = host(a), host(b)
    return a.shape == np.asarray(b).shape and np.array_equal(a, b)


def copy(x):
    return x.clone() if DEVICE else x.copy()


def is_array_type(x, T=None):
    ok = isinstance(x, torch.Tensor) and x.is_cuda if DEVICE else isinstance(x, np.ndarray)
    return ok and (T is None or host(x).dtype == np.dtype(T))


# ---------------------------------------------------------------------------
def t_allreduce(comm):
    """test/test_allreduce.jl:13-55"""
    comm_size = MPI.Comm_size(comm)
    operators = [MPI.SUM, operator.add, lambda x, y: 2 * x + y - x]
    T = np.int64  # `for T = [Int]`
    for dims in (1, 2, 3):
        send_arr = np.zeros((3,) * dims, dtype=T)
        send_arr.reshape(-1)[:] = np.arange(1, send_arr.size + 1)
        send_arr = arr(send_arr)
        for op in operators:
            recv_arr = undef(host(send_arr).shape, T)
            MPI.Allreduce_(send_arr, recv_arr, op, comm)
            check(eq(recv_arr, comm_size * host(send_arr)), ("allreduce", dims))
            recv_short = undef(tuple(d - 1 for d in host(send_arr).shape), T)
            raises(AssertionError, lambda: MPI.Allreduce_(send_arr, recv_short, _len(send_arr), op, comm),
                   "allreduce short recv")
            recv_arr = copy(send_arr)
            MPI.Allreduce_(recv_arr, op, comm)
            check(eq(recv_arr, comm_size * host(send_arr)), ("allreduce IN_PLACE", dims))
            val = MPI.Allreduce(2, op, comm)
            check(val == comm_size * 2, ("allreduce scalar", val))
            vals = MPI.Allreduce(send_arr, op, comm)
            check(is_array_type(vals, T), "allreduce alloc type")
            check(eq(vals, comm_size * host(send_arr)), ("allreduce alloc", dims))
    MPI.Barrier(comm)


def _len(a):
    return host(a).size


def t_reduce(comm):
    """test/test_reduce.jl:11-101"""
    sz, rank = MPI.Comm_size(comm), MPI.Comm_rank(comm)
    root = sz - 1
    isroot = rank == root
    val = sum(range(sz)) if isroot else None
    check(MPI.Reduce(rank, MPI.SUM, root, comm) == val, "reduce SUM scalar")
    check(MPI.Reduce(rank, operator.add, root, comm) == val, "reduce + scalar")
    val = sz - 1 if isroot else None
    check(MPI.Reduce(rank, MPI.MAX, root, comm) == val, "reduce MAX")
    check(MPI.Reduce(rank, max, root, comm) == val, "reduce max")
    val = 0 if isroot else None
    check(MPI.Reduce(rank, MPI.MIN, root, comm) == val, "reduce MIN")
    check(MPI.Reduce(rank, min, root, comm) == val, "reduce min")
    val = sz if isroot else None
    check(MPI.Reduce(1, operator.add, root, comm) == val, "reduce 1")
    mesg = arr(np.arange(1.0, 6.0))
    sum_mesg = MPI.Reduce(mesg, operator.add, root, comm)
    if isroot:
        check(is_array_type(sum_mesg, np.float64), "reduce float64 type")
        check(eq(sum_mesg, sz * host(mesg)), "reduce mesg")
    operators = [MPI.SUM, operator.add, lambda x, y: 2 * x + y - x]
    T = np.int64
    for dims in (1, 2, 3):
        base = np.zeros((3,) * dims, dtype=T)
        base.reshape(-1)[:] = np.arange(1, base.size + 1)
        send_arr = arr(base)
        for op in operators:
            recv_arr = undef(base.shape, T)
            MPI.Reduce_(send_arr, recv_arr, op, root, comm)
            if isroot:
                check(eq(recv_arr, sz * base), ("reduce", dims))
            recv_short = undef(tuple(d - 1 for d in base.shape), T)
            if isroot:
                raises(AssertionError, lambda: MPI.Reduce_(send_arr, recv_short, base.size, op, root, comm),
                       "reduce short recv")
            recv_arr = copy(send_arr)
            MPI.Reduce_(recv_arr, op, root, comm)
            if isroot:
                check(eq(recv_arr, sz * base), ("reduce IN_PLACE", dims))
            val = MPI.Reduce(2, op, root, comm)
            if isroot:
                check(val == sz * 2, "reduce alloc scalar")
            recv_arr = MPI.Reduce(send_arr, op, root, comm)
            if isroot:
                check(is_array_type(recv_arr, T), "reduce alloc type")
                check(eq(recv_arr, sz * base), ("reduce alloc", dims))
            else:
                check(recv_arr is None, "reduce non-root nothing")
            # view(send_arr, 2:3): a contiguous sub-array
            sub = send_arr.reshape(-1)[1:3]
            recv_arr = MPI.Reduce(sub, op, root, comm)
            if isroot:
                check(eq(recv_arr, sz * base.reshape(-1)[1:3]), "reduce subarray")
    MPI.Barrier(comm)


def _prodrank(k, T):
    return np.array(np.prod(np.arange(1, k + 1, dtype=np.float64)), dtype=T)


def t_scan(comm):
    """test/test_scan.jl:11-31 (`*` -> MPI.PROD; all MPIDatatypes but Char/Int8/UInt8)"""
    rank = MPI.Comm_rank(comm)
    for T in [t for t in TYPES if t not in (np.int8, np.uint8)]:
        pr = _prodrank(rank + 1, T)
        A = arr(np.full(4, rank + 1), T)
        B = undef(4, T)
        MPI.Scan_(A, B, operator.mul, comm)
        check(eq(B, np.full(4, pr, dtype=T)), ("scan", T.__name__))
        B = MPI.Scan(A, operator.mul, comm)
        check(is_array_type(B, T), "scan alloc type")
        check(eq(B, np.full(4, pr, dtype=T)), ("scan alloc", T.__name__))
        b = MPI.Scan(T(rank + 1), operator.mul, comm)
        check(b == pr, ("scan scalar", T.__name__))


def t_exscan(comm):
    """test/test_exscan.jl:11-37"""
    rank = MPI.Comm_rank(comm)
    for T in [t for t in TYPES if t not in (np.int8, np.uint8)]:
        pr = _prodrank(rank, T)
        A = arr(np.full(4, rank + 1), T)
        B = undef(4, T)
        MPI.Exscan_(A, B, operator.mul, comm)
        if rank > 0:
            check(eq(B, np.full(4, pr, dtype=T)), ("exscan", T.__name__))
        B = MPI.Exscan(A, operator.mul, comm)
        check(is_array_type(B, T), "exscan alloc type")
        if rank > 0:
            check(eq(B, np.full(4, pr, dtype=T)), ("exscan alloc", T.__name__))
        b = MPI.Exscan(T(rank + 1), operator.mul, comm)
        if rank > 0:
            check(b == pr, ("exscan scalar", T.__name__))


def t_bcast(comm):
    """test/test_bcast.jl:13-36 (array part; the serialized `bcast` of Julia
    objects is host-only and not on the device path)."""
    root = 0
    rng = np.random.default_rng(17)  # Random.seed!(17)
    for T in TYPES + [np.uint32]:  # + Char (a UInt32 bit pattern, datatypes.jl:281-284)
        if np.issubdtype(T, np.complexfloating):
            a = (rng.random((17, 17)) + 1j * rng.random((17, 17))).astype(T)
        elif np.issubdtype(T, np.floating):
            a = rng.random((17, 17)).astype(T)
        else:
            info = np.iinfo(T)
            a = rng.integers(info.min, info.max, size=(17, 17), dtype=T, endpoint=True)
        A = arr(a)
        B = A if MPI.Comm_rank(comm) == root else undef(a.shape, T)
        MPI.Bcast_(B, root, comm)
        check(eq(B, a), ("bcast", T.__name__))


def t_allgather(comm):
    """test/test_allgather.jl:12-54"""
    size, rank = MPI.Comm_size(comm), MPI.Comm_rank(comm)
    for T in TYPES:
        A = arr([rank + 1], T)
        Cc = MPI.Allgather(A, comm)
        check(is_array_type(Cc, T), "allgather type")
        check(eq(Cc, np.arange(1, size + 1, dtype=T)), ("allgather", T.__name__))
        Cs = MPI.Allgather(T(rank + 1), comm)
        check(isinstance(Cs, list) and Cs == list(np.arange(1, size + 1, dtype=T)), ("allgather scalar", T.__name__))
        Cb = undef(size, T)
        MPI.Allgather_(A, Cb, _len(A), comm)
        check(eq(Cb, np.arange(1, size + 1, dtype=T)), "allgather!")
        Cshort = undef(size - 1, T)
        raises(AssertionError, lambda: MPI.Allgather_(A, Cshort, _len(A), comm), "allgather short")
        Ci = arr([i if i == rank else size + 1 for i in range(size)], T)
        MPI.Allgather_(MPI.IN_PLACE, Ci, 1, comm)
        check(eq(Ci, np.arange(size, dtype=T)), ("allgather IN_PLACE", T.__name__))
        Ci = arr([i if i == rank else size + 1 for i in range(size)], T)
        MPI.Allgather_(Ci, 1, comm)
        check(eq(Ci, np.arange(size, dtype=T)), ("allgather implicit IN_PLACE", T.__name__))


def t_alltoall(comm):
    """test/test_alltoall.jl:11-35"""
    size, rank = MPI.Comm_size(comm), MPI.Comm_rank(comm)
    for T in TYPES:
        a = arr(np.full(size, rank), T)
        b = MPI.Alltoall(a, 1, comm)
        check(is_array_type(b, T), "alltoall type")
        check(eq(b, np.arange(size, dtype=T)), ("alltoall", T.__name__))
        a = arr(np.full(size, rank), T)
        b = undef(size, T)
        MPI.Alltoall_(a, b, 1, comm)
        check(eq(b, np.arange(size, dtype=T)), "alltoall!")
        a = arr(np.full(size, rank), T)
        MPI.Alltoall_(MPI.IN_PLACE, a, 1, comm)
        check(eq(a, np.arange(size, dtype=T)), ("alltoall IN_PLACE", T.__name__))


def t_gather(comm):
    """test/test_gather.jl:12-70"""
    root, rank, sz = 0, MPI.Comm_rank(comm), MPI.Comm_size(comm)
    isroot = rank == root
    for T in TYPES:
        A = arr(np.full(4, rank + 1), T)
        C = MPI.Gather(A, root, comm)
        if isroot:
            check(is_array_type(C, T), "gather type")
            check(eq(C, np.repeat(np.arange(1, sz + 1), 4).astype(T)), ("gather", T.__name__))
        Cs = MPI.Gather(T(rank + 1), root, comm)
        if isroot:
            check(isinstance(Cs, list) and Cs == list(np.arange(1, sz + 1, dtype=T)), ("gather obj", T.__name__))
        A = arr([rank + 1, 0], T)
        C = MPI.Gather(A, 1, root, comm)
        if isroot:
            check(eq(C, np.arange(1, sz + 1, dtype=T)), "gather explicit length")
        C = MPI.Gather(A[0:1], root, comm)  # view(A, 1:1)
        if isroot:
            check(eq(C, np.arange(1, sz + 1, dtype=T)), "gather view")
        A = arr(np.full(4, rank + 1), T)
        C = undef(4 * sz, T)
        MPI.Gather_(A, C, _len(A), root, comm)
        if isroot:
            check(eq(C, np.repeat(np.arange(1, sz + 1), 4).astype(T)), "gather!")
        A = arr(np.full(4 * sz if isroot else 4, rank + 1), T)
        if isroot:
            MPI.Gather_(None, A, 4, root, comm)
            check(eq(A, np.repeat(np.arange(1, sz + 1), 4).astype(T)), ("gather IN_PLACE", T.__name__))
        else:
            MPI.Gather_(A, None, 4, root, comm)


def t_gatherv(comm):
    """test/test_gatherv.jl:12-58"""
    root, size, rank = 0, MPI.Comm_size(comm), MPI.Comm_rank(comm)
    isroot = rank == root
    counts = [i % 2 + 1 for i in range(size)]
    chk = np.concatenate([np.full(counts[r], r) for r in range(size)])
    for T in TYPES:
        A = arr(np.full(rank % 2 + 1, rank), T)
        B = MPI.Gatherv(A, counts, root, comm)
        if isroot:
            check(is_array_type(B, T) and eq(B, chk.astype(T)), ("gatherv", T.__name__))
        B = undef(sum(counts), T)
        MPI.Gatherv_(A, B, counts, root, comm)
        if isroot:
            check(eq(B, chk.astype(T)), "gatherv!")
        B = undef(sum(counts) - 1, T)
        if isroot:
            raises(AssertionError, lambda: MPI.Gatherv_(A, B, counts, root, comm), "gatherv short")
        B = arr(np.full(sum(counts), rank), T)
        if isroot:
            MPI.Gatherv_(None, B, counts, root, comm)
            check(eq(B, chk.astype(T)), ("gatherv IN_PLACE", T.__name__))
        else:
            MPI.Gatherv_(B, None, counts, root, comm)


def t_scatter(comm):
    """test/test_scatter.jl:12-44"""
    size, rank, root = MPI.Comm_size(comm), MPI.Comm_rank(comm), 0
    isroot = rank == root
    for T in TYPES:
        A = arr(np.arange(1, size + 1), T) if isroot else undef(1, T)
        B = MPI.Scatter(A, 1, root, comm)
        check(is_array_type(B, T) and host(B)[0] == T(rank + 1), ("scatter", T.__name__))
        B = undef(1, T)
        MPI.Scatter_(A, B, 1, root, comm)
        check(host(B)[0] == T(rank + 1), "scatter!")
        B = copy(A) if isroot else undef(1, T)
        if isroot:
            MPI.Scatter_(B, None, 1, root, comm)
        else:
            MPI.Scatter_(None, B, 1, root, comm)
        check(host(B)[0] == T(rank + 1), ("scatter IN_PLACE", T.__name__))
        B = undef(0, T)
        raises(AssertionError, lambda: MPI.Scatter_(A, B, 1, root, comm), "scatter short")


def t_scatterv(comm):
    """test/test_scatterv.jl:12-50"""
    size, rank, root = MPI.Comm_size(comm), MPI.Comm_rank(comm), 0
    isroot = rank == root
    counts = [i % 2 + 1 for i in range(size)]
    ref = np.concatenate([np.full(counts[r], r) for r in range(size)])
    for T in TYPES:
        A = arr(ref, T) if isroot else undef(1, T)
        B = MPI.Scatterv(A, counts, root, comm)
        check(is_array_type(B, T) and eq(B, np.full(counts[rank], rank, dtype=T)), ("scatterv", T.__name__))
        B = undef(counts[rank], T)
        MPI.Scatterv_(A, B, counts, root, comm)
        check(eq(B, np.full(counts[rank], rank, dtype=T)), "scatterv!")
        B = copy(A) if isroot else undef(counts[rank], T)
        if isroot:
            MPI.Scatterv_(B, None, counts, root, comm)
            check(eq(B, host(A)), "scatterv IN_PLACE root")
        else:
            MPI.Scatterv_(None, B, counts, root, comm)
            check(eq(B, np.full(counts[rank], rank, dtype=T)), ("scatterv IN_PLACE", T.__name__))


def t_allgatherv(comm):
    """test/test_allgatherv.jl:12-44"""
    size, rank = MPI.Comm_size(comm), MPI.Comm_rank(comm)
    counts = [i % 2 + 1 for i in range(size)]
    chk = np.concatenate([np.full(counts[r], r) for r in range(size)])
    for T in TYPES:
        A = arr(np.full(counts[rank], rank), T)
        B = MPI.Allgatherv(A, counts, comm)
        check(is_array_type(B, T) and eq(B, chk.astype(T)), ("allgatherv", T.__name__))
        B = undef(sum(counts), T)
        MPI.Allgatherv_(A, B, counts, comm)
        check(eq(B, chk.astype(T)), "allgatherv!")
        B = undef(sum(counts) - 1, T)
        raises(AssertionError, lambda: MPI.Allgatherv_(A, B, counts, comm), "allgatherv short")
        B = arr(np.full(sum(counts), rank), T)
        MPI.Allgatherv_(MPI.IN_PLACE, B, counts, comm)
        check(eq(B, chk.astype(T)), ("allgatherv IN_PLACE", T.__name__))


def t_alltoallv(comm):
    """test/test_alltoallv.jl:12-38"""
    size, rank = MPI.Comm_size(comm), MPI.Comm_rank(comm)
    send_counts = list(range(1, size + 1))
    recv_counts = [rank + 1] * size
    send_vals = np.concatenate([np.arange(1, i + 1) for i in range(1, size + 1)])
    recv_vals = np.concatenate([np.arange(1, rank + 2) for _ in range(size)])
    for T in TYPES:
        A = arr(send_vals, T)
        B = MPI.Alltoallv(A, send_counts, recv_counts, comm)
        check(is_array_type(B, T) and eq(B, recv_vals.astype(T)), ("alltoallv", T.__name__))
        C = undef(sum(recv_counts), T)
        MPI.Alltoallv_(A, C, send_counts, recv_counts, comm)
        check(eq(C, recv_vals.astype(T)), "alltoallv!")
        C = undef(sum(recv_counts) - 1, T)
        raises(AssertionError, lambda: MPI.Alltoallv_(A, C, send_counts, recv_counts, comm), "alltoallv short")


def main():
    comm = MPI.Init()
    for t in (t_allreduce, t_reduce, t_scan, t_exscan, t_bcast, t_allgather, t_alltoall, t_gather, t_gatherv,
              t_scatter, t_scatterv, t_allgatherv, t_alltoallv):
        try:
            t(comm)
        except Exception:  # noqa: BLE001
            FAIL.append(f"{t.__name__}: {traceback.format_exc()[-800:]}")
            break  # collective sequence is broken; stop here
    MPI.Finalize()
    check(MPI.Finalized(), "Finalized")
    print(json.dumps({"rank": MPI.Comm_rank(comm), "device": DEVICE, "checks": NCHECK[0],
                      "failures": [str(f) for f in FAIL[:10]], "nfail": len(FAIL)}), flush=True)
    sys.exit(1 if FAIL else 0)


if __name__ == "__main__":
    main()
