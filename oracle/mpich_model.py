"""CPU oracle: a numpy restatement of the arithmetic behind MPI.jl's collectives.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker.  The mpigx
product path never routes through it (there is no CPU fallback).

What it restates
----------------
MPI.jl v0.14.2 performs no arithmetic itself: every collective on the hot path
is one ccall into libmpi (src/collective.jl:34 Bcast, :304 Allgather,
:498 Alltoall, :615 Reduce, :698 Allreduce, :765 Scan, :839 Exscan).  The
default libmpi is MPICH 3.3.2 (Project.toml:10 MPICH_jll, deps/build.jl:139-152,
conf/travis-install-mpi.sh:11 MPICHVER=3.3.2).  MPICH is a third-party
dependency that is NOT vendored under /root/reference, so this module restates
its published algorithms (MPICH 3.3.2 src/mpi/coll/...):

* built-in op loops (src/mpi/coll/op/op*.c): ``inout[i] = OP(inout[i], in[i])``
  with ``MPL_MAX(a,b) = a > b ? a : b``, ``MPL_MIN(a,b) = a < b ? a : b``,
  ``LAND/LOR/LXOR`` producing 0/1 in the element type, two's-complement wrap
  for integers, complex PROD as ``(ar*br - ai*bi, ar*bi + ai*br)`` without FMA;
* MPIR_Allreduce_intra_smp: with MPIR_CVAR_ENABLE_SMP_COLLECTIVES=1 (the
  MPICH 3.3.2 default, `mpivars`) and every rank on one node, Allreduce is an
  intra-node MPIR_Reduce to rank 0 followed by MPIR_Bcast, so every rank
  receives rank 0's reduction (pinned: all ranks' outputs in the fixtures,
  NaN/±0 cases included);
* MPIR_Reduce_intra_auto: binomial tree over relative ranks
  (``relrank = (rank - root) mod n``, the lower subtree is ``inout``) when
  ``count*size <= 2048`` or ``count < pof2``, else Rabenseifner
  reduce-scatter (recursive halving) + gather, with the non-power-of-two
  pre-step in which odd rank ``2i+1`` folds rank ``2i`` into itself
  (``inout`` = odd);
* MPIR_Scan / MPIR_Exscan recursive doubling (partial_scan / recvbuf model);
* Bcast / Allgather / Alltoall are byte copies.

The restatement simulates the message-passing schedule on in-memory per-rank
buffers, so operand roles (which operand is ``inout``) — which decide NaN and
signed-zero outcomes of MIN/MAX — are reproduced, not only the association.

Pinning: tests/test_oracle_golden.py checks every function here bit-for-bit
against tests/golden/mpich_golden.npz, which gen_mpich_golden.c recorded from
MPICH 3.3.2 itself with the reference's ccall argument shapes.
"""
from __future__ import annotations

import numpy as np

# ---------------------------------------------------------------------------
# MPICH handle values (deps/consts_mpich.jl:30-72)
# ---------------------------------------------------------------------------
OPS = {
    "MAX": 1476395009, "MIN": 1476395010, "SUM": 1476395011, "PROD": 1476395012,
    "LAND": 1476395013, "BAND": 1476395014, "LOR": 1476395015, "BOR": 1476395016,
    "LXOR": 1476395017, "BXOR": 1476395018,
}
OP_NAMES = {v: k for k, v in OPS.items()}

# name -> (handle, numpy dtype, kind); kind in {"int", "uint", "float", "complex", "byte", "bf16", "none"}
DTYPES = {
    "INT8_T": (1275068727, np.int8, "int"),
    "UINT8_T": (1275068731, np.uint8, "uint"),
    "INT16_T": (1275068984, np.int16, "int"),
    "UINT16_T": (1275068988, np.uint16, "uint"),
    "INT32_T": (1275069497, np.int32, "int"),
    "UINT32_T": (1275069501, np.uint32, "uint"),
    "INT64_T": (1275070522, np.int64, "int"),
    "UINT64_T": (1275070526, np.uint64, "uint"),
    "BYTE": (1275068685, np.uint8, "byte"),
    "SHORT": (1275068931, np.int16, "int"),
    "UNSIGNED_SHORT": (1275068932, np.uint16, "uint"),
    "INT": (1275069445, np.int32, "int"),
    "UNSIGNED": (1275069446, np.uint32, "uint"),
    "LONG": (1275070471, np.int64, "int"),
    "UNSIGNED_LONG": (1275070472, np.uint64, "uint"),
    "CHAR": (1275068673, np.int8, "int"),
    "SIGNED_CHAR": (1275068696, np.int8, "int"),
    "UNSIGNED_CHAR": (1275068674, np.uint8, "uint"),
    "WCHAR": (1275069454, np.int32, "none"),
    "FLOAT": (1275069450, np.float32, "float"),
    "DOUBLE": (1275070475, np.float64, "float"),
    "C_FLOAT_COMPLEX": (1275070528, np.complex64, "complex"),
    "C_DOUBLE_COMPLEX": (1275072577, np.complex128, "complex"),
    # mpigx extension (no MPICH counterpart; parity unpinned): bf16 stored as
    # uint16 bit patterns, computed in fp32, RNE-rounded after every op.
    "BFLOAT16": (1275068912, np.uint16, "bf16"),
}
DTYPE_BY_HANDLE = {v[0]: k for k, v in DTYPES.items()}

MPI_SUCCESS, MPI_ERR_TYPE, MPI_ERR_OP = 0, 3, 9

ARITH = ("SUM", "PROD")
ORDERED = ("MIN", "MAX")
LOGICAL = ("LAND", "LOR", "LXOR")
BITWISE = ("BAND", "BOR", "BXOR")


def op_valid(dtname: str, opname: str) -> int:
    """Error class MPICH returns for (datatype, op) (op_type_matrix.json pins it).

    SUM/PROD: integers, floats, complex, (CHAR); MIN/MAX/LAND/LOR/LXOR:
    integers and floats; BAND/BOR/BXOR: integers and BYTE.  WCHAR: nothing.
    """
    if dtname not in DTYPES:
        return MPI_ERR_TYPE
    if opname not in OPS:
        return MPI_ERR_OP
    kind = DTYPES[dtname][2]
    ok = {
        "int": True, "uint": True,
        "float": opname not in BITWISE,
        "bf16": opname not in BITWISE,
        "complex": opname in ARITH,
        "byte": opname in BITWISE,
        "none": False,
    }[kind]
    return MPI_SUCCESS if ok else MPI_ERR_OP


# ---------------------------------------------------------------------------
# bf16 helpers (mpigx definition)
# ---------------------------------------------------------------------------
def bf16_to_f32(u16: np.ndarray) -> np.ndarray:
    return (u16.astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16(f: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even fp32 -> bf16; NaN stays NaN (quiet)."""
    u = np.ascontiguousarray(f, dtype=np.float32).view(np.uint32)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    q = ((u >> 16) | 0x0040).astype(np.uint16)
    return np.where(nan, q, r)


# ---------------------------------------------------------------------------
# elementwise op: MPIR op loops, a = inout, b = in  ->  new inout
# ---------------------------------------------------------------------------
def apply_op(opname: str, dtname: str, inout: np.ndarray, inv: np.ndarray) -> np.ndarray:
    """``inout[i] = OP(inout[i], in[i])`` exactly as MPICH's MPIR_*_check loops."""
    kind = DTYPES[dtname][2]
    if kind == "bf16":
        a = bf16_to_f32(inout)
        b = bf16_to_f32(inv)
        return f32_to_bf16(apply_op(opname, "FLOAT", a, b))
    a, b = inout, inv
    with np.errstate(all="ignore"):
        if opname == "SUM":
            if kind == "complex":
                return _cplx(a.real + b.real, a.imag + b.imag, a.dtype)
            return (a + b).astype(a.dtype)
        if opname == "PROD":
            if kind == "complex":
                # no FMA contraction: each product and sum rounds separately
                re = a.real * b.real
                re = re - a.imag * b.imag
                im = a.real * b.imag
                im = im + a.imag * b.real
                return _cplx(re, im, a.dtype)
            return (a * b).astype(a.dtype)
        if opname == "MAX":
            return np.where(a > b, a, b)
        if opname == "MIN":
            return np.where(a < b, a, b)
        if opname == "LAND":
            return ((a != 0) & (b != 0)).astype(a.dtype)
        if opname == "LOR":
            return ((a != 0) | (b != 0)).astype(a.dtype)
        if opname == "LXOR":
            return ((a != 0) != (b != 0)).astype(a.dtype)
        if opname == "BAND":
            return a & b
        if opname == "BOR":
            return a | b
        if opname == "BXOR":
            return a ^ b
    raise ValueError(opname)


def _cplx(re, im, dt):
    out = np.empty(re.shape, dtype=dt)
    out.real = re
    out.imag = im
    return out


def reduce_local(inv, inout, dtname, opname):
    """MPI_Reduce_local(inbuf, inoutbuf, ...) (mpi.h:1357) -> new inoutbuf."""
    return apply_op(opname, dtname, inout, inv)


def _esize(dtname):
    return np.dtype(DTYPES[dtname][1]).itemsize


def _pof2(n):
    p = 1
    while p * 2 <= n:
        p *= 2
    return p


# ---------------------------------------------------------------------------
# Allreduce: MPIR_Allreduce_intra_smp = Reduce(root 0) + Bcast on one node.
# (_allreduce_rd is MPIR_Allreduce_intra_recursive_doubling, kept for the
#  multi-node / SMP-disabled configuration; it is not what one node runs.)
# ---------------------------------------------------------------------------
def allreduce(inputs, dtname, opname, short_msg=2048):
    """Per-rank outputs of MPI_Allreduce (collective.jl:698-700)."""
    n = len(inputs)
    res = reduce(inputs, dtname, opname, 0, short_msg)
    return [res.copy() for _ in range(n)]


def _prestep(bufs, dtname, opname, n, pof2, keep_even=False):
    """Non-power-of-two pre-step between ranks 2i and 2i+1 (i < rem).
    Allreduce (MPIR_Allreduce_intra_recursive_doubling /
    _reduce_scatter_allgather): the even rank sends, the odd rank folds,
    inout = odd, newrank i = rank 2i+1.  Reduce (MPIR_Reduce_intra_
    reduce_scatter_gather, keep_even=True): the odd rank sends, the EVEN rank
    folds, inout = even, newrank i = rank 2i.  The roles show only where
    operands are ordered: MIN/MAX with NaN or +-0 (pinned by the large-count
    MPICH fixtures, tests/golden/mpich_large.npz, n = 5)."""
    rem = n - pof2
    for i in range(rem):
        if keep_even:
            bufs[2 * i] = apply_op(opname, dtname, bufs[2 * i], bufs[2 * i + 1])
        else:
            bufs[2 * i + 1] = apply_op(opname, dtname, bufs[2 * i + 1], bufs[2 * i])
    newrank = {}
    for r in range(n):
        if r < 2 * rem:
            if (r % 2 == 0) == keep_even:
                newrank[r] = r // 2
        else:
            newrank[r] = r - rem
    real = {v: k for k, v in newrank.items()}  # newrank -> rank
    return rem, newrank, real


def _poststep(bufs, n, rem):
    for i in range(rem):
        bufs[2 * i] = bufs[2 * i + 1].copy()


def _allreduce_rd(inputs, dtname, opname):
    n = len(inputs)
    pof2 = _pof2(n)
    bufs = [x.copy() for x in inputs]
    rem, newrank, real = _prestep(bufs, dtname, opname, n, pof2)
    mask = 1
    while mask < pof2:
        snap = {nr: bufs[real[nr]].copy() for nr in range(pof2)}
        for nr in range(pof2):
            dst = nr ^ mask
            r = real[nr]
            # commutative builtin: reduce_local(tmp=partner, recvbuf=own)
            bufs[r] = apply_op(opname, dtname, snap[nr], snap[dst])
        mask <<= 1
    _poststep(bufs, n, rem)
    return bufs


def _allreduce_rsag(inputs, dtname, opname, out_ranks=None):
    """Reduce-scatter + gather over newranks — the schedule of
    MPIR_Reduce_intra_reduce_scatter_gather, which one node's Allreduce runs
    (Reduce to rank 0 + Bcast, MPIR_Allreduce_intra_smp): pre-step with the
    even rank as inout (_prestep keep_even)."""
    n = len(inputs)
    count = inputs[0].shape[0]
    pof2 = _pof2(n)
    bufs = [x.copy() for x in inputs]
    rem, newrank, real = _prestep(bufs, dtname, opname, n, pof2, keep_even=True)
    cnts = [count // pof2] * (pof2 - 1) + [count - (count // pof2) * (pof2 - 1)]
    disps = [0]
    for i in range(1, pof2):
        disps.append(disps[-1] + cnts[i - 1])
    # state per newrank
    st = {nr: dict(send_idx=0, recv_idx=0, last_idx=pof2) for nr in range(pof2)}
    mask = 1
    while mask < pof2:
        snap = {nr: bufs[real[nr]].copy() for nr in range(pof2)}
        plan = {}
        for nr in range(pof2):
            s = st[nr]
            dst = nr ^ mask
            if nr < dst:
                s["send_idx"] = s["recv_idx"] + pof2 // (mask * 2)
                lo, hi = s["recv_idx"], s["send_idx"]
            else:
                s["recv_idx"] = s["send_idx"] + pof2 // (mask * 2)
                lo, hi = s["recv_idx"], s["last_idx"]
            plan[nr] = (dst, disps[lo], (disps[hi] if hi < pof2 else count))
        for nr in range(pof2):
            dst, a, b = plan[nr]
            r = real[nr]
            seg = apply_op(opname, dtname, snap[nr][a:b], snap[dst][a:b])
            bufs[r][a:b] = seg
        for nr in range(pof2):
            s = st[nr]
            s["send_idx"] = s["recv_idx"]
        mask <<= 1
        if mask < pof2:
            for nr in range(pof2):
                s = st[nr]
                s["last_idx"] = s["recv_idx"] + pof2 // mask
    # each newrank now owns [disps[recv_idx] .. +block); allgather = copies
    owned = {}
    for nr in range(pof2):
        s = st[nr]
        lo = s["recv_idx"]
        a = disps[lo]
        b = disps[lo + 1] if lo + 1 < pof2 else count
        owned[nr] = (a, b, bufs[real[nr]][a:b].copy())
    result = np.empty_like(bufs[0])
    for nr, (a, b, v) in owned.items():
        result[a:b] = v
    return [result.copy() for _ in range(n)]


# ---------------------------------------------------------------------------
# Reduce: MPIR_Reduce_intra_auto (binomial | reduce-scatter + gather)
# ---------------------------------------------------------------------------
def reduce(inputs, dtname, opname, root, short_msg=2048):
    """Result at `root` of MPI_Reduce (collective.jl:615-617)."""
    n = len(inputs)
    count = inputs[0].shape[0]
    pof2 = _pof2(n)
    if count * _esize(dtname) > short_msg and count >= pof2:
        return _allreduce_rsag(inputs, dtname, opname)[root]
    # binomial over relative ranks, lroot = root (commutative builtin)
    bufs = {rel: inputs[(rel + root) % n].copy() for rel in range(n)}
    mask = 1
    while mask < n:
        for rel in range(n):
            if rel & (mask - 1):
                continue  # already sent
            if (rel & mask) == 0:
                src = rel | mask
                if src < n:
                    bufs[rel] = apply_op(opname, dtname, bufs[rel], bufs[src])
        mask <<= 1
    return bufs[0]


# ---------------------------------------------------------------------------
# Scan / Exscan: recursive doubling (MPIR_Scan_intra_recursive_doubling,
# MPIR_Exscan_intra_recursive_doubling)
# ---------------------------------------------------------------------------
def scan(inputs, dtname, opname):
    n = len(inputs)
    partial = [x.copy() for x in inputs]
    recv = [x.copy() for x in inputs]
    mask = 1
    while mask < n:
        snap = [p.copy() for p in partial]
        for r in range(n):
            dst = r ^ mask
            if dst < n:
                t = snap[dst]
                if r > dst:
                    partial[r] = apply_op(opname, dtname, snap[r], t)
                    recv[r] = apply_op(opname, dtname, recv[r], t)
                else:
                    partial[r] = apply_op(opname, dtname, snap[r], t)
        mask <<= 1
    return recv


def exscan(inputs, dtname, opname, untouched=None):
    """Per-rank outputs; rank 0's output is `untouched` (its prior recvbuf)."""
    n = len(inputs)
    partial = [x.copy() for x in inputs]
    recv = [None] * n
    mask = 1
    while mask < n:
        snap = [p.copy() for p in partial]
        for r in range(n):
            dst = r ^ mask
            if dst < n:
                t = snap[dst]
                partial[r] = apply_op(opname, dtname, snap[r], t)
                if r > dst and r != 0:
                    recv[r] = t.copy() if recv[r] is None else apply_op(opname, dtname, recv[r], t)
        mask <<= 1
    recv[0] = untouched
    return recv


# ---------------------------------------------------------------------------
# byte-copy collectives
# ---------------------------------------------------------------------------
def bcast(buffers, root):
    return [buffers[root].copy() for _ in buffers]


def allgather(inputs):
    full = np.concatenate(inputs)
    return [full.copy() for _ in inputs]


def alltoall(inputs, count):
    n = len(inputs)
    return [np.concatenate([inputs[j][r * count:(r + 1) * count] for j in range(n)]) for r in range(n)]


# ---------------------------------------------------------------------------
# mpigx-defined folds (no MPICH counterpart), used by the engine's
# deterministic modes and by the local multi-buffer reduce (config 2)
# ---------------------------------------------------------------------------
def fold_linear(inputs, dtname, opname):
    """Rank-ordered fold ((x0 op x1) op x2) ... with the running value as inout."""
    v = inputs[0].copy()
    for x in inputs[1:]:
        v = apply_op(opname, dtname, v, x)
    return v


def ring_strides(n, want):
    """Ring strides of mpigx's ring Allreduce (csrc/mpigx.cpp ring_strides):
    candidates 1, n-1, 2, n-2, ... coprime with n, distinct, at most `want`."""
    from math import gcd
    st = []
    for d in range(1, n):
        for cand in (d, n - d):
            if len(st) < want and gcd(cand, n) == 1 and cand not in st:
                st.append(cand)
    return st


def fold_ring(inputs, dtname, opname, nch=1, round_elems=None):
    """mpigx ring reduce-scatter + allgather (MPIGX_ALGO=ring; csrc/kernels.hpp
    ring_body) — an mpigx schedule with no MPICH counterpart.  Per round of
    ``round_elems`` elements the message is cut into ``nch`` parts of
    ceil(cnt/nch) elements rounded up to n*vec (vec = 16 B of elements); part k
    rides the ring of stride s_k, whose position i is rank (i*s_k) mod n, and
    is cut into n chunks; chunk c is folded left to right along the ring
    starting at position c, the running partial as inout:
    ((x_q(c) op x_q(c+1)) op x_q(c+2)) ... op x_q(c+n-1)."""
    n = len(inputs)
    count = inputs[0].shape[0]
    es = _esize(dtname)
    vec = max(1, 16 // es)
    strides = ring_strides(n, nch)
    nch = len(strides)
    out = np.empty_like(inputs[0])
    rnd = round_elems or max(count, 1)
    for off in range(0, count, rnd):
        cnt = min(rnd, count - off)
        part = -(-(-(-cnt // nch)) // (n * vec)) * (n * vec)
        chunk = part // n
        for k, st in enumerate(strides):
            p0 = min(k * part, cnt)
            p1 = min(p0 + part, cnt)
            for c in range(n):
                lo = min(p0 + c * chunk, p1)
                hi = min(lo + chunk, p1)
                if lo == hi:
                    continue
                acc = inputs[(c * st) % n][off + lo:off + hi].copy()
                for i in range(1, n):
                    acc = apply_op(opname, dtname, acc, inputs[((c + i) * st) % n][off + lo:off + hi])
                out[off + lo:off + hi] = acc
    return out


def ring_round_elems(stage_bytes, n, dtname, nch=1):
    """Elements per round of the ring (mpigx.cpp allreduce_ring): the staging
    arena (rounded up to 4 KiB) in elements, a multiple of nch*n*vec."""
    es = _esize(dtname)
    vec = max(1, 16 // es)
    nch = len(ring_strides(n, nch))
    sb = (stage_bytes + 4095) // 4096 * 4096
    q = nch * n * vec
    return (sb // es) // q * q


def sum_tolerance(inputs, dtname):
    """|a - b| bound between two summation orders of the same n values
    (2 (n-1) u sum|x|, u = unit roundoff): the stated tolerance of the ring's
    float SUM against MPICH's pairwise tree."""
    n = len(inputs)
    u = {"FLOAT": 2.0 ** -24, "DOUBLE": 2.0 ** -53, "BFLOAT16": 2.0 ** -8}[dtname]
    if dtname == "BFLOAT16":
        mag = sum(np.abs(bf16_to_f32(x).astype(np.float64)) for x in inputs)
    else:
        mag = sum(np.abs(x.astype(np.float64)) for x in inputs)
    return 2 * (n - 1) * u * mag


def fold_tree(inputs, dtname, opname):
    """MPICH single-node Allreduce result (binomial tree to rank 0, <= 2 KiB regime)."""
    return reduce(list(inputs), dtname, opname, 0, short_msg=1 << 62)


def fold_rsag(inputs, dtname, opname):
    """MPICH single-node Allreduce result in the Rabenseifner regime."""
    return _allreduce_rsag(list(inputs), dtname, opname)[0]


# ---------------------------------------------------------------------------
# v-collectives / rooted variants (byte movement; MPI.jl passes packed
# displacements: disps = cumsum(counts) - counts, collective.jl:169/365/425/551)
# ---------------------------------------------------------------------------
def vcnt(seed, a, b, base):
    """Count pattern of the golden v-cases (gen_mpich_golden.c vcnt)."""
    return ((a * 7 + b * 3 + seed) % 5) * base


def _disps(counts):
    d, acc = [], 0
    for c in counts:
        d.append(acc)
        acc += c
    return d


def gather(inputs, count, root):
    """Result at root of MPI_Gather (collective.jl:230-246)."""
    return np.concatenate([x[:count] for x in inputs])


def gatherv(inputs, counts):
    """Result at root of MPI_Gatherv (collective.jl:363-382)."""
    return np.concatenate([x[:c] for x, c in zip(inputs, counts)])


def scatter(root_buf, count, n):
    """Per-rank outputs of MPI_Scatter (collective.jl:90-106)."""
    return [root_buf[r * count:(r + 1) * count].copy() for r in range(n)]


def scatterv(root_buf, counts):
    """Per-rank outputs of MPI_Scatterv (collective.jl:156-175)."""
    d = _disps(counts)
    return [root_buf[d[r]:d[r] + counts[r]].copy() for r in range(len(counts))]


def allgatherv(inputs, counts):
    full = gatherv(inputs, counts)
    return [full.copy() for _ in inputs]


def alltoallv(inputs, S):
    """S[p][q] = elements rank p sends to rank q (collective.jl:545-559)."""
    n = len(inputs)
    sd = [_disps(S[p]) for p in range(n)]
    return [np.concatenate([inputs[p][sd[p][r]:sd[p][r] + S[p][r]] for p in range(n)]) for r in range(n)]
