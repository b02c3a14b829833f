"""MPI.jl's point-to-point API (src/pointtopoint.jl) over libmpigx / libmpi.

Same split as the collectives (api.py): torch tensors on a ROCm device go to
``mpigx_<fn>`` (p2p.cpp: rendezvous through shm mailboxes, the receiver pulls
over xGMI with one copy kernel per progress pass), numpy arrays go to
``MPI_<Fn>`` of the process's libmpi.  Names follow MPI.jl (``!`` -> ``_``);
``Status`` has MPICH's 20-byte layout (pointtopoint.jl:4-60) and request
handles are MPICH ``int``s, so the ctypes calls are identical either way.

Index conventions are the reference's: ``Waitany_`` / ``Testany_`` return the
1-based index of the completed request (0 when none is active) and
``Waitsome_`` / ``Testsome_`` 1-based index lists, as pointtopoint.jl:546-660
do, so the restated reference tests read like the Julia ones.

Departure from the reference: ``Wait_`` returns the request's Status
(pointtopoint.jl:410 returns the unrelated function ``stat``, a typo).
"""
from __future__ import annotations

import ctypes
import pickle

import numpy as np

from . import consts as C
from . import hostmpi
from ._lib import lib
from .api import Buffer, MPIError, _check, _eltype, _is_host, _len, _ptr, _scalar_ref, _stream, _torch, _unwrap

__all__ = ["Status", "STATUS_EMPTY", "Request", "REQUEST_NULL", "ANY_SOURCE", "ANY_TAG", "PROC_NULL", "UNDEFINED",
           "Get_source", "Get_tag", "Get_error", "Get_count", "Test_cancelled", "isnull", "free_request",
           "Send", "Isend", "Recv_", "Irecv_", "Recv", "Sendrecv_", "send", "recv", "isend", "irecv",
           "Probe", "Iprobe", "Wait_", "Test_", "Waitall_", "Testall_", "Waitany_", "Testany_", "Waitsome_",
           "Testsome_", "Cancel_", "Buffer_send"]

ANY_SOURCE = C.MPI_ANY_SOURCE
ANY_TAG = C.MPI_ANY_TAG
PROC_NULL = C.MPI_PROC_NULL
UNDEFINED = C.MPI_UNDEFINED
_IGNORE = ctypes.c_void_p(1)  # MPI_STATUS(ES)_IGNORE


class Status(ctypes.Structure):
    """MPI.Status: MPICH's MPI_Status (mpi.h:585-591); fields `source`, `tag`,
    `error` as in pointtopoint.jl:4-60."""
    _fields_ = [("count_lo", ctypes.c_int), ("count_hi_and_cancelled", ctypes.c_int), ("source", ctypes.c_int),
                ("tag", ctypes.c_int), ("error", ctypes.c_int)]

    def __eq__(self, o):
        return isinstance(o, Status) and bytes(self) == bytes(o)

    def __hash__(self):
        return hash(bytes(self))

    def __repr__(self):
        return (f"MPI.Status(source={self.source}, tag={self.tag}, error={self.error}, "
                f"bytes={self.count_lo}, cancelled={self.count_hi_and_cancelled & 1})")


def _empty():
    return Status(0, 0, ANY_SOURCE, ANY_TAG, C.MPI_SUCCESS)


STATUS_EMPTY = _empty()


def Get_source(st: Status) -> int:
    return int(st.source)


def Get_tag(st: Status) -> int:
    return int(st.tag)


def Get_error(st: Status) -> int:
    return int(st.error)


def Get_count(st: Status, T) -> int:
    """pointtopoint.jl:150-157: entries received, MPI_UNDEFINED if the byte
    count is not a multiple of sizeof(T)."""
    from .api import Datatype
    dt = T if isinstance(T, Datatype) else Datatype(T)
    out = ctypes.c_int()
    _check(lib().mpigx_get_count(ctypes.byref(st), dt.val, ctypes.byref(out)))
    return out.value


def Test_cancelled(st: Status) -> bool:
    return bool(st.count_hi_and_cancelled & 1)


class Request:
    """MPI.Request (pointtopoint.jl:72-90): handle + the buffer it keeps alive.
    `backend` is 'dev' (libmpigx) or 'host' (libmpi)."""
    __slots__ = ("val", "buffer", "backend")

    def __init__(self, val=C.MPI_REQUEST_NULL, buffer=None, backend=None):
        self.val, self.buffer, self.backend = val, buffer, backend

    def __eq__(self, o):
        return isinstance(o, Request) and o.val == self.val

    def __hash__(self):
        return hash(self.val)

    def __repr__(self):
        return "MPI.REQUEST_NULL" if isnull(self) else f"MPI.Request({self.val:#x}, {self.backend})"


REQUEST_NULL = Request()


def isnull(req: Request) -> bool:
    return req.val == C.MPI_REQUEST_NULL


def _be(backend):
    return lib() if backend == "dev" else hostmpi.lib()


def _fn(backend, name):
    f = getattr(_be(backend), ("mpigx_" + name.lower()) if backend == "dev" else ("MPI_" + name))
    if backend == "dev":
        return f
    from .types import _host_args  # derived datatypes have their own host handles

    return lambda *a: f(*_host_args(a))


def free_request(req: Request):
    """MPI.free(::Request) (pointtopoint.jl:94-101)."""
    if not isnull(req):
        h = ctypes.c_int(req.val)
        _check(_fn(req.backend, "Request_free")(ctypes.byref(h)))
        req.val, req.buffer = C.MPI_REQUEST_NULL, None


# ---------------------------------------------------------------------------
# buffers
# ---------------------------------------------------------------------------
def Buffer_send(data, comm=None):
    """buffers.jl Buffer_send: isbits scalars travel as a 1-element Ref."""
    if isinstance(data, Buffer) or isinstance(data, np.ndarray) or hasattr(data, "data_ptr"):
        return data if isinstance(data, Buffer) else Buffer(data)
    return Buffer(_scalar_ref(data, comm))


def _args(buf):
    b = buf if isinstance(buf, Buffer) else Buffer(buf)
    return b, _ptr(b), int(b.count), b.datatype.val


def _route(buf, comm):
    """('host', MPI_Comm) for numpy buffers, ('dev', mpigx_comm) for tensors."""
    if _is_host(buf):
        if comm.host is None:
            raise TypeError("host buffers need host libmpi (start the ranks with mpiexec)")
        return "host", comm.host
    if not comm.val:
        raise TypeError("device buffers need a ROCm device")
    _stream(comm)
    return "dev", comm.val


# ---------------------------------------------------------------------------
# blocking / nonblocking send and receive
# ---------------------------------------------------------------------------
def Send(buf, dest: int, tag: int, comm):
    """pointtopoint.jl:179-209 (arrays, Buffers and isbits scalars)."""
    b, p, cnt, dt = _args(Buffer_send(buf, comm))
    be, ch = _route(b, comm)
    _check(_fn(be, "Send")(p, cnt, dt, int(dest), int(tag), ch))


def Isend(buf, dest: int, tag: int, comm) -> Request:
    """pointtopoint.jl:221-236."""
    b, p, cnt, dt = _args(Buffer_send(buf, comm))
    be, ch = _route(b, comm)
    h = ctypes.c_int(C.MPI_REQUEST_NULL)
    _check(_fn(be, "Isend")(p, cnt, dt, int(dest), int(tag), ch, ctypes.byref(h)))
    return Request(h.value, b, be)


def Recv_(buf, src: int, tag: int, comm) -> Status:
    """pointtopoint.jl:266-276."""
    b, p, cnt, dt = _args(buf)
    be, ch = _route(b, comm)
    st = _empty()
    _check(_fn(be, "Recv")(p, cnt, dt, int(src), int(tag), ch, ctypes.byref(st)))
    return st


def Recv(T, src: int, tag: int, comm):
    """pointtopoint.jl:293-297: receive one isbits value -> (value, status)."""
    ref = _scalar_ref(np.dtype(T).type(0), comm)
    st = Recv_(ref, src, tag, comm)
    return (ref[0].item() if isinstance(ref, np.ndarray) else ref.cpu()[0].item()), st


def Irecv_(buf, src: int, tag: int, comm) -> Request:
    """pointtopoint.jl:325-339."""
    b, p, cnt, dt = _args(buf)
    be, ch = _route(b, comm)
    h = ctypes.c_int(C.MPI_REQUEST_NULL)
    _check(_fn(be, "Irecv")(p, cnt, dt, int(src), int(tag), ch, ctypes.byref(h)))
    return Request(h.value, b, be)


def Sendrecv_(sendbuf, dest, sendtag, recvbuf, source, recvtag, comm) -> Status:
    """pointtopoint.jl:370-391."""
    sb, sp, sc, sd = _args(sendbuf)
    rb, rp, rc_, rd = _args(recvbuf)
    be, ch = _route(rb, comm)
    if _is_host(sb) != (be == "host"):
        raise TypeError("Sendrecv! needs both buffers on the same side (host or device)")
    st = _empty()
    _check(_fn(be, "Sendrecv")(sp, sc, sd, int(dest), int(sendtag), rp, rc_, rd, int(source), int(recvtag), ch,
                               ctypes.byref(st)))
    return st


# serialized objects (pointtopoint.jl:210-218, 242-251, 299-312, 341-352)
def _bytes_buf(raw: bytes, comm):
    a = np.frombuffer(raw, dtype=np.uint8).copy()
    if comm.host is not None:
        return a
    return _torch().from_numpy(a).to(f"cuda:{comm.device}")


def send(obj, dest: int, tag: int, comm):
    Send(_bytes_buf(pickle.dumps(obj), comm), dest, tag, comm)


def isend(obj, dest: int, tag: int, comm) -> Request:
    return Isend(_bytes_buf(pickle.dumps(obj), comm), dest, tag, comm)


def _unpickle(buf):
    raw = buf.tobytes() if isinstance(buf, np.ndarray) else buf.cpu().numpy().tobytes()
    return pickle.loads(raw)  # payload produced by send()/isend() of this program


def recv(src: int, tag: int, comm):
    st = Probe(src, tag, comm)
    n = Get_count(st, np.uint8)
    buf = _bytes_buf(bytes(n), comm)
    st = Recv_(buf, Get_source(st), Get_tag(st), comm)
    return _unpickle(buf), st


def irecv(src: int, tag: int, comm):
    flag, st = Iprobe(src, tag, comm)
    if not flag:
        return False, None, None
    n = Get_count(st, np.uint8)
    buf = _bytes_buf(bytes(n), comm)
    st = Recv_(buf, Get_source(st), Get_tag(st), comm)
    return True, _unpickle(buf), st


# ---------------------------------------------------------------------------
# probe
# ---------------------------------------------------------------------------
def _backends(comm):
    bes = []
    if comm.val:
        bes.append(("dev", comm.val))
    if comm.host is not None:
        bes.append(("host", comm.host))
    return bes


def Iprobe(src: int, tag: int, comm):
    """pointtopoint.jl:126-137 -> (flag, Status | None); checks the device
    engine and host libmpi (messages may come from either side)."""
    for be, ch in _backends(comm):
        flag = ctypes.c_int(0)
        st = _empty()
        _check(_fn(be, "Iprobe")(int(src), int(tag), ch, ctypes.byref(flag), ctypes.byref(st)))
        if flag.value:
            return True, st
    return False, None


def Probe(src: int, tag: int, comm) -> Status:
    """pointtopoint.jl:107-115."""
    bes = _backends(comm)
    if len(bes) == 1:
        be, ch = bes[0]
        st = _empty()
        _check(_fn(be, "Probe")(int(src), int(tag), ch, ctypes.byref(st)))
        return st
    while True:
        flag, st = Iprobe(src, tag, comm)
        if flag:
            return st


# ---------------------------------------------------------------------------
# completion (pointtopoint.jl:398-681)
# ---------------------------------------------------------------------------
def _done(req):
    req.val, req.buffer = C.MPI_REQUEST_NULL, None


def Wait_(req: Request) -> Status:
    st = _empty()
    if isnull(req):
        return st
    h = ctypes.c_int(req.val)
    rc = _fn(req.backend, "Wait")(ctypes.byref(h), ctypes.byref(st))
    _done(req)
    _check(rc)
    return st


def Test_(req: Request):
    st = _empty()
    if isnull(req):
        return True, st
    h = ctypes.c_int(req.val)
    flag = ctypes.c_int(0)
    rc = _fn(req.backend, "Test")(ctypes.byref(h), ctypes.byref(flag), ctypes.byref(st))
    _check(rc)
    if not flag.value:
        return False, None
    _done(req)
    return True, st


def _groups(reqs):
    """Indices of the active requests per backend."""
    g = {}
    for i, r in enumerate(reqs):
        if not isnull(r):
            g.setdefault(r.backend, []).append(i)
    return g


def Waitall_(reqs):
    stats = [_empty() for _ in reqs]
    for be, idx in _groups(reqs).items():
        n = len(idx)
        hv = (ctypes.c_int * n)(*[reqs[i].val for i in idx])
        sv = (Status * n)()
        rc = _fn(be, "Waitall")(n, hv, sv)
        for k, i in enumerate(idx):
            stats[i] = Status.from_buffer_copy(sv[k])
            _done(reqs[i])
        _check(rc)
    return stats


def Testall_(reqs):
    """-> (True, statuses) if every request completed (all freed), else
    (False, None) with no request modified."""
    g = _groups(reqs)
    if len(g) > 1:
        raise TypeError("Testall! over a mix of host and device requests cannot be all-or-nothing; use Waitall!")
    stats = [_empty() for _ in reqs]
    for be, idx in g.items():
        n = len(idx)
        hv = (ctypes.c_int * n)(*[reqs[i].val for i in idx])
        sv = (Status * n)()
        flag = ctypes.c_int(0)
        rc = _fn(be, "Testall")(n, hv, ctypes.byref(flag), sv)
        if not flag.value:
            _check(rc)
            return False, None
        for k, i in enumerate(idx):
            stats[i] = Status.from_buffer_copy(sv[k])
            _done(reqs[i])
        _check(rc)
    return True, stats


def _any(reqs, blocking):
    g = _groups(reqs)
    if not g:
        return True, 0, _empty()
    while True:
        for be, idx in g.items():
            n = len(idx)
            hv = (ctypes.c_int * n)(*[reqs[i].val for i in idx])
            ind, flag = ctypes.c_int(0), ctypes.c_int(0)
            st = _empty()
            if blocking and len(g) == 1:
                rc = _fn(be, "Waitany")(n, hv, ctypes.byref(ind), ctypes.byref(st))
                flag.value = 1
            else:
                rc = _fn(be, "Testany")(n, hv, ctypes.byref(ind), ctypes.byref(flag), ctypes.byref(st))
            if flag.value and ind.value != C.MPI_UNDEFINED:
                i = idx[ind.value]
                _done(reqs[i])
                _check(rc)
                return True, i + 1, st
            _check(rc)
        if not blocking:
            return False, 0, None


def Waitany_(reqs):
    """-> (1-based index, Status); (0, empty Status) if no request is active."""
    _, i, st = _any(reqs, True)
    return i, st


def Testany_(reqs):
    """-> (flag, 1-based index, Status | None) as pointtopoint.jl:559-598."""
    flag, i, st = _any(reqs, False)
    if flag and i == 0:
        return True, 0, None
    return flag, i, st


def _some(reqs, blocking):
    g = _groups(reqs)
    if not g:
        return [], []
    while True:
        inds, stats = [], []
        for be, idx in g.items():
            n = len(idx)
            hv = (ctypes.c_int * n)(*[reqs[i].val for i in idx])
            out = ctypes.c_int(0)
            iv = (ctypes.c_int * n)()
            sv = (Status * n)()
            name = "Waitsome" if blocking and len(g) == 1 else "Testsome"
            rc = _fn(be, name)(n, hv, ctypes.byref(out), iv, sv)
            k = 0 if out.value == C.MPI_UNDEFINED else out.value
            for j in range(k):
                i = idx[iv[j]]
                _done(reqs[i])
                inds.append(i + 1)
                stats.append(Status.from_buffer_copy(sv[j]))
            _check(rc)
        if inds or not blocking:
            return inds, stats


def Waitsome_(reqs):
    """-> (1-based indices, statuses) of the requests that completed."""
    return _some(reqs, True)


def Testsome_(reqs):
    return _some(reqs, False)


def Cancel_(req: Request):
    """pointtopoint.jl:671-681 (the request stays valid until waited on)."""
    if isnull(req):
        raise MPIError(C.MPI_ERR_REQUEST)
    h = ctypes.c_int(req.val)
    _check(_fn(req.backend, "Cancel")(ctypes.byref(h)))
