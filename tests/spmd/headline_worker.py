"""SPMD worker: parity at the headline sizes (BASELINE configs 3-5) on the
DEFAULT paths (the algorithm the size selects — zero-copy at these sizes):

* Allreduce! 256 MiB f32 SUM: bit-exact against the oracle (fold_rsag, the
  MPICH Rabenseifner association) on sampled slices spanning every two-shot
  chunk boundary, the prefix and the tail;
* Bcast! / Allgather! / Alltoall! at 512 MiB: exact (torch.equal) against
  the regenerated inputs;
* Scan! / Exscan! / Reduce! on 64 Mi Int32 / Int64 elements with BAND / BOR /
  MAX: exact against the prefix folds of the regenerated inputs (integer ops
  are association-free).
Every rank regenerates every rank's seeded input on its own device.
Launched by tests/test_headline_gpu.py.
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "mpi.jl_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpigx as MPI  # noqa: E402
from oracle import mpich_model as M  # noqa: E402


# every MPIGX_ALGO at 16 MiB and 1 MiB; "auto" = the size's own choice
# (tuners included); where an algorithm cannot take a size the engine runs
# the static choice (e.g. "ll" above its 256 KiB capacity)
ALGOS = ("auto", "ll", "ll2", "oneshot", "twoshot", "push", "ring", "pull", "pull_generic", "pullpush")


def extra(comm, r, n, f32_input, fails):
    """The production grid (no MPIGX_MAX_BLOCKS: the default 256-block grid,
    capped only by the ranks-per-device residency rule) through every
    algorithm at 16 MiB and 1 MiB — whole buffers against the oracle (the
    ring against its own association, fold_ring) — and one 1 GiB Allreduce
    on the default path, sampled at the chunk and Rabenseifner boundaries."""
    for mib in (16, 1):
        count = (mib << 20) // 4
        xs = [f32_input(q, count, 5000 + mib) for q in range(n)]
        hs = [x.cpu().numpy() for x in xs]
        tree = M.fold_rsag(hs, "FLOAT", "SUM")
        for algo in ALGOS:
            MPI.set_knob(comm, "ALGO", None if algo == "auto" else algo)
            recv = torch.empty_like(xs[r])
            for _ in range(4 if algo == "auto" else 1):  # auto: the tuners' sampling calls too
                recv.zero_()
                MPI.Allreduce_(xs[r], recv, MPI.SUM, comm)
                got = recv.cpu().numpy()
                if algo == "ring" and count * 4 >= MPI.get_knob(comm, "ZC_MIN"):  # the ring is a zero-copy-size path
                    stage = MPI.get_knob(comm, "STAGING_BYTES")
                    exp = M.fold_ring(hs, "FLOAT", "SUM", 1, M.ring_round_elems(stage, n, "FLOAT", 1))
                else:
                    exp = tree
                if not np.array_equal(got.view(np.uint32), exp.view(np.uint32)):
                    bad = np.nonzero(got.view(np.uint32) != exp.view(np.uint32))[0]
                    fails.append(("allreduce", mib, algo, int(bad.size), int(bad[0])))
                    break
        MPI.set_knob(comm, "ALGO", None)
        del xs, hs
    # 1 GiB on the default path, sampled spans
    count = (1 << 30) // 4
    send = f32_input(r, count, 6000)
    recv = torch.empty_like(send)
    MPI.Allreduce_(send, recv, MPI.SUM, comm)
    chunk = -(-(-(-count // n)) // 4) * 4
    spans = [(0, 1 << 15), (count - (1 << 15), count)] + \
            [(c * chunk - 2048, c * chunk + 2048) for c in range(1, n)] + \
            [(count // 8 * k - 1024, count // 8 * k + 1024) for k in range(1, 8)]
    samples = {}
    for q in range(n):
        x = f32_input(q, count, 6000)
        for lo, hi in spans:
            samples.setdefault((lo, hi), []).append(x[lo:hi].cpu().numpy())
        del x
    for (lo, hi), ins in samples.items():
        ref = M.fold_rsag(ins, "FLOAT", "SUM")
        if not np.array_equal(recv[lo:hi].cpu().numpy().view(np.uint32), ref.view(np.uint32)):
            fails.append(("allreduce-1GiB", lo, hi))
    del send, recv


def main():
    comm = MPI.Init()
    r, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
    dev = torch.device("cuda")
    fails = []

    def f32_input(q, count, seed):
        g = torch.Generator(device=dev).manual_seed(seed + q)
        return torch.rand(count, device=dev, generator=g) * 2 - 1

    # --- Allreduce 256 MiB f32 SUM, default path
    count = (256 << 20) // 4
    send = f32_input(r, count, 1000)
    recv = torch.empty_like(send)
    MPI.Allreduce_(send, recv, MPI.SUM, comm)
    xs = [f32_input(q, count, 1000) for q in range(n)]
    # the WHOLE buffer against the oracle: rank r checks the r-th of n equal
    # parts (f32 SUM's MPICH association depends on the element's position
    # only through the operand roles, which SUM does not see, so a part folds
    # like the whole) and every rank's recvbuf must hash like rank 0's (sha1
    # over the host control plane's gloo group, not through the engine)
    lo, hi = count * r // n, count * (r + 1) // n
    ref = M.fold_rsag([x[lo:hi].cpu().numpy() for x in xs], "FLOAT", "SUM")
    mine = recv[lo:hi].cpu().numpy()
    if not np.array_equal(mine.view(np.uint32), ref.view(np.uint32)):
        bad = np.nonzero(mine.view(np.uint32) != ref.view(np.uint32))[0]
        fails.append(("allreduce-256MiB-whole", lo + int(bad[0]), int(bad.size)))
    del ref, mine
    import hashlib
    import torch.distributed as dist
    digests = [None] * n
    dist.all_gather_object(digests, hashlib.sha1(recv.cpu().numpy().tobytes()).hexdigest())
    if len(set(digests)) != 1:
        fails.append(("allreduce-256MiB-ranks-differ", digests.index(digests[r])))
    # the same call again (cached zero-copy view) gives the same bits
    again = torch.empty_like(send)
    MPI.Allreduce_(send, again, MPI.SUM, comm)
    if not torch.equal(again.view(torch.int32), recv.view(torch.int32)):
        fails.append(("allreduce-repeat",))
    # the large-Allreduce tuner: call 2 above timed the pull two-shot, call 3
    # times the push two-shot, call 4 the pull-push two-shot and decides,
    # call 5 runs the choice; every call gives the same bits (same fold
    # schedule)
    import ctypes
    for k in (3, 4, 5):
        again.zero_()
        MPI.Allreduce_(send, again, MPI.SUM, comm)
        if not torch.equal(again.view(torch.int32), recv.view(torch.int32)):
            fails.append(("allreduce-tuner-call", k))
    ch = ctypes.c_int(-2)
    MPI.lib().mpigx_comm_ar_choice(comm.val, ctypes.byref(ch), None, None)
    if ch.value not in (0, 1, 2):
        fails.append(("ar-tune-undecided", ch.value))
    del send, recv, again, xs

    if os.environ.get("MPIGX_HEADLINE_EXTRA"):
        extra(comm, r, n, f32_input, fails)

    # --- Bcast / Allgather / Alltoall at 512 MiB
    nb = 512 << 20
    cnt = nb // 4
    for root in sorted({0, n - 1}):
        buf = f32_input(r, cnt, 2000) if r == root else torch.zeros(cnt, device=dev)
        MPI.Bcast_(buf, root, comm)
        if not torch.equal(buf, f32_input(root, cnt, 2000)):
            fails.append(("bcast-512MiB", root))
        del buf
    per = cnt // n
    src = f32_input(r, per, 3000)
    dst = torch.empty(per * n, device=dev)
    MPI.Allgather_(src, dst, per, comm)
    for q in range(n):
        if not torch.equal(dst[q * per:(q + 1) * per], f32_input(q, per, 3000)):
            fails.append(("allgather-512MiB", q))
    # in place
    dst.zero_()
    dst[r * per:(r + 1) * per] = src
    MPI.Allgather_(dst, per, comm)
    for q in range(n):
        if not torch.equal(dst[q * per:(q + 1) * per], f32_input(q, per, 3000)):
            fails.append(("allgather-inplace-512MiB", q))
    del src, dst
    a2s = f32_input(r, per * n, 4000)
    a2r = torch.empty_like(a2s)
    MPI.Alltoall_(a2s, a2r, per, comm)
    for q in range(n):
        if not torch.equal(a2r[q * per:(q + 1) * per], f32_input(q, per * n, 4000)[r * per:(r + 1) * per]):
            fails.append(("alltoall-512MiB", q))
    del a2s, a2r

    # --- Scan / Exscan / Reduce, 64 Mi elements of Int32 / Int64
    ops = (("BAND", MPI.BAND, torch.bitwise_and), ("BOR", MPI.BOR, torch.bitwise_or), ("MAX", MPI.MAX, torch.maximum))
    cnt = 64 << 20
    for tdt, lim in ((torch.int32, 1 << 31), (torch.int64, 1 << 62)):
        def gen(q):
            g = torch.Generator(device=dev).manual_seed(7000 + 31 * q)
            return torch.randint(-lim, lim, (cnt,), dtype=tdt, device=dev, generator=g)
        mine = gen(r)
        for oname, op, fn in ops:
            pref = None
            for q in range(r + 1):  # prefix through my rank
                pref = gen(q) if pref is None else fn(pref, gen(q))
            out = torch.zeros_like(mine)
            MPI.Scan_(mine, out, op, comm)
            if not torch.equal(out, pref):
                fails.append(("scan", str(tdt), oname))
            out.fill_(7)
            MPI.Exscan_(mine, out, op, comm)
            if r > 0:
                ex = None
                for q in range(r):
                    ex = gen(q) if ex is None else fn(ex, gen(q))
                if not torch.equal(out, ex):
                    fails.append(("exscan", str(tdt), oname))
            elif not bool((out == 7).all()):
                fails.append(("exscan-rank0-touched", str(tdt), oname))
            root = n - 1
            rout = torch.zeros_like(mine) if r == root else None
            MPI.Reduce_(mine, rout, op, root, comm)
            if r == root:
                tot = pref
                for q in range(r + 1, n):
                    tot = fn(tot, gen(q))
                if not torch.equal(rout, tot):
                    fails.append(("reduce", str(tdt), oname))
            del out, rout, pref
        del mine
    MPI.Barrier(comm)
    pm = list(MPI.peer_memory(comm))  # signalling protocol per peer pair (rw_mask, same_device)
    MPI.Finalize()
    print(json.dumps({"rank": r, "n": n, "peer_mem": pm, "nfail": len(fails), "failures": [str(f) for f in fails[:20]]}), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
