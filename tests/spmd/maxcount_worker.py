"""SPMD worker: the largest message MPI.jl can pass — `count` is a Cint
(collective.jl:698-700 `ccall(..., Cint, ...)`), so 2^31 - 1 elements — on
every collective's default path, with byte offsets past 2^31 (int8) and
2^33 (f32) and, for Allgather / Alltoall, totals of n·count elements past
2^31.  Exact against results recomputed on the device from the regenerated
seeded inputs:

* integer SUM / BXOR wrap and are association-free;
* f32 SUM at n = 2 is x0 + x1 and at n = 3 MPICH's Reduce-based association
  (x0 + x1) + x2 (the Rabenseifner pre-step folds rank 1 into rank 0, then
  the pairwise tree) — computed in that order by torch, bit for
  bit.

Rank 0 also runs the local MPI.Op kernel (config 2's API) over 8 int8 inputs
of 2^31 - 1 elements.  Launched by tests/test_maxcount_gpu.py."""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "mpi.jl_amd")):
    sys.path.insert(0, p)

import torch  # noqa: E402

import mpigx as MPI  # noqa: E402

CMAX = int(os.environ.get("MAXCOUNT_ELEMS", (1 << 31) - 1))  # smaller for diagnosis only


def main():
    comm = MPI.Init()
    r, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
    dev = torch.device("cuda")
    fails, times = [], {}
    if os.environ.get("MAXCOUNT_WATCH"):  # diagnosis: where a stuck call is
        import ctypes
        import faulthandler
        import threading
        faulthandler.dump_traceback_later(30, repeat=True, file=sys.stderr)
        L = MPI.lib()

        def watch():
            while True:
                time.sleep(5.0)
                st8 = (ctypes.c_ulonglong * 8)()
                L.mpigx_comm_diag_state(comm.val, st8)
                print(f"r{r} watch {list(st8)}", file=sys.stderr, flush=True)

        threading.Thread(target=watch, daemon=True).start()

    def i8(q, seed, count=CMAX):
        g = torch.Generator(device=dev).manual_seed(seed + 101 * q)
        return torch.randint(-128, 128, (count,), dtype=torch.int8, device=dev, generator=g)

    def timed(name, fn):
        torch.cuda.synchronize()
        print(f"r{r} {name} ...", file=sys.stderr, flush=True)
        t0 = time.time()
        fn()
        torch.cuda.synchronize()
        times[name] = round(time.time() - t0, 4)
        print(f"r{r} {name} {times[name]} s", file=sys.stderr, flush=True)

    import ctypes
    hip_rt = ctypes.c_int(0)
    ctypes.CDLL("libamdhip64.so").hipRuntimeGetVersion(ctypes.byref(hip_rt))
    capped = hip_rt.value < 70200000  # runtime.hpp ipc_alloc_max: no IPC export of allocations >= 2 GiB

    def zc_hits():  # launches made on an agreed zero-copy view
        h, x = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        MPI.lib().mpigx_comm_zc_stats(comm.val, ctypes.byref(h), ctypes.byref(x))
        return h.value

    # --- Allreduce int8 SUM: calls 1-4 are the zero-copy tuner's (register,
    # pull, push, pull-push), call 5 runs its choice; every call exact
    x = i8(r, 10)
    exp = i8(0, 10)
    for q in range(1, n):
        exp += i8(q, 10)
    out = torch.empty_like(x)
    for k in range(5):
        out.zero_()
        timed(f"allreduce_i8_sum_call{k + 1}", lambda: MPI.Allreduce_(x, out, MPI.SUM, comm))
        if not torch.equal(out, exp):
            fails.append(("allreduce-i8-sum", k + 1))
    # an allocation the loaded HIP runtime cannot IPC-map goes staged on every
    # rank: no zero-copy view was ever built for it
    if capped and CMAX >= (1 << 31) - 1 and zc_hits() != 0:
        fails.append(("zero-copy view over a >= 2 GiB allocation on a capped runtime", zc_hits()))
    # in place
    out.copy_(x)
    timed("allreduce_i8_sum_inplace", lambda: MPI.Allreduce_(out, MPI.SUM, comm))
    if not torch.equal(out, exp):
        fails.append(("allreduce-i8-sum-inplace",))
    # staged path (zero-copy off: the arena-sized rounds)
    zc0 = MPI.get_knob(comm, "ZC_MIN")
    MPI.set_knob(comm, "ZC_MIN", 0)
    out.zero_()
    timed("allreduce_i8_sum_staged", lambda: MPI.Allreduce_(x, out, MPI.SUM, comm))
    if not torch.equal(out, exp):
        fails.append(("allreduce-i8-sum-staged",))
    MPI.set_knob(comm, "ZC_MIN", zc0)

    # --- point-to-point from / into the middle of the 2 GiB buffers: the
    # sender's allocation is staged through a pooled temporary where the
    # runtime cannot IPC-map it (p2p.cpp mpigx_isend)
    seg = 16 << 20
    lo = CMAX // 2 - seg // 2
    peer = (r + 1) % n
    src = (r - 1) % n
    out.fill_(0)
    timed("sendrecv_i8_16MiB_in_2GiB", lambda: MPI.Sendrecv_(x[lo:lo + seg], peer, 7, out[lo:lo + seg], src, 7, comm))
    if not torch.equal(out[lo:lo + seg], i8(src, 10)[lo:lo + seg]):
        fails.append(("sendrecv-in-2GiB",))

    # --- Reduce int8 BXOR to the last rank
    root = n - 1
    exp = i8(0, 10)
    for q in range(1, n):
        exp ^= i8(q, 10)
    rout = torch.zeros_like(x) if r == root else None
    timed("reduce_i8_bxor", lambda: MPI.Reduce_(x, rout, MPI.BXOR, root, comm))
    if r == root and not torch.equal(rout, exp):
        fails.append(("reduce-i8-bxor",))
    del rout

    # --- Scan / Exscan int8 SUM
    pref = i8(0, 10)
    for q in range(1, r + 1):
        pref += i8(q, 10)
    out.zero_()
    timed("scan_i8_sum", lambda: MPI.Scan_(x, out, MPI.SUM, comm))
    if not torch.equal(out, pref):
        fails.append(("scan-i8-sum",))
    out.fill_(7)
    timed("exscan_i8_sum", lambda: MPI.Exscan_(x, out, MPI.SUM, comm))
    if r > 0:
        pref -= x  # exclusive prefix = inclusive minus my own contribution (wrapping)
        if not torch.equal(out, pref):
            fails.append(("exscan-i8-sum",))
    elif not bool((out == 7).all()):
        fails.append(("exscan-rank0-touched",))
    del pref, exp

    # --- Bcast int8 from rank 1 (or 0 at n = 1)
    broot = 1 % n
    buf = x.clone() if r == broot else torch.zeros_like(x)
    timed("bcast_i8", lambda: MPI.Bcast_(buf, broot, comm))
    if not torch.equal(buf, i8(broot, 10)):
        fails.append(("bcast-i8",))
    del buf, out

    # --- Allgather: count = 2^31 - 1 per rank, n·count elements in recvbuf
    dst = torch.empty(n * CMAX, dtype=torch.int8, device=dev)
    timed("allgather_i8", lambda: MPI.Allgather_(x, dst, CMAX, comm))
    for q in range(n):
        if not torch.equal(dst[q * CMAX:(q + 1) * CMAX], i8(q, 10)):
            fails.append(("allgather-i8", q))
    del dst, x

    # --- Alltoall: blocks of 2^30 elements, n·2^30 per rank (2^31 at n = 2)
    blk = (CMAX + 1) // 2
    a2s = i8(r, 20, n * blk)
    a2r = torch.empty_like(a2s)
    timed("alltoall_i8", lambda: MPI.Alltoall_(a2s, a2r, blk, comm))
    for q in range(n):
        if not torch.equal(a2r[q * blk:(q + 1) * blk], i8(q, 20, n * blk)[r * blk:(r + 1) * blk]):
            fails.append(("alltoall-i8", q))
    del a2s, a2r
    torch.cuda.empty_cache()

    # --- Allreduce f32 SUM, 2^31 - 1 elements (8 GiB per buffer)
    def f32(q):
        g = torch.Generator(device=dev).manual_seed(30 + 101 * q)
        return torch.rand(CMAX, device=dev, generator=g) * 2 - 1

    if n in (2, 3):
        xf = f32(r)
        expf = f32(0)
        expf += f32(1)  # rank 0 inout, rank 1 in: x0 + x1 (IEEE add commutes)
        if n == 3:
            expf += f32(2)
        outf = torch.empty_like(xf)
        for k in range(2):
            outf.zero_()
            timed(f"allreduce_f32_sum_call{k + 1}", lambda: MPI.Allreduce_(xf, outf, MPI.SUM, comm))
            if not torch.equal(outf.view(torch.int32), expf.view(torch.int32)):
                fails.append(("allreduce-f32-sum", k + 1))
        del xf, expf, outf
        torch.cuda.empty_cache()

    # --- the local MPI.Op kernel (config 2's API) at the maximum count
    if r == 0:
        ins = [i8(q, 40) for q in range(8)]
        expl = ins[0].clone()
        for t in ins[1:]:
            expl += t
        outl = torch.empty_like(expl)
        timed("reduce_local_multi_i8_sum_8in", lambda: MPI.reduce_local_multi(ins, outl, MPI.SUM))
        if not torch.equal(outl, expl):
            fails.append(("reduce-local-multi-i8",))
        del ins, expl, outl

    MPI.Barrier(comm)
    MPI.Finalize()
    print(json.dumps({"rank": r, "n": n, "nfail": len(fails), "fails": fails[:10], "hip_runtime": hip_rt.value,
                      "ipc_capped": capped, "times_s": times}), flush=True)


if __name__ == "__main__":
    main()
