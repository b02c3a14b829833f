"""test/test_threads.jl restated on the Python mirror, device mode: MPI
initialized with THREAD_MULTIPLE, then every rank posts N Irecv! / Isend
pairs of one-element device views from a pool of threads at once
(`Threads.@threads for i = 1:N`, test_threads.jl:33-36) and waits for all of
them on the main thread.  ctypes releases the GIL around each call, so the
threads really are inside libmpigx together (rt::big_lock, runtime.hpp).
Beyond the reference's N = 10: the same with 256 pairs, 8 threads and three
rounds, and a thread that waits on its own receive while other threads keep
posting, and a thread in Win_fence while another sends the message the
peer needs before its own fence, and collectives on three duplicated
communicators from three threads at once (MPIGX_CONCURRENT_COMMS=4 set by
the launcher so the three grids fit on the GPU together).  Launched by
tests/test_reference_suite_gpu.py."""
import json
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))

import torch  # noqa: E402

import mpigx as MPI  # noqa: E402

FAIL = []
NCHECK = [0]


def check(cond, what):
    NCHECK[0] += 1
    if not bool(cond):
        FAIL.append(what)


def exchange(comm, n_msgs, nthreads, tag0):
    size, rank = MPI.Comm_size(comm), MPI.Comm_rank(comm)
    dst, src = (rank + 1) % size, (rank - 1) % size
    send_arr = torch.arange(1, n_msgs + 1, dtype=torch.float64, device="cuda") + 1000 * rank
    recv_arr = torch.zeros(n_msgs, dtype=torch.float64, device="cuda")
    reqs = [None] * (2 * n_msgs)

    def work(i):
        reqs[n_msgs + i] = MPI.Irecv_(recv_arr[i:i + 1], src, tag0 + i, comm)
        reqs[i] = MPI.Isend(send_arr[i:i + 1], dst, tag0 + i, comm)

    with ThreadPoolExecutor(max_workers=nthreads) as ex:
        list(ex.map(work, range(n_msgs)))
    MPI.Waitall_(reqs)
    want = torch.arange(1, n_msgs + 1, dtype=torch.float64, device="cuda") + 1000 * src
    return torch.equal(recv_arr, want)


def concurrent_comms(comm, size, rank):
    """Collectives on distinct communicators from distinct threads at once
    (each communicator's calls stay ordered, as MPI requires): every thread
    runs a loop of Allreduce! (LL, one-shot and zero-copy sizes) and Bcast!
    on its own Comm_dup of COMM_WORLD.  MPIGX_CONCURRENT_COMMS covers the
    three communicators: every result must be exact."""
    comms = [MPI.Comm_dup(comm) for _ in range(3)]
    results = [None] * len(comms)

    def loop(i):
        cm = comms[i]
        ok = True
        # each thread on its own stream (the mirror runs a communicator's
        # collectives on the caller's current stream; two communicators'
        # kernels queued on ONE stream in different orders on different
        # ranks would wait for each other — the rule NCCL / RCCL state
        # for concurrent communicators too)
        torch.cuda.set_stream(torch.cuda.Stream())
        for it, cnt in enumerate((7, 1000, 60000, (32 << 20) // 4, 5)):
            x = torch.full((cnt,), float(rank + 1 + i), device="cuda")
            y = MPI.Allreduce(x, MPI.SUM, cm)
            ok &= bool((y == float(sum(q + 1 + i for q in range(size)))).all())
            b = torch.full((cnt,), float(it) if rank == 0 else -1.0, device="cuda")
            MPI.Bcast_(b, 0, cm)
            ok &= bool((b == float(it)).all())
        torch.cuda.synchronize()
        results[i] = ok

    ths = [threading.Thread(target=loop, args=(i,)) for i in range(len(comms))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(120)
    check(all(results) and not any(t.is_alive() for t in ths), f"concurrent collectives on {len(comms)} comms: {results}")
    for cm in comms:
        MPI.free(cm)


def stuck_case(comm, size, rank, stream_ordered=False):
    """More communicators in flight than the GPU holds resident together
    (VERDICT r05 item 2), made deterministic: three communicators, each
    Allreduce! of 64 MiB (zero-copy) on its own thread and stream, grids at
    their residency cap (MPIGX_MAX_BLOCKS raised by the launcher, so each
    grid takes its share of the device: with MPIGX_CONCURRENT_COMMS = 1 the
    three of one rank fill it).  Rank 0 launches first; the other ranks
    0.5 s later find no room, and their launches never start while rank 0's
    grids wait for them.  With MPIGX_CONCURRENT_COMMS = 1 every call must
    come back with MPI_ERR_OTHER within about MPIGX_TIMEOUT_MS (mpigx.cpp
    stuck_peer / the stall rule; stderr names the knob); with the knob at
    the number of communicators every result must be exact.
    stream_ordered: the same with RCCL-style launches: the process-wide
    watcher (mpigx.cpp watch_one) cancels a stuck or partially resident
    launch, and the error comes from mpigx_comm_synchronize."""
    ncomm = 3
    comms = [MPI.Comm_dup(comm) for _ in range(ncomm)]
    cnt = (64 << 20) // 4
    xs = [torch.full((cnt,), float(rank + 1 + i), device="cuda") for i in range(ncomm)]
    ys = [torch.empty_like(x) for x in xs]
    want = [float(sum(q + 1 + i for q in range(size))) for i in range(ncomm)]
    streams = [torch.cuda.Stream() for _ in range(ncomm)]
    # one communicator at a time first: buffer registration and the
    # algorithm tuner's sampling calls, so the concurrent calls below launch
    # straight away (no host exchange that would line the ranks up)
    L = MPI.lib()
    for i in range(ncomm):
        with torch.cuda.stream(streams[i]):
            for _ in range(6):
                MPI.Allreduce_(xs[i], ys[i], MPI.SUM, comms[i])
            check(bool((ys[i] == want[i]).all()), f"warm-up comm {i}")
        if stream_ordered:
            MPI.api._check(L.mpigx_comm_set_blocking(comms[i].val, 0))
    torch.cuda.synchronize()
    MPI.Barrier(comm)
    results, secs = [None] * ncomm, [None] * ncomm

    def run(i):
        torch.cuda.set_stream(streams[i])
        if rank != 0:
            time.sleep(0.5)
        t0 = time.time()
        try:
            ys[i].fill_(-1)
            MPI.Allreduce_(xs[i], ys[i], MPI.SUM, comms[i])
            if stream_ordered:
                MPI.api._check(L.mpigx_comm_synchronize(comms[i].val))
            results[i] = bool((ys[i] == want[i]).all())
        except MPI.MPIError as e:
            results[i] = f"MPIError {e.code}"
        secs[i] = round(time.time() - t0, 3)

    ths = [threading.Thread(target=run, args=(i,)) for i in range(ncomm)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(180)
    alive = any(t.is_alive() for t in ths)
    check(not alive, f"every thread came back: {results}")
    check(all(r is True or r == f"MPIError {MPI.consts.MPI_ERR_OTHER}" for r in results), f"results: {results}")
    print(json.dumps({"rank": rank, "stuck_results": results, "call_s": secs,
                      "errors": sum(isinstance(r, str) for r in results)}), flush=True)
    for cm in comms:
        try:
            MPI.free(cm)
        except MPI.MPIError:
            pass  # a communicator that failed above

def main():
    provided = MPI.Init_thread(MPI.THREAD_MULTIPLE)       # test_threads.jl:11
    if os.environ.get("THREADS_MODE") in ("stuck", "stuck_so"):
        comm = MPI.COMM_WORLD
        stuck_case(comm, MPI.Comm_size(comm), MPI.Comm_rank(comm), os.environ["THREADS_MODE"] == "stuck_so")
        MPI.Barrier(comm)
        MPI.Finalize()
        print(json.dumps({"rank": MPI.Comm_rank(comm), "provided": provided, "checks": NCHECK[0],
                          "failures": FAIL[:10], "nfail": len(FAIL)}), flush=True)
        sys.exit(1 if FAIL else 0)
    check(MPI.THREAD_SINGLE <= provided <= MPI.THREAD_MULTIPLE, "provided range")  # :13
    check(MPI.Query_thread() == provided, "Query_thread")   # :14
    check(MPI.Is_thread_main(), "Is_thread_main")           # :15
    comm = MPI.COMM_WORLD
    check(provided == MPI.THREAD_MULTIPLE, "engine provides THREAD_MULTIPLE")
    if provided == MPI.THREAD_MULTIPLE:
        check(exchange(comm, 10, 10, 0), "N = 10 threaded Isend / Irecv")  # :26-40
        for rnd in range(3):
            check(exchange(comm, 256, 8, 1000 + 300 * rnd), f"256 pairs, 8 threads, round {rnd}")
        # a thread blocked in Wait must not hold up another thread's Isend
        size, rank = MPI.Comm_size(comm), MPI.Comm_rank(comm)
        dst, src = (rank + 1) % size, (rank - 1) % size
        got = torch.zeros(4, dtype=torch.float64, device="cuda")
        out = torch.full((4,), float(rank), dtype=torch.float64, device="cuda")
        waiter = threading.Thread(target=lambda: MPI.Wait_(MPI.Irecv_(got, src, 9000, comm)))
        waiter.start()
        MPI.Wait_(MPI.Isend(out, dst, 9000, comm))
        waiter.join(60)
        check(not waiter.is_alive() and bool((got == float(src)).all()), "blocked waiter + concurrent Isend")
        # one thread in a collective RMA call that waits (Win_fence), another
        # sending the message its peer needs before the peer can reach the
        # fence: the waiting call must let the Isend through (the big lock
        # is yielded while it polls, rt::yield_big_lock)
        win_buf = torch.zeros(64, dtype=torch.float64, device="cuda")
        win = MPI.Win_create(win_buf, comm)
        MPI.Win_fence(0, win)
        token = torch.full((8,), 5.0 + rank, dtype=torch.float64, device="cuda")
        if rank == 0:
            fencer = threading.Thread(target=lambda: MPI.Win_fence(0, win))
            fencer.start()
            for q in range(1, size):
                MPI.Send(token, q, 9100, comm)
            fencer.join(60)
            check(not fencer.is_alive(), "fence with a concurrent Send on another thread")
        else:
            got2 = torch.zeros(8, dtype=torch.float64, device="cuda")
            MPI.Recv_(got2, 0, 9100, comm)
            check(bool((got2 == 5.0).all()), "message sent beside a fence")
            MPI.Win_fence(0, win)
        MPI.free(win)
        # Puts to one target from 8 threads inside one fence epoch, 64 each:
        # far more than the 16-envelope ring per (origin, target), so threads
        # wait for slots while others post (rma.cpp post claims its sequence
        # number before it can yield the lock)
        nput = 8 * 64
        win_buf2 = torch.zeros(nput, dtype=torch.float64, device="cuda")
        win2 = MPI.Win_create(win_buf2, comm)
        vals = torch.arange(nput, dtype=torch.float64, device="cuda") + 10000.0 * rank
        MPI.Win_fence(0, win2)

        def putter(k):
            for j in range(64):
                i = k * 64 + j
                MPI.Put(vals[i:i + 1], 1, dst, i, win2)

        with ThreadPoolExecutor(max_workers=8) as ex:
            list(ex.map(putter, range(8)))
        MPI.Win_fence(0, win2)
        want2 = torch.arange(nput, dtype=torch.float64, device="cuda") + 10000.0 * src
        check(torch.equal(win_buf2, want2), "512 Puts to one target from 8 threads in one epoch")
        MPI.free(win2)
        concurrent_comms(comm, size, rank)
    MPI.Barrier(comm)
    MPI.Finalize()
    print(json.dumps({"rank": MPI.Comm_rank(comm), "provided": provided, "checks": NCHECK[0],
                      "failures": FAIL[:10], "nfail": len(FAIL)}), flush=True)
    sys.exit(1 if FAIL else 0)


if __name__ == "__main__":
    main()
