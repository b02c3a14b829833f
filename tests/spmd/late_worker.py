"""SPMD worker: a rank that reaches a collective late, or never.  With the
host gate (ranks sharing one GPU, mpigx.cpp shared_gate) the early ranks wait
on the host; with MPIGX_SHARED_GATE=0 (and MPIGX_PEER_MEM=xdev: the
one-rank-per-GPU protocol) their kernels wait on the device while their hosts
watch the peers (mpigx.cpp finish, PeerView.cancel).

* late — the last rank sleeps on the host for 2.5 x MPIGX_TIMEOUT_MS before
  a 16 MiB zero-copy Allreduce (`late`) or a 4 KiB one (`late_small`, the LL
  step / staged one-shot); the others are already in it.  MPI semantics
  (collective.jl:698-700 blocks until every rank arrives): the call waits for
  it and every rank gets the exact sum.  A second call right after must be
  exact too.
* late_stream — the last rank is late on its GPU, not on its host: its
  stream holds 2.5 x MPIGX_TIMEOUT_MS of earlier work (torch.cuda._sleep)
  when it makes the blocking call, so its host waits in the call from the
  start while its GPU has not reached the launch.  That rank is the late
  one and must not declare a protocol stall (its peers are all
  in the launch, its own GPU is still in the previous one); exact results;
* late_vx — the same, before an Allgatherv (its rounds are agreed over the
  host control plane before any launch, so the early ranks wait on the host,
  host_allgather);
* late_so — the same on a stream-ordered communicator with fresh 16 MiB
  buffers (a stream-ordered zero-copy call agrees on the view over the host
  control plane before its launch);
* late_so_small — stream-ordered (RCCL-style): the early ranks' 4 KiB
  Allreduce KERNELS are already waiting on the device (no host exchange at
  this size) while the last rank sleeps; stream-ordered launches have no
  time limit either, so the synchronize after them returns exact results
  once the late rank arrives;
* gone_so — stream-ordered, the last rank exits: the early ranks' waiting
  kernels are cancelled by their peer watcher (mpigx.cpp watch_peers) and
  the synchronize fails within seconds;
* late_p2p — point-to-point: rank 0 posts a blocking Recv! from the last
  rank, which sleeps 2.5 x MPIGX_TIMEOUT_MS before its Send (pointtopoint.jl
  Recv! blocks until the message arrives): exact, no error;
* gone_p2p — rank 0's Recv! from the last rank, which exits instead: the
  Recv fails within seconds (the peer is gone), not after a timeout and not
  never;
* gone — after one good call the last rank exits without finalizing; the
  others' next Allreduce must fail (MPIError) within seconds instead of
  waiting for ever.
* broken — after one good call the last rank's communicator fails
  (mpigx_comm_diag_break, a fault injection) and its next call returns
  MPI_ERR_OTHER at once; the others' next Allreduce must fail within seconds
  too (ShmRank.broken), not wait for a rank that will never come.
Launched by tests/test_late_rank_gpu.py.
"""
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


def main():
    scenario = sys.argv[1]
    comm = MPI.Init()
    r, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
    timeout_s = int(os.environ["MPIGX_TIMEOUT_MS"]) / 1000.0
    count = (16 << 20) // 4
    send = torch.full((count,), float(r + 1), device="cuda")
    recv = torch.empty(count, device="cuda")
    want = float(n * (n + 1) // 2)
    out = {"rank": r, "n": n, "scenario": scenario}
    fails = []

    MPI.Allreduce_(send, recv, MPI.SUM, comm)
    if not bool((recv == want).all()):
        fails.append("first call")
    out["peer_mem"] = list(MPI.peer_memory(comm))
    if scenario in ("late", "late_small"):
        if scenario == "late_small":
            send, recv = send[:1024].clone(), recv[:1024].clone()
        if r == n - 1:
            time.sleep(2.5 * timeout_s)
        recv.fill_(-1)
        t0 = time.time()
        MPI.Allreduce_(send, recv, MPI.SUM, comm)
        out["late_call_s"] = round(time.time() - t0, 3)
        if not bool((recv == want).all()):
            fails.append("late call")
        recv.fill_(-1)
        MPI.Allreduce_(send, recv, MPI.SUM, comm)
        if not bool((recv == want).all()):
            fails.append("call after")
        MPI.Barrier(comm)
        MPI.Finalize()
    elif scenario == "late_stream":
        # calibrate torch.cuda._sleep (clock cycles) on this box, then queue
        # 2.5 x the timeout of it on the last rank's stream
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        torch.cuda._sleep(10_000_000)
        b.record()
        torch.cuda.synchronize()
        per_cycle_s = a.elapsed_time(b) / 1e3 / 10_000_000
        MPI.Barrier(comm)
        recv.fill_(-1)
        torch.cuda.synchronize()
        t0 = time.time()
        if r == n - 1:
            torch.cuda._sleep(int(3.0 * timeout_s / per_cycle_s))
        MPI.Allreduce_(send, recv, MPI.SUM, comm)
        out["late_call_s"] = round(time.time() - t0, 3)
        if not bool((recv == want).all()):
            fails.append("call behind a busy stream")
        recv.fill_(-1)
        MPI.Allreduce_(send, recv, MPI.SUM, comm)
        if not bool((recv == want).all()):
            fails.append("call after")
        MPI.Barrier(comm)
        MPI.Finalize()
    elif scenario in ("late_vx", "late_so"):
        if r == n - 1:
            time.sleep(2.5 * timeout_s)
        t0 = time.time()
        if scenario == "late_vx":
            counts = [1000 + 17 * q for q in range(n)]
            mine = torch.full((counts[r],), float(r + 1), device="cuda")
            got = torch.full((sum(counts),), -1.0, device="cuda")
            MPI.Allgatherv_(mine, got, counts, comm)
            exp = torch.cat([torch.full((counts[q],), float(q + 1), device="cuda") for q in range(n)])
            if not torch.equal(got, exp):
                fails.append("late allgatherv")
        else:
            MPI.api._check(MPI.lib().mpigx_comm_set_blocking(comm.val, 0))
            send2 = torch.full((count,), float(r + 1), device="cuda")
            recv2 = torch.full((count,), -1.0, device="cuda")
            MPI.Allreduce_(send2, recv2, MPI.SUM, comm)
            torch.cuda.synchronize()
            if not bool((recv2 == want).all()):
                fails.append("late stream-ordered call")
            MPI.api._check(MPI.lib().mpigx_comm_set_blocking(comm.val, 1))
        out["late_call_s"] = round(time.time() - t0, 3)
        recv.fill_(-1)
        MPI.Allreduce_(send, recv, MPI.SUM, comm)
        if not bool((recv == want).all()):
            fails.append("call after")
        MPI.Barrier(comm)
        MPI.Finalize()
    elif scenario == "late_so_small":
        L = MPI.lib()
        small, sres = send[:1024].clone(), torch.full((1024,), -1.0, device="cuda")
        MPI.api._check(L.mpigx_comm_set_blocking(comm.val, 0))
        if r == n - 1:
            time.sleep(2.5 * timeout_s)
        t0 = time.time()
        MPI.Allreduce_(small, sres, MPI.SUM, comm)
        MPI.api._check(L.mpigx_comm_synchronize(comm.val))
        torch.cuda.synchronize()
        out["late_call_s"] = round(time.time() - t0, 3)
        if not bool((sres == want).all()):
            fails.append("late stream-ordered kernel")
        MPI.api._check(L.mpigx_comm_set_blocking(comm.val, 1))
        recv.fill_(-1)
        MPI.Allreduce_(send, recv, MPI.SUM, comm)
        if not bool((recv == want).all()):
            fails.append("call after")
        MPI.Barrier(comm)
        MPI.Finalize()
    elif scenario == "gone_so":
        L = MPI.lib()
        if r == n - 1:
            sys.stdout.flush()
            os._exit(0)
        small, sres = send[:1024].clone(), torch.full((1024,), -1.0, device="cuda")
        MPI.api._check(L.mpigx_comm_set_blocking(comm.val, 0))
        t0 = time.time()
        rc = 0
        try:
            MPI.Allreduce_(small, sres, MPI.SUM, comm)
            rc = L.mpigx_comm_synchronize(comm.val)
        except MPI.MPIError as e:
            out["error"] = str(e)
            rc = -1
        if rc == 0:
            fails.append("no error with a vanished peer (stream-ordered)")
        out["gone_call_s"] = round(time.time() - t0, 3)
        torch.cuda.synchronize()
        out["fails"] = fails
        print(json.dumps(out), flush=True)
        os._exit(1 if fails else 0)
    elif scenario in ("late_p2p", "gone_p2p"):
        last = n - 1
        msg = torch.full((4096,), float(r + 1), device="cuda")
        box = torch.zeros(4096, device="cuda")
        if r == last:
            if scenario == "gone_p2p":
                sys.stdout.flush()
                os._exit(0)
            time.sleep(2.5 * timeout_s)
            MPI.Send(msg, 0, 77, comm)
        elif r == 0:
            t0 = time.time()
            try:
                MPI.Recv_(box, last, 77, comm)
                if scenario == "gone_p2p":
                    fails.append("no error with a vanished sender")
                elif not bool((box == float(last + 1)).all()):
                    fails.append("late message")
            except MPI.MPIError as e:
                out["error"] = str(e)
                if scenario == "late_p2p":
                    fails.append("error waiting for a late sender")
            out["late_call_s" if scenario == "late_p2p" else "gone_call_s"] = round(time.time() - t0, 3)
        if scenario == "gone_p2p":
            out.setdefault("gone_call_s", 0.0)  # ranks other than the receiver wait for nothing
            out["fails"] = fails
            print(json.dumps(out), flush=True)
            os._exit(1 if fails else 0)
        if r != 0:
            out["late_call_s"] = 999.0  # not the waiting rank
        MPI.Barrier(comm)
        MPI.Finalize()
    elif scenario == "broken":
        if r == n - 1:
            MPI.lib().mpigx_comm_diag_break(comm.val)
            try:
                MPI.Allreduce_(send, recv, MPI.SUM, comm)
                fails.append("no error on the broken rank")
            except MPI.MPIError:
                pass
            out["fails"] = fails
            print(json.dumps(out), flush=True)
            os._exit(1 if fails else 0)
        t0 = time.time()
        try:
            MPI.Allreduce_(send, recv, MPI.SUM, comm)
            fails.append("no error with a broken peer")
        except MPI.MPIError as e:
            out["error"] = str(e)
        out["broken_call_s"] = round(time.time() - t0, 3)
        torch.cuda.synchronize()
        out["fails"] = fails
        print(json.dumps(out), flush=True)
        os._exit(1 if fails else 0)
    elif scenario == "gone":
        if r == n - 1:
            sys.stdout.flush()
            os._exit(0)
        t0 = time.time()
        try:
            MPI.Allreduce_(send, recv, MPI.SUM, comm)
            fails.append("no error with a vanished peer")
        except MPI.MPIError as e:
            out["error"] = str(e)
        out["gone_call_s"] = round(time.time() - t0, 3)
        torch.cuda.synchronize()
        out["fails"] = fails
        print(json.dumps(out), flush=True)
        os._exit(1 if fails else 0)  # no Finalize: a peer is gone
    out["fails"] = fails
    print(json.dumps(out), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
