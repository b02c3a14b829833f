"""SPMD worker for the communicator-agreement guards (one scenario per launch,
MPIGX_TEST_SCENARIO):

* mismatch_init   — rank 1 alone sets MPIGX_ALGO=ring: every rank's Init must
                    fail with MPI_ERR_ARG at once (knobs are compared at init),
                    not spin until the device timeout;
* bad_name        — an unknown MPIGX_ALGO fails Init with MPI_ERR_ARG;
* set_knob        — mpigx_comm_set_knob is collective: differing values give
                    MPI_ERR_ARG on every rank and change nothing; agreed values
                    switch the algorithm (ring / push / pull_generic / oneshot,
                    results checked against the oracle); init-only knobs reject;
* share           — ranks sharing the GPU: device_share reports them and the
                    compute units per rank; with MAX_BLOCKS raised to 1024 the
                    per-kernel residency caps still keep every grid resident;
* share_limit     — MPIGX_MAX_RANKS_PER_DEVICE below the ranks on the GPU:
                    Init fails with MPI_ERR_OTHER at once;
* import_fail     — rank 1 fails its first peer import (MPIGX_TEST_IMPORT_FAIL):
                    the zero-copy exchange agrees on the failure and every rank
                    takes the staged path, stream-ordered and blocking, with
                    the right result (the failure used to leave recvbuf
                    unwritten on the other ranks in stream-ordered mode);
* ll_wrap         — MPIGX_EPOCH_BASE just below 2^31: LL launches cross the LL
                    flag generation (the area is cleared there), blocking and
                    stream-ordered, every result vs the oracle.
Launched by tests/test_knobs_gpu.py; prints one JSON line per rank.
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "mpi.jl_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpigx as MPI  # noqa: E402
from gen_inputs import make  # noqa: E402
from golden_io import same_bits  # noqa: E402
from oracle import mpich_model as M  # noqa: E402


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to("cuda")


def main():
    sc = os.environ["MPIGX_TEST_SCENARIO"]
    rank, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    fails, out = [], {"rank": rank, "scenario": sc}
    if sc == "mismatch_init" and rank == 1:
        os.environ["MPIGX_ALGO"] = "ring"
    if sc == "import_fail" and rank == 1:
        os.environ["MPIGX_TEST_IMPORT_FAIL"] = "1"
    if sc in ("mismatch_init", "bad_name", "share_limit"):
        t0 = time.time()
        try:
            MPI.Init()
            fails.append("init succeeded")
        except MPI.MPIError as e:
            out["code"] = e.code
            want = MPI.consts.MPI_ERR_OTHER if sc == "share_limit" else MPI.consts.MPI_ERR_ARG
            if e.code != want:
                fails.append(("code", e.code))
        out["init_s"] = round(time.time() - t0, 2)
        if out["init_s"] > 20:
            fails.append(("slow", out["init_s"]))
    else:
        comm = MPI.Init()
        r = MPI.Comm_rank(comm)
        if sc == "set_knob":
            try:
                MPI.set_knob(comm, "ALGO", "ring" if r == 0 else "push")
                fails.append("mismatched set_knob accepted")
            except MPI.MPIError as e:
                if e.code != MPI.consts.MPI_ERR_ARG:
                    fails.append(("mismatch code", e.code))
            if MPI.get_knob(comm, "ALGO") != 0:
                fails.append("mismatched set_knob changed the knob")
            for knob in ("STAGING_BYTES", "LL_MAX"):
                try:
                    MPI.set_knob(comm, knob, 1 << 20)
                    fails.append(("init-only knob set", knob))
                except MPI.MPIError:
                    pass
            MPI.set_knob(comm, "ZC_MIN", 1)
            for algo in ("ring", "push", "pull", "pull_generic", "pullpush", "oneshot", "twoshot", "ll", None):
                MPI.set_knob(comm, "ALGO", algo)
                if MPI.get_knob(comm, "ALGO") != MPI.ALGOS[algo]:
                    fails.append(("get_knob", algo))
                ins = make("INT32_T", "SUM", n, 50_001, 31)
                recv = torch.empty(50_001, dtype=torch.int32, device="cuda")
                MPI.Allreduce_(dev(ins[r]), recv, MPI.SUM, comm)
                if not same_bits(recv.cpu().numpy(), M.allreduce(ins, "INT32_T", "SUM")[r]):
                    fails.append(("result", algo))
            # the pull-push two-shot's dynamic slice hand-out: ticket counters
            # carry over launches (monotone bases), across slice counts, the
            # static variant and other algorithms in between
            MPI.set_knob(comm, "ALGO", "pullpush")
            for count in (50_001, (3 << 20) + 5):
                ins = make("FLOAT", "SUM", n, count, 41)
                exp = M.allreduce(ins, "FLOAT", "SUM")[r]
                src = dev(ins[r])
                for slices in (0, 1, 7, 64, 4, 0, 4):
                    MPI.set_knob(comm, "AR_SLICES", slices)
                    if MPI.get_knob(comm, "AR_SLICES") != slices:
                        fails.append(("AR_SLICES knob", slices))
                    for _ in range(2):
                        recv = torch.zeros(count, dtype=torch.float32, device="cuda")
                        MPI.Allreduce_(src, recv, MPI.SUM, comm)
                        if not same_bits(recv.cpu().numpy(), exp):
                            fails.append(("pullpush slices", count, slices))
                    MPI.set_knob(comm, "ALGO", "pull")
                    MPI.Allreduce_(src, recv, MPI.SUM, comm)
                    MPI.set_knob(comm, "ALGO", "pullpush")
            MPI.set_knob(comm, "AR_SLICES", 0)
            MPI.set_knob(comm, "ALGO", None)
            MPI.set_knob(comm, "ZC_MIN", 16 << 20)
        elif sc == "share":
            ranks, cap = MPI.device_share(comm)
            out.update(ranks_per_device=ranks, cap=cap, max_blocks=MPI.get_knob(comm, "MAX_BLOCKS"))
            cus = torch.cuda.get_device_properties(0).multi_processor_count
            if ranks != n:
                fails.append(("ranks", ranks))
            # cap = compute units per rank on the shared device; each launch's
            # grid is capped at cap x that kernel's resident blocks per CU
            if cap != cus // ranks:
                fails.append(("cap", cap))
            MPI.set_knob(comm, "MAX_BLOCKS", 1024)  # the per-kernel caps keep every grid resident
            if MPI.get_knob(comm, "MAX_BLOCKS") != 1024:
                fails.append("MAX_BLOCKS knob")
            ins = make("FLOAT", "SUM", n, (64 << 20) // 4 + 3, 77)  # zero-copy two-shot at the full grid
            recv = torch.empty(ins[r].size, dtype=torch.float32, device="cuda")
            MPI.Allreduce_(dev(ins[r]), recv, MPI.SUM, comm)
            if not same_bits(recv.cpu().numpy(), M.allreduce(ins, "FLOAT", "SUM")[r]):
                fails.append("full-grid allreduce")
        elif sc == "import_fail":
            count = (32 << 20) // 4  # zero-copy size
            ins = make("INT64_T", "BXOR", n, count // 2, 55)
            exp = M.allreduce(ins, "INT64_T", "BXOR")[r]
            s = dev(ins[r])
            MPI.lib().mpigx_comm_set_blocking(comm.val, 0)  # stream-ordered: no abort verdict reaches the host
            d = torch.zeros_like(s)
            MPI.Allreduce_(s, d, MPI.BXOR, comm)
            MPI.lib().mpigx_comm_synchronize(comm.val)
            MPI.lib().mpigx_comm_set_blocking(comm.val, 1)
            if not same_bits(d.cpu().numpy(), exp):
                fails.append("stream-ordered result after a failed import")
            d2 = torch.zeros_like(s)
            MPI.Allreduce_(s, d2, MPI.BXOR, comm)  # blocking, imports now succeed
            if not same_bits(d2.cpu().numpy(), exp):
                fails.append("blocking result after a failed import")
        elif sc == "ll_wrap":
            cases = []
            for k in range(48):
                cnt = (1, 7, 512, 4000)[k % 4] + k
                cases.append(make("FLOAT", "SUM", n, cnt, 900 + k))
            # 24 stream-ordered LL launches, then 24 blocking ones; the test
            # sets MPIGX_EPOCH_BASE so that 2^31 falls inside one or the other
            MPI.lib().mpigx_comm_set_blocking(comm.val, 0)
            pairs = [(dev(ins[r]), torch.empty(ins[r].size, dtype=torch.float32, device="cuda")) for ins in cases[:24]]
            for s, d in pairs:
                MPI.Allreduce_(s, d, MPI.SUM, comm)
            MPI.lib().mpigx_comm_synchronize(comm.val)
            MPI.lib().mpigx_comm_set_blocking(comm.val, 1)
            for k, (ins, (s, d)) in enumerate(zip(cases[:24], pairs)):
                if not same_bits(d.cpu().numpy(), M.allreduce(ins, "FLOAT", "SUM")[r]):
                    fails.append(("ll-stream", k))
            for k, ins in enumerate(cases[24:]):
                recv = torch.empty(ins[r].size, dtype=torch.float32, device="cuda")
                MPI.Allreduce_(dev(ins[r]), recv, MPI.SUM, comm)
                if not same_bits(recv.cpu().numpy(), M.allreduce(ins, "FLOAT", "SUM")[r]):
                    fails.append(("ll-blocking", k))
        MPI.Barrier(comm)
        MPI.Finalize()
    out.update(nfail=len(fails), failures=[str(f) for f in fails[:20]])
    print(json.dumps(out), flush=True)
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
