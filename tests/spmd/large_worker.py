"""SPMD worker: the MPICH-recorded large-count fixtures (tests/golden/
mpich_large.npz, recorded by make_large_golden.sh with MPICH 3.3.2) through
the HIP path, at the headline regime where the Rabenseifner pre-step operand
roles matter (even rank inout; NaN on the odd rank of a pair under MAX):

* Allreduce! / Reduce! at 4,194,307 elements — f32 SUM, f64 SUM, f32 MAX with
  +-0 / +-inf / NaN / denormal edges — through the default path (the tuner's
  sampling calls included), pull, push, pull-push, pull_generic (the
  all-modes fold kernel), the staged two-shot (zero-copy off) and the staged
  one-shot rounds;
* Scan! / Exscan! at 1,048,579 elements (Int64 BOR, f64 SUM) staged and
  zero-copy.

Inputs are regenerated from the fixture's splitmix64 seeds
(gen_inputs.splitmix_input); the recorded output spans (prefix, tail, +-64
elements around every Rabenseifner block boundary) are compared bit for bit
(any NaN matches any NaN: x86 and AMDGPU generate different payloads).
Launched by tests/test_large_gpu.py at n = 5 and 8 (the fixture's rank
counts), all ranks on the test box's one GPU."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "mpi.jl_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mpigx as MPI  # noqa: E402
from gen_inputs import splitmix_input  # noqa: E402
from golden_io import same_bits  # noqa: E402

OPS = {"SUM": MPI.SUM, "MAX": MPI.MAX, "BOR": MPI.BOR}
TORCH = {"f32": torch.float32, "f64": torch.float64, "i64": torch.int64}

# (name, knobs); "staged" switches the zero-copy paths off, "zc" lowers the
# zero-copy threshold under the 8 MiB prefix-collective cases
REDUCE_ALGOS = (("auto", {}), ("pull", {"ALGO": "pull"}), ("push", {"ALGO": "push"}),
                ("pullpush", {"ALGO": "pullpush"}), ("pull_generic", {"ALGO": "pull_generic"}),
                ("staged_twoshot", {"ZC_MIN": 0, "ALGO": "twoshot"}), ("staged_oneshot", {"ZC_MIN": 0, "ALGO": "oneshot"}))
ROOTED_ALGOS = (("auto", {}), ("pull_generic", {"ALGO": "pull_generic"}), ("staged", {"ZC_MIN": 0}))
SCAN_ALGOS = (("staged", {}), ("zc", {"ZC_MIN": 1 << 20}))


def main():
    comm = MPI.Init()
    r, n = MPI.Comm_rank(comm), MPI.Comm_size(comm)
    dev = torch.device("cuda")
    with open(os.path.join(ROOT, "tests", "golden", "mpich_large_manifest.json")) as f:
        cases = [c for c in json.load(f) if c["n"] == n]
    arr = np.load(os.path.join(ROOT, "tests", "golden", "mpich_large.npz"))
    defaults = {k: MPI.get_knob(comm, k) for k in ("ALGO", "ZC_MIN")}
    fails, checked = [], 0

    def with_knobs(knobs):
        for k in ("ALGO", "ZC_MIN"):
            MPI.set_knob(comm, k, knobs.get(k, None if k == "ALGO" else defaults[k]))

    for case in cases:
        coll, kind, count = case["coll"], case["kind"], case["count"]
        x = splitmix_input(kind, case["seed"], r, count, bool(case["edge"]))
        send = torch.from_numpy(np.ascontiguousarray(x)).to(dev)
        op = OPS[case["op"]]
        if coll in ("allreduce", "reduce"):
            algos = REDUCE_ALGOS if coll == "allreduce" else ROOTED_ALGOS
            root = case["root"]
            want_rank = 0 if coll == "allreduce" else root
            exp = arr[f"{case['id']}.r{want_rank}"]
            for name, knobs in algos:
                with_knobs(knobs)
                recv = torch.empty_like(send) if (coll == "allreduce" or r == root) else None
                for call in range(4 if name == "auto" else 1):  # auto: the tuner's sampling calls
                    if recv is not None:
                        recv.fill_(0)
                    if coll == "allreduce":
                        MPI.Allreduce_(send, recv, op, comm)
                    else:
                        MPI.Reduce_(send, recv, op, root, comm)
                    if recv is None:
                        continue
                    got = recv.cpu().numpy()
                    part = np.concatenate([got[lo:hi] for lo, hi in case["spans"]])
                    checked += 1
                    if not same_bits(part.view(got.dtype), exp.view(got.dtype)):
                        bad = np.nonzero(~_eq(part, exp.view(got.dtype)))[0]
                        fails.append((case["id"], name, call, int(bad.size), int(bad[0])))
                        break
                del recv
        else:
            excl = coll == "exscan"
            for name, knobs in SCAN_ALGOS:
                with_knobs(knobs)
                recv = torch.full_like(send, 7) if excl else torch.empty_like(send)
                (MPI.Exscan_ if excl else MPI.Scan_)(send, recv, op, comm)
                got = recv.cpu().numpy()
                checked += 1
                if excl and r == 0:
                    if not (got == 7).all():  # rank 0's recvbuf untouched (collective.jl Exscan!)
                        fails.append((case["id"], name, "rank0-touched"))
                    continue
                exp = arr[f"{case['id']}.r{r}"].view(got.dtype)
                part = np.concatenate([got[lo:hi] for lo, hi in case["spans"]])
                if not same_bits(part, exp):
                    bad = np.nonzero(~_eq(part, exp))[0]
                    fails.append((case["id"], name, int(bad.size), int(bad[0])))
                del recv
        del send
    with_knobs({})
    MPI.Barrier(comm)
    pm = list(MPI.peer_memory(comm))  # signalling protocol per peer pair (rw_mask, same_device)
    MPI.Finalize()
    print(json.dumps({"rank": r, "n": n, "peer_mem": pm, "cases": len(cases), "checked": checked, "nfail": len(fails),
                      "failures": [str(f) for f in fails[:20]]}), flush=True)
    sys.exit(1 if fails else 0)


def _eq(a, b):
    if a.dtype.kind == "f":
        return (a.view(np.uint8).reshape(a.size, -1) == b.view(np.uint8).reshape(b.size, -1)).all(1) | \
            (np.isnan(a) & np.isnan(b))
    return a == b


if __name__ == "__main__":
    main()
