"""Randomized parity sweep (tests/spmd/fuzz_worker.py): seeded random
collectives — every valid (op, type) pair, counts across the LL / one-shot /
two-shot / zero-copy thresholds, unaligned buffers, IN_PLACE, every root,
every Allreduce algorithm — plus Gatherv / Scatterv / Allgatherv /
Alltoallv with random counts (zeros included) and gapped displacements
(the gaps must stay untouched) and the local MPI.Op kernel over 2-16
unaligned inputs, against the MPICH-pinned oracle, bit for bit (any NaN =
any NaN).  The zero-copy threshold is lowered to 1 MiB so the
zero-copy kernels see odd counts and unaligned buffers too.  Run with the
same-GPU protocol and, at n = 3 and 8, with the cross-GPU one
(MPIGX_PEER_MEM=xdev, no host gate)."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_TIMEOUT_MS": "30000",
       "MPIGX_ZC_MIN": str(1 << 20), "FUZZ_CASES": os.environ.get("FUZZ_CASES", "120")}
# a longer campaign: FUZZ_SEED_BASE shifts every seed, FUZZ_CASES raises the
# case count (profiles/r05zo_*)
SEED_BASE = int(os.environ.get("FUZZ_SEED_BASE", 0))
XDEV = dict(ENV, MPIGX_PEER_MEM="xdev", MPIGX_SHARED_GATE="0")


@pytest.mark.parametrize("cfg,n,seed", [("same", 2, 11), ("same", 3, 12), ("same", 5, 13), ("same", 8, 14),
                                        ("xdev", 3, 15), ("xdev", 8, 16)])
def test_fuzz_collectives(cfg, n, seed):
    """(~38 s) Seeded random collectives (every valid (op, type), counts across every algorithm threshold, unaligned buffers, IN_PLACE, every root and Allreduce algorithm, float edge values), random v-collectives and local folds, bit for bit against the MPICH-pinned oracle."""
    env = dict(ENV if cfg == "same" else XDEV, FUZZ_SEED=str(seed + SEED_BASE))
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "fuzz_worker.py"), n, timeout=600, extra_env=env)
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}" for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    res = [json.loads(l) for o in outs for l in o.splitlines() if l.startswith("{") and '"nfail"' in l]
    assert len(res) == n, msg
    print(json.dumps({"cfg": cfg, "n": n, "seed": seed + SEED_BASE, "ran_per_rank": [x["ran"] for x in res],
                      "nfail": sum(x["nfail"] for x in res)}), flush=True)  # shown with -s
    assert all(x["nfail"] == 0 and x["ran"] >= 100 for x in res), [x for x in res if x["nfail"]][:2]
