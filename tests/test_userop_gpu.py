"""User-defined ops on device buffers (operators.jl:56-88).
tests/spmd/userop_worker.py — test_allreduce.jl / test_reduce.jl's custom
`(x, y) -> 2x + y - x`, and a non-commutative affine-composition op over a
contiguous derived pair type through Allreduce / Reduce / Scan / Exscan — on
ROCm tensors must reproduce MPICH's MPI_Op_create results
(tests/golden/userop_golden.json) through BOTH engine paths: the device
callback (torch ops on device pointers) and the host-staged
MPI_User_function callback (what MPI.jl's @cfunction(OpWrapper) binds) —
and, "libmpi", an op handed over as the reference's MPI.Op(f, T) holds it (a
libmpi handle plus that function pointer), which the API re-registers with
libmpigx; the same handle without a function stays MPI_ERR_OP."""
import json
import os

import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_MAX_BLOCKS": "16", "MPIGX_TIMEOUT_MS": "30000",
       "MPIGX_STAGING_BYTES": str(32 << 20), "MPIGX_TEST_ARRAYTYPE": "ROCArray"}


@pytest.mark.parametrize("n", [2, 3, 4])
@pytest.mark.parametrize("hostcb", ["0", "1", "libmpi"])
def test_user_ops_device_match_mpich(n, hostcb, tmp_path):
    """(~29 s) User ops (host-staged, device callback, libmpi MPI_Op_create) reproduce MPICH's results at n = 2, 3, 4."""
    env = dict(ENV, UO_OUT=str(tmp_path / "uo"), USEROP_HOSTCB=hostcb)
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "userop_worker.py"), n, timeout=300, extra_env=env)
    recs = {}
    for r in range(n):
        p = tmp_path / f"uo.{r}"
        if p.exists():
            recs[r] = json.loads(p.read_text())
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}\n{recs.get(r, {}).get('failed')}"
                    for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    with open(os.path.join(ROOT, "tests", "golden", "userop_golden.json")) as f:
        gold = json.load(f)["runs"][str(n)]
    for r in range(n):
        assert recs[r]["device"] is True and recs[r]["failed"] is None
        assert recs[r]["records"] == gold[r], (r, recs[r]["records"], gold[r])
