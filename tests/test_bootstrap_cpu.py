"""world_size 2/3 gloo test (CPU) of the N>1 bootstrap: rank 0's unique id
must reach every rank bit-exactly (the step MPI_Bcast plays in the Julia
glue)."""
import os

import pytest

from spmd_launch import ROOT, launch


@pytest.mark.parametrize("n", [2, 3])
def test_unique_id_broadcast(n):
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "bootstrap_worker.py"), n, timeout=180,
                       extra_env={"CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""})
    assert all(rc == 0 for rc in rcs), outs
    ids = [l.split()[2] for o in outs for l in o.splitlines() if l.startswith("BOOT")]
    assert len(ids) == n and len(set(ids)) == 1
