"""Config 1 (plumbing, no GPU): MPI.jl's own collective test scripts,
restated on the Python mirror (tests/spmd/ref_tests.py), run on host arrays
under `mpiexec -n 4` — the reference's test strategy (test/runtests.jl:28-45)
with libmpi = MPICH 3.3.2.  Exercises the mirror's argument handling
(asserts, IN_PLACE, count defaults, allocating and scalar forms, user ops via
MPI_Op_create) end to end."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = "/opt/conda/bin/mpiexec"


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="needs MPICH (/opt/conda)")
@pytest.mark.parametrize("n", [2, 4])
def test_reference_suite_host(n):
    env = dict(os.environ, MPIGX_HOST_ONLY="1", OMP_NUM_THREADS="1")
    p = subprocess.run([MPIEXEC, "-n", str(n), sys.executable, os.path.join(ROOT, "tests", "spmd", "ref_tests.py")],
                       env=env, capture_output=True, text=True, timeout=600)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert len(lines) == n and all('"nfail": 0' in l for l in lines), lines
