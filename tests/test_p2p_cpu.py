"""Point-to-point, CPU side:

* the scenario script (tests/spmd/p2p_worker.py) on host arrays under MPICH
  reproduces the committed golden fixture (tests/golden/p2p_golden.json) —
  i.e. the fixture is deterministic and the mirror's host path is the
  reference's own libmpi path;
* p2p constants of include/mpigx.h are MPICH's and the Status layout is the
  20-byte MPI_Status (pointtopoint.jl:4-60 asserts the same offsets).
"""
import ctypes
import json
import os
import re
import subprocess
import sys

import pytest

import mpigx
from mpigx import consts as C

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MPIEXEC = "/opt/conda/bin/mpiexec"
GOLDEN = os.path.join(ROOT, "tests", "golden", "p2p_golden.json")


def golden_runs():
    with open(GOLDEN) as f:
        return json.load(f)["runs"]


def records_of(stdout):
    recs = {}
    for line in stdout.splitlines():
        if line.startswith("{") and '"records"' in line:
            d = json.loads(line)
            assert d["failed"] is None, d["failed"]
            recs[d["rank"]] = d["records"]
    return recs


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="needs MPICH (/opt/conda)")
@pytest.mark.parametrize("n", [2, 3])
def test_p2p_scenarios_host_match_golden(n):
    env = dict(os.environ, MPIGX_HOST_ONLY="1", OMP_NUM_THREADS="1")
    p = subprocess.run([MPIEXEC, "-n", str(n), sys.executable, os.path.join(ROOT, "tests", "spmd", "p2p_worker.py")],
                       env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    recs = records_of(p.stdout)
    gold = golden_runs()[str(n)]
    for r in range(n):
        assert recs[r] == gold[r], (r, recs[r], gold[r])


def test_golden_covers_semantics():
    gold = golden_runs()
    assert sorted(gold) == ["2", "3", "4"]
    cases = {rec["case"] for rec in gold["2"][0]}
    for c in ("ring_waitall", "chain", "waitsome", "null_arrays", "waitany_self", "cancel", "procnull", "truncation",
              "probe_self", "tag_order", "many_outstanding", "sendrecv", "big", "errors"):
        assert c in cases
    r1 = {rec["case"]: rec for rec in gold["2"][1]}
    assert r1["truncation"]["err"] == C.MPI_ERR_TRUNCATE
    assert r1["truncation"]["counts"] == [C.MPI_UNDEFINED, 3, C.MPI_UNDEFINED]
    assert r1["null_arrays"]["testany"] == [True, 0, None]


def test_p2p_header_constants():
    with open(mpigx.HEADER_PATH) as f:
        txt = f.read()
    d = {k: int(v, 0) for k, v in re.findall(r"#define\s+(MPIGX_\w+)\s+\(?(-?(?:0x)?[0-9a-fA-F]+)\)?", txt)}
    for name in ("ERR_TAG", "ERR_RANK", "ERR_TRUNCATE", "ERR_IN_STATUS", "ERR_REQUEST", "ANY_SOURCE", "ANY_TAG",
                 "PROC_NULL", "UNDEFINED", "REQUEST_NULL", "TAG_UB"):
        assert d[f"MPIGX_{name}"] == getattr(C, f"MPI_{name}"), name


def test_status_layout_and_get_count():
    assert ctypes.sizeof(mpigx.Status) == 20
    s = mpigx.Status(24, 0, 1, 7, 0)
    assert mpigx.Get_count(s, mpigx.Datatype(__import__("numpy").float64)) == 3
    assert mpigx.Get_count(s, mpigx.Datatype(__import__("numpy").int16)) == 12
    s = mpigx.Status(3, 1, 0, 0, 0)
    assert mpigx.Get_count(s, mpigx.Datatype(__import__("numpy").float64)) == C.MPI_UNDEFINED
    assert mpigx.Test_cancelled(s)
    assert mpigx.STATUS_EMPTY == mpigx.Status(0, 0, C.MPI_ANY_SOURCE, C.MPI_ANY_TAG, 0)


def test_null_request_calls_need_no_gpu():
    """Null-request completion calls are pure host logic (no device touched)."""
    L = mpigx.lib()
    h = (ctypes.c_int * 2)(C.MPI_REQUEST_NULL, C.MPI_REQUEST_NULL)
    idx, flag, out = ctypes.c_int(0), ctypes.c_int(0), ctypes.c_int(0)
    st = mpigx.Status(9, 9, 9, 9, 9)
    assert L.mpigx_waitany(2, h, ctypes.byref(idx), ctypes.byref(st)) == 0
    assert idx.value == C.MPI_UNDEFINED and (st.source, st.tag, st.count_lo, st.error) == (-2, -1, 0, 9)
    assert L.mpigx_testany(2, h, ctypes.byref(idx), ctypes.byref(flag), ctypes.byref(st)) == 0
    assert flag.value == 1 and idx.value == C.MPI_UNDEFINED
    assert L.mpigx_waitsome(2, h, ctypes.byref(out), None, None) == 0 and out.value == C.MPI_UNDEFINED
    assert L.mpigx_testsome(2, h, ctypes.byref(out), None, None) == 0 and out.value == C.MPI_UNDEFINED
    bad = ctypes.c_int(0x6c00ffff)
    assert L.mpigx_wait(ctypes.byref(bad), None) == C.MPI_ERR_REQUEST


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="needs MPICH (/opt/conda)")
@pytest.mark.parametrize("seed", [7, 11])
def test_matching_model_pinned_by_mpich(seed):
    """oracle/p2p_model.match_unexpected_first predicts which message every
    receive gets; MPICH agrees on random traffic (sizes, tags, ANY_TAG)."""
    env = dict(os.environ, MPIGX_HOST_ONLY="1", OMP_NUM_THREADS="1", P2P_SEED=str(seed))
    p = subprocess.run([MPIEXEC, "-n", "3", sys.executable,
                        os.path.join(ROOT, "tests", "spmd", "p2p_random_worker.py")],
                       env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 3 and all(d["nbad"] == 0 and d["failed"] is None for d in lines), lines
    assert sum(d["checks"] for d in lines) > 40


def test_matching_model_matches_golden_tag_order():
    from oracle.p2p_model import ANY_TAG, match_posted_first, match_unexpected_first
    tags = [5, 6, 5, 7, 6]
    pattern = [7, 5, ANY_TAG, 5, 6]
    arrived = [(0, t, k) for k, t in enumerate(tags)]
    recvs = [(0, t) for t in pattern]
    want = [r for r in golden_runs()["2"][1] if r["case"] == "tag_order"][0]
    assert [float(k) for k in match_unexpected_first(arrived, recvs)] == want["unexpected_first"]["data"]
    assert [float(k) for k in match_posted_first(recvs, arrived)] == want["posted_first"]["data"]
