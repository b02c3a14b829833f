"""Derived datatypes on device buffers.

* The device pack / unpack kernels (mpigx_pack / mpigx_unpack, types.cpp
  pack_kernel) must produce exactly the bytes MPICH 3.3.2's MPI_Pack /
  MPI_Unpack produce for every type of tests/spmd/types_cases.py at counts 1
  and 3 (tests/golden/types_golden.json) — gaps left untouched by unpack.
* tests/spmd/dtype_worker.py — the reference's test_subarray.jl and
  test_datatype.jl restated, plus Bcast / Allgather / Alltoall / Gather /
  Scatter with struct, vector and subarray types — on ROCm tensors must
  reproduce the records MPICH produced on host arrays
  (tests/golden/dtype_golden.json) at 2, 3 and 4 ranks sharing the GPU."""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

from spmd_launch import ROOT, launch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "spmd"))


def test_pack_unpack_match_mpich():
    """(~1 s) MPI_Pack / MPI_Unpack bytes equal MPICH's for the recorded derived types."""
    import torch

    import mpigx as MPI
    from types_cases import build, typed_input

    with open(os.path.join(HERE, "golden", "types_golden.json")) as f:
        gold = {t["name"]: t for t in json.load(f)["types"]}
    dev = torch.device("cuda:0")
    L = MPI.lib()
    for name, dt in build(MPI):
        g = gold[name]
        for count in (1, 3):
            inp = typed_input(g["extent"], g["true_lb"] + g["true_extent"], count)
            d_in = torch.from_numpy(inp).to(dev)
            nb = g["size"] * count
            d_pk = torch.zeros(max(1, nb), dtype=torch.uint8, device=dev)
            pos = ctypes.c_longlong(0)
            assert L.mpigx_pack(ctypes.c_void_p(d_in.data_ptr()), count, dt.val, ctypes.c_void_p(d_pk.data_ptr()),
                                d_pk.numel(), ctypes.byref(pos), None) == 0
            assert pos.value == nb
            assert d_pk.cpu().numpy()[:nb].tobytes().hex() == g["pack"][str(count)], (name, count)
            back = torch.zeros_like(d_in)
            pos = ctypes.c_longlong(0)
            assert L.mpigx_unpack(ctypes.c_void_p(d_pk.data_ptr()), d_pk.numel(), ctypes.byref(pos),
                                  ctypes.c_void_p(back.data_ptr()), count, dt.val, None) == 0
            assert back.cpu().numpy().tobytes().hex() == g["unpack"][str(count)], (name, count)


ENV = {"MPIGX_DEVICE": "0", "MPIGX_INIT_TIMEOUT_MS": "60000", "MPIGX_MAX_BLOCKS": "16", "MPIGX_TIMEOUT_MS": "30000",
       "MPIGX_STAGING_BYTES": str(32 << 20), "MPIGX_TEST_ARRAYTYPE": "ROCArray"}


@pytest.mark.parametrize("n", [2, 3, 4])
def test_dtype_scenarios_device_match_mpich(n, tmp_path):
    """(~10 s) Derived-datatype collectives and p2p reproduce MPICH records at n = 2, 3, 4."""
    env = dict(ENV, DT_OUT=str(tmp_path / "dt"))
    rcs, outs = launch(os.path.join(ROOT, "tests", "spmd", "dtype_worker.py"), n, timeout=600, extra_env=env)
    recs = {}
    for r in range(n):
        p = tmp_path / f"dt.{r}"
        if p.exists():
            recs[r] = json.loads(p.read_text())
    msg = "\n".join(f"--- rank {r} rc={rc}\n{o[-3000:]}\n{recs.get(r, {}).get('failed')}"
                    for r, (rc, o) in enumerate(zip(rcs, outs)))
    assert all(rc == 0 for rc in rcs), msg
    with open(os.path.join(ROOT, "tests", "golden", "dtype_golden.json")) as f:
        gold = json.load(f)["runs"][str(n)]
    for r in range(n):
        assert recs[r]["device"] is True and recs[r]["failed"] is None
        assert len(recs[r]["dev_checks"]) == 2 and all(c["ok"] for c in recs[r]["dev_checks"]), recs[r]["dev_checks"]
        assert len(recs[r]["records"]) == len(gold[r])
        for got, want in zip(recs[r]["records"], gold[r]):
            assert got == want, (r, got, want)
