"""Records MPICH 3.3.2's view of the derived datatypes in
tests/spmd/types_cases.py: lb/extent, true lb/extent, size, and MPI_Pack /
MPI_Unpack bytes of a deterministic byte pattern at counts 1 and 3.  Run in
the build container under `mpiexec -n 1` (tests/golden/make_types_golden.sh);
the JSON is committed; tests/test_types_cpu.py (host-side constructors) and
tests/test_types_gpu.py (device pack / unpack kernels) must reproduce it."""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mpi.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "spmd"))

import numpy as np  # noqa: E402

import mpigx as MPI  # noqa: E402
from mpigx import hostmpi  # noqa: E402
from types_cases import build, typed_input  # noqa: E402

comm = MPI.Init()
L = hostmpi.lib()
out = []
for name, dt in build(MPI):
    h = dt.host
    lb, ex, tlb, tex = (ctypes.c_long() for _ in range(4))
    sz = ctypes.c_int()
    L.MPI_Type_get_extent(h, ctypes.byref(lb), ctypes.byref(ex))
    L.MPI_Type_get_true_extent(h, ctypes.byref(tlb), ctypes.byref(tex))
    L.MPI_Type_size(h, ctypes.byref(sz))
    rec = {"name": name, "lb": lb.value, "extent": ex.value, "true_lb": tlb.value, "true_extent": tex.value,
           "size": sz.value, "pack": {}, "unpack": {}}
    for count in (1, 3):
        inp = typed_input(ex.value, tlb.value + tex.value, count)
        packed = np.zeros(max(1, sz.value * count), np.uint8)
        pos = ctypes.c_int(0)
        rc = L.MPI_Pack(ctypes.c_void_p(inp.ctypes.data), count, h, ctypes.c_void_p(packed.ctypes.data),
                        packed.size, ctypes.byref(pos), comm.host)
        assert rc == 0 and pos.value == sz.value * count, (name, rc, pos.value)
        back = np.zeros_like(inp)
        pos = ctypes.c_int(0)
        rc = L.MPI_Unpack(ctypes.c_void_p(packed.ctypes.data), packed.size, ctypes.byref(pos),
                          ctypes.c_void_p(back.ctypes.data), count, h, comm.host)
        assert rc == 0, (name, rc)
        rec["pack"][str(count)] = packed[:sz.value * count].tobytes().hex()
        rec["unpack"][str(count)] = back.tobytes().hex()
    out.append(rec)
json.dump({"source": "MPICH 3.3.2 (/opt/conda) MPI_Type_get_extent / MPI_Type_get_true_extent / MPI_Type_size / "
                     "MPI_Pack / MPI_Unpack over tests/spmd/types_cases.py", "types": out},
          open(os.path.join(HERE, "types_golden.json"), "w"), indent=None, separators=(",", ":"))
MPI.Finalize()
