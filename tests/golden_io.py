"""Loader for the MPICH golden fixtures (tests/golden/, made by make_golden.sh)."""
import json
import os

import numpy as np

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load():
    with open(os.path.join(HERE, "mpich_golden_manifest.json")) as f:
        cases = json.load(f)
    arrays = np.load(os.path.join(HERE, "mpich_golden.npz"), allow_pickle=False)
    return cases, arrays


def op_type_matrix():
    with open(os.path.join(HERE, "op_type_matrix.json")) as f:
        return json.load(f)


def typed(raw_rows, npdtype):
    """[n, bytes] uint8 -> list of per-rank typed arrays."""
    return [np.ascontiguousarray(r).view(npdtype) for r in raw_rows]


def same_bits(a, b, bf16=False):
    """Bitwise equality, except any NaN matches any NaN (payloads and the sign
    of a generated NaN differ by ISA: x86 default NaN is 0xFFC00000, AMDGPU
    0x7FC00000).  bf16=True compares uint16 bf16 patterns that way too."""
    a = np.asarray(a)
    b = np.asarray(b)
    if bf16:
        a = (a.astype(np.uint32) << 16).view(np.float32)
        b = (b.astype(np.uint32) << 16).view(np.float32)
    if a.shape != b.shape:
        return False
    if a.dtype.kind in "fc":
        fa = a.view(a.real.dtype) if a.dtype.kind == "c" else a
        fb = b.view(b.real.dtype) if b.dtype.kind == "c" else b
        na, nb = np.isnan(fa), np.isnan(fb)
        if not np.array_equal(na, nb):
            return False
        return np.array_equal(fa[~na].view(np.uint8 if False else fa.dtype).tobytes(), fb[~nb].tobytes()) and \
            np.array_equal(np.signbit(fa[~na]), np.signbit(fb[~nb]))
    return np.array_equal(a.view(np.uint8), b.view(np.uint8))
