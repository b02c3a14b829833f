"""Operand generator of the RMA accumulate matrix (tests/spmd/rma_worker.py),
shared with the CPU oracle test (tests/test_rma_oracle.py) so both see the
same values."""
import numpy as np

TYPES = [np.int8, np.uint8, np.int16, np.uint16, np.int32, np.uint32, np.int64, np.uint64, np.float32, np.float64,
         np.complex64, np.complex128]
OPS = ["SUM", "PROD", "MIN", "MAX", "LAND", "LOR", "LXOR", "BAND", "BOR", "BXOR", "REPLACE", "NO_OP"]
K = 12


def operands(dt, opname, who, salt):
    """Deterministic window / origin values for rank `who`."""
    rng = np.random.default_rng(1000 * who + salt)
    d = np.dtype(dt)
    if d.kind in "iu":
        info = np.iinfo(d)
        if opname in ("SUM", "PROD"):
            v = rng.integers(info.min // 2 if d.kind == "i" else 0, info.max // 2, K, dtype=np.int64, endpoint=True)
            v = v.astype(d)
            v[0] = info.max  # wraparound
        else:
            v = rng.integers(-3 if d.kind == "i" else 0, 4, K).astype(d)
        return v
    if d.kind == "f":
        v = rng.integers(-4, 5, K).astype(d) * d.type(0.5)
        if opname in ("MIN", "MAX", "LAND", "LOR", "LXOR", "REPLACE", "NO_OP"):
            v[1] = np.nan if who % 2 else v[1]
            v[2] = d.type(-0.0) if who % 2 else d.type(0.0)
            v[3] = d.type(2.0)
        return v
    re = rng.integers(-3, 4, K).astype(np.float64)
    im = rng.integers(-3, 4, K).astype(np.float64)
    return (re + 1j * im).astype(d)
