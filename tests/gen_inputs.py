"""Seeded synthetic inputs (numpy) for parity tests, per MPI datatype name."""
import numpy as np

from oracle import mpich_model as M


def make(dtname, opname, n, count, seed, edge=False):
    """n per-rank arrays of `count` elements of MPI type `dtname`."""
    rng = np.random.default_rng(seed)
    npdt = M.DTYPES[dtname][1]
    kind = M.DTYPES[dtname][2]
    logical = opname in M.LOGICAL
    out = []
    for r in range(n):
        if kind in ("int", "uint", "byte"):
            info = np.iinfo(npdt)
            x = rng.integers(info.min, info.max, size=count, dtype=npdt, endpoint=True)
            if opname == "PROD":
                x = rng.integers(-3 if kind == "int" else 0, 4, size=count).astype(npdt)
        elif kind == "float":
            x = rng.uniform(-1, 1, size=count).astype(npdt)
            if edge and count:
                e = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45 if npdt == np.float32 else 5e-324],
                             dtype=npdt)
                idx = rng.integers(0, count, size=max(1, count // 8))
                x[idx] = e[rng.integers(0, len(e), size=idx.size)]
        elif kind == "complex":
            x = (rng.uniform(-1, 1, size=count) + 1j * rng.uniform(-1, 1, size=count)).astype(npdt)
        elif kind == "bf16":
            f = rng.uniform(-1, 1, size=count).astype(np.float32)
            x = M.f32_to_bf16(f)
            if edge and count:
                e = M.f32_to_bf16(np.array([0.0, -0.0, np.inf, -np.inf, np.nan], dtype=np.float32))
                idx = rng.integers(0, count, size=max(1, count // 8))
                x[idx] = e[rng.integers(0, len(e), size=idx.size)]
        else:
            raise KeyError(dtname)
        if logical and count:
            z = rng.random(count) < 0.35
            x = x.copy()
            x[z] = 0
        out.append(np.ascontiguousarray(x))
    return out


def valid_pairs(dtypes=None):
    names = dtypes or [d for d in M.DTYPES if M.DTYPES[d][2] != "none"]
    return [(d, o) for d in names for o in M.OPS if M.op_valid(d, o) == 0]
