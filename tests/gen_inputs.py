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


# ---------------------------------------------------------------------------
# splitmix64 inputs of the large-count MPICH fixtures (tests/golden/
# gen_mpich_large.c gen(): same keying, same bit-to-value maps), regenerated
# here so the fixture holds outputs only
# ---------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def splitmix_input(kind, seed, rank, count, edge=False):
    """Rank `rank`'s input of a large fixture case: kind "f32" / "f64" / "i64"."""
    i = np.arange(count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * np.uint64(0x100000001B3) ^ (np.uint64(rank) << np.uint64(40))
    r = _splitmix64(base ^ i)
    if kind == "i64":
        return r.view(np.int64)
    if kind == "f32":
        v = ((r >> np.uint64(40)).astype(np.int64) - (1 << 23)).astype(np.float32) / np.float32(1 << 23)
        tiny = np.float32(np.ldexp(np.float32(1), -149))
        table = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, tiny, 1.0, -1.0], dtype=np.float32)
    else:
        v = ((r >> np.uint64(11)).astype(np.int64) - (1 << 52)).astype(np.float64) / 4503599627370496.0
        table = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, np.ldexp(1.0, -1074), 1.0, -1.0])
    if edge:
        m = (r & np.uint64(15)) == 0
        v[m] = table[((r[m] >> np.uint64(4)) & np.uint64(7)).astype(np.int64)]
    return v
