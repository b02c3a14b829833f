"""Pack the raw MPICH golden dumps (gen_mpich_golden.c) into one .npz.

Each case becomes arrays `<id>.in` (uint8, [n, in_bytes]) and `<id>.out`
(uint8, [n, out_bytes]); the manifest (JSON lines) and the op x type error
matrix are stored as JSON text next to it.  Load with numpy.load (no pickle).
"""
import json
import os
import sys

import numpy as np


def main(raw, dest):
    cases = []
    for fn in sorted(os.listdir(raw)):
        if fn.startswith("manifest_") and fn.endswith(".jsonl"):
            with open(os.path.join(raw, fn)) as f:
                cases += [json.loads(l) for l in f if l.strip()]
    arrays = {}
    for c in cases:
        nr = c["n"]  # rows = ranks (reduce_local: in = [in, inout])
        for tag in ("in", "out"):
            b = np.fromfile(os.path.join(raw, f"{c['id']}.{tag}.bin"), dtype=np.uint8)
            per = c[f"{tag}_bytes"]
            rows = b.size // per if per else nr
            arrays[f"{c['id']}.{tag}"] = b.reshape(rows, per)
    np.savez_compressed(os.path.join(dest, "mpich_golden.npz"), **arrays)
    with open(os.path.join(dest, "mpich_golden_manifest.json"), "w") as f:
        json.dump(cases, f, indent=0)
    with open(os.path.join(raw, "op_type_matrix.json")) as f:
        matrix = json.load(f)
    with open(os.path.join(dest, "op_type_matrix.json"), "w") as f:
        json.dump(matrix, f, indent=1, sort_keys=True)
    print(f"packed {len(cases)} cases, {sum(a.nbytes for a in arrays.values())} raw bytes")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
