"""Pack gen_mpich_large.c's dumps into tests/golden/mpich_large.npz (uint8
arrays `<id>.r<rank>`: that rank's output bytes at the manifest's spans,
concatenated) + mpich_large_manifest.json.  Load with numpy.load (no pickle)."""
import json
import os
import sys

import numpy as np


def main(raw, dest):
    cases = []
    for fn in sorted(os.listdir(raw)):
        if fn.startswith("manifest_large_") and fn.endswith(".jsonl"):
            with open(os.path.join(raw, fn)) as f:
                cases += [json.loads(l) for l in f if l.strip()]
    arrays = {}
    for c in cases:
        for fn in sorted(os.listdir(raw)):
            if fn.startswith(c["id"] + ".r") and fn.endswith(".bin"):
                arrays[fn[:-4]] = np.fromfile(os.path.join(raw, fn), dtype=np.uint8)
    np.savez_compressed(os.path.join(dest, "mpich_large.npz"), **arrays)
    with open(os.path.join(dest, "mpich_large_manifest.json"), "w") as f:
        json.dump(cases, f, indent=0)
    print(f"{len(cases)} cases, {len(arrays)} arrays, {sum(a.size for a in arrays.values())} bytes")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
