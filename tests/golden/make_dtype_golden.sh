#!/bin/bash
# Regenerates tests/golden/dtype_golden.json: the derived-datatype scenarios
# of tests/spmd/dtype_worker.py on host arrays under MPICH 3.3.2 (/opt/conda).
# Build container only; the device run (tests/test_types_gpu.py) must match.
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
root="$(dirname "$(dirname "$here")")"
work="$(mktemp -d)"
for n in 2 3 4; do
  MPIGX_HOST_ONLY=1 OMP_NUM_THREADS=1 DT_OUT="$work/n$n" /opt/conda/bin/mpiexec -n $n \
    python3 "$root/tests/spmd/dtype_worker.py"
done
python3 - "$work" "$here/dtype_golden.json" <<'PY'
import json, sys
work, dest = sys.argv[1], sys.argv[2]
out = {}
for n in (2, 3, 4):
    recs = []
    for r in range(n):
        d = json.load(open(f"{work}/n{n}.{r}"))
        assert d["failed"] is None, d["failed"]
        recs.append(d["records"])
    out[str(n)] = recs
json.dump({"source": "MPICH 3.3.2 (/opt/conda), tests/spmd/dtype_worker.py on host arrays", "runs": out},
          open(dest, "w"), indent=None, separators=(",", ":"))
PY
rm -rf "$work"
