#!/bin/bash
# Regenerates tests/golden/userop_golden.json: tests/spmd/userop_worker.py on
# host arrays with MPICH 3.3.2's MPI_Op_create (build container only).
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
root="$(dirname "$(dirname "$here")")"
work="$(mktemp -d)"
for n in 2 3 4; do
  MPIGX_HOST_ONLY=1 OMP_NUM_THREADS=1 UO_OUT="$work/n$n" /opt/conda/bin/mpiexec -n $n \
    python3 "$root/tests/spmd/userop_worker.py"
done
python3 - "$work" "$here/userop_golden.json" <<'PY'
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
json.dump({"source": "MPICH 3.3.2 (/opt/conda) MPI_Op_create, tests/spmd/userop_worker.py on host arrays",
           "runs": out}, open(dest, "w"), indent=None, separators=(",", ":"))
PY
rm -rf "$work"
