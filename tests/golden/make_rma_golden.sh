#!/bin/bash
# Regenerates tests/golden/rma_golden.json: the one-sided scenarios of
# tests/spmd/rma_worker.py run on host arrays under MPICH 3.3.2 (/opt/conda),
# the libmpi MPI.jl ccalls (src/onesided.jl).  Run in the build container; the
# JSON is committed and the device run (tests/test_rma_gpu.py) must reproduce
# it exactly.
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
root="$(dirname "$(dirname "$here")")"
work="$(mktemp -d)"
for n in 2 3 4; do
  MPIGX_HOST_ONLY=1 OMP_NUM_THREADS=1 RMA_OUT="$work/n$n" /opt/conda/bin/mpiexec -n $n \
    python3 "$root/tests/spmd/rma_worker.py"
done
python3 - "$work" "$here/rma_golden.json" <<'PY'
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
json.dump({"source": "MPICH 3.3.2 (/opt/conda), tests/spmd/rma_worker.py on host arrays", "runs": out},
          open(dest, "w"), indent=None, separators=(",", ":"))
PY
rm -rf "$work"
