#!/bin/bash
# Regenerates tests/golden/p2p_golden.json: the point-to-point scenarios of
# tests/spmd/p2p_worker.py run on host arrays under MPICH 3.3.2 (/opt/conda),
# the libmpi MPI.jl ccalls.  Run in the build container; the JSON is committed
# and the device run (tests/test_p2p_gpu.py) must reproduce it exactly.
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
root="$(dirname "$(dirname "$here")")"
work="$(mktemp -d)"
for n in 2 3 4; do
  MPIGX_HOST_ONLY=1 OMP_NUM_THREADS=1 /opt/conda/bin/mpiexec -n $n python3 "$root/tests/spmd/p2p_worker.py" \
    > "$work/n$n.log"
done
python3 - "$work" "$here/p2p_golden.json" <<'PY'
import json, sys
work, dest = sys.argv[1], sys.argv[2]
out = {}
for n in (2, 3, 4):
    recs = {}
    for line in open(f"{work}/n{n}.log"):
        if line.startswith("{"):
            d = json.loads(line)
            assert d["failed"] is None, d["failed"]
            recs[d["rank"]] = d["records"]
    out[str(n)] = [recs[r] for r in range(n)]
json.dump({"source": "MPICH 3.3.2 (/opt/conda), tests/spmd/p2p_worker.py on host arrays", "runs": out},
          open(dest, "w"), indent=None, separators=(",", ":"))
PY
rm -rf "$work"
