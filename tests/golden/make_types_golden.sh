#!/bin/bash
# Regenerates tests/golden/types_golden.json from MPICH 3.3.2 (build container only).
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
MPIGX_HOST_ONLY=1 OMP_NUM_THREADS=1 /opt/conda/bin/mpiexec -n 1 python3 "$here/gen_types_golden.py"
