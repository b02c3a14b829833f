#!/bin/bash
# Regenerates tests/golden/mpich_large.npz + mpich_large_manifest.json from
# MPICH 3.3.2 (/opt/conda): large-count Allreduce / Reduce / Scan / Exscan at
# n = 5 and 8, sampled spans only (gen_mpich_large.c).  Run in the build
# container (needs /opt/conda MPICH); the outputs are committed.
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
work="$(mktemp -d)"
gcc -O2 -std=c99 -o "$work/gen" "$here/gen_mpich_large.c" -I/opt/conda/include \
    -L/opt/conda/lib -lmpi -lm -Wl,-rpath,/opt/conda/lib
mkdir -p "$work/raw"
for n in 5 8; do
  /opt/conda/bin/mpiexec -n $n "$work/gen" "$work/raw"
done
python3 "$here/pack_large_golden.py" "$work/raw" "$here"
rm -rf "$work"
