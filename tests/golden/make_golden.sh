#!/bin/bash
# Regenerates tests/golden/mpich_golden.npz from MPICH 3.3.2 (/opt/conda), the
# libmpi MPI.jl v0.14.2 ccalls by default. Run in the build container (needs
# /opt/conda MPICH); the packed .npz + matrix JSON are committed.
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
work="$(mktemp -d)"
gcc -O2 -std=c99 -o "$work/gen" "$here/gen_mpich_golden.c" -I/opt/conda/include \
    -L/opt/conda/lib -lmpi -lm -Wl,-rpath,/opt/conda/lib
mkdir -p "$work/raw"
for n in 1 2 3 4 5 6 8; do
  /opt/conda/bin/mpiexec -n $n "$work/gen" "$work/raw"
done
python3 "$here/pack_golden.py" "$work/raw" "$here"
rm -rf "$work"
