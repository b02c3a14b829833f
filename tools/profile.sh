#!/bin/bash
# Round profile of bench.py on the GPU box: kernel trace + stats, then HBM
# traffic from PMC in separate passes (FETCH_SIZE and WRITE_SIZE do not fit
# one TCC pass; MI355X_MICROARCH.md "rocprofv3 PMC slots").  Summaries are
# written to profiles/ by tools/summarize_prof.py.
#   usage: tools/profile.sh <round-tag> [bench args...]
set -euo pipefail
TAG=${1:-r01}; shift || true
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export TMPDIR=/tmp
OUT=$R/gpurun_out/prof_$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-sweep --steps 10 "$@" > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/fetch" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-sweep --steps 5 --warmup 1 "$@" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/write" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline --no-sweep --steps 5 --warmup 1 "$@" > "$OUT/write.log" 2>&1
# summaries into the box's profiles/ and beside the raw CSVs under
# gpurun_out/ (the only part of a gpurun box's tree that comes back)
python3 "$R/tools/summarize_prof.py" "$OUT" "$R/profiles" "$TAG"
python3 "$R/tools/summarize_prof.py" "$OUT" "$OUT/summary" "$TAG" > /dev/null
