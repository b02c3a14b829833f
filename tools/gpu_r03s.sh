#!/bin/bash
# Round-3 final GPU pass (completion-word write-back + host stream fallback):
# the 8-rank same-device repro, the full GPU suite, the N=2 same-device and
# N=1 bench lines.  Timeouts / crashes stop it.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03s}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${T}_${name}.log" 2>&1
  local rc=$?
  echo "STEP $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step repro8 300 python3 tools/scan_repro_launch.py 8
step pytest 600 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread
step bench2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline
step bench1 200 python bench.py
echo ALL_DONE
