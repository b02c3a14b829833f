#!/bin/bash
# Round-3 closing GPU pass: the same-device Scan/Exscan/Reduce repro at n = 8
# (pull-push Scan off), the N=2 same-device and N=1 bench lines, and the
# rocprofv3 kernel trace + PMC traffic of the N=1 bench (tools/profile.sh).  Timeouts / crashes stop it.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03r}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${T}_${name}.log" 2>&1
  local rc=$?
  echo "STEP $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step repro8 300 python3 tools/scan_repro_launch.py 8
step bench2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline
step bench1 300 python bench.py
step prof 800 bash tools/profile.sh $T
echo ALL_DONE
