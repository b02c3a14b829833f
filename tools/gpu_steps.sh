#!/bin/bash
# One GPU call = a list of steps, each under its own time limit, output to
# gpurun_out/<TAG>_<name>.log; the call stops after the first step that timed
# out, crashed or aborted (rc >= 124), so nothing more touches a GPU in a bad
# state.  Usage (from the repo root, e.g. through gpurun):
#
#   TAG=r04a tools/gpu_steps.sh 'repro8|300|python3 tools/scan_repro_launch.py 8' \
#                               'pytest|900|python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread'
#
# Predefined step names (pass just the name): pytest, bench1, bench2, repro8.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-gpu}
STOP_ON_FAIL=${STOP_ON_FAIL:-0}
declare -A PRE=(
  [pytest]="pytest|900|python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread"
  [bench1]="bench1|240|python bench.py"
  [bench2]="bench2|300|python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline"
  [repro8]="repro8|300|python3 tools/scan_repro_launch.py 8"
)
for spec in "$@"; do
  [ -n "${PRE[$spec]}" ] && spec=${PRE[$spec]}
  name=${spec%%|*}
  rest=${spec#*|}
  t=${rest%%|*}
  cmd=${rest#*|}
  start=$(date +%s)
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/${T}_${name}.log" 2>&1
  rc=$?
  echo "STEP $name rc=$rc $(( $(date +%s) - start ))s"
  tail -n 4 "gpurun_out/${T}_${name}.log"
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  if [ $rc -ne 0 ] && [ "$STOP_ON_FAIL" = 1 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
done
echo ALL_DONE
