#!/bin/bash
# Round-3 GPU pass: guards, collective-kernel profile (n = 2 on one GPU), the
# full GPU suite, the N=2 same-device bench line (driver command shape) and
# the N=1 line.  A step that fails its assertions does not stop the pass; a
# step that times out, aborts or crashes does (nothing more runs on the GPU).
set -o pipefail
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/r03b_${name}.log" 2>&1
  local rc=$?
  echo "STEP $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step knobs 400 python -u -m pytest tests/test_knobs_gpu.py -x -v --timeout 200 --timeout-method thread
step coll 900 python3 tools/coll_prof.py gpurun_out/coll_r03b r03b --n 2
step pytest 1000 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread
step bench2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline
step tune 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 tools/tune_cost.py
step bench1 300 python bench.py --no-cpu-baseline
echo ALL_DONE
