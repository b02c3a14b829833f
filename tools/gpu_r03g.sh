#!/bin/bash
# Round-3 GPU pass (pull-push Scan / Exscan, zero-copy Reduce chunks owned by
# the non-roots): the cross-XCD visibility probe, zero-copy + headline parity
# (golden cases through the new paths, in place too; 64 Mi-element Scan /
# Exscan / Reduce at n = 2, 4, 8), and the N=2 / N=4 same-device bench lines
# (config 5 section).  A step that fails its assertions does not stop the
# pass; a step that times out, aborts or crashes does (nothing more runs on
# the GPU).
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03g}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${T}_${name}.log" 2>&1
  local rc=$?
  echo "STEP $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step xcd 60 tools/xcd_coherence
step quick 800 python -u -m pytest tests/test_collectives_gpu.py::test_golden_collectives_zero_copy tests/test_headline_gpu.py -x -v --timeout 500 --timeout-method thread
step bench2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline
step bench4 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 4 --steps 10 --warmup 3 --no-cpu-baseline
echo ALL_DONE
