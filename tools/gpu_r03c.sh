#!/bin/bash
# Round-3 GPU pass (pull-push two-shot, fence-free exit barriers): zero-copy
# and headline parity first, then the collective-kernel profile (n = 2 on one GPU), the
# N=2 same-device bench line (driver command shape), the N=1 line and the
# N=1 rocprof kernel-trace + PMC traffic passes (tools/profile.sh).  A step that fails its assertions does not stop the pass; a
# step that times out, aborts or crashes does (nothing more runs on the GPU).
set -o pipefail
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/r03c_${name}.log" 2>&1
  local rc=$?
  echo "STEP $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step quick 700 python -u -m pytest tests/test_collectives_gpu.py::test_golden_collectives_zero_copy tests/test_headline_gpu.py -x -v --timeout 400 --timeout-method thread
step coll 900 python3 tools/coll_prof.py gpurun_out/coll_r03c r03c --n 2
step bench2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline
step bench1 300 python bench.py --no-cpu-baseline
step prof 960 bash tools/profile.sh r03
echo ALL_DONE
