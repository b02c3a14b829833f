#!/bin/bash
# Round-3 GPU pass (dynamic slice hand-out in the pull-push two-shot): knob
# guards (incl. MPIGX_AR_SLICES sequences), zero-copy and headline parity,
# the collective-kernel profile of slice counts 0 / 4 / 8 / 16 at n = 2 on one
# GPU, and the N=2 same-device bench line.  A step that fails its
# assertions does not stop the pass; a step that times out, aborts or
# crashes does (nothing more runs on the GPU).
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03e}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${T}_${name}.log" 2>&1
  local rc=$?
  echo "STEP $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step knobs 300 python -u -m pytest tests/test_knobs_gpu.py -x -v --timeout 200 --timeout-method thread
step quick 600 python -u -m pytest tests/test_collectives_gpu.py::test_golden_collectives_zero_copy tests/test_headline_gpu.py -x -v --timeout 400 --timeout-method thread
step coll 700 python3 tools/coll_prof.py gpurun_out/coll_$T $T --n 2 --configs 256:pullpush,256:pullpush/0,256:pullpush/8,256:pullpush/16,256:pull,64:pullpush,64:pullpush/0,16:pullpush,16:pullpush/0 --pmc-configs 256:pullpush
step bench2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline
echo ALL_DONE
