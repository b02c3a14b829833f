#!/bin/bash
# Round-3 GPU pass (zero-copy Reduce into the root's recvbuf, static slices
# by default): copy roofline of the box, the full GPU suite, the N=2
# same-device and N=1 bench lines.  A step that fails its assertions does
# not stop the pass; a step that times out, aborts or crashes does.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03f}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${T}_${name}.log" 2>&1
  local rc=$?
  echo "STEP $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step copyroof 120 python3 tools/copy_roof.py --mib 512
step pytest 900 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread
step bench2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline
step bench1 300 python bench.py
echo ALL_DONE
