#!/bin/bash
# Round-3 GPU pass after the flag write-back fix: the same-device
# Scan/Exscan/Reduce sequence that timed out (tools/scan_repro.py, n = 4
# and n = 8) with the headline / zero-copy parity (PART=1); the full GPU
# suite and the N=2 / N=1 bench lines (PART=2).
# Assertion failures do not stop the pass; timeouts / aborts / crashes do.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03p}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${T}_${name}.log" 2>&1
  local rc=$?
  echo "STEP $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
export MPIGX_DIAG_TRACE=1
if [ "${PART:-1}" = 1 ]; then
step repro4a 300 python3 tools/scan_repro_launch.py 4
step repro8 300 python3 tools/scan_repro_launch.py 8
unset MPIGX_DIAG_TRACE
step quick 700 python -u -m pytest tests/test_headline_gpu.py tests/test_collectives_gpu.py::test_golden_collectives_zero_copy -v --timeout 500 --timeout-method thread
echo ALL_DONE
exit 0
fi
unset MPIGX_DIAG_TRACE
step pytest 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread
step bench2 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline
step bench1 300 python bench.py
echo ALL_DONE
