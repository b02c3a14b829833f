#!/bin/bash
# Round-3 first GPU pass: the new agreement guards, the collective-kernel
# profile (tools/coll_prof.py, n = 2 ranks on the one GPU), the full GPU suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_knobs_gpu.py -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/r03a_knobs.log 2>&1 || { echo KNOBS_FAILED; exit 1; }
timeout -k 10 900 python3 tools/coll_prof.py gpurun_out/coll_r03a r03a --n 2 > gpurun_out/r03a_coll.log 2>&1 \
  || { echo COLLPROF_FAILED; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread \
  > gpurun_out/r03a_pytest_gpu.log 2>&1 || { echo PYTEST_FAILED; exit 1; }
echo ALL_OK
