#!/bin/bash
# A/B for the n = 8 same-device Scan / Reduce timeouts seen after the
# pull-push Scan landed: the 64 Mi-element Int32/Int64 Scan/Exscan/Reduce
# sequence (tools/scan_repro.py) with the previous commit's library, with the
# new one on a small grid, and with the new one at n = 4.  Assertion failures
# do not stop the pass; timeouts / aborts / crashes do.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r03h}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${T}_${name}.log" 2>&1
  local rc=$?
  echo "STEP $name rc=$rc"
  if [ $rc -ge 124 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step old8 400 python3 tools/scan_repro_launch.py 8 mpi.jl_amd/lib_old/libmpigx.so
MPIGX_MAX_BLOCKS=32 step new8_g32 400 python3 tools/scan_repro_launch.py 8
step new4 400 python3 tools/scan_repro_launch.py 4
echo ALL_DONE
