set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { echo PYTEST_FAILED; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { echo BENCH1_FAILED; exit 1; }
bash tools/profile.sh r02 > gpurun_out/prof_r02.log 2>&1 || { echo PROF_FAILED; exit 1; }
echo ALL_OK
