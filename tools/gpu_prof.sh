set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_local_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_local.log 2>&1 || { echo LOCAL_FAILED; exit 1; }
bash tools/profile.sh r02 > gpurun_out/prof_r02.log 2>&1 || { echo PROF_FAILED; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { echo BENCH1_FAILED; exit 1; }
MPIGX_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/latency.py > gpurun_out/latency_n2.json 2> gpurun_out/latency_n2.err || { echo LAT_FAILED; exit 1; }
echo ALL_OK
