set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_headline_gpu.py tests/test_collectives_gpu.py tests/test_zero_copy_gpu.py -x -v --timeout 500 --timeout-method thread > gpurun_out/pytest_tune.log 2>&1 || { echo TESTS_FAILED; exit 1; }
MPIGX_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { echo BENCH2_FAILED; exit 1; }
echo ALL_OK
