set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_collectives_gpu.py tests/test_zero_copy_gpu.py -x -v --timeout 500 --timeout-method thread > gpurun_out/pytest_coll.log 2>&1 || { echo COLL_FAILED; exit 1; }
for algo in ll oneshot; do
MPIGX_ALGO=$algo MPIGX_DEVICE=0 LAT_SIZES=8,4096,16384,65536 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/latency.py > gpurun_out/latency_${algo}_n2.json 2> gpurun_out/latency_${algo}_n2.err || { echo LAT_FAILED; exit 1; }
done
echo ALL_OK
