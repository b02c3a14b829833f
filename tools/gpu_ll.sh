set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_collectives_gpu.py -x -v --timeout 500 --timeout-method thread > gpurun_out/pytest_coll.log 2>&1 || { echo COLL_FAILED; exit 1; }
MPIGX_DEVICE=0 LAT_SIZES=8,4096,65536,262144,1048576 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/latency.py > gpurun_out/latency_ll_n2.json 2> gpurun_out/latency_ll_n2.err || { echo LAT_FAILED; exit 1; }
MPIGX_ALGO=oneshot MPIGX_DEVICE=0 LAT_SIZES=8,4096,65536,262144 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 tools/latency.py > gpurun_out/latency_os_n2.json 2> gpurun_out/latency_os_n2.err || { echo LAT2_FAILED; exit 1; }
MPIGX_DEVICE=0 LAT_SIZES=8,4096,65536,262144 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29514 tools/latency.py > gpurun_out/latency_ll_n4.json 2> gpurun_out/latency_ll_n4.err || { echo LAT3_FAILED; exit 1; }
MPIGX_ALGO=oneshot MPIGX_DEVICE=0 LAT_SIZES=8,4096,65536,262144 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29515 tools/latency.py > gpurun_out/latency_os_n4.json 2> gpurun_out/latency_os_n4.err || { echo LAT4_FAILED; exit 1; }
echo ALL_OK
