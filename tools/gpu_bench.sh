set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { echo BENCH1_FAILED; exit 1; }
MPIGX_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err || { echo BENCH2_FAILED; exit 1; }
bash tools/profile.sh r02 > gpurun_out/prof_r02.log 2>&1 || { echo PROF_FAILED; exit 1; }
echo ALL_OK
