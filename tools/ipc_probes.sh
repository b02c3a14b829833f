#!/bin/bash
# The IPC probes behind DESIGN §13 ("IPC imports of >= 2 GiB allocations hang
# under the HIP 7.0 runtime"), one mode per GPU call:
#   tools/ipc_probes.sh seq     tools/ipc_big seq: one owner, one peer, imports in sequence (system HIP 7.2)
#   tools/ipc_probes.sh torch   tools/ipc_torch.py variants in torch processes (PyTorch's HIP 7.0):
#                               each rank leaves by itself 15 s into a stuck open, so no step hits its limit
# (tools/ipc_big with no mode / `bidir`: one-way / both-way opens per size;
#  tools/ipc_reuse: buffer id / handle reuse after free)
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
case "${1:-seq}" in
  seq)
    for v in "2048" "64 2048" "1024 1024" "1024 2047" "1024 2048" "2048 2048" "512 1536" "1536 1536"; do
      timeout -k 5 60 ./tools/ipc_big seq $v
      echo "rc=$? ($v)"
    done ;;
  torch)
    for v in "torch 0 2048" "hip 0 2048" "hip 0 1024,2048" "torch 0 1536,2047" "torch 0 3072" "hip 1 2048"; do
      set -- $v
      tag="alloc_$1_mpigx_$2_$3"
      IPC_ALLOC=$1 IPC_MPIGX=$2 SIZES_MIB=$3 MPIGX_DEVICE=0 timeout -k 5 90 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29700 + RANDOM % 100)) tools/ipc_torch.py \
        > gpurun_out/ipc_$tag.log 2>&1
      rc=$?
      echo "VARIANT $tag rc=$rc"; grep '^{' gpurun_out/ipc_$tag.log | grep -v '"alloc"'
      if [ $rc -ge 124 ]; then echo STOP; exit 0; fi
    done ;;
  *) echo "usage: $0 seq|torch"; exit 2 ;;
esac
