#!/bin/bash
# tools/ipc_big seq variants: which sequence of IPC imports hangs
cd ${GRAFT_REPO_ROOT:-.}
for v in "2048" "64 2048" "1024 1024" "1024 2047" "1024 2048" "2048 2048" "512 1536" "1536 1536"; do
  timeout -k 5 60 ./tools/ipc_big seq $v
  echo "rc=$? ($v)"
done
