#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29611 tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1
rc=$?; grep -E "rank|Error|error|Duplicate" gpurun_out/rccl_probe.log | head -20; echo "rc=$rc"
