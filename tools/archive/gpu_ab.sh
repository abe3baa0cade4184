#!/bin/bash
# A/B of bench.py under environment variants: gpu_ab.sh "VAR=a" "VAR=b" ...
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for v in "$@"; do
  env $v timeout -k 10 300 python bench.py --steps 8 --warmup 2 > gpurun_out/ab_$i.log 2>&1 || { tail -20 gpurun_out/ab_$i.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/ab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["phase_s"]["ProofVerification"], d["phase_s"]["JustExecution"])')"
  i=$((i+1))
done
