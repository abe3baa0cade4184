#!/bin/bash
# Full-config bench + rocprofv3 kernel stats (kernel trace only; no PMC in the same run).
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_full.log 2>&1 && tail -1 gpurun_out/bench_full.log \
 && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT \
 && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_run.log 2>&1 \
 && find gpurun_out/prof -name "*stats*" | head -5
