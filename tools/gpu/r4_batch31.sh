#!/bin/bash
# rocprofv3 kernel statistics of the final tree's headline (3 timed steps).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kstats -o run -- python3 -u bench.py --steps 3 --warmup 2 > gpurun_out/kstats_run.log 2>&1 || { tail -30 gpurun_out/kstats_run.log; exit 1; }
find gpurun_out/kstats -name "*kernel_stats.csv" | head -3
tail -2 gpurun_out/kstats_run.log | cut -c1-200
