#!/bin/bash
# rocprofv3 kernel trace + stats of the headline (2 timed queries after 1 warmup);
# per-kernel totals and the per-query kernel timeline summary.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_run.log 2>&1; rc=$?
tail -1 gpurun_out/prof_run.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
ls -R gpurun_out/prof | head -20
