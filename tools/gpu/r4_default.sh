#!/bin/bash
# bench.py with no flags (the driver's N=1 default) on the final tree.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/default_bench.log 2>&1 || { tail -30 gpurun_out/default_bench.log; exit 1; }
tail -1 gpurun_out/default_bench.log | cut -c1-300
