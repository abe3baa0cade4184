#!/bin/bash
# Ledger A/B + kernel-trace occupancy of the bench.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
DRYNX_LEDGER_RANGE=off timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_ledger_off.log 2>&1
rc=$?; tail -1 gpurun_out/bench_ledger_off.log | cut -c1-330; fatal $rc bench-off
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_run.log 2>&1
rc=$?; echo "prof rc=$rc"; fatal $rc prof; tail -1 gpurun_out/prof_run.log | cut -c1-330
python tools/gpu_busy.py gpurun_out/prof/bench_kernel_trace.csv > gpurun_out/gpu_busy.txt; cat gpurun_out/gpu_busy.txt
