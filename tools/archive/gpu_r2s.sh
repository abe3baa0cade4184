#!/bin/bash
# Current-state baseline: headline bench, host span trace, kernel-trace timeline + stats.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 > gpurun_out/bench_s.log 2>&1
rc=$?; tail -1 gpurun_out/bench_s.log | cut -c1-330; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
DRYNX_TRACE=gpurun_out/trace_s timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_s_trace.log 2>&1
rc=$?; fatal $rc bench_trace; [ $rc -eq 0 ] || exit $rc
python tools/host_trace.py gpurun_out/trace_s.r0.json 0.5 > gpurun_out/host_trace_s.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_run.log 2>&1
rc=$?; echo "prof rc=$rc"; fatal $rc prof
python tools/gpu_busy.py gpurun_out/prof/bench_kernel_trace.csv timeline > gpurun_out/gpu_busy_s.txt; head -40 gpurun_out/gpu_busy_s.txt
