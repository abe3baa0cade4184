#!/bin/bash
# Round 2 iteration: new GPU tests, bench, host-span trace of the last step.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "fold or fb4 or layouts or early_range" > gpurun_out/pytest_gpu_new.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu_new.log; fatal $rc pytest
DRYNX_TRACE=gpurun_out/trace timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
python tools/host_trace.py gpurun_out/trace.r0.json 0.3 > gpurun_out/host_trace.txt; echo trace rc=$?
