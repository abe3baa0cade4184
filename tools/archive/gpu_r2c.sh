#!/bin/bash
# Round 2: full GPU test suite + traced bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; fatal $rc pytest
DRYNX_TRACE=gpurun_out/trace timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log | cut -c1-700; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
python tools/host_trace.py gpurun_out/trace.r0.json 0.3 > gpurun_out/host_trace.txt; echo trace rc=$?
