#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; fatal $rc pytest
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1
rc=$?; tail -1 gpurun_out/bench.log | cut -c1-330; fatal $rc bench
timeout -k 10 1000 bash tools/gpu_multirank.sh; echo "multirank rc=$?"
