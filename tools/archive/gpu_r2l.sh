#!/bin/bash
# Folds queued before the MSM plans: range GPU tests + traced bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "range or fold or survey" > gpurun_out/pytest_l.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_l.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
DRYNX_TRACE=gpurun_out/trace_l timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 > gpurun_out/bench_l.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_l.log; fatal $rc bench
