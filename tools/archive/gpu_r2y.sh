#!/bin/bash
# GT multi-exp with 11-bit windows + gT^t from a signed 16-bit table: GPU tests, then the headline bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_rpmsm.py -m gpu -x -q --timeout 250 --timeout-method thread -k "layout or msm or joint or range or lr or logreg or encod" > gpurun_out/pytest_y.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_y.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
DRYNX_TRACE=gpurun_out/trace_y timeout -k 10 500 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench_y.log 2>&1
rc=$?; echo "$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_y.log) $(grep -o '"all_proofs_valid": [a-z]*' gpurun_out/bench_y.log)"; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
python tools/host_trace.py gpurun_out/trace_y.r0.json 0.5 > gpurun_out/host_trace_y.txt
