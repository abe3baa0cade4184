#!/bin/bash
# msm verifier, plans-first schedule: GPU tests, traced bench, kernel timeline.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 150 python -u -m pytest tests/test_rpmsm.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_u.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_u.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
DRYNX_TRACE=gpurun_out/trace_u timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 > gpurun_out/bench_u.log 2>&1
rc=$?; echo "$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_u.log) $(grep -o '"all_proofs_valid": [a-z]*' gpurun_out/bench_u.log)"; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
python tools/host_trace.py gpurun_out/trace_u.r0.json 0.5 > gpurun_out/host_trace_u.txt
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_run.log 2>&1
rc=$?; echo "prof rc=$rc"; fatal $rc prof
python tools/gpu_busy.py gpurun_out/prof/bench_kernel_trace.csv timeline > gpurun_out/gpu_busy_u.txt; sed -n '/step 1/,/step 2/p' gpurun_out/gpu_busy_u.txt | head -20
