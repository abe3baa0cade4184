#!/bin/bash
# ScaleDPs after batching the ledger copies / aggregation decode; configs 2 and 3.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "int_moments or batched_dp or every_operation or survey" > gpurun_out/pytest_h.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_h.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
for q in mean variance lin_reg; do
  timeout -k 10 300 python -u bench.py --query $q --steps 5 --warmup 1 > gpurun_out/bench_$q.log 2>&1
  rc=$?; tail -1 gpurun_out/bench_$q.log | cut -c1-260; fatal $rc bench_$q
done
DRYNX_TRACE=gpurun_out/trace6000.json timeout -k 10 300 python -u tools/profile_many_dps.py 6000 gpurun_out/prof6000.txt > gpurun_out/prof6000.log 2>&1
rc=$?; head -1 gpurun_out/prof6000.txt; fatal $rc prof
timeout -k 10 300 python -u tools/bench_scaling.py 1 dps > gpurun_out/scaling_dps.log 2>&1
rc=$?; cut -c1-200 gpurun_out/scaling_dps.log; fatal $rc scaling
