#!/bin/bash
# Checkpoint: full GPU suite, smoke(), headline bench, traced bench, configs 2/3.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/pytest_q.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_q.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_q.log 2>&1
rc=$?; tail -1 gpurun_out/smoke_q.log; fatal $rc smoke; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench_q.log 2>&1
rc=$?; tail -1 gpurun_out/bench_q.log | cut -c1-330; fatal $rc bench
DRYNX_TRACE=gpurun_out/trace_q timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_q_trace.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_q_trace.log; fatal $rc bench_trace
for q in mean variance lin_reg; do
  timeout -k 10 300 python -u bench.py --query $q --steps 5 --warmup 1 > gpurun_out/bench_q_$q.log 2>&1
  rc=$?; echo "$q $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_q_$q.log)"; fatal $rc bench_$q
done
