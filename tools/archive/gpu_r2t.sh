#!/bin/bash
# Verifier mode "msm" (bilinearity regrouping): GPU tests, headline bench A/B vs the per-item fold.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 150 python -u -m pytest tests/test_rpmsm.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_t0.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_t0.log; fatal $rc pytest0; [ $rc -eq 0 ] || exit $rc
for mode in msm fold; do
  DRYNX_RPV=$mode DRYNX_TRACE=gpurun_out/trace_t_$mode timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 > gpurun_out/bench_t_$mode.log 2>&1
  rc=$?; echo "$mode $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_t_$mode.log) $(grep -o '"all_proofs_valid": [a-z]*' gpurun_out/bench_t_$mode.log)"; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
  python tools/host_trace.py gpurun_out/trace_t_$mode.r0.json 0.5 > gpurun_out/host_trace_t_$mode.txt
done
