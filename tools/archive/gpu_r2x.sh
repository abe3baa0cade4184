#!/bin/bash
# Prover table mode 7 (GLS-2 signed 8-bit): GPU layout tests, then the headline bench (mode 7 default) + mode 6 A/B.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_rpmsm.py -m gpu -x -q --timeout 250 --timeout-method thread -k "layout or rpmsm or msm or joint" > gpurun_out/pytest_x.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_x.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
for b in 7 6; do
  DRYNX_PROVER_TABLE_BITS=$b DRYNX_TRACE=gpurun_out/trace_x$b timeout -k 10 500 python -u bench.py --steps 4 --warmup 1 > gpurun_out/bench_x$b.log 2>&1
  rc=$?; echo "bits=$b $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_x$b.log) $(grep -o '"all_proofs_valid": [a-z]*' gpurun_out/bench_x$b.log)"; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
  python tools/host_trace.py gpurun_out/trace_x$b.r0.json 0.5 > gpurun_out/host_trace_x$b.txt
done
