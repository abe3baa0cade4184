#!/bin/bash
# GLS-2 6-bit prover tables: GPU layout tests + bench A/B (mode 6 vs 4).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread \
  -k "layouts or oracle or range_proofs" > gpurun_out/pytest_o.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_o.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
for bits in 6 4; do
  DRYNX_PROVER_TABLE_BITS=$bits DRYNX_TRACE=gpurun_out/trace_tb$bits timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 > gpurun_out/bench_tb$bits.log 2>&1
  rc=$?; echo "bits=$bits $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_tb$bits.log) $(grep -o '"all_proofs_valid": [a-z]*' gpurun_out/bench_tb$bits.log)"; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
done
