#!/bin/bash
# A/B: prover kernels at 1 wave/SIMD (no scratch) vs 2 waves/SIMD (spills), alternating.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "layout" > gpurun_out/pytest_ab.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_ab.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
for w in 1 2 1 2; do
  DRYNX_PROVE_WAVES=$w timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench_ab.log 2>&1
  rc=$?; echo "waves=$w $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_ab.log) $(grep -o '"all_proofs_valid": [a-z]*' gpurun_out/bench_ab.log)"; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
done
DRYNX_PROVE_WAVES=1 timeout -k 10 200 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "layout" > gpurun_out/pytest_ab1.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_ab1.log; fatal $rc pytest1
