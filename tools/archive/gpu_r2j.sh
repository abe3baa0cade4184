#!/bin/bash
# Shared-V fold: GPU tests, fold microbench, headline bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "fold or range_proofs" > gpurun_out/pytest_j.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_j.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/fold_bench.py > gpurun_out/fold_j.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/fold_j.log; fatal $rc fold
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_j.log 2>&1
rc=$?; tail -1 gpurun_out/bench_j.log | cut -c1-300; fatal $rc bench
