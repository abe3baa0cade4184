#!/bin/bash
# K14 kernel + batched DP encoding on the GPU, then the ScaleDPs sweep and a
# cProfile of the 6000-DP survey.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "int_moments or batched_dp or every_operation or native_loaded" > gpurun_out/pytest_k14.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_k14.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_scaling.py 1 dps > gpurun_out/scaling_dps.log 2>&1
rc=$?; cat gpurun_out/scaling_dps.log | cut -c1-200; fatal $rc scaling
timeout -k 10 300 python -u tools/profile_many_dps.py 6000 gpurun_out/prof6000.txt > gpurun_out/prof6000.log 2>&1
rc=$?; head -3 gpurun_out/prof6000.txt; fatal $rc prof
