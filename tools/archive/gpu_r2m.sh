#!/bin/bash
# Paired-line accumulation: fold tests + microbench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "fold" > gpurun_out/pytest_m.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_m.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/fold_bench.py > gpurun_out/fold_m.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/fold_m.log; fatal $rc fold
