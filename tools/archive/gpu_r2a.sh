#!/bin/bash
# Round 2: GPU tests + headline bench at the reference configuration + kernel stats.
# A GPU step that faults, aborts or times out ends the script (no further GPU step).
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; fatal $rc pytest
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1
rc=$?; tail -2 gpurun_out/bench.log; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_run.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
