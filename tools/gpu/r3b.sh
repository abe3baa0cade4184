#!/bin/bash
# RCCL one-rank plane tests, then clean vs fault-injected headline with spans.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_rccl_plane.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_rccl.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_rccl.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_rccl.log; exit $rc; }
bash tools/gpu/fault2.sh
