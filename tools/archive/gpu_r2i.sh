#!/bin/bash
# ScaleDPs after batching envelope packing / digests / signatures and the VN decode.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "batched_dp or every_operation or survey or range_proofs" > gpurun_out/pytest_i.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_i.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
DRYNX_TRACE=gpurun_out/trace6000.json timeout -k 10 300 python -u tools/profile_many_dps.py 6000 gpurun_out/prof6000.txt > gpurun_out/prof6000.log 2>&1
rc=$?; head -1 gpurun_out/prof6000.txt; fatal $rc prof
timeout -k 10 300 python -u tools/bench_scaling.py 3 dps > gpurun_out/scaling_dps.log 2>&1
rc=$?; cut -c1-200 gpurun_out/scaling_dps.log; fatal $rc scaling
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lr -o lr -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/bench_prof.log 2>&1
rc=$?; tail -1 gpurun_out/bench_prof.log | cut -c1-200; fatal $rc rocprof
