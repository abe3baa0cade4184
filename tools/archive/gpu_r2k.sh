#!/bin/bash
# Full GPU suite, traced headline bench, kernel stats of the headline bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_k.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_k.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
DRYNX_TRACE=gpurun_out/trace_lr timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench_k.log 2>&1
rc=$?; tail -1 gpurun_out/bench_k.log | cut -c1-250; fatal $rc bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k -o lr -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/bench_prof_k.log 2>&1
rc=$?; grep '^{' gpurun_out/bench_prof_k.log | cut -c1-200; fatal $rc rocprof
