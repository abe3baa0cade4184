#!/bin/bash
# GLV batch weights: GPU tests + bench (glv vs 64-bit weights) + kernel stats.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "glv or range or fold or survey or oracle" > gpurun_out/pytest_n.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_n.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
for rho in glv 64 glv; do
  DRYNX_RHO=$rho timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 > gpurun_out/bench_rho_$rho.log 2>&1
  rc=$?; echo "rho=$rho $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_rho_$rho.log) $(grep -o '"all_proofs_valid": [a-z]*' gpurun_out/bench_rho_$rho.log)"; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_n -o lr -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/bench_prof_n.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_prof_n.log; fatal $rc rocprof
