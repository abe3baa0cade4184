#!/bin/bash
# Normalised-line fold (mode 4): GPU tests + fold microbench + bench A/B (4 vs 3).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread \
  -k "fold or range_proofs or glv" > gpurun_out/pytest_p.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_p.log; fatal $rc pytest; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/fold_bench.py > gpurun_out/fold_p.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/fold_p.log | grep -i "normal\|sharedV\|check"; fatal $rc fold
for f in 4 3; do
  DRYNX_FOLD=$f timeout -k 10 400 python -u bench.py --steps 4 --warmup 1 > gpurun_out/bench_fold$f.log 2>&1
  rc=$?; echo "fold=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_fold$f.log) $(grep -o '"all_proofs_valid": [a-z]*' gpurun_out/bench_fold$f.log)"; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
done
