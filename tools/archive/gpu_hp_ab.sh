#!/bin/bash
# A/B: survey work on a high-priority stream (default) vs off.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
for hp in 1 0 1; do
  DRYNX_HP_STREAM=$hp DRYNX_TRACE=gpurun_out/trace_hp$hp timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 > gpurun_out/bench_hp$hp.log 2>&1
  rc=$?; echo "hp=$hp $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_hp$hp.log)"; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
done
