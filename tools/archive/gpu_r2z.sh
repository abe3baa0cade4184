#!/bin/bash
# CU reservation A/B: pool / prover streams on CU-masked streams leaving k CUs to the latency-bound launches.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
for cfg in "0 0" "64 0" "96 0" "48 0" "0 0" "128 0" "64 0"; do
  set -- $cfg
  DRYNX_POOL_RESERVE_CUS=$1 DRYNX_PROVE_RESERVE_CUS=$2 timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench_z.log 2>&1
  rc=$?; echo "pool=$1 prove=$2 $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_z.log) $(grep -o '"all_proofs_valid": [a-z]*' gpurun_out/bench_z.log)"; fatal $rc bench; [ $rc -eq 0 ] || exit $rc
done
