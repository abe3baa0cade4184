#!/bin/bash
# torch.profiler over one timed query: which torch ops cost GPU time beside the framework kernels.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
DRYNX_TORCH_PROF=gpurun_out/torch_prof.txt timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 > gpurun_out/bench_w.log 2>&1
rc=$?; tail -1 gpurun_out/bench_w.log | cut -c1-120; fatal $rc bench
sed -n "/# GPU time of torch ops/,\$p" gpurun_out/torch_prof.txt | head -62
