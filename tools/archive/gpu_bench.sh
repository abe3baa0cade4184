#!/bin/bash
# Bench sweep on one GPU: small LR first (d=8), then the full SPECTF-shaped config.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench.py --features 8 --records 1000000 --steps 2 --warmup 1 > gpurun_out/bench_d8.log 2>&1 && tail -1 gpurun_out/bench_d8.log \
 && timeout -k 10 900 python bench.py --features 44 --records 1000000 --steps 1 --warmup 1 > gpurun_out/bench_d44.log 2>&1 && tail -1 gpurun_out/bench_d44.log
