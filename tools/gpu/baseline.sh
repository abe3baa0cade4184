#!/bin/bash
# Round-start baseline on one GPU: GPU tests, headline bench, traced bench,
# RangeProofMode 1 A/B (cost of the per-V G2 subgroup check), non-pooled A/B.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-400 \
 && timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --range-mode 1 > gpurun_out/bench_mode1.log 2>&1 && tail -1 gpurun_out/bench_mode1.log | cut -c1-300 \
 && DRYNX_VN_POOL=0 timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > gpurun_out/bench_nopool.log 2>&1 && tail -1 gpurun_out/bench_nopool.log | cut -c1-300 \
 && DRYNX_TRACE=gpurun_out/trace timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_trace.log 2>&1 \
 && python tools/host_trace.py gpurun_out/trace.r0.json 0.3 > gpurun_out/host_trace.txt && echo trace ok
