#!/bin/bash
# One build -> measure iteration: GPU tests, headline bench, torch-op GPU time
# by framework call site (DRYNX_TORCH_PROF), u = l = 0 bench with host spans.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-400; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.log; exit $rc; }
DRYNX_TORCH_PROF=gpurun_out/torch_prof.txt timeout -k 10 400 python -u bench.py --steps 2 --warmup 2 > gpurun_out/bench_tprof.log 2>&1 || exit 1
DRYNX_TRACE=gpurun_out/trace timeout -k 10 400 python bench.py --steps 3 --warmup 2 > gpurun_out/bench_trace.log 2>&1 \
 && python tools/host_trace.py gpurun_out/trace.r0.json 0.3 > gpurun_out/host_trace.txt && echo trace ok
