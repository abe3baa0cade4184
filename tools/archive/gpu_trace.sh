#!/bin/bash
# Bench with the host span trace on (DRYNX_TRACE) -> gpurun_out/trace.r0.json
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DRYNX_TRACE=gpurun_out/trace timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_trace.log 2>&1 && tail -1 gpurun_out/bench_trace.log \
 && python tools/host_trace.py gpurun_out/trace.r0.json 0.5 > gpurun_out/host_trace.txt && echo trace ok
