#!/bin/bash
# The no-range-proof line (everything but the range proofs) with host spans.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DRYNX_TRACE=gpurun_out/trace_u0l0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --u 0 --l 0 > gpurun_out/bench_u0l0.log 2>&1; rc=$?
tail -1 gpurun_out/bench_u0l0.log | cut -c1-300; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_u0l0.log; exit $rc; }
python tools/host_trace.py gpurun_out/trace_u0l0.r0.json 0.05 > gpurun_out/host_trace_u0l0.txt && echo trace ok
