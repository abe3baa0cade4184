#!/bin/bash
# Headline host trace (span timeline of one rank, 6 steps).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
DRYNX_TRACE=gpurun_out/q_head_trace step q_head_tr 300 python -u bench.py --steps 6 --warmup 2 --json-out gpurun_out/q_head_tr.json
python3 tools/host_trace.py gpurun_out/q_head_trace.r0.json 0.1 > gpurun_out/q_host_trace_head.txt
