#!/bin/bash
# Span trace of two W=8 pool parts (a VN rank and a 2-DP helper) on the final tree.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
DRYNX_TRACE=gpurun_out/s_parts_trace.json RANK_SHARE_PARTS=3,6 RANK_SHARE_TRACE_ONLY=1 timeout -k 10 400 python -u tools/rank_share.py --world 8 --reps 1 > gpurun_out/s_parts.log 2>&1 || { tail -30 gpurun_out/s_parts.log; exit 1; }
python3 tools/host_trace.py gpurun_out/s_parts_trace.json 0.1 > gpurun_out/s_host_trace_parts.txt
tail -3 gpurun_out/s_host_trace_parts.txt
