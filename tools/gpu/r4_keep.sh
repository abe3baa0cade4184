#!/bin/bash
# Span-synchronised cost of the whole 1-GPU pooled range check (3 VNs, the
# full inbox as one part) with and without the kept per-segment buckets.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-220; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
DRYNX_TRACE=gpurun_out/trace_w1_keep.json DRYNX_SPAN_SYNC=1 RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=0 step w1_keep 400 python -u tools/rank_share.py --world 1 --reps 1
python tools/host_trace.py gpurun_out/trace_w1_keep.json 0.1 > gpurun_out/host_trace_w1_keep.txt
DRYNX_SEG_KEEP=0 DRYNX_TRACE=gpurun_out/trace_w1_nokeep.json DRYNX_SPAN_SYNC=1 RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=0 step w1_nokeep 400 python -u tools/rank_share.py --world 1 --reps 1
python tools/host_trace.py gpurun_out/trace_w1_nokeep.json 0.1 > gpurun_out/host_trace_w1_nokeep.txt
DRYNX_TRACE=gpurun_out/trace_pool.json DRYNX_SPAN_SYNC=1 RANK_SHARE_TRACE_ONLY=1 step share_trace 400 python -u tools/rank_share.py --world 8 --reps 1
python tools/host_trace.py gpurun_out/trace_pool.json 0.1 > gpurun_out/host_trace_pool.txt
