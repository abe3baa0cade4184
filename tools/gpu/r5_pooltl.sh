#!/bin/bash
# Concurrent timeline of one W=8 pool part (rank 6 helper) + its host trace.
set -o pipefail
O=gpurun_out/r5tl; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
DRYNX_TRACE=$O/trace.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=6 RANK_SHARE_TRACE_REPS=3 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -u tools/rank_share.py --world 8 --reps 1 > $O/run.log 2>&1 || { tail -30 $O/run.log; exit 1; }
T=$(find $O/kt -name "*kernel_trace.csv" -print -quit)
python3 tools/kernel_timeline.py $T --gap 500 --burst -1 > $O/timeline_part6.txt
python3 tools/host_trace.py $O/trace.json 0.1 > $O/host_trace.txt
rm -rf $O/kt
head -3 $O/timeline_part6.txt
