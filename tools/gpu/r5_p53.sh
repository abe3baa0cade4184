#!/bin/bash
set -o pipefail
O=gpurun_out/${R5_OUT:-r5p53}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
DRYNX_TRACE=$O/trace.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=5,3 RANK_SHARE_TRACE_REPS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -u tools/rank_share.py --world 8 --reps 1 > $O/tl.log 2>&1 || { tail -20 $O/tl.log; exit 1; }
T=$(find $O/kt -name "*kernel_trace.csv" -print -quit)
python3 tools/kernel_timeline.py $T --gap 500 --burst -3 > $O/timeline_part5.txt
python3 tools/kernel_timeline.py $T --gap 500 --burst -1 > $O/timeline_part3.txt
python3 tools/host_trace.py $O/trace.json 0.1 > $O/host_trace.txt
rm -rf $O/kt
head -1 $O/timeline_part5.txt; head -1 $O/timeline_part3.txt; grep "pool_part" $O/host_trace.txt
