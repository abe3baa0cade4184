#!/bin/bash
# Kernel statistics of the headline (5 timed steps) + one W=8 pool part's host trace and kernel timeline.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6prof}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step stats 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o run -- python3 -u bench.py --steps 5 --warmup 2
S=$(find $O/st -name "*kernel_stats.csv" -print -quit); cp $S $O/kernel_stats_bench5.csv; rm -rf $O/st
DRYNX_TRACE=$O/trace.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=6,3 RANK_SHARE_TRACE_REPS=2 step tl 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -u tools/rank_share.py --world 8 --reps 1
T=$(find $O/kt -name "*kernel_trace.csv" -print -quit)
python3 tools/kernel_timeline.py $T --gap 500 --burst -3 > $O/timeline_part6.txt
python3 tools/kernel_timeline.py $T --gap 500 --burst -1 > $O/timeline_part3.txt
python3 tools/host_trace.py $O/trace.json 0.05 > $O/host_trace.txt
rm -rf $O/kt
head -1 $O/timeline_part6.txt; head -1 $O/timeline_part3.txt
