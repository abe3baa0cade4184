#!/bin/bash
# Radix-sort plans back: headline, W=8 rank share, traced pool parts, and a span-synced
# trace of the setup-share emulation (where its 1/8 build spends its time).
set -o pipefail
O=gpurun_out/${R5_OUT:-r5it11}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-250; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step pyt 300 python -u -m pytest tests/test_rpmsm.py tests/test_timers.py -m gpu -x -v --timeout 120 --timeout-method thread
step bench 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json
step share 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json profiles/r5/it10/u0l0.json --ctrl-json profiles/r5/it10/ctrl_w8.json --json-out $O/rank_share_w8.json
DRYNX_TRACE=$O/setup_trace.json DRYNX_SPAN_SYNC=1 step setup 400 python -u tools/setup_share.py --world 8 --rank 0 --bench-json $O/bench.json --json-out $O/setup_share_w8.json
python3 tools/host_trace.py $O/setup_trace.json 1 > $O/setup_host_trace.txt || true
DRYNX_TRACE=$O/trace.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=6,3 RANK_SHARE_TRACE_REPS=2 step tl 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -u tools/rank_share.py --world 8 --reps 1
T=$(find $O/kt -name "*kernel_trace.csv" -print -quit)
python3 tools/kernel_timeline.py $T --gap 500 --burst -3 > $O/timeline_part6.txt
python3 tools/kernel_timeline.py $T --gap 500 --burst -1 > $O/timeline_part3.txt
python3 tools/host_trace.py $O/trace.json 0.1 > $O/host_trace.txt
rm -rf $O/kt
head -1 $O/timeline_part6.txt; head -1 $O/timeline_part3.txt
