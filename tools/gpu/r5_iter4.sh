#!/bin/bash
# Profile: per-kernel cost of the headline query (concurrent and serialized), a traced 1-DP
# proving (host spans + kernel timeline), and the setup-share emulation.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5it4}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step kt 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -u bench.py --steps 3 --warmup 2
python3 tools/kernel_cost.py $(find $O/kt -name "*kernel_trace.csv" -print -quit) > $O/kcost_headline.txt
AMD_SERIALIZE_KERNEL=3 step kts 500 rocprofv3 --kernel-trace --output-format csv -d $O/kts -o run -- python3 -u bench.py --steps 3 --warmup 2
python3 tools/kernel_cost.py $(find $O/kts -name "*kernel_trace.csv" -print -quit) > $O/kcost_headline_ser.txt
rm -rf $O/kt $O/kts
DRYNX_TRACE=$O/trace_prove.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS= RANK_SHARE_PROVE=0,6 RANK_SHARE_TRACE_REPS=2 step ptl 400 rocprofv3 --kernel-trace --output-format csv -d $O/pt -o run -- python3 -u tools/rank_share.py --world 8 --reps 1
T=$(find $O/pt -name "*kernel_trace.csv" -print -quit)
python3 tools/kernel_timeline.py $T --gap 500 --burst -3 > $O/timeline_prove0.txt
python3 tools/kernel_timeline.py $T --gap 500 --burst -1 > $O/timeline_prove6.txt
python3 tools/host_trace.py $O/trace_prove.json 0.1 > $O/host_trace_prove.txt
rm -rf $O/pt
step setup 400 python -u tools/setup_share.py --world 8 --rank 0 --bench-json profiles/r5/it3/bench.json --json-out $O/setup_share_w8.json
head -1 $O/timeline_prove0.txt; head -25 $O/kcost_headline.txt
