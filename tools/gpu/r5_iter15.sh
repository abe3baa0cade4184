#!/bin/bash
# Host tails under the multi-exponentiation: GPU tests, same-box headline A/B vs the it8 tree
# (abtmp/r8), W=8 rank share, traced pool parts.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5it15}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$(pwd)
step() { local name=$1; shift; timeout -k 10 "$@" > $R/$O/$name.log 2>&1; local rc=$?; tail -1 $R/$O/$name.log | cut -c1-160; if [ $rc -ne 0 ]; then tail -40 $R/$O/$name.log; exit $rc; fi; }
step pyt 600 python -u -m pytest tests/test_rpmsm.py tests/test_gpu.py tests/test_multirank_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
step head1 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/head1.json
(cd abtmp/r8 && step old1 300 python -u bench.py --steps 20 --warmup 5 --json-out $R/$O/old1.json) || exit 1
step head2 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/head2.json
(cd abtmp/r8 && step old2 300 python -u bench.py --steps 20 --warmup 5 --json-out $R/$O/old2.json) || exit 1
step share 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json profiles/r5/it10/u0l0.json --ctrl-json profiles/r5/it10/ctrl_w8.json --json-out $O/rank_share_w8.json
DRYNX_TRACE=$O/trace.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=6,3 RANK_SHARE_TRACE_REPS=2 step tl 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -u tools/rank_share.py --world 8 --reps 1
T=$(find $O/kt -name "*kernel_trace.csv" -print -quit)
python3 tools/kernel_timeline.py $T --gap 500 --burst -3 > $O/timeline_part6.txt
python3 tools/kernel_timeline.py $T --gap 500 --burst -1 > $O/timeline_part3.txt
python3 tools/host_trace.py $O/trace.json 0.1 > $O/host_trace.txt
rm -rf $O/kt
for f in head1 old1 head2 old2; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['ms_per_step'])"; done
head -1 $O/timeline_part6.txt; head -1 $O/timeline_part3.txt
