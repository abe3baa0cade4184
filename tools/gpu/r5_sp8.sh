#!/bin/bash
set -o pipefail
O=gpurun_out/r5sp8; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rpmsm.py -v --timeout 200 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RS="import sys, runpy; from drynx_amd import native as nt; nt.U_JOINT_SP8_BELOW = 0; sys.argv = ['tools/rank_share.py'] + sys.argv[1:]; runpy.run_path('tools/rank_share.py', run_name='__main__')"
for i in 1 2; do
timeout -k 10 400 python -u -c "$RS" --world 8 --reps 3 --json-out $O/share_old$i.json > $O/share_old$i.log 2>&1 || { tail -20 $O/share_old$i.log; exit 1; }
echo "old $(tail -1 $O/share_old$i.log | cut -c1-300)"
timeout -k 10 400 python -u tools/rank_share.py --world 8 --reps 3 --json-out $O/share_new$i.json > $O/share_new$i.log 2>&1 || { tail -20 $O/share_new$i.log; exit 1; }
echo "new $(tail -1 $O/share_new$i.log | cut -c1-300)"
done
DRYNX_TRACE=$O/trace.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=6,3 RANK_SHARE_TRACE_REPS=2 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -u tools/rank_share.py --world 8 --reps 1 > $O/tl.log 2>&1 || { tail -20 $O/tl.log; exit 1; }
T=$(find $O/kt -name "*kernel_trace.csv" -print -quit)
python3 tools/kernel_timeline.py $T --gap 500 --burst -3 > $O/timeline_part6.txt
rm -rf $O/kt
head -1 $O/timeline_part6.txt; grep u_joint $O/timeline_part6.txt
