#!/bin/bash
set -o pipefail
O=gpurun_out/r5sp2; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for i in 1 2; do
for sp in 2 4; do
RS="import sys, runpy; from drynx_amd import native as nt; nt.U_JOINT_SP_SMALL = $sp; sys.argv = ['tools/rank_share.py'] + sys.argv[1:]; runpy.run_path('tools/rank_share.py', run_name='__main__')"
timeout -k 10 400 python -u -c "$RS" --world 8 --reps 3 --json-out $O/share_sp${sp}_$i.json > $O/share_sp${sp}_$i.log 2>&1 || { tail -20 $O/share_sp${sp}_$i.log; exit 1; }
echo "sp=$sp $(tail -1 $O/share_sp${sp}_$i.log | cut -c1-300)"
done
done
