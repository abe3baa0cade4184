#!/bin/bash
# Same-box A/B of the HIP hardware-queue count per process (streams beyond it share queues
# and run in order): headline and W=8 rank share at 4 (the box default), 8 and 16.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5ab13}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-100; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
for q in 4 8 16 4 8 16; do
  GPU_MAX_HW_QUEUES=$q step b_q$q 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/b_q${q}_$RANDOM.json
done
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q step s_q$q 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json profiles/r5/it10/u0l0.json --ctrl-json profiles/r5/it10/ctrl_w8.json --json-out $O/share_q$q.json
done
for f in $O/b_q*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['ms_per_step'])"; done
