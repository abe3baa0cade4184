#!/bin/bash
# Same-box A/B, interleaved: HIP hardware queues per process 4 (box default) vs 8.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5ab17}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
for i in 1 2 3 4; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q step b_q${q}_$i 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/b_q${q}_$i.json
  done
done
for f in $O/b_q*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['ms_per_step'])"; done
