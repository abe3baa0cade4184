#!/bin/bash
# Same-box A/B, HEAD vs abtmp/prev (the tree before the last change, same native library):
# serial path x3 each, headline x2 each.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5ab19}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$(pwd)
step() { local name=$1; shift; timeout -k 10 "$@" > $R/$O/$name.log 2>&1; local rc=$?; if [ $rc -ne 0 ]; then tail -40 $R/$O/$name.log; exit $rc; fi; }
U="--steps 20 --warmup 5 --u 0 --l 0"
for i in 1 2 3; do
  step u_head$i 300 python -u bench.py $U --json-out $O/u_head$i.json
  (cd abtmp/prev && step u_prev$i 300 python -u bench.py $U --json-out $R/$O/u_prev$i.json) || exit 1
done
for i in 1 2; do
  step h_head$i 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/h_head$i.json
  (cd abtmp/prev && step h_prev$i 300 python -u bench.py --steps 20 --warmup 5 --json-out $R/$O/h_prev$i.json) || exit 1
done
for f in $O/*.json; do python3 -c "import json,statistics;d=json.load(open('$f'));print('$f', d['ms_per_step'], statistics.median(d['ranks'][0]['step_ms']))"; done
