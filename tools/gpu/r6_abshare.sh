#!/bin/bash
# Same-box A/B of the W=8 pool parts: working tree vs the ab_base/ snapshot (new, old, new, old).
set -o pipefail
O=gpurun_out/${R6_OUT:-r6abshare}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$(pwd)
step() { local name=$1; shift; timeout -k 10 "$@" > $R/$O/$name.log 2>&1; local rc=$?; tail -1 $R/$O/$name.log | cut -c1-160; if [ $rc -ne 0 ]; then tail -40 $R/$O/$name.log; exit $rc; fi; }
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu.py
for k in 1 2; do
  step new$k 500 python -u tools/rank_share.py --world 8 --reps 3 --ctrl-json profiles/r5/final/ctrl_w8.json --json-out $O/new$k.json
  (cd ab_base && step old$k 500 python -u tools/rank_share.py --world 8 --reps 3 --ctrl-json $R/profiles/r5/final/ctrl_w8.json --json-out $R/$O/old$k.json) || exit 1
done
