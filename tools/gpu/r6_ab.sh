#!/bin/bash
# Same-box A/B of a runtime switch on the headline (A, B, A), then the W=8 pool share.
# R6_AB="ENV=VALUE" is the B side.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6ab}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step a1 300 python -u bench.py --steps 10 --warmup 3 --json-out $O/a1.json
step b1 300 env ${R6_AB} python -u bench.py --steps 10 --warmup 3 --json-out $O/b1.json
step a2 300 python -u bench.py --steps 10 --warmup 3 --json-out $O/a2.json
step b2 300 env ${R6_AB} python -u bench.py --steps 10 --warmup 3 --json-out $O/b2.json
if [ -n "${R6_SHARE:-}" ]; then
  step share 500 python -u tools/rank_share.py --world 8 --reps 3 --ctrl-json profiles/r5/final/ctrl_w8.json --json-out $O/rank_share_w8.json
fi
