#!/bin/bash
# Round-6 baseline: headline (driver form), serial line, W=8 rank share.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6base}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step bench 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json
step u0l0 300 python -u bench.py --steps 20 --warmup 5 --u 0 --l 0 --json-out $O/u0l0.json
step share 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json $O/u0l0.json --ctrl-json profiles/r5/final/ctrl_w8.json --json-out $O/rank_share_w8.json
