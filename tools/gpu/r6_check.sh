#!/bin/bash
# Round-6 checkpoint: GPU suite (device assertion on), smoke, headline, W=8 share in pool and vn-local modes.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6check}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step pytest 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json
step share 500 python -u tools/rank_share.py --world 8 --reps 3 --ctrl-json profiles/r5/final/ctrl_w8.json --json-out $O/rank_share_w8.json
step sharel 500 python -u tools/rank_share.py --world 8 --reps 3 --vn-mode local --ctrl-json profiles/r5/final/ctrl_w8.json --json-out $O/rank_share_w8_local.json
