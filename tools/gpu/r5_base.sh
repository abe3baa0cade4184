#!/bin/bash
# Round-5 baseline on a fresh box: GPU suite, driver-form headline, serial line, W=8 rank share.
set -o pipefail
mkdir -p gpurun_out/r5base
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
O=gpurun_out/r5base
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -30 $O/$name.log; exit $rc; fi; }
step pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
step bench 400 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json
step u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out $O/u0l0.json
step share 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json $O/u0l0.json --json-out $O/rank_share_w8.json
