#!/bin/bash
# Checkpoint: GPU suite (incl. the 2-rank device tests), driver-form headline, a 100-step durable-ledger run.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5chk}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread
step bench 400 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json
step bench100 600 python -u bench.py --steps 100 --warmup 5 --json-out $O/bench100.json
df -h /tmp > $O/df.txt
