#!/bin/bash
# Small-grid ledger copy: its GPU test, then headline vs the no-copy diagnostic on one box.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5it8}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step pyt 300 python -u -m pytest tests/test_gpu.py -m gpu -k "copy_to_host or batched_copy" -v --timeout 120 --timeout-method thread
step b1 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/b1.json --check-ledger
step nc1 300 python -u tools/ab_ledger_copy.py --steps 20 --warmup 5 --json-out $O/nc1.json
step b2 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/b2.json
step nc2 300 python -u tools/ab_ledger_copy.py --steps 20 --warmup 5 --json-out $O/nc2.json
for f in b1 nc1 b2 nc2; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['ms_per_step'], d['ranks'][0].get('ledger_readback'))"; done
