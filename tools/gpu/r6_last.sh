#!/bin/bash
# Last check of a tree: full GPU suite, smoke, 20-step headline (driver form), lr_dro, 8-rank rehearsal.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6last}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step pytest 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json
step lrdro 300 python -u bench.py --query lr_dro --steps 5 --warmup 2 --json-out $O/lrdro.json
REH_OUT=${R6_OUT:-r6last}/reh8 bash tools/gpu/reh8.sh
