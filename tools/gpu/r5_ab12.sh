#!/bin/bash
# Same-box A/B: the tree at the ledger-copy commit (abtmp/r8, same native library) vs HEAD.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5ab12}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$(pwd)
step() { local name=$1; shift; timeout -k 10 "$@" > $R/$O/$name.log 2>&1; local rc=$?; tail -1 $R/$O/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -40 $R/$O/$name.log; exit $rc; fi; }
step head1 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/head1.json
(cd abtmp/r8 && step old1 300 python -u bench.py --steps 20 --warmup 5 --json-out $R/$O/old1.json) || exit 1
step head2 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/head2.json
(cd abtmp/r8 && step old2 300 python -u bench.py --steps 20 --warmup 5 --json-out $R/$O/old2.json) || exit 1
for f in head1 old1 head2 old2; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['ms_per_step'])"; done
