#!/bin/bash
# Same-box A/B of the working tree against a snapshot of another commit in ab_base/
# (same native library): headline A B A B, then the W=8 pool share of each.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6abtree}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$(pwd)
step() { local name=$1; shift; timeout -k 10 "$@" > $R/$O/$name.log 2>&1; local rc=$?; tail -1 $R/$O/$name.log | cut -c1-160; if [ $rc -ne 0 ]; then tail -40 $R/$O/$name.log; exit $rc; fi; }
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_rpmsm.py tests/test_range_hardening.py tests/test_gpu.py tests/test_ledger_codec.py
step new1 300 python -u bench.py --steps 10 --warmup 3 --json-out $O/new1.json
(cd ab_base && step old1 300 python -u bench.py --steps 10 --warmup 3 --json-out $R/$O/old1.json) || exit 1
step new2 300 python -u bench.py --steps 10 --warmup 3 --json-out $O/new2.json
(cd ab_base && step old2 300 python -u bench.py --steps 10 --warmup 3 --json-out $R/$O/old2.json) || exit 1
step sharenew 500 python -u tools/rank_share.py --world 8 --reps 3 --ctrl-json profiles/r5/final/ctrl_w8.json --json-out $O/share_new.json
(cd ab_base && step shareold 500 python -u tools/rank_share.py --world 8 --reps 3 --ctrl-json $R/profiles/r5/final/ctrl_w8.json --json-out $R/$O/share_old.json) || exit 1
