#!/bin/bash
# Equal pool parts: multi-rank GPU test, W=8 rank share with the synchronised projection.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5it16}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step pyt 400 python -u -m pytest tests/test_multirank_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread
step share 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json profiles/r5/it10/u0l0.json --ctrl-json profiles/r5/it10/ctrl_w8.json --json-out $O/rank_share_w8.json
grep rank $O/share.log
