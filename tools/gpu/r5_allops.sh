#!/bin/bash
# Every AllOps operation and the scaling sweeps on the final tree.
set -o pipefail
O=gpurun_out/r5allops; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python -u tools/bench_allops.py > $O/allops.log 2>&1 || { tail -30 $O/allops.log; exit 1; }
tail -16 $O/allops.log | cut -c1-160
timeout -k 10 500 python -u tools/bench_scaling.py 3 dps > $O/scaling_dps.log 2>&1 || { tail -30 $O/scaling_dps.log; exit 1; }
tail -10 $O/scaling_dps.log | cut -c1-200
