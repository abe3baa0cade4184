#!/bin/bash
set -o pipefail
O=gpurun_out/r5spank; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
DRYNX_ROCTX=1 DRYNX_SPAN_SYNC=1 timeout -k 10 600 rocprofv3 --runtime-trace --output-format csv -d $O/rt -o run -- python3 -u bench.py --steps 3 --warmup 2 > $O/run.log 2>&1 || { tail -30 $O/run.log; exit 1; }
python3 tools/span_kernels.py $O/rt --queries 3 --out $O/span_kernels_sync.txt > $O/sk.log 2>&1 || { tail -20 $O/sk.log; exit 1; }
rm -rf $O/rt
head -60 $O/span_kernels_sync.txt
