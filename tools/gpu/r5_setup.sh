#!/bin/bash
set -o pipefail
O=gpurun_out/${R5_OUT:-r5setup}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u tools/setup_share.py --mode full --json-out $O/setup_full.json > $O/setup_full.log 2>&1 || { tail -30 $O/setup_full.log; exit 1; }
DRYNX_TRACE=$O/setup_trace.json timeout -k 10 400 python -u tools/setup_share.py --world 8 --rank 0 --full-json $O/setup_full.json --bench-json ${BENCH_JSON:-profiles/r5/final/bench.json} --json-out $O/setup_share_w8.json > $O/setup.log 2>&1 || { tail -30 $O/setup.log; exit 1; }
tail -1 $O/setup.log | cut -c1-600
python3 tools/host_trace.py $O/setup_trace.json 1 > $O/setup_host_trace.txt
head -12 $O/setup_host_trace.txt
