#!/bin/bash
set -o pipefail
O=gpurun_out/r5dps2; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
RS="import sys, runpy; from drynx_amd.protocols import proof_collection as pc; pc.LEDGER_PREFETCH = False; sys.argv = ['tools/bench_scaling.py', '3', 'dps']; runpy.run_path('tools/bench_scaling.py', run_name='__main__')"
timeout -k 10 500 python -u -c "$RS" > $O/dps_nopf.log 2>&1 || { tail -30 $O/dps_nopf.log; exit 1; }
grep '#DPs' $O/dps_nopf.log | cut -c1-160
