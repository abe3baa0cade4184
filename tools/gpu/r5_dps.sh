#!/bin/bash
set -o pipefail
O=gpurun_out/r5dps; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 500 python -u tools/bench_scaling.py 3 dps > $O/dps_new.log 2>&1 || { tail -30 $O/dps_new.log; exit 1; }
grep '#DPs' $O/dps_new.log | cut -c1-160
RS="import sys, runpy; from drynx_amd.services import service; service.LEDGER_GT_T2 = False; sys.argv = ['tools/bench_scaling.py', '3', 'dps']; runpy.run_path('tools/bench_scaling.py', run_name='__main__')"
timeout -k 10 500 python -u -c "$RS" > $O/dps_raw.log 2>&1 || { tail -30 $O/dps_raw.log; exit 1; }
grep '#DPs' $O/dps_raw.log | cut -c1-160
