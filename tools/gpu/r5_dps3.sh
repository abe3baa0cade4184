#!/bin/bash
set -o pipefail
O=gpurun_out/r5dps3; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
DRYNX_TRACE=$O/t.json timeout -k 10 500 python -u -c "
import sys, runpy
from drynx_amd.utils import timers
sys.argv = ['tools/bench_scaling.py', '1', 'dps']
runpy.run_path('tools/bench_scaling.py', run_name='__main__')
timers.dump_trace('$O/t.json')
" > $O/run.log 2>&1 || { tail -30 $O/run.log; exit 1; }
python3 tools/host_trace.py $O/t.json 5 > $O/host_trace.txt || true
grep -A45 "totals" $O/host_trace.txt | head -45
rm -f $O/t.json
