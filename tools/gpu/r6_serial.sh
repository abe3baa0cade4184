#!/bin/bash
# The serial (no range proof) path: 20-step --u 0 --l 0 in the driver's form + a host span trace of it.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6serial}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step u0l0 300 python -u bench.py --u 0 --l 0 --steps 20 --warmup 3 --json-out $O/u0l0.json
DRYNX_TRACE=$O/tr step u0l0tr 300 python -u bench.py --u 0 --l 0 --steps 5 --warmup 3
python3 tools/host_trace.py $O/tr.r0.json 0.1 > $O/host_trace_u0l0.txt && rm -f $O/tr.r0.json
