#!/bin/bash
# Kernel time per framework span of the timed headline queries (roctx ranges + runtime trace).
set -o pipefail
O=gpurun_out/${R6_OUT:-r6spank}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
DRYNX_ROCTX=1 step rt 400 rocprofv3 --runtime-trace --output-format csv -d $O/rt -o run -- python3 -u bench.py --steps 3 --warmup 1
python3 tools/span_kernels.py $O/rt --queries 3 > $O/span_kernels.txt && rm -rf $O/rt && head -40 $O/span_kernels.txt
