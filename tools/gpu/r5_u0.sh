#!/bin/bash
# Serial path (--u 0 --l 0): timed run, host span trace, kernel timeline of the last step.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5u0}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-150; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step u0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out $O/u0l0.json
DRYNX_TRACE=$O/u0 step u0t 300 python -u bench.py --steps 5 --warmup 2 --u 0 --l 0 --json-out $O/u0l0_traced.json
python3 tools/host_trace.py $O/u0.r0.json 0.1 > $O/host_trace_u0l0.txt
step u0k 300 rocprofv3 --kernel-trace --output-format csv -d $O/uk -o run -- python3 -u bench.py --steps 5 --warmup 2 --u 0 --l 0
python3 tools/trace_step.py $(find $O/uk -name "*kernel_trace.csv" -print -quit) 0.05 > $O/u0l0_step_kernels.txt
rm -rf $O/uk
