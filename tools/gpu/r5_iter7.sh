#!/bin/bash
# Ledger-copy A/B (tools/ab_ledger_copy.py: no device-to-host copy, diagnostic only) and a
# host span trace + kernel timeline of the serial path (--u 0 --l 0).
set -o pipefail
O=gpurun_out/${R5_OUT:-r5it7}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step b1 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/b1.json
step nc1 300 python -u tools/ab_ledger_copy.py --steps 20 --warmup 5 --json-out $O/nc1.json
step b2 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/b2.json
step nc2 300 python -u tools/ab_ledger_copy.py --steps 20 --warmup 5 --json-out $O/nc2.json
DRYNX_TRACE=$O/u0 step u0t 300 python -u bench.py --steps 5 --warmup 2 --u 0 --l 0 --json-out $O/u0l0_traced.json
python3 tools/host_trace.py $O/u0.r0.json 0.1 > $O/host_trace_u0l0.txt
step u0k 300 rocprofv3 --kernel-trace --output-format csv -d $O/uk -o run -- python3 -u bench.py --steps 5 --warmup 2 --u 0 --l 0
python3 tools/trace_step.py $(find $O/uk -name "*kernel_trace.csv" -print -quit) 0.05 > $O/u0l0_step_kernels.txt
rm -rf $O/uk
head -3 $O/u0l0_step_kernels.txt
