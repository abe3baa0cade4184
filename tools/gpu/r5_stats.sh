#!/bin/bash
set -o pipefail
O=gpurun_out/r5stats; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
S=$(find $O/prof -name "*kernel_stats.csv" -print -quit)
cp $S $O/kernel_stats.csv
T=$(find $O/prof -name "*kernel_trace.csv" -print -quit)
python3 tools/trace_step.py $T 0.05 > $O/step_kernels.txt || true
rm -rf $O/prof
head -30 $O/kernel_stats.csv | cut -c1-200
