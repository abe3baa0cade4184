#!/bin/bash
# rocprofv3 kernel trace of the headline with every kernel serialized
# (AMD_SERIALIZE_KERNEL=3): each kernel's cost alone on the chip, no overlap
# inflation -> tools/kernel_cost.py gives the per-query cost table.
set -o pipefail
mkdir -p gpurun_out/prof_ser
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
export AMD_SERIALIZE_KERNEL=3
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ser -o bench -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_ser_run.log 2>&1; rc=$?
tail -1 gpurun_out/prof_ser_run.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
python3 tools/kernel_cost.py gpurun_out/prof_ser/bench_kernel_trace.csv > gpurun_out/kernel_cost_serial.txt
