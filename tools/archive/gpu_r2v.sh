#!/bin/bash
# True per-kernel cost of one query: kernel trace with every launch serialized (AMD_SERIALIZE_KERNEL=3).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
rm -rf gpurun_out/profv
AMD_SERIALIZE_KERNEL=3 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/profv -o bench -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/profv_run.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/profv_run.log | cut -c1-200; fatal $rc prof
python tools/kernel_cost.py gpurun_out/profv/bench_kernel_trace.csv > gpurun_out/kernel_cost_serial.txt; head -45 gpurun_out/kernel_cost_serial.txt
