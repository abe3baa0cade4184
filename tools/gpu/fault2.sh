#!/bin/bash
# Fault-injected headline (DP 3's range proof corrupted) with host spans,
# against the clean headline on the same box.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-600; if [ $rc -ne 0 ]; then tail -20 gpurun_out/$name.log; exit $rc; fi; }
step bench 400 python -u bench.py --steps 6 --warmup 2
DRYNX_TRACE=gpurun_out/trace_fault step bench_fault 400 python -u bench.py --steps 4 --warmup 1 --fault-dp 3
python tools/host_trace.py gpurun_out/trace_fault.r0.json 0.3 > gpurun_out/host_trace_fault.txt && echo trace ok
