#!/bin/bash
# Spans as profiler ranges: GPU time per framework span and per torch op of
# the 1-GPU pooled check + proving; headline, fault, no-range-proof line.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-220; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step pytest_it 300 python -u -m pytest tests/test_gpu.py tests/test_rpmsm.py -m gpu -x -q --timeout 200 --timeout-method thread
RANK_SHARE_TRACE_ONLY=1 DRYNX_TRACE=gpurun_out/trace_dummy.json RANK_SHARE_PARTS=0 step glue 400 python -u tools/rank_share.py --world 1 --reps 1 --torch-prof gpurun_out/torch_glue.txt
step bench_it 300 python -u bench.py --steps 10 --warmup 2
step bench_fault 300 python -u bench.py --steps 5 --warmup 1 --fault-dp 3
DRYNX_TRACE=gpurun_out/trace_u0l0 step bench_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python tools/host_trace.py gpurun_out/trace_u0l0.r0.json 0.05 > gpurun_out/host_trace_u0l0.txt
