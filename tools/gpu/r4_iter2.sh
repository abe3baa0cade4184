#!/bin/bash
# Round-4 iteration 2: range GPU tests (rocPRIM bucket sort, device slice
# plans, kept per-segment buckets), headline, fault-injected headline, the
# per-rank share of the 8-rank schedule with torch-op attribution.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-600; if [ $rc -ne 0 ]; then tail -25 gpurun_out/$name.log; exit $rc; fi; }
step pytest_it 300 python -u -m pytest tests/test_rpmsm.py tests/test_range_hardening.py tests/test_sigma.py tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread
DRYNX_TRACE=gpurun_out/trace step bench_it 300 python -u bench.py --steps 10 --warmup 2
python tools/host_trace.py gpurun_out/trace.r0.json 0.3 > gpurun_out/host_trace.txt
DRYNX_TRACE=gpurun_out/trace_fault step bench_fault_it 300 python -u bench.py --steps 5 --warmup 1 --fault-dp 3
python tools/host_trace.py gpurun_out/trace_fault.r0.json 0.3 > gpurun_out/host_trace_fault.txt
step rank_share 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json profiles/r4/bench_u0l0_event_timers.json --json-out gpurun_out/rank_share.json --torch-prof gpurun_out/torch_glue.txt
