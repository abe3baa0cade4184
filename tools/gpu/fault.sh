#!/bin/bash
# Attribution check: range-proof GPU tests, clean headline, fault-injected
# headline (DP 3's range proof corrupted), and a host trace of the
# no-range-proof line.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-900; if [ $rc -ne 0 ]; then tail -20 gpurun_out/$name.log; exit $rc; fi; }
step pytest_rp 300 python -u -m pytest tests/test_rpmsm.py tests/test_range_hardening.py -m gpu -x -q --timeout 120 --timeout-method thread
step bench 400 python -u bench.py --steps 10 --warmup 2
step bench_fault 400 python -u bench.py --steps 5 --warmup 1 --fault-dp 3
DRYNX_TRACE=gpurun_out/trace_u0l0 step bench_u0l0_trace 400 python -u bench.py --steps 3 --warmup 1 --u 0 --l 0
python tools/host_trace.py gpurun_out/trace_u0l0.r0.json 0.05 > gpurun_out/host_trace_u0l0.txt && echo trace ok
