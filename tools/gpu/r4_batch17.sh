#!/bin/bash
# Priority policy by query (range work on the GPU or not): u0l0 twice, the
# headline, a u0l0 host trace; the service GPU tests.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step j_tests 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu.py
step j_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/j_u0l0.json
step j_head 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/j_head.json
step j_u0l0b 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/j_u0l0b.json
DRYNX_TRACE=gpurun_out/j_u0l0_trace step j_u0l0_tr 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python3 tools/host_trace.py gpurun_out/j_u0l0_trace.r0.json 0.1 > gpurun_out/j_host_trace_u0l0.txt
