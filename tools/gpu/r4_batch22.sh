#!/bin/bash
# No early range plane without range proofs: u0l0 x3 + trace, headline once,
# the proof-collection GPU tests.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step o_tests 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu.py tests/test_pool.py
step o_u0l0_1 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/o_u0l0_1.json
step o_u0l0_2 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/o_u0l0_2.json
step o_head 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/o_head.json
step o_u0l0_3 300 python -u bench.py --steps 20 --warmup 5 --u 0 --l 0 --json-out gpurun_out/o_u0l0_3.json
DRYNX_TRACE=gpurun_out/o_u0l0_trace step o_u0l0_tr 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python3 tools/host_trace.py gpurun_out/o_u0l0_trace.r0.json 0.1 > gpurun_out/o_host_trace_u0l0.txt
