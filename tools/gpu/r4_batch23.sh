#!/bin/bash
# Batched LR encoder (one reduction launch for all DPs of a rank): GPU tests,
# u0l0 x2 + trace, headline x2.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step p_tests 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu.py tests/test_encoding.py
step p_u0l0_1 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/p_u0l0_1.json
step p_head_1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/p_head_1.json
step p_u0l0_2 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/p_u0l0_2.json
step p_head_2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/p_head_2.json
DRYNX_TRACE=gpurun_out/p_u0l0_trace step p_u0l0_tr 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python3 tools/host_trace.py gpurun_out/p_u0l0_trace.r0.json 0.1 > gpurun_out/p_host_trace_u0l0.txt
