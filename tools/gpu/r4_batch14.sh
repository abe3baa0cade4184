#!/bin/bash
# Stream-priority A/B for the serial path: querier at normal priority with
# the CN-proof stream high (the CN proofs' signing waits behind the querier's
# decryption in the u0l0 trace), on both lines; plus the generator tests.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step h_tests 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_digest_rng.py tests/test_sigma.py
step h_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/h_u0l0.json
DRYNX_HP_STREAM=0 DRYNX_CNP_PRIORITY=-1 step h_u0l0_prio 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/h_u0l0_prio.json
step h_head 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/h_head.json
DRYNX_HP_STREAM=0 DRYNX_CNP_PRIORITY=-1 step h_head_prio 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/h_head_prio.json
DRYNX_HP_STREAM=0 DRYNX_CNP_PRIORITY=-1 DRYNX_TRACE=gpurun_out/h_u0l0_trace step h_u0l0_prio_tr 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python3 tools/host_trace.py gpurun_out/h_u0l0_trace.r0.json 0.1 > gpurun_out/h_host_trace_u0l0_prio.txt
