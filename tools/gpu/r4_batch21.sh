#!/bin/bash
# CN-proof jobs wait for their inputs when they start (event), not at submit:
# device signing vs host signing of small batches (DRYNX_SIGN_DEVICE_MIN=8), alternating.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step n_u0l0_dev 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/n_u0l0_dev.json
DRYNX_SIGN_DEVICE_MIN=8 step n_u0l0_host8 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/n_u0l0_host8.json
step n_u0l0_dev2 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/n_u0l0_dev2.json
DRYNX_SIGN_DEVICE_MIN=8 step n_u0l0_host8b 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/n_u0l0_host8b.json
step n_head_dev 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/n_head_dev.json
DRYNX_SIGN_DEVICE_MIN=8 step n_head_host8 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/n_head_host8.json
step n_head_dev2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/n_head_dev2.json
DRYNX_SIGN_DEVICE_MIN=8 step n_head_host8b 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/n_head_host8b.json
DRYNX_TRACE=gpurun_out/n_u0l0_trace step n_u0l0_tr 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python3 tools/host_trace.py gpurun_out/n_u0l0_trace.r0.json 0.1 > gpurun_out/n_host_trace_u0l0.txt
