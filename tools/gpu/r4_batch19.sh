#!/bin/bash
# Host Schnorr signing of small envelope batches (the CN proofs' signing waits
# ~4 ms behind the key-switch proof kernels on the device): u0l0 and headline.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step l_u0l0_dev 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/l_u0l0_dev.json
DRYNX_SIGN_DEVICE_MIN=8 step l_u0l0_host8 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/l_u0l0_host8.json
step l_u0l0_dev2 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/l_u0l0_dev2.json
DRYNX_SIGN_DEVICE_MIN=8 step l_u0l0_host8b 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/l_u0l0_host8b.json
step l_head_dev 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/l_head_dev.json
DRYNX_SIGN_DEVICE_MIN=8 step l_head_host8 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/l_head_host8.json
DRYNX_SIGN_DEVICE_MIN=8 DRYNX_TRACE=gpurun_out/l_u0l0_trace step l_u0l0_tr 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python3 tools/host_trace.py gpurun_out/l_u0l0_trace.r0.json 0.1 > gpurun_out/l_host_trace_u0l0_host8.txt
