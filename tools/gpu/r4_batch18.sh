#!/bin/bash
# Querier start after the first CN proofs are signed (default) vs at once
# (DRYNX_CLIENT_EARLY=1), alternating on one box: u0l0 and the headline.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step k_u0l0_late1 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/k_u0l0_late1.json
DRYNX_CLIENT_EARLY=1 step k_u0l0_early1 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/k_u0l0_early1.json
step k_u0l0_late2 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/k_u0l0_late2.json
DRYNX_CLIENT_EARLY=1 step k_u0l0_early2 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/k_u0l0_early2.json
step k_head_late1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/k_head_late1.json
DRYNX_CLIENT_EARLY=1 step k_head_early1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/k_head_early1.json
step k_head_late2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/k_head_late2.json
DRYNX_TRACE=gpurun_out/k_u0l0_trace step k_u0l0_tr 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python3 tools/host_trace.py gpurun_out/k_u0l0_trace.r0.json 0.1 > gpurun_out/k_host_trace_u0l0.txt
