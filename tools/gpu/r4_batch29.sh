#!/bin/bash
# GIL switch interval (DRYNX_SWITCH_INTERVAL=0.0005 vs the 5 ms default):
# u0l0 and headline, alternating.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step v_u0l0_def1 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/v_u0l0_def1.json
DRYNX_SWITCH_INTERVAL=0.0005 step v_u0l0_sw1 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/v_u0l0_sw1.json
step v_u0l0_def2 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/v_u0l0_def2.json
DRYNX_SWITCH_INTERVAL=0.0005 step v_u0l0_sw2 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/v_u0l0_sw2.json
step v_head_def1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/v_head_def1.json
DRYNX_SWITCH_INTERVAL=0.0005 step v_head_sw1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/v_head_sw1.json
step v_head_def2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/v_head_def2.json
DRYNX_SWITCH_INTERVAL=0.0005 step v_head_sw2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/v_head_sw2.json
DRYNX_SWITCH_INTERVAL=0.0005 DRYNX_TRACE=gpurun_out/v_u0l0_trace step v_u0l0_tr 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python3 tools/host_trace.py gpurun_out/v_u0l0_trace.r0.json 0.1 > gpurun_out/v_host_trace_u0l0_sw.txt
