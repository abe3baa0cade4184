#!/bin/bash
# GIL switch interval default (0.5 ms) vs the interpreter's 5 ms
# (DRYNX_SWITCH_INTERVAL=0): W=8 rank shares and the headline, alternating.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-160; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step w_share_sw 600 python -u tools/rank_share.py --world 8 --reps 3 --order 4,5,3,0,1,2,6,7 --json-out gpurun_out/w_share_sw.json
DRYNX_SWITCH_INTERVAL=0 step w_share_def 600 python -u tools/rank_share.py --world 8 --reps 3 --order 4,5,3,0,1,2,6,7 --json-out gpurun_out/w_share_def.json
step w_head_sw1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/w_head_sw1.json
DRYNX_SWITCH_INTERVAL=0 step w_head_def1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/w_head_def1.json
step w_head_sw2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/w_head_sw2.json
DRYNX_SWITCH_INTERVAL=0 step w_head_def2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/w_head_def2.json
