#!/bin/bash
# Weighted pool parts: W=8 rank shares, plus the headline.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step f_share 600 python -u tools/rank_share.py --world 8 --reps 3 --serial-json profiles/r4/checkpoint_u0l0.json --json-out gpurun_out/f_rank_share_w8.json
DRYNX_POOL_BALANCE=0 step f_share_eq 600 python -u tools/rank_share.py --world 8 --reps 3 --serial-json profiles/r4/checkpoint_u0l0.json --json-out gpurun_out/f_rank_share_w8_equal.json
step f_bench 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/f_bench.json
