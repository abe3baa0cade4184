#!/bin/bash
# Round-4 iteration 5: GPU tests (split U combinations, GLV key-switch
# check), headline + plan-sort A/B, one rank's pool share (adaptive R
# window, split U), then the multi-rank path on this one GPU over gloo with
# bench.py's own launcher: 4 ranks at d = 20 and the 8-rank placement at
# d = 12 (sharded prover tables, 1/W pool slices).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-500; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step pytest_it 300 python -u -m pytest tests/test_rpmsm.py tests/test_ks_direct_gpu.py tests/test_gpu.py tests/test_range_hardening.py -m gpu -x -q --timeout 200 --timeout-method thread
step bench_it 300 python -u bench.py --steps 10 --warmup 2
DRYNX_PLAN_SORT=torch step bench_torchsort 300 python -u bench.py --steps 10 --warmup 2
step rank_share 400 python -u tools/rank_share.py --world 8 --reps 3 --serial-json profiles/r4/bench_u0l0_event_timers.json --json-out gpurun_out/rank_share.json
DRYNX_DIST_BACKEND=gloo step rehearsal_4rank 400 python -u bench.py --gpus 4 --steps 3 --warmup 1 --features 20 --device cuda:0
DRYNX_DIST_BACKEND=gloo step rehearsal_8rank 500 python -u bench.py --gpus 8 --steps 3 --warmup 1 --features 12 --device cuda:0
