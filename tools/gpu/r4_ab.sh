#!/bin/bash
# A/B of the round-4 headline changes (10 steps each): as built, without the
# kept per-segment buckets, with synchronising phase timers, with 32-bit
# GT-membership weights (diagnostic only), with torch's plan sort; then the
# no-range-proof line with host spans.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-220; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step ab_base 300 python -u bench.py --steps 10 --warmup 2
DRYNX_SEG_KEEP=0 step ab_nokeep 300 python -u bench.py --steps 10 --warmup 2
DRYNX_TIMER_SYNC=1 step ab_timersync 300 python -u bench.py --steps 10 --warmup 2
DRYNX_GAMMA_BITS=32 step ab_gamma32 300 python -u bench.py --steps 10 --warmup 2
DRYNX_PLAN_SORT=torch step ab_torchsort 300 python -u bench.py --steps 10 --warmup 2
DRYNX_TRACE=gpurun_out/trace_u0l0 step bench_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python tools/host_trace.py gpurun_out/trace_u0l0.r0.json 0.05 > gpurun_out/host_trace_u0l0.txt
