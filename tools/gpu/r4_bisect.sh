#!/bin/bash
# Same-box bisection of the round-4 headline against the round-3 tree
# (_r3ref/, this call only): r4 with one change reverted at a time.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
(cd _r3ref && timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > ../gpurun_out/bs_r3.log 2>&1) && tail -1 gpurun_out/bs_r3.log | cut -c1-120
step bs_r4 300 python -u bench.py --steps 10 --warmup 2
DRYNX_TIMER_SYNC=1 step bs_timersync 300 python -u bench.py --steps 10 --warmup 2
DRYNX_CNP_PRIORITY=0 step bs_cnp0 300 python -u bench.py --steps 10 --warmup 2
DRYNX_PROOF_STAGES=1 step bs_stages1 300 python -u bench.py --steps 10 --warmup 2
DRYNX_SIGN_DEVICE_MIN=1 step bs_signdev 300 python -u bench.py --steps 10 --warmup 2
DRYNX_GAMMA_BITS=32 step bs_gamma32 300 python -u bench.py --steps 10 --warmup 2
(cd _r3ref && timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > ../gpurun_out/bs_r3b.log 2>&1) && tail -1 gpurun_out/bs_r3b.log | cut -c1-120
