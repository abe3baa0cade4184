#!/bin/bash
# Same-box comparison with the round-3 tree (copied under _r3ref/ for this
# call only): r3, r4, r3, r4 headline runs of 10 timed queries.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-150; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
(cd _r3ref && timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > ../gpurun_out/vs_r3_a.log 2>&1) && tail -1 gpurun_out/vs_r3_a.log | cut -c1-150
step vs_r4_a 300 python -u bench.py --steps 10 --warmup 2
(cd _r3ref && timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > ../gpurun_out/vs_r3_b.log 2>&1) && tail -1 gpurun_out/vs_r3_b.log | cut -c1-150
step vs_r4_b 300 python -u bench.py --steps 10 --warmup 2
DRYNX_PLAN_SORT=rocprim step vs_r4_rocprim 300 python -u bench.py --steps 10 --warmup 2
step vs_r4_fault 300 python -u bench.py --steps 5 --warmup 1 --fault-dp 3
DRYNX_SEG_KEEP=1 step vs_r4_fault_keep 300 python -u bench.py --steps 5 --warmup 1 --fault-dp 3
