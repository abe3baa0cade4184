#!/bin/bash
# Same-box A/B of the plan sort (counting / torch onesweep / rocPRIM pairs)
# and of the kept per-segment buckets; serialized torch-op attribution.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-150; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step ab_count 300 python -u bench.py --steps 10 --warmup 2
DRYNX_PLAN_SORT=torch step ab_torch 300 python -u bench.py --steps 10 --warmup 2
DRYNX_PLAN_SORT=rocprim step ab_rocprim 300 python -u bench.py --steps 10 --warmup 2
DRYNX_SEG_KEEP=0 step ab_count_nokeep 300 python -u bench.py --steps 10 --warmup 2
DRYNX_SEG_KEEP=0 DRYNX_PLAN_SORT=torch step ab_torch_nokeep 300 python -u bench.py --steps 10 --warmup 2
AMD_SERIALIZE_KERNEL=3 RANK_SHARE_TRACE_ONLY=1 DRYNX_TRACE=gpurun_out/trace_dummy.json RANK_SHARE_PARTS=0 step glue 500 python -u tools/rank_share.py --world 1 --reps 1 --torch-prof gpurun_out/torch_glue_ser.txt
