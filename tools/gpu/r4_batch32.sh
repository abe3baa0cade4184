#!/bin/bash
# Hardware queues per process: GPU_MAX_HW_QUEUES=8 vs the default 4 (the
# node uses ~8 streams: survey, plans, pool, prover, CN proofs, querier,
# digests, ledger), headline and u0l0, alternating.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step x_head_q4a 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/x_head_q4a.json
GPU_MAX_HW_QUEUES=8 step x_head_q8a 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/x_head_q8a.json
step x_head_q4b 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/x_head_q4b.json
GPU_MAX_HW_QUEUES=8 step x_head_q8b 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/x_head_q8b.json
step x_u0l0_q4 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/x_u0l0_q4.json
GPU_MAX_HW_QUEUES=8 step x_u0l0_q8 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/x_u0l0_q8.json
