#!/bin/bash
# N-rank rehearsal of the multi-GPU path on ONE GPU (gloo data plane, every
# rank on cuda:0), d = 20, with per-rank host spans.  $1 = N (2 or 4).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
N=${1:-2}
DRYNX_DIST_BACKEND=gloo DRYNX_TRACE=gpurun_out/trace_${N}rank timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29533 + N)) bench.py --gpus $N --steps 3 --warmup 1 \
  --features 20 --device cuda:0 > gpurun_out/rehearsal_${N}rank.log 2>&1; rc=$?
tail -1 gpurun_out/rehearsal_${N}rank.log | cut -c1-400; [ $rc -eq 0 ] || { tail -30 gpurun_out/rehearsal_${N}rank.log; exit $rc; }
for r in $(seq 0 $((N - 1))); do python tools/host_trace.py gpurun_out/trace_${N}rank.r$r.json 0.3 > gpurun_out/host_trace_${N}rank_r$r.txt; done; echo traces ok
