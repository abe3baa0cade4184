#!/bin/bash
# Multi-rank rehearsal on ONE GPU: 2 and 4 ranks over gloo, all on cuda:0 (the
# RCCL data plane needs a GPU per rank; the driver's 8-GPU run covers that).
# SPECTF-like LR with 20 features (462 outputs) keeps 4 ranks' prover tables
# (10 GB each) inside one GPU's HBM.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for N in 2 4; do
  DRYNX_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29533 + N)) bench.py --gpus $N --steps 2 --warmup 1 --features 20 \
    --device cuda:0 > gpurun_out/bench_${N}rank_gloo.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -30 gpurun_out/bench_${N}rank_gloo.log; exit $rc; fi
  tail -1 gpurun_out/bench_${N}rank_gloo.log | cut -c1-600
done
