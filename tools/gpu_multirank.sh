#!/bin/bash
# Multi-rank rehearsal on ONE GPU: 2 ranks over gloo, both on cuda:0 (the RCCL
# data plane needs a GPU per rank; the driver's 8-GPU run covers that).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
DRYNX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --records 200000 --device cuda:0 > gpurun_out/bench_2rank_gloo.log 2>&1; rc=$?; tail -2 gpurun_out/bench_2rank_gloo.log; exit $rc
