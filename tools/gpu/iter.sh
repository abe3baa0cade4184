#!/bin/bash
# One build -> measure iteration on one GPU: GPU tests, headline bench,
# traced bench (host spans), optional 2/4-rank gloo rehearsal ($1 = "multi").
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-2000; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench.log; exit $rc; }
DRYNX_TRACE=gpurun_out/trace timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_trace.log 2>&1 \
 && python tools/host_trace.py gpurun_out/trace.r0.json 0.3 > gpurun_out/host_trace.txt && echo trace ok || exit 1
if [ "$1" = "multi" ]; then
  for N in 2 4; do
    DRYNX_DIST_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
      --master-addr 127.0.0.1 --master-port $((29533 + N)) bench.py --gpus $N --steps 2 --warmup 1 --features 20 \
      --device cuda:0 > gpurun_out/bench_${N}rank_gloo.log 2>&1
    rc=$?; tail -1 gpurun_out/bench_${N}rank_gloo.log | cut -c1-1500; [ $rc -eq 0 ] || { tail -30 gpurun_out/bench_${N}rank_gloo.log; exit $rc; }
  done
fi
