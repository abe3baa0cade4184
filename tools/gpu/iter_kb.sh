#!/bin/bash
# iteration + GT-chain microbenchmark + multi-rank rehearsal
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u tools/kbench_gt.py > gpurun_out/kbench_gt.json 2> gpurun_out/kbench_gt.err; rc=$?; cat gpurun_out/kbench_gt.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/kbench_gt.err; exit $rc; }
bash tools/gpu/iter.sh "$@"
