#!/bin/bash
# A/B of the two-phase fold variants (tools/fold_bench.py) on one GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/fold_bench.py > gpurun_out/fold_ab.log 2>&1
rc=$?; cat gpurun_out/fold_ab.log | grep -v amdgpu.ids; exit $rc
