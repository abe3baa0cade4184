#!/bin/bash
# Iteration loop on one GPU: correctness, smoke, kernel microbench, full bench, kernel profile.
# Every GPU step has its own time limit; steps are chained so the first failure ends the run.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log \
 && timeout -k 10 300 python tools/microbench.py > gpurun_out/microbench.json 2> gpurun_out/microbench.err && cat gpurun_out/microbench.json \
 && timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_full.log 2>&1 && tail -1 gpurun_out/bench_full.log \
 && export TMPDIR=/tmp \
 && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_run.log 2>&1 \
 && echo prof ok
