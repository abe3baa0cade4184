#!/bin/bash
# Iteration loop on one GPU: correctness, kernel microbench, full bench, kernel profile.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log \
 && timeout -k 10 300 python tools/microbench.py > gpurun_out/microbench.json 2> gpurun_out/microbench.err && cat gpurun_out/microbench.json \
 && timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_full.log 2>&1 && tail -1 gpurun_out/bench_full.log \
 && timeout -k 10 600 python -m cProfile -o gpurun_out/bench.prof bench.py --steps 2 --warmup 1 > gpurun_out/bench_cprof.log 2>&1 \
 && python -c "import pstats; s=pstats.Stats('gpurun_out/bench.prof'); s.sort_stats('tottime').print_stats(45); s.sort_stats('cumtime').print_stats(60)" > gpurun_out/cprof.txt \
 && export TMPDIR=/tmp \
 && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_run.log 2>&1 \
 && echo prof ok
