#!/bin/bash
# Bench + host-side cProfile (where the Python/host time between kernels goes).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_full.log 2>&1 && tail -1 gpurun_out/bench_full.log \
 && timeout -k 10 600 python -m cProfile -o gpurun_out/bench.prof bench.py --steps 3 --warmup 1 > gpurun_out/bench_cprof.log 2>&1 \
 && python -c "import pstats; s=pstats.Stats('gpurun_out/bench.prof'); s.sort_stats('tottime').print_stats(50); s.sort_stats('cumtime').print_stats(90)" > gpurun_out/cprof.txt \
 && echo cprof ok
