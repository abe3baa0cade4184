#!/bin/bash
# One GPU session: tests, smoke, kernel microbench, small benches. Every GPU step
# has its own time limit and steps are chained so the first failure ends the run.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest gpu ok" \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo "smoke ok" \
 && timeout -k 10 300 python tools/microbench.py > gpurun_out/microbench.json 2> gpurun_out/microbench.err && cat gpurun_out/microbench.json \
 && timeout -k 10 600 python bench.py --features 8 --records 1000000 --steps 2 --warmup 1 > gpurun_out/bench_d8.log 2>&1 && tail -1 gpurun_out/bench_d8.log
