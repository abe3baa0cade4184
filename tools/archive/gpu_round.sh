#!/bin/bash
# Round-end evidence on one GPU: GPU tests, smoke, kernel microbench, traced
# bench (host spans), rocprofv3 kernel stats + per-step kernel timeline.
# Every GPU step has its own limit; steps are chained so the first failure ends the run.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log \
 && timeout -k 10 300 python tools/microbench.py > gpurun_out/microbench.json 2> gpurun_out/microbench.err && cat gpurun_out/microbench.json \
 && timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log \
 && DRYNX_TRACE=gpurun_out/trace timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_trace.log 2>&1 \
 && python tools/host_trace.py gpurun_out/trace.r0.json 0.3 > gpurun_out/host_trace.txt \
 && export TMPDIR=/tmp \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_run.log 2>&1 \
 && python tools/trace_step.py gpurun_out/prof/bench_kernel_trace.csv 0.25 > gpurun_out/kernel_step.txt && echo prof ok
