#!/bin/bash
# Kernel time per framework span (roctx ranges + HIP runtime trace), one
# timed bench run: tools/span_kernels.py joins kernels -> launches -> spans.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
# one hardware queue + serialized kernels: every kernel alone on the chip, so its
# duration is its own cost (AMD_SERIALIZE_KERNEL=3 alone still overlaps streams)
GPU_MAX_HW_QUEUES=1 AMD_SERIALIZE_KERNEL=3 DRYNX_ROCTX=1 timeout -k 10 400 rocprofv3 --runtime-trace --output-format csv -d gpurun_out/spans -o run -- python3 -u bench.py --steps 4 --warmup 2 > gpurun_out/spans_run.log 2>&1 || { tail -30 gpurun_out/spans_run.log; exit 1; }
tail -1 gpurun_out/spans_run.log | cut -c1-200
python3 tools/span_kernels.py gpurun_out/spans --queries 3 --out gpurun_out/span_kernels.txt | head -60
