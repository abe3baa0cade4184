#!/bin/bash
# One W=8 pool part (rank 6: a helper; rank 3: a VN rank) on one GPU under a
# HIP runtime trace with roctx spans: wall vs device-busy time of the part and
# the kernel time of each span (tools/span_kernels.py), plus the host trace.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
DRYNX_ROCTX=1 DRYNX_TRACE=gpurun_out/pp_trace.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=6,3 timeout -k 10 500 rocprofv3 --runtime-trace --output-format csv -d gpurun_out/pp -o run -- python3 -u tools/rank_share.py --world 8 --reps 1 > gpurun_out/pp_run.log 2>&1 || { tail -30 gpurun_out/pp_run.log; exit 1; }
python3 tools/span_kernels.py gpurun_out/pp --queries 1 --window "pool_part[6]" --out gpurun_out/pp_span_kernels_part6.txt | head -45
python3 tools/span_kernels.py gpurun_out/pp --queries 1 --window "pool_part[3]" --out gpurun_out/pp_span_kernels_part3.txt | head -8
python3 tools/host_trace.py gpurun_out/pp_trace.json 0.1 > gpurun_out/pp_host_trace.txt
