#!/bin/bash
# Where one rank's 1/8 share of the pooled range check spends its time: a
# span-synchronised trace and a serialized kernel trace of rank 3's and rank
# 6's share, each run alone after an idle gap.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then tail -25 gpurun_out/$name.log; exit $rc; fi; }
DRYNX_TRACE=gpurun_out/trace_pool.json DRYNX_SPAN_SYNC=1 RANK_SHARE_TRACE_ONLY=1 step share_trace 400 python -u tools/rank_share.py --world 8 --reps 1
python tools/host_trace.py gpurun_out/trace_pool.json 0.1 > gpurun_out/host_trace_pool.txt
DRYNX_TRACE=gpurun_out/trace_pool2.json RANK_SHARE_TRACE_ONLY=1 AMD_SERIALIZE_KERNEL=3 step share_prof 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_share -o share -- python3 tools/rank_share.py --world 8 --reps 1
python tools/kernel_bursts.py gpurun_out/prof_share/share_kernel_trace.csv --gap 500 --last 2 > gpurun_out/kernel_bursts_share.txt
