#!/bin/bash
# Per-kernel cost of one W=8 pool part (rank 6 helper, rank 3 VN rank) on one GPU:
# kernel trace of the parts (concurrent) and again with every kernel serialized.
set -o pipefail
O=gpurun_out/r5pp; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
DRYNX_TRACE=$O/trace.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=6,3 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -u tools/rank_share.py --world 8 --reps 1 > $O/run.log 2>&1 || { tail -30 $O/run.log; exit 1; }
python3 tools/kernel_bursts.py $(find $O/kt -name "*kernel_trace.csv" -print -quit) --gap 500 --last 2 > $O/bursts.txt
python3 tools/host_trace.py $O/trace.json 0.1 > $O/host_trace.txt
AMD_SERIALIZE_KERNEL=3 GPU_MAX_HW_QUEUES=1 DRYNX_STREAM_PRIO=0 DRYNX_TRACE=$O/trace_ser.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=6,3 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kts -o run -- python3 -u tools/rank_share.py --world 8 --reps 1 > $O/run_ser.log 2>&1 || { tail -30 $O/run_ser.log; exit 1; }
python3 tools/kernel_bursts.py $(find $O/kts -name "*kernel_trace.csv" -print -quit) --gap 500 --last 2 > $O/bursts_ser.txt
rm -rf $O/kt $O/kts
head -40 $O/bursts_ser.txt
