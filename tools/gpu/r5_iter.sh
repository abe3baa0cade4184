#!/bin/bash
# Iteration: GPU suite, driver-form headline, W=8 rank share, pool-part kernel bursts (serialized).
set -o pipefail
O=gpurun_out/${R5_OUT:-r5it}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step pytest 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
step bench 400 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json
step u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out $O/u0l0.json
step share 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json $O/u0l0.json --json-out $O/rank_share_w8.json
AMD_SERIALIZE_KERNEL=3 GPU_MAX_HW_QUEUES=1 DRYNX_STREAM_PRIO=0 DRYNX_TRACE=$O/trace_ser.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=6,3 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/kts -o run -- python3 -u tools/rank_share.py --world 8 --reps 1 > $O/run_ser.log 2>&1 || { tail -30 $O/run_ser.log; exit 1; }
python3 tools/kernel_bursts.py $(find $O/kts -name "*kernel_trace.csv" -print -quit) --gap 500 --last 2 > $O/bursts_ser.txt
rm -rf $O/kts
head -30 $O/bursts_ser.txt
