#!/bin/bash
# Closing evidence: the serialized per-span kernel table of the final tree and
# the client-priority A/B on the serial path.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
DRYNX_CLIENT_PRIORITY=0 DRYNX_CNP_PRIORITY=-1 step i_u0l0_cprio 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/i_u0l0_cprio.json
DRYNX_CLIENT_PRIORITY=0 DRYNX_CNP_PRIORITY=-1 step i_head_cprio 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/i_head_cprio.json
step i_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/i_u0l0.json
DRYNX_STREAM_PRIO=0 GPU_MAX_HW_QUEUES=1 AMD_SERIALIZE_KERNEL=3 DRYNX_ROCTX=1 timeout -k 10 400 rocprofv3 --runtime-trace --output-format csv -d gpurun_out/spans_final -o run -- python3 -u bench.py --steps 4 --warmup 2 > gpurun_out/spans_final_run.log 2>&1 || { tail -30 gpurun_out/spans_final_run.log; exit 1; }
python3 tools/span_kernels.py gpurun_out/spans_final --queries 3 --out gpurun_out/span_kernels_final.txt | head -12
