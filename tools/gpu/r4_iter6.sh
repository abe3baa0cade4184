#!/bin/bash
# GPU tests of the touched paths, the clean headline twice, then the
# serialized per-span kernel table (one hardware queue, every stream at normal
# priority, AMD_SERIALIZE_KERNEL=3).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-220; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step i6_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_copy.py tests/test_ks_direct_gpu.py tests/test_sigma.py tests/test_rpmsm.py
step i6_clean 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/i6_clean.json
step i6_clean2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/i6_clean2.json
DRYNX_STREAM_PRIO=0 GPU_MAX_HW_QUEUES=1 AMD_SERIALIZE_KERNEL=3 DRYNX_ROCTX=1 timeout -k 10 400 rocprofv3 --runtime-trace --output-format csv -d gpurun_out/spans6 -o run -- python3 -u bench.py --steps 4 --warmup 2 > gpurun_out/spans6_run.log 2>&1 || { tail -30 gpurun_out/spans6_run.log; exit 1; }
tail -1 gpurun_out/spans6_run.log | cut -c1-200
python3 tools/span_kernels.py gpurun_out/spans6 --queries 3 --out gpurun_out/span_kernels6.txt | head -50
