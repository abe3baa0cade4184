#!/bin/bash
# Serialized per-kernel cost of the last headline query (AMD_SERIALIZE_KERNEL=3: each kernel alone on the chip)
# + the GPU checks of the kernels touched, + a 10-step headline.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6cost}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${R6_TESTS:-tests/test_gpu.py tests/test_ledger_codec.py tests/test_rpmsm.py}
step bench 300 python -u bench.py --steps 10 --warmup 2 --json-out $O/bench.json
AMD_SERIALIZE_KERNEL=3 step kt 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -u bench.py --steps 2 --warmup 1
T=$(find $O/kt -name "*kernel_trace.csv" -print -quit)
python3 tools/kernel_cost.py $T --inner > $O/kernel_cost.txt && rm -rf $O/kt && head -30 $O/kernel_cost.txt
