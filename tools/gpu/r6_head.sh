#!/bin/bash
# Headline: GPU checks of the touched kernels, 10-step bench, and a host span trace of the query.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6head}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu ${R6_TESTS:-tests/test_gpu.py tests/test_ledger_codec.py tests/test_rpmsm.py}
step bench 300 python -u bench.py --steps 10 --warmup 2 --json-out $O/bench.json
DRYNX_TRACE=$O/tr step trace 300 python -u bench.py --steps 3 --warmup 2
python3 tools/host_trace.py $O/tr.r0.json 0.3 > $O/host_trace.txt && rm -f $O/tr.r0.json
