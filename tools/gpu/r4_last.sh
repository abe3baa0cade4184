#!/bin/bash
# Last check of the final tree: the whole GPU suite, smoke, the driver-form headline.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step z_pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
step z_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step z_bench 400 python -u bench.py --steps 20 --warmup 5 --json-out gpurun_out/z_bench.json
step z_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/z_u0l0.json
