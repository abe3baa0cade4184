#!/bin/bash
# Masked first pass + hinted attribution: GPU numerics of the attribution
# tests, then the clean headline and the fault-injected run on the same box,
# with and without the masked weights.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-220; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step mk_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_copy.py tests/test_rpmsm.py tests/test_sigma.py
step mk_clean 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/mk_clean.json
step mk_fault 300 python -u bench.py --steps 10 --warmup 2 --fault-dp 3 --json-out gpurun_out/mk_fault.json
DRYNX_RP_MASK=0 step mk_fault_nomask 300 python -u bench.py --steps 10 --warmup 2 --fault-dp 3 --json-out gpurun_out/mk_fault_nomask.json
step mk_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/mk_u0l0.json
step mk_clean2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/mk_clean2.json
