#!/bin/bash
# iter6 (tests, clean headline x2, serialized span table), the W=8 pool-part
# profile, then the ledger persistence run (100 steps with three VN copies of
# every proof against a 20-step run).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
bash tools/gpu/r4_iter6.sh && bash tools/gpu/r4_pool_prof.sh || exit 1
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-220; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
DRYNX_LEDGER_COPIES=3 step ledger20 300 python -u bench.py --steps 20 --warmup 2 --json-out gpurun_out/ledger20.json
DRYNX_LEDGER_COPIES=3 step ledger100 400 python -u bench.py --steps 100 --warmup 2 --json-out gpurun_out/ledger100.json
