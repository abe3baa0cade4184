#!/bin/bash
# Tests of the touched paths, clean headline x2, the W=8 pool-part profile,
# the u0l0 host trace, then the ledger persistence run (three VN copies of
# every proof, 20 vs 100 steps: the blob generations prune at the disk reserve).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-220; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step b8_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_copy.py tests/test_rpmsm.py tests/test_sigma.py tests/test_ks_direct_gpu.py
step b8_clean 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/b8_clean.json
bash tools/gpu/r4_pool_prof.sh || exit 1
DRYNX_TRACE=gpurun_out/b8_u0l0_trace.json step b8_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/b8_u0l0.json
python3 tools/host_trace.py gpurun_out/b8_u0l0_trace.json 0.1 > gpurun_out/b8_host_trace_u0l0.txt
step b8_clean2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/b8_clean2.json
df -h /tmp | tee gpurun_out/ledger_df.txt
DRYNX_LEDGER_COPIES=3 step ledger20 300 python -u bench.py --steps 20 --warmup 2 --json-out gpurun_out/ledger20.json
DRYNX_LEDGER_COPIES=3 step ledger100 600 python -u bench.py --steps 100 --warmup 2 --json-out gpurun_out/ledger100.json
df -h /tmp | tee -a gpurun_out/ledger_df.txt
