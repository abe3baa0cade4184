#!/bin/bash
# msm-verifier trims (no Zphi B, one uv(-Y) for all VNs): GPU tests of the
# verifier, the headline twice and the W=8 rank shares.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step g_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_rpmsm.py tests/test_range_hardening.py tests/test_range_proof.py tests/test_pool.py
step g_bench 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/g_bench.json
step g_fault 300 python -u bench.py --steps 5 --warmup 2 --fault-dp 3 --json-out gpurun_out/g_fault.json
step g_share 600 python -u tools/rank_share.py --world 8 --reps 3 --serial-json profiles/r4/checkpoint_u0l0.json --json-out gpurun_out/g_rank_share_w8.json
step g_bench2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/g_bench2.json
