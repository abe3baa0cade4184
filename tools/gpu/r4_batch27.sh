#!/bin/bash
# R-MSM / D-check passes on their own stream beside the GT multi-exp
# (DRYNX_RUN_SPLIT=1): verifier GPU tests with it, W=8 rank shares and the
# headline, A/B against the default.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-160; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
DRYNX_RUN_SPLIT=1 step t_tests 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_rpmsm.py tests/test_range_hardening.py tests/test_range_proof.py tests/test_pool.py
DRYNX_RUN_SPLIT=1 step t_share_split 600 python -u tools/rank_share.py --world 8 --reps 3 --order 4,5,3,0,1,2,6,7 --json-out gpurun_out/t_share_split.json
step t_share_def 600 python -u tools/rank_share.py --world 8 --reps 3 --order 4,5,3,0,1,2,6,7 --json-out gpurun_out/t_share_def.json
DRYNX_RUN_SPLIT=1 step t_head_split1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/t_head_split1.json
step t_head_def1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/t_head_def1.json
DRYNX_RUN_SPLIT=1 step t_head_split2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/t_head_split2.json
step t_head_def2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/t_head_def2.json
