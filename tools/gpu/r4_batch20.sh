#!/bin/bash
# Same-box A/B of the headline: the tree at 10ed65d (ab_old/, a git worktree
# with the same native library) vs this tree, alternating.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$PWD
step() { local name=$1; shift; timeout -k 10 "$@" > $R/gpurun_out/$name.log 2>&1; local rc=$?; tail -1 $R/gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -30 $R/gpurun_out/$name.log; exit $rc; fi; }
step m_new1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/m_new1.json
(cd ab_old && step m_old1 300 python -u bench.py --steps 10 --warmup 2 --json-out $R/gpurun_out/m_old1.json) || exit 1
step m_new2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/m_new2.json
(cd ab_old && step m_old2 300 python -u bench.py --steps 10 --warmup 2 --json-out $R/gpurun_out/m_old2.json) || exit 1
step m_new3 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/m_new3.json
