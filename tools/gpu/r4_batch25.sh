#!/bin/bash
# Headline: CN-proof stream high priority (DRYNX_CNP_PRIORITY=-1) vs default,
# alternating, with the event-ordered CN-proof jobs.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step r_head_def1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r_head_def1.json
DRYNX_CNP_PRIORITY=-1 step r_head_cnp1 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r_head_cnp1.json
step r_head_def2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r_head_def2.json
DRYNX_CNP_PRIORITY=-1 step r_head_cnp2 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r_head_cnp2.json
step r_head_def3 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r_head_def3.json
DRYNX_CNP_PRIORITY=-1 step r_head_cnp3 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/r_head_cnp3.json
