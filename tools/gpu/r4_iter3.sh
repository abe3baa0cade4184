#!/bin/bash
# Round-4 iteration 3: GLV key-switch batch check, A/B of the kept
# per-segment buckets, span-synchronised cost breakdowns of the headline and
# of one rank's share of the 8-rank pool.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then tail -25 gpurun_out/$name.log; exit $rc; fi; }
step pytest_it 300 python -u -m pytest tests/test_ks_direct_gpu.py tests/test_gpu.py tests/test_rpmsm.py -m gpu -x -q --timeout 200 --timeout-method thread
step bench_it 300 python -u bench.py --steps 10 --warmup 2
DRYNX_SEG_KEEP=0 step bench_nokeep 300 python -u bench.py --steps 10 --warmup 2
DRYNX_TRACE=gpurun_out/trace_sync DRYNX_SPAN_SYNC=1 step bench_sync 300 python -u bench.py --steps 2 --warmup 1
python tools/host_trace.py gpurun_out/trace_sync.r0.json 0.2 > gpurun_out/host_trace_sync.txt
DRYNX_TRACE=gpurun_out/trace_pool.json DRYNX_SPAN_SYNC=1 step rank_share 500 python -u tools/rank_share.py --world 8 --reps 1
python tools/host_trace.py gpurun_out/trace_pool.json 0.1 > gpurun_out/host_trace_pool.txt
