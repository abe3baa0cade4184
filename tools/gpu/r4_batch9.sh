#!/bin/bash
# Round-4 closing measurements: the W=8 per-rank projection (rank_share, with
# the u0l0 serial JSON), the D2H engine probe, a PMC pass over one query
# (VALU busy, LDS, scratch per kernel), and the driver-form headline.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -25 gpurun_out/$name.log; exit $rc; fi; }
step b9_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/b9_u0l0.json
# A/B of the CN-proof signing placement on both lines (u0l0: the signatures
# sit on the critical path; headline: host signing competes with the query)
DRYNX_CNP_PRIORITY=-1 step b9_u0l0_cnp 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/b9_u0l0_cnp.json
DRYNX_SIGN_DEVICE_MIN=256 step b9_u0l0_hostsign 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/b9_u0l0_hostsign.json
step b9_head 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/b9_head.json
DRYNX_CNP_PRIORITY=-1 step b9_head_cnp 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/b9_head_cnp.json
DRYNX_SIGN_DEVICE_MIN=256 step b9_head_hostsign 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/b9_head_hostsign.json
step b9_share 600 python -u tools/rank_share.py --world 8 --reps 3 --serial-json gpurun_out/b9_u0l0.json --json-out gpurun_out/b9_rank_share_w8.json
bash tools/gpu/r4_d2h.sh || exit 1
step b9_pmc 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS --output-format csv -d gpurun_out/b9_pmc -o pmc -- python3 bench.py --steps 1 --warmup 1
step b9_kt 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/b9_kt -o kt -- python3 bench.py --steps 2 --warmup 1
step b9_bench 400 python -u bench.py --steps 20 --warmup 2 --json-out gpurun_out/b9_bench.json
