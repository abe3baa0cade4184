#!/bin/bash
# Checkpoint: the whole GPU suite + smoke, the driver-form headline, the W=8
# per-rank projection, fault-injected headline, configs 2-4 and the u0l0 line.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step c_pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
step c_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step c_bench 400 python -u bench.py --steps 20 --warmup 5 --json-out gpurun_out/c_bench.json
step c_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/c_u0l0.json
step c_share 600 python -u tools/rank_share.py --world 8 --reps 3 --serial-json gpurun_out/c_u0l0.json --json-out gpurun_out/c_rank_share_w8.json
step c_fault 300 python -u bench.py --steps 10 --warmup 2 --fault-dp 3 --json-out gpurun_out/c_fault.json
step c_mean 200 python -u bench.py --steps 5 --warmup 2 --query mean --json-out gpurun_out/c_mean.json
step c_variance 200 python -u bench.py --steps 5 --warmup 2 --query variance --json-out gpurun_out/c_variance.json
step c_linreg 200 python -u bench.py --steps 5 --warmup 2 --query lin_reg --json-out gpurun_out/c_linreg.json
step c_lrdro 300 python -u bench.py --steps 5 --warmup 2 --query lr_dro --json-out gpurun_out/c_lrdro.json
