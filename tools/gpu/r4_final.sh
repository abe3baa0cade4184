#!/bin/bash
# Final checkpoint: the whole GPU suite + smoke, the driver-form headline, the W=8
# per-rank projection (VN rank 3 measured after 4 and 5), fault-injected headline, configs 2-4, u0l0.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step f_pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
step f_smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step f_bench 400 python -u bench.py --steps 20 --warmup 5 --json-out gpurun_out/f_bench.json
step f_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/f_u0l0.json
step f_share 600 python -u tools/rank_share.py --world 8 --reps 3 --serial-json gpurun_out/f_u0l0.json --order 4,5,3,0,1,2,6,7 --json-out gpurun_out/f_rank_share_w8.json
step f_fault 300 python -u bench.py --steps 10 --warmup 2 --fault-dp 3 --json-out gpurun_out/f_fault.json
step f_mean 200 python -u bench.py --steps 5 --warmup 2 --query mean --json-out gpurun_out/f_mean.json
step f_variance 200 python -u bench.py --steps 5 --warmup 2 --query variance --json-out gpurun_out/f_variance.json
step f_linreg 200 python -u bench.py --steps 5 --warmup 2 --query lin_reg --json-out gpurun_out/f_linreg.json
step f_lrdro 300 python -u bench.py --steps 5 --warmup 2 --query lr_dro --json-out gpurun_out/f_lrdro.json
