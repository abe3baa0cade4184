#!/bin/bash
# End-of-session checkpoint: GPU tests, smoke, headline, BASELINE configs
# 2/3/4, a 6-CN SPECTF query, the fault-injected headline and a 2-rank
# rehearsal -- each step under its own time limit, stopping at the first
# failure.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then tail -25 gpurun_out/$name.log; exit $rc; fi; }
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python -u bench.py --steps 10 --warmup 3
step bench_mean 300 python -u bench.py --query mean --steps 5 --warmup 1
step bench_variance 300 python -u bench.py --query variance --steps 5 --warmup 1
step bench_lin_reg 300 python -u bench.py --query lin_reg --steps 5 --warmup 1
step bench_lr_dro 400 python -u bench.py --query lr_dro --steps 3 --warmup 1
step bench_fault 400 python -u bench.py --steps 4 --warmup 1 --fault-dp 3
step bench_6cn 600 python -u bench.py --cns 6 --steps 2 --warmup 1
bash tools/gpu/rehearse.sh 2
