#!/bin/bash
# BASELINE configs 2-4 and the 6-CN headline on a tree.
set -o pipefail
O=gpurun_out/${CFG_OUT:-configs}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-200; if [ $rc -ne 0 ]; then tail -30 $O/$name.log; exit $rc; fi; }
step mean 300 python -u bench.py --query mean --steps 5 --warmup 2 --json-out $O/mean.json
step variance 300 python -u bench.py --query variance --steps 5 --warmup 2 --json-out $O/variance.json
step linreg 300 python -u bench.py --query lin_reg --steps 5 --warmup 2 --json-out $O/linreg.json
step lrdro 400 python -u bench.py --query lr_dro --steps 5 --warmup 2 --json-out $O/lrdro.json
step cn6 600 python -u bench.py --cns 6 --steps 5 --warmup 2 --json-out $O/bench_6cn.json
