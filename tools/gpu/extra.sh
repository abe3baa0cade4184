#!/bin/bash
# torch-op attribution of the headline's GPU time, fault-injected headline,
# 6-CN signature set (GLS table budget), BASELINE config 4 (lr_dro) and the
# pure-execution line (no range proofs).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-600; if [ $rc -ne 0 ]; then tail -20 gpurun_out/$name.log; exit $rc; fi; }
DRYNX_TORCH_PROF=gpurun_out/torch_prof.txt step bench_torchprof 400 python -u bench.py --steps 2 --warmup 1
step bench_fault 400 python -u bench.py --steps 5 --warmup 1 --fault-dp 3
step bench_u0l0 400 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
step bench_lr_dro 400 python -u bench.py --query lr_dro --steps 5 --warmup 1
step bench_cns6 600 python -u bench.py --cns 6 --steps 3 --warmup 1
