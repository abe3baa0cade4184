#!/bin/bash
# Iteration: headline, 100-step durable-ledger run, serial line, control-round latency on the
# box's CPUs, setup share (1/8 table build + landing), W=8 rank share with the control term.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5it3}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step bench 400 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json
step bench100 600 python -u bench.py --steps 100 --warmup 5 --check-ledger --json-out $O/bench100.json
step u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out $O/u0l0.json
OMP_NUM_THREADS=1 step ctrl 300 python -u tools/ctrl_round.py --world 8 --rounds 300 --json-out $O/ctrl_w8.json
step setup 400 python -u tools/setup_share.py --world 8 --rank 0 --bench-json $O/bench.json --json-out $O/setup_share_w8.json
step share 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json $O/u0l0.json --ctrl-json $O/ctrl_w8.json --json-out $O/rank_share_w8.json
