#!/bin/bash
# Checkpoint of a tree: full GPU suite + smoke, headline (driver form), 100-step durable ledger,
# fault path, serial line, control rounds, W=8 rank share (pool and vn-local), setup share (span trace),
# pool-part traces.  FINAL_STEPS=quick: suite, headline, W=8 shares only.
set -o pipefail
O=gpurun_out/${FINAL_OUT:-final}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-300; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step pytest 900 python -u -m pytest ${FINAL_TESTS:-tests} -m gpu -v --timeout 400 --timeout-method thread
if [ "${FINAL_STEPS:-all}" = quick ]; then
  step bench 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json
  step share 500 python -u tools/rank_share.py --world 8 --reps 3 --ctrl-json profiles/r5/final/ctrl_w8.json --json-out $O/rank_share_w8.json
  step sharel 500 python -u tools/rank_share.py --world 8 --reps 3 --vn-mode local --ctrl-json profiles/r5/final/ctrl_w8.json --json-out $O/rank_share_w8_local.json
  exit 0
fi
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json
step bench100 600 python -u bench.py --steps 100 --warmup 5 --check-ledger --json-out $O/bench100.json
step fault 300 python -u bench.py --steps 10 --warmup 3 --fault-dp 3 --json-out $O/fault.json
step u0l0 300 python -u bench.py --steps 20 --warmup 5 --u 0 --l 0 --json-out $O/u0l0.json
OMP_NUM_THREADS=1 step ctrl 300 python -u tools/ctrl_round.py --world 8 --rounds 300 --json-out $O/ctrl_w8.json
step share 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json $O/u0l0.json --ctrl-json $O/ctrl_w8.json --json-out $O/rank_share_w8.json
step sharel 500 python -u tools/rank_share.py --world 8 --reps 3 --vn-mode local --serial-json $O/u0l0.json --ctrl-json $O/ctrl_w8.json --json-out $O/rank_share_w8_local.json
step setupf 400 python -u tools/setup_share.py --mode full --json-out $O/setup_full.json
DRYNX_TRACE=$O/setup_trace.json step setup 400 python -u tools/setup_share.py --world 8 --rank 0 --full-json $O/setup_full.json --bench-json $O/bench.json --json-out $O/setup_share_w8.json
python3 tools/host_trace.py $O/setup_trace.json 1 > $O/setup_host_trace.txt || true
DRYNX_TRACE=$O/trace.json RANK_SHARE_TRACE_ONLY=1 RANK_SHARE_PARTS=6,3 RANK_SHARE_TRACE_REPS=2 step tl 400 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 -u tools/rank_share.py --world 8 --reps 1
T=$(find $O/kt -name "*kernel_trace.csv" -print -quit)
python3 tools/kernel_timeline.py $T --gap 500 --burst -3 > $O/timeline_part6.txt
python3 tools/kernel_timeline.py $T --gap 500 --burst -1 > $O/timeline_part3.txt
python3 tools/host_trace.py $O/trace.json 0.1 > $O/host_trace.txt
rm -rf $O/kt
head -1 $O/timeline_part6.txt; head -1 $O/timeline_part3.txt
