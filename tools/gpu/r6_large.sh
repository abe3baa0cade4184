#!/bin/bash
# Round-6: the reference's large-output (MaxOptimized) and large-noise (DiffPri) rows end to end.
# R6_LARGE=small: 1k / 10k / 100k max ranges + 100k noise list; R6_LARGE=big: the 1M rows.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6large}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
# heartbeat: the long single-query steps print only at their end
( while true; do date +%s > $O/heartbeat; sleep 45; done ) &
HB=$!
trap "kill $HB" EXIT
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
if [ "${R6_LARGE:-small}" = small ]; then
  step max1k 300 python -u bench.py --query max --range 1000 --steps 3 --warmup 1 --json-out $O/max_1k.json
  step max10k 300 python -u bench.py --query max --range 10000 --steps 2 --warmup 1 --json-out $O/max_10k.json
  step max100k 500 python -u bench.py --query max --range 100000 --steps 1 --warmup 1 --json-out $O/max_100k.json
  step dro100k 300 python -u bench.py --query lr_dro --dro 100000 --steps 2 --warmup 1 --json-out $O/lrdro_100k.json
  step sweeps 500 python -u tools/bench_scaling.py 3 servers,vns,threshold
else
  step max1m 900 python -u bench.py --query max --range 1000000 --steps 1 --warmup 1 --json-out $O/max_1m.json
  step dro1m 600 python -u bench.py --query lr_dro --dro 1000000 --steps 1 --warmup 1 --json-out $O/lrdro_1m.json
fi
