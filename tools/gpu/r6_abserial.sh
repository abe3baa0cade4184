#!/bin/bash
# Same-box A/B of the serial line (--u 0 --l 0, 20 steps): working tree vs the ab_base/ snapshot.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6abserial}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
R=$(pwd)
step() { local name=$1; shift; timeout -k 10 "$@" > $R/$O/$name.log 2>&1; local rc=$?; tail -1 $R/$O/$name.log | cut -c1-160; if [ $rc -ne 0 ]; then tail -40 $R/$O/$name.log; exit $rc; fi; }
true
for k in 1 2; do
  step new$k 300 python -u bench.py --u 0 --l 0 --steps 20 --warmup 5 --json-out $O/new$k.json
  (cd ab_base && step old$k 300 python -u bench.py --u 0 --l 0 --steps 20 --warmup 5 --json-out $R/$O/old$k.json) || exit 1
done
DRYNX_TRACE=$O/tr step trace 300 python -u bench.py --u 0 --l 0 --steps 5 --warmup 3
python3 tools/host_trace.py $O/tr.r0.json 0.1 > $O/host_trace_u0l0.txt && rm -f $O/tr.r0.json
