#!/bin/bash
set -o pipefail
O=gpurun_out/${R5_OUT:-r5lp}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for i in 1 2 3 4; do
  timeout -k 10 200 python -u tools/ab_patch.py --no-ledger-prefetch -- --steps 20 --warmup 5 --u 0 --l 0 --json-out $O/u0_old$i.json > $O/u0_old$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --u 0 --l 0 --json-out $O/u0_new$i.json > $O/u0_new$i.log 2>&1 || exit 1
done
DRYNX_TRACE=$O/u0 timeout -k 10 200 python -u bench.py --steps 5 --warmup 2 --u 0 --l 0 --json-out $O/u0l0_traced.json > $O/u0t.log 2>&1 || exit 1
python3 tools/host_trace.py $O/u0.r0.json 0.1 > $O/host_trace_u0l0.txt
timeout -k 10 300 python -u tools/ab_patch.py --no-ledger-prefetch -- --steps 20 --warmup 5 --json-out $O/h_old.json > $O/h_old.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/h_new.json > $O/h_new.log 2>&1 || exit 1
python3 - <<'PY'
import json
import os; O="gpurun_out/"+os.environ.get("R5_OUT","r5lp")
for k in ("u0_old","u0_new"):
    print(k, [round(json.load(open(f"{O}/{k}{i}.json"))["ms_per_step"],2) for i in (1,2,3,4)])
for k in ("h_old","h_new"):
    print(k, round(json.load(open(f"{O}/{k}.json"))["ms_per_step"],2))
PY
