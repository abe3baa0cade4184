#!/bin/bash
set -o pipefail
O=gpurun_out/r5glv; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_glv_split.py tests/test_gpu.py -v --timeout 200 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -u tools/bench_g1mul.py > $O/micro.txt 2>&1 || { tail -20 $O/micro.txt; exit 1; }
cat $O/micro.txt
for i in 1 2; do
  timeout -k 10 200 python -u tools/ab_patch.py --no-glv --no-ledger-prefetch -- --steps 20 --warmup 5 --u 0 --l 0 --json-out $O/u0_old$i.json > $O/u0_old$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/ab_patch.py --no-ledger-prefetch -- --steps 20 --warmup 5 --u 0 --l 0 --json-out $O/u0_glv$i.json > $O/u0_glv$i.log 2>&1 || exit 1
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --u 0 --l 0 --json-out $O/u0_new$i.json > $O/u0_new$i.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/ab_patch.py --no-glv --no-ledger-prefetch -- --steps 20 --warmup 5 --json-out $O/h_old$i.json > $O/h_old$i.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/h_new$i.json > $O/h_new$i.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
O="gpurun_out/r5glv"
for k in ("u0_old","u0_glv","u0_new","h_old","h_new"):
    print(k, [round(json.load(open(f"{O}/{k}{i}.json"))["ms_per_step"],2) for i in (1,2)])
PY
