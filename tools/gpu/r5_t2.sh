#!/bin/bash
set -o pipefail
O=gpurun_out/r5t2; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ledger_codec.py tests/test_ledger_retention.py tests/test_multirank_gpu.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u tools/ab_patch.py --raw-ledger -- --steps 20 --warmup 5 --check-ledger --json-out $O/h_old$i.json > $O/h_old$i.log 2>&1 || { tail -20 $O/h_old$i.log; exit 1; }
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --check-ledger --json-out $O/h_new$i.json > $O/h_new$i.log 2>&1 || { tail -20 $O/h_new$i.log; exit 1; }
done
python3 - <<'PY'
import json
O="gpurun_out/r5t2"
for k in ("h_old","h_new"):
    for i in (1,2):
        d=json.load(open(f"{O}/{k}{i}.json"))
        r=d.get("ranks",[{}])
        r0=r[0] if isinstance(r,list) and r else {}
        print(k, i, d["ms_per_step"], "ledger_blob_bytes/step", r0.get("ledger_blob_bytes",0)/d["steps"]/1e6, "MB", "readback", r0.get("ledger_readback"), "ok", d.get("result_ok"), d.get("proofs_ok"))
PY
