#!/bin/bash
# 8-rank rehearsal on ONE GPU (gloo data plane, every rank on cuda:0): the
# multi-rank device paths end to end -- placement, pooled VN checks, fan-out,
# node-shared compact ledger payloads (read back), fault blame.
set -o pipefail
O=gpurun_out/${REH_OUT:-reh8}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp DRYNX_DIST_BACKEND=gloo DRYNX_PROVER_TABLE_BITS=7
SMALL="--steps 2 --warmup 1 --records 20000 --features 6 --max-iter 20"
timeout -k 10 500 python -u bench.py --gpus 8 $SMALL --check-ledger --json-out $O/reh8.json > $O/reh8.log 2>&1 || { tail -40 $O/reh8.log; exit 1; }
tail -1 $O/reh8.log | cut -c1-400
timeout -k 10 500 python -u bench.py --gpus 8 $SMALL --fault-dp 3 --json-out $O/reh8_fault.json > $O/reh8_fault.log 2>&1 || { tail -40 $O/reh8_fault.log; exit 1; }
timeout -k 10 500 python -u bench.py --gpus 8 $SMALL --vn-mode local --fault-dp 3 --json-out $O/reh8_local_fault.json > $O/reh8_local_fault.log 2>&1 || { tail -40 $O/reh8_local_fault.log; exit 1; }
O=$O python3 - <<'PY'
import json, os
for f in ("reh8", "reh8_fault", "reh8_local_fault"):
    d=json.load(open(f"{os.environ['O']}/{f}.json"))
    print(f, d["n_gpus"], d["ms_per_step"], d["config"].get("trust_model"), "valid", d.get("all_proofs_valid"),
          "blame", d.get("blame_ok"), "result", d.get("result_ok"),
          "readback", [r.get("ledger_readback") for r in d.get("ranks", []) if r.get("ledger_readback")],
          "blob MB/step", sum(r.get("ledger_blob_bytes",0) for r in d.get("ranks",[]))/d["steps"]/1e6)
PY
