#!/bin/bash
# Pool-part times by measurement order (is a rank's part slow, or the slot it is measured in?)
set -o pipefail
O=gpurun_out/r5order; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 500 python -u tools/rank_share.py --world 8 --reps 3 --order 5,3,4,0,1,2,6,7 --json-out $O/share_o1.json > $O/o1.log 2>&1 || { tail -20 $O/o1.log; exit 1; }
timeout -k 10 500 python -u tools/rank_share.py --world 8 --reps 3 --order 7,6,2,1,0,4,3,5 --json-out $O/share_o2.json > $O/o2.log 2>&1 || { tail -20 $O/o2.log; exit 1; }
python3 - <<'PY'
import json
for f in ("o1", "o2"):
    d = json.load(open(f"gpurun_out/r5order/share_{f}.json"))
    print(f, [(k, v["pool_ms"]) for k, v in d["ranks"].items()], d["projection_terms_ms"])
PY
