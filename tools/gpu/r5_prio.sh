#!/bin/bash
set -o pipefail
O=gpurun_out/r5prio; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
RS="import sys, runpy; from drynx_amd.proofs import range_proof as rp; rp.AUX_PRIORITY = 0; sys.argv = ['tools/rank_share.py'] + sys.argv[1:]; runpy.run_path('tools/rank_share.py', run_name='__main__')"
timeout -k 10 400 python -u -c "$RS" --world 8 --reps 3 --json-out $O/share_new.json > $O/share_new.log 2>&1 || { tail -20 $O/share_new.log; exit 1; }
tail -1 $O/share_new.log | cut -c1-400
timeout -k 10 400 python -u tools/rank_share.py --world 8 --reps 3 --json-out $O/share_old.json > $O/share_old.log 2>&1 || { tail -20 $O/share_old.log; exit 1; }
tail -1 $O/share_old.log | cut -c1-400
for i in 1 2 3; do
  timeout -k 10 300 python -u tools/ab_patch.py --aux-priority 0 -- --steps 20 --warmup 5 --json-out $O/h_new$i.json > $O/h_new$i.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/h_old$i.json > $O/h_old$i.log 2>&1 || exit 1
done
python3 - <<'PY'
import json
O="gpurun_out/r5prio"
for k in ("h_old","h_new"):
    print(k, [round(json.load(open(f"{O}/{k}{i}.json"))["ms_per_step"],2) for i in (1,2,3)])
PY
