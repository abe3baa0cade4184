#!/bin/bash
set -o pipefail
O=gpurun_out/r5prio2; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
run() {  # name aux val pool
  local RS="import sys, runpy; from drynx_amd.proofs import range_proof as rp; from drynx_amd.protocols import proof_collection as pc; rp.AUX_PRIORITY = $2; rp.VAL_PRIORITY = $3; pc.POOL_PRIORITY = $4; sys.argv = ['tools/rank_share.py'] + sys.argv[1:]; runpy.run_path('tools/rank_share.py', run_name='__main__')"
  timeout -k 10 400 python -u -c "$RS" --world 8 --reps 3 --json-out $O/share_$1.json > $O/share_$1.log 2>&1 || { tail -20 $O/share_$1.log; exit 1; }
  echo "$1 aux=$2 val=$3 pool=$4 $(tail -1 $O/share_$1.log | cut -c1-400)"
}
run A -1 0 0
run B -1 0 -1
run C -1 -1 -1
run D -1 -1 0
