#!/bin/bash
# Same-box A/B of the 1-GPU verifier windows: R MSM 13 (default) vs 14 / 15 bits,
# GT multi-exponentiation 16 (default) vs 14.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5ab18}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
B="--steps 20 --warmup 5"
for i in 1 2; do
  step def_$i 300 python -u bench.py $B --json-out $O/def_$i.json
  step r15_$i 300 python -u tools/ab_patch.py --r-window 15 -- $B --json-out $O/r15_$i.json
done
step r14_1 300 python -u tools/ab_patch.py --r-window 14 -- $B --json-out $O/r14_1.json
step me14_1 300 python -u tools/ab_patch.py --me-window 14 -- $B --json-out $O/me14_1.json
step def_3 300 python -u bench.py $B --json-out $O/def_3.json
for f in $O/*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['ms_per_step'], d['all_proofs_valid'], d['phase_s']['vn0_VerifyRange'])"; done
