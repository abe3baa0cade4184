#!/bin/bash
# safegcd inversion: full GPU suite, then same-box A/B against the previous library build
# (abtmp/libdrynx_native_old.so, DRYNX_NATIVE_LIB): headline x2 each, W=8 rank share each.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5it6}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-250; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step pytest 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread
OLD=abtmp/libdrynx_native_old.so
step b_new1 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/b_new1.json
DRYNX_NATIVE_LIB=$OLD step b_old1 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/b_old1.json
step b_new2 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/b_new2.json
DRYNX_NATIVE_LIB=$OLD step b_old2 300 python -u bench.py --steps 20 --warmup 5 --json-out $O/b_old2.json
step s_new 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json profiles/r5/it3/u0l0.json --ctrl-json profiles/r5/it3/ctrl_w8.json --json-out $O/share_new.json
DRYNX_NATIVE_LIB=$OLD step s_old 500 python -u tools/rank_share.py --world 8 --reps 3 --serial-json profiles/r5/it3/u0l0.json --ctrl-json profiles/r5/it3/ctrl_w8.json --json-out $O/share_old.json
