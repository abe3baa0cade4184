#!/bin/bash
# iter6 (tests, clean headline x2, serialized span table), the W=8 pool-part
# profile, then the ledger persistence run (100 steps with three VN copies of
# every proof against a 20-step run).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
bash tools/gpu/r4_iter6.sh && bash tools/gpu/r4_pool_prof.sh || exit 1
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-220; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
# ~0.55 GB of range payloads per query and copy: size the long run to half the free space
df -h /tmp | tee gpurun_out/ledger_df.txt
N=$(python3 -c "import shutil; f=shutil.disk_usage('/tmp').free; print(max(0, min(100, int(0.5 * f / (3 * 0.56e9)) - 4)))")
echo "ledger long run: $N steps" | tee -a gpurun_out/ledger_df.txt
[ "$N" -ge 30 ] || { echo "not enough disk for the ledger run"; exit 0; }
DRYNX_LEDGER_COPIES=3 step ledger20 300 python -u bench.py --steps 20 --warmup 2 --json-out gpurun_out/ledger20.json
DRYNX_LEDGER_COPIES=3 step ledgerN 500 python -u bench.py --steps $N --warmup 2 --json-out gpurun_out/ledgerN.json
