#!/bin/bash
# PMC counters over one headline query (counters only: no trace domains in the same run).
set -o pipefail
mkdir -p gpurun_out/pmc2
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/pmc2
timeout -s KILL 500 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc2 -o q -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pmc2_run.log 2>&1; rc=$?
echo "rc=$rc"; tail -2 gpurun_out/pmc2_run.log | cut -c1-200; f=$(find gpurun_out/pmc2 -name "*counter_collection*.csv" | head -1); echo "$f"
[ -n "$f" ] && python tools/pmc_summary.py "$f" > gpurun_out/pmc2_summary.txt && head -40 gpurun_out/pmc2_summary.txt
exit $rc
