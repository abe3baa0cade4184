#!/bin/bash
# PMC counters for the kernel microbenchmarks (counters only: no trace domains in the same run).
set -o pipefail
mkdir -p gpurun_out/pmc
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc -o mb -- python3 tools/microbench.py > gpurun_out/pmc_run.log 2>&1; rc=$?
tail -3 gpurun_out/pmc_run.log; find gpurun_out/pmc -name "*.csv" | head; exit $rc
