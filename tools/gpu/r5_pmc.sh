#!/bin/bash
# One PMC pass over a short headline run (5 SQ counters, nothing else collected).
set -o pipefail
O=gpurun_out/${R5_OUT:-r5pmc}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS --output-format csv -d $O/pmc -o run -- python3 -u bench.py --steps 2 --warmup 1 > $O/pmc_run.log 2>&1 || { tail -30 $O/pmc_run.log; exit 1; }
C=$(find $O/pmc -name "*counter_collection.csv" -print -quit)
python3 tools/pmc_summary.py $C > $O/pmc_summary.txt
rm -rf $O/pmc
head -40 $O/pmc_summary.txt
