#!/bin/bash
# Round-4 start on one GPU: GPU tests, smoke, headline (driver form), the
# no-range-proof line with host spans, a rocprofv3 kernel trace of the
# headline and a PMC pass (VALU busy, LDS, scratch) over one query.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-700; if [ $rc -ne 0 ]; then tail -25 gpurun_out/$name.log; exit $rc; fi; }
step pytest_gpu 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python -u bench.py --steps 20 --warmup 2
DRYNX_TRACE=gpurun_out/trace_u0l0 step bench_u0l0 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python tools/host_trace.py gpurun_out/trace_u0l0.r0.json 0.05 > gpurun_out/host_trace_u0l0.txt
step prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --steps 2 --warmup 1
step pmc 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc -o pmc -- python3 bench.py --steps 1 --warmup 1
ls -R gpurun_out/prof gpurun_out/pmc | head
