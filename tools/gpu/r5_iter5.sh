#!/bin/bash
# Lane-major coop fold output: fold tests, headline, per-kernel cost (names fixed) with the
# last query's trace kept, a torch-profiler glue table of one whole query, the W=8 rank share,
# and a kernel trace of the setup-share emulation.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5it5}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1; local rc=$?; tail -1 $O/$name.log | cut -c1-400; if [ $rc -ne 0 ]; then tail -40 $O/$name.log; exit $rc; fi; }
step pyt 600 python -u -m pytest tests/test_gpu.py tests/test_rpmsm.py -m gpu -x -v --timeout 300 --timeout-method thread
step bench 400 python -u bench.py --steps 20 --warmup 5 --json-out $O/bench.json
AMD_SERIALIZE_KERNEL=3 step kts 500 rocprofv3 --kernel-trace --output-format csv -d $O/kts -o run -- python3 -u bench.py --steps 3 --warmup 2
T=$(find $O/kts -name "*kernel_trace.csv" -print -quit)
python3 tools/kernel_cost.py $T > $O/kcost_headline_ser.txt
python3 tools/trace_step.py $T 0.2 > $O/step_kernels_ser.txt
rm -rf $O/kts
step glue 500 python -u tools/rank_share.py --world 8 --reps 3 --torch-prof-query $O/glue_query.txt --serial-json profiles/r5/it3/u0l0.json --ctrl-json profiles/r5/it3/ctrl_w8.json --json-out $O/rank_share_w8.json
step sst 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ss -o run -- python3 -u tools/setup_share.py --world 8 --rank 0 --json-out $O/setup_share_w8.json
find $O/ss -name "*kernel_stats.csv" -exec cp {} $O/setup_kernel_stats.csv \;
python3 tools/kernel_timeline.py $(find $O/ss -name "*kernel_trace.csv" -print -quit) --gap 50 --burst -1 --min-ms 5 > $O/setup_share_build_timeline.txt
rm -rf $O/ss
head -30 $O/kcost_headline_ser.txt
