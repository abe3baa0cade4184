#!/bin/bash
# Round-4 iteration: range / sigma GPU tests, headline, fault-injected
# headline (kept per-segment buckets), no-range-proof line with host spans,
# a serialized kernel trace (each kernel's cost alone) and the torch-op
# attribution of the non-hand-written kernels.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-600; if [ $rc -ne 0 ]; then tail -25 gpurun_out/$name.log; exit $rc; fi; }
step pytest_it 300 python -u -m pytest tests/test_rpmsm.py tests/test_range_hardening.py tests/test_sigma.py tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread
step bench_it 300 python -u bench.py --steps 10 --warmup 2
DRYNX_TRACE=gpurun_out/trace_fault step bench_fault_it 300 python -u bench.py --steps 5 --warmup 1 --fault-dp 3
python tools/host_trace.py gpurun_out/trace_fault.r0.json 0.3 > gpurun_out/host_trace_fault.txt
DRYNX_TRACE=gpurun_out/trace_u0l0 step bench_u0l0_it 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0
python tools/host_trace.py gpurun_out/trace_u0l0.r0.json 0.05 > gpurun_out/host_trace_u0l0.txt
AMD_SERIALIZE_KERNEL=3 step prof_ser 500 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_ser -o bench -- python3 bench.py --steps 2 --warmup 1
python tools/kernel_cost.py gpurun_out/prof_ser/bench_kernel_trace.csv > gpurun_out/kernel_cost_serial.txt
DRYNX_TORCH_PROF=gpurun_out/torch_prof.txt step bench_tprof 400 python -u bench.py --steps 2 --warmup 1
