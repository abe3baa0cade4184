#!/bin/bash
# Co-hosted VNs' Schnorr checks on the device for small inboxes
# (DRYNX_SIG_DEVICE_MIN=16) vs the host below 256 checks: u0l0 and headline.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-120; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step y_tests 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_sigma.py tests/test_gpu.py
step y_u0l0_host1 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/y_u0l0_host1.json
DRYNX_SIG_DEVICE_MIN=16 step y_u0l0_dev1 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/y_u0l0_dev1.json
step y_u0l0_host2 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/y_u0l0_host2.json
DRYNX_SIG_DEVICE_MIN=16 step y_u0l0_dev2 300 python -u bench.py --steps 10 --warmup 2 --u 0 --l 0 --json-out gpurun_out/y_u0l0_dev2.json
step y_head_host 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/y_head_host.json
DRYNX_SIG_DEVICE_MIN=16 step y_head_dev 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/y_head_dev.json
