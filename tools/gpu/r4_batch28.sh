#!/bin/bash
# One-round control framing: the RCCL plane tests (nccl data plane + gloo
# control group on one GPU), distributed CPU tests on the box, headline once.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
step() { local name=$1; shift; timeout -k 10 "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -1 gpurun_out/$name.log | cut -c1-160; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
step u_tests 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_plane.py tests/test_comm_exchange.py
step u_head 300 python -u bench.py --steps 10 --warmup 2 --json-out gpurun_out/u_head.json
