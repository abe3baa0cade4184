"""The RCCL ("nccl" backend) code path of the data plane on one GPU: the
DistComm planes under torchrun with one rank (DRYNX_FORCE_DIST=1) -- the
only RCCL configuration a one-GPU box can run (RCCL refuses two ranks on
one device) -- and a small verifiable LR query through bench.py on that
communicator."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun(args, port, timeout=240):
    env = dict(os.environ, DRYNX_FORCE_DIST="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), *args]
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


def test_rccl_dist_comm_one_rank():
    r = _torchrun(["tools/dist_smoke.py"], 29641)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "dist smoke ok: backend nccl" in r.stdout


def test_bench_on_rccl_comm_one_rank():
    r = _torchrun(["bench.py", "--steps", "1", "--warmup", "1", "--features", "6", "--records", "20000"], 29643)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["all_proofs_valid"] and line["result_ok"] and line["n_gpus"] == 1
