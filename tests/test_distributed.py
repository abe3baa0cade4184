"""Multi-process (gloo, world_size 2) surveys: parties spread over ranks, EC
collectives over torch.distributed, proof fan-out, shared skipchain block."""
import os
import socket
import subprocess
import sys
import tempfile

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import json

    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drynx_amd.parallel.comm import DistComm
    from drynx_amd.services.api import DrynxClient
    from drynx_amd.services.local import local_cluster, make_survey

    comm = DistComm("cpu")
    cl, node = local_cluster(3, 4, 2, comm=comm, device="cpu", workdir=os.path.join(outdir, f"r{rank}"))
    out = {}
    for op, kw in [("sum", {}), ("variance", {}), ("frequencyCount", {}), ("sum", {"proofs": 1, "ranges": [16, 3]}),
                   ("max", {"proofs": 1, "ranges": [2, 1], "obfuscation": True})]:
        if rank == 0:
            client = DrynxClient(node)
            sq = make_survey(client, cl, op, query_min=0, query_max=4, rows=6, **kw)
            _, vals, res = client.send_survey_query(sq)
            out[f"{op}{len(out)}"] = {"vals": vals[0], "block": res.block.Hash if res.block else None,
                                      "codes": sorted(set(res.block.data_block().Proofs.values())) if res.block else []}
        else:
            res = node.run_survey(None)
            out[f"{op}{len(out)}"] = {"block": res.block.Hash if res.block else None,
                                      "clear": res.clear_dp}
    with open(os.path.join(outdir, f"out{rank}.json"), "w") as f:
        json.dump(out, f, default=str)
    node.close()
    dist.destroy_process_group()


def test_two_rank_gloo_surveys():
    import json

    outdir = tempfile.mkdtemp()
    mp.spawn(_worker, args=(2, _free_port(), outdir), nprocs=2, join=True)
    o0 = json.load(open(os.path.join(outdir, "out0.json")))
    o1 = json.load(open(os.path.join(outdir, "out1.json")))
    for k in o0:
        assert o0[k]["block"] == o1[k]["block"]
    assert o0["sum3"]["codes"] == [1] and o0["max4"]["codes"] == [1]
    assert o0["max4"]["vals"][0] <= 4.0


@pytest.mark.slow
def test_bench_two_ranks_torchrun():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "1", "--warmup", "0", "--records", "2000", "--features", "2", "--max-iter", "5", "--device", "cpu"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line) if (json := __import__("json")) else None
    assert d["n_gpus"] == 2 and d["all_proofs_valid"] and d["value"] > 0
