"""A DP whose answer does not fit the query aborts the survey on EVERY rank
(gloo, world 2): the DP's rank announces the abort in the DataCollection
route's size round, so a rank hosting no DP raises too instead of waiting in
the CN collectives (services/service.py, protocols/data_collection.py)."""
import json
import os
import socket
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


def _worker(rank, world, port, outdir, mode):
    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drynx_amd.parallel.comm import DistComm, ExchangeAborted
    from drynx_amd.query import LogisticRegressionParameters
    from drynx_amd.services.api import DrynxClient
    from drynx_amd.services.local import local_cluster, make_survey

    comm = DistComm("cpu")
    # CN + VN on rank 0, the only DP on rank 1
    cl, node = local_cluster(1, 1, 1, comm=comm, device="cpu", workdir=os.path.join(outdir, f"r{rank}"),
                             offsets={"cn": 0, "vn": 0, "dp": 1})
    d = 3
    if rank == 1 and mode == "width":  # the DP's rank reads the query as one output wider
        from drynx_amd.protocols import data_collection as dcp

        orig = dcp.expected_n_out
        dcp.expected_n_out = lambda sq: orig(sq) + 1
    if rank == 1 and mode == "raise":  # one feature too many: the DP's encoder fails
        g = torch.Generator().manual_seed(5)
        node.dp_data = {cl.dps[0].id: (torch.rand((20, d + 1), generator=g, dtype=torch.float64),
                                       torch.randint(0, 2, (20,), generator=g))}
    lp = LogisticRegressionParameters(NbrRecords=20, NbrFeatures=d, Means=[0.5] * d, StandardDeviations=[0.3] * d,
                                      Lambda=1.0, Step=0.1, MaxIterations=5, InitialWeights=[0.1] * (d + 1), K=2,
                                      PrecisionApproxCoefficients=10.0)
    out = {"raised": None}
    try:
        if rank == 0:
            client = DrynxClient(node)
            sq = make_survey(client, cl, "logistic regression", proofs=0, lr_params=lp)
            client.send_survey_query(sq)
        else:
            node.run_survey(None)
    except ExchangeAborted as e:
        out["raised"] = str(e)
    with open(os.path.join(outdir, f"p{rank}.json"), "w") as f:
        json.dump(out, f)
    node.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["raise", "width"])
def test_dp_failure_aborts_every_rank(mode):
    outdir = tempfile.mkdtemp()
    mp.spawn(_worker, args=(2, _free_port(), outdir, mode), nprocs=2, join=True)
    outs = [json.load(open(os.path.join(outdir, f"p{r}.json"))) for r in range(2)]
    msg = "failed to encode" if mode == "raise" else "the query announces"
    assert outs[1]["raised"] and msg in outs[1]["raised"], outs
    assert outs[0]["raised"] and "aborted by rank(s) [1]" in outs[0]["raised"], outs
