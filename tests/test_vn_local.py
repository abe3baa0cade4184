"""vn-local verification (proof_collection.verification_mode "local"): each
VN's range lists are checked only by its own rank and helper ranks assigned
to that VN alone.  At 8 ranks (gloo, the bench's placement: CNs on ranks
0-2, VNs on 3-5, DPs round robin from rank 6) one helper of the first VN
reports every list it checks as false: only that VN blames the DPs; the other
VNs' verdicts do not depend on it (in the single-operator pool the same
helper would sway every VN), and that helper never receives another VN's
seed."""
import json
import os
import socket
import sys
import tempfile

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = 8


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, mode, op="frequencyCount", lie=True):
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      OMP_NUM_THREADS="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drynx_amd.parallel.comm import DistComm
    from drynx_amd.protocols import proof_collection as pcp
    from drynx_amd.proofs import requests as prq
    from drynx_amd.services.api import DrynxClient
    from drynx_amd.services.local import local_cluster, make_survey

    comm = DistComm("cpu")
    cl, node = local_cluster(3, 10, 3, comm=comm, device="cpu", workdir=os.path.join(outdir, f"r{rank}"),
                             offsets={"cn": 0, "vn": 3, "dp": 6})
    node.pool_policy = mode
    dps, vns, vn_ranks = [0] * W, [0] * W, [v.rank for v in cl.vns]
    for d in cl.dps:
        dps[d.rank] += 1
    for r in vn_ranks:
        vns[r] += 1
    groups, _ = pcp.verification_groups(pcp.verification_mode(node), W, dps, vns, vn_ranks)
    bad = groups[0][1]  # a helper of the first VN (a rank hosting no VN)
    if rank == bad and lie:
        orig = prq.verify_range_pool_part

        def liar(reqs, vn_idxs, *a, **k):
            res, dig = orig(reqs, vn_idxs, *a, **k)
            return {v: {i: False for i in r} for v, r in res.items()}, dig
        prq.verify_range_pool_part = liar
    seen = {}
    orig_fan = pcp.fan_out

    def spy(ctx, sq, reqs, pool=False, stage=0):
        out = orig_fan(ctx, sq, reqs, pool, stage)
        seen.update(getattr(ctx, "_pool_seeds", {}).get((sq.SurveyID, stage), {}))
        return out
    pcp.fan_out = spy
    out = {"bad": bad, "groups": groups}
    if rank == 0:
        client = DrynxClient(node)
        # frequencyCount: 16-output lists, every helper of a group checks a non-empty slice
        sq = make_survey(client, cl, op, query_min=0, query_max=15, rows=5, proofs=1, ranges=[16, 2])
        _, vals, res = client.send_survey_query(sq)
        codes = {}
        for key, c in res.block.data_block().Proofs.items():
            if "/range/" in key:
                vn = key.rsplit("/", 1)[-1]
                codes.setdefault(vn, set()).add(c)
        out["codes"] = {vn: sorted(c) for vn, c in codes.items()}
        out["vns"] = [v.id for v in cl.vns]
    else:
        node.run_survey(None)
    out["seeds"] = sorted(seen)
    with open(os.path.join(outdir, f"p{rank}.json"), "w") as f:
        json.dump(out, f)
    node.close()
    dist.destroy_process_group()


def test_verification_groups_partition():
    from drynx_amd.protocols.proof_collection import verification_groups

    dps, vns, vn_ranks = [1, 1, 1, 1, 1, 1, 2, 2], [0, 0, 0, 1, 1, 1, 0, 0], [3, 4, 5]
    g, parts = verification_groups("local", 8, dps, vns, vn_ranks)
    assert [x[0] for x in g] == vn_ranks
    helpers = [k for x in g for k in x[1:]]
    assert sorted(helpers) == [0, 1, 2, 6, 7]  # every rank without a VN serves exactly one VN
    assert max(map(len, g)) - min(map(len, g)) <= 1
    for grp, p in zip(g, parts):
        assert sorted(p) == sorted(grp) and all(p[k][1] == len(grp) for k in grp)
    gp, pp = verification_groups("pool", 8, dps, vns, vn_ranks)
    assert all(x == list(range(8)) for x in gp) and pp[0] == pp[1] == pp[2]
    go, po = verification_groups("own", 8, dps, vns, vn_ranks)
    assert go == [[3], [4], [5]] and po == [{3: (0, 1)}, {4: (0, 1)}, {5: (0, 1)}]


@pytest.mark.slow
@pytest.mark.parametrize("mode", ["local", "pool"])
def test_vn_local_verdicts_independent_w8(mode):
    outdir = tempfile.mkdtemp()
    mp.spawn(_worker, args=(W, _free_port(), outdir, mode), nprocs=W, join=True)
    outs = [json.load(open(os.path.join(outdir, f"p{r}.json"))) for r in range(W)]
    o0 = outs[0]
    first, others = o0["vns"][0], o0["vns"][1:]
    assert o0["codes"][first] == [0]  # the lying helper's VN blames the range lists
    bad = o0["bad"]
    if mode == "local":
        assert all(o0["codes"][v] == [1] for v in others), o0["codes"]  # nobody else is swayed
        assert outs[bad]["seeds"] == [first]  # the helper learned only its own VN's seed
    else:
        assert all(o0["codes"][v] == [0] for v in others), o0["codes"]  # the pool: every VN trusts every rank
        assert outs[bad]["seeds"] == sorted(o0["vns"])


@pytest.mark.slow
@pytest.mark.parametrize("mode", ["pool", "local"])
def test_short_lists_w8(mode):
    """One-proof lists (sum) over 8 ranks: most helpers' slices are empty and
    they report nothing for them; that must not count as a false verdict."""
    outdir = tempfile.mkdtemp()
    mp.spawn(_worker, args=(W, _free_port(), outdir, mode, "sum", False), nprocs=W, join=True)
    o0 = json.load(open(os.path.join(outdir, "p0.json")))
    assert all(c == [1] for c in o0["codes"].values()), o0["codes"]
