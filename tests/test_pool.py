"""Pooled range verification over several ranks (gloo, world 3, one VN):
helper ranks receive only their slice of each range bundle (~1/W of the
payload), check it with coins derived from the VN's seed, and report a slice
digest; the VN accepts a helper's verdict only for exactly the bytes it
received itself.  A prover that sends a helper a different (forged) slice is
caught by the digest and the VN re-checks that slice on its own."""
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


def _worker(rank, world, port, outdir, equivocate, threshold=1.0):
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      DRYNX_VN_POOL="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drynx_amd.parallel.comm import DistComm
    from drynx_amd.proofs import requests as prq
    from drynx_amd.services.api import DrynxClient
    from drynx_amd.services.local import local_cluster, make_survey

    if equivocate:
        from drynx_amd.protocols import proof_collection as pcp

        def forged(lists, sq, part):  # the prover hands helpers a tampered slice
            out = prq.slice_lists(lists, sq, part)
            for r in out:
                if r.zr is not None:
                    r.zr = r.zr.clone()
                    r.zr[:, 0] ^= 1
            return out
        pcp._helper_slice = forged
    comm = DistComm("cpu")
    # 1 VN: ranks without it are pool helpers; DPs on every rank
    cl, node = local_cluster(3, 3, 1, comm=comm, device="cpu", workdir=os.path.join(outdir, f"r{rank}"),
                             offsets={"cn": 0, "vn": 0, "dp": 0})
    out = {}
    before = comm.bytes_recv
    if rank == 0:
        client = DrynxClient(node)
        sq = make_survey(client, cl, "frequencyCount", query_min=0, query_max=5, rows=8, proofs=1, ranges=[2, 4],
                         thresholds=[threshold, 1.0, 1.0, 0.0, 1.0])
        _, vals, res = client.send_survey_query(sq)
        out["codes"] = sorted(set(res.block.data_block().Proofs.values()))
        out["vals"] = [float(v) for v in vals[0]]
        out["clear_dp"] = res.clear_dp
    else:
        res = node.run_survey(None)
        out["clear_dp"] = res.clear_dp
    out["recv"] = comm.bytes_recv - before
    out["vn_rank"] = cl.vns[0].rank
    with open(os.path.join(outdir, f"p{rank}.json"), "w") as f:
        json.dump(out, f, default=str)
    node.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("equivocate,threshold", [(False, 1.0), (True, 1.0), (True, 0.0)])
def test_pool_slices_and_digests_world3(equivocate, threshold):
    """threshold 0: the VN samples no list; a helper digest mismatch must not
    turn those lists into code 0 (its re-check covers only sampled lists)."""
    outdir = tempfile.mkdtemp()
    mp.spawn(_worker, args=(3, _free_port(), outdir, equivocate, threshold), nprocs=3, join=True)
    outs = [json.load(open(os.path.join(outdir, f"p{r}.json"))) for r in range(3)]
    o0 = outs[0]
    # every proof verified (the forged helper slices were re-checked by the VN);
    # with threshold 0 every proof is received, not checked (code 2)
    assert o0["codes"] == ([1] if threshold == 1.0 else [2]), o0["codes"]
    clear = [0] * 6
    for o in outs:
        for v in o["clear_dp"].values():
            v = json.loads(v.replace("'", '"')) if isinstance(v, str) else v
            clear = [a + b for a, b in zip(clear, v[0])]
    assert o0["vals"] == [float(x) for x in clear]
    vn_rank = o0["vn_rank"]
    helpers = [r for r in range(3) if r != vn_rank]
    assert helpers
    # a helper receives its slices only: far less than the VN's full inbox
    for h in helpers:
        assert outs[h]["recv"] < 0.8 * outs[vn_rank]["recv"], (h, outs[h]["recv"], outs[vn_rank]["recv"])


def test_balanced_pool_parts_partition_every_list():
    """Weighted pool parts (prq.balanced_parts) cut every list into disjoint,
    covering slices; a rank hosting a VN gets a shorter one, a rank proving
    more DPs does not (every part starts at the fan-out, after the slowest
    rank's proving); DRYNX_POOL_BALANCE=0 gives the equal slices."""
    from drynx_amd.proofs import requests as prq

    class _Sq:
        RangeProofThreshold = 1.0
    dps, vns = [1, 1, 1, 1, 1, 1, 2, 2], [0, 0, 0, 1, 1, 1, 0, 0]
    parts = prq.balanced_parts(8, dps, vns)
    for n in (1, 7, 8, 100, 2070, 12345):
        b = [prq.sampled_bounds(_Sq, n, p) for p in parts]
        assert b[0][0] == 0 and b[-1][1] == n and all(b[k][1] == b[k + 1][0] for k in range(7))
    b = [prq.sampled_bounds(_Sq, 2070, p) for p in parts]
    size = [hi - lo for lo, hi in b]
    assert size[3] < size[0] and abs(size[6] - size[0]) <= 1 and abs(size[6] - size[7]) <= 1
    assert prq.balanced_parts(1, [10], [3]) == [(0, 1)]
