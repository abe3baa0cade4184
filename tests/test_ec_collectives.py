"""EC collectives over torch.distributed (gloo, world 3: uneven shard bounds):
sum_to_root (direct and reduce-scatter paths), all_reduce_cv, broadcast_cv,
route.  Mirrors the reference's tree aggregation (services/service.go:676,
unlynx CollectiveAggregation) with the full-mesh data plane of SURVEY §2.4."""
import json
import os
import socket
import sys
import tempfile

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SECRET = 0x1234567


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drynx_amd.crypto import elgamal as eg
    from drynx_amd.crypto import oracle as O
    from drynx_amd.parallel import ec_collectives as ec
    from drynx_amd.parallel.comm import DistComm

    comm = DistComm("cpu")
    pk = eg.pk_table(O.g1_mul(SECRET, O.G1_GEN))
    n = 7
    mine = [(rank + 1) * (i + 1) - 3 for i in range(n)]
    cv, _ = eg.encrypt_ints(pk, mine)
    out = {}
    out["all_reduce"] = eg.decrypt_ints(SECRET, ec.all_reduce_cv(comm, [cv], n))
    direct = ec.sum_to_root(comm, [cv], n, root=1)
    sharded = ec.sum_to_root(comm, [cv, cv], n, root=0, shard_threshold=2)
    out["direct"] = eg.decrypt_ints(SECRET, direct) if direct is not None else None
    out["sharded"] = eg.decrypt_ints(SECRET, sharded) if sharded is not None else None
    b = ec.broadcast_cv(comm, cv if rank == 2 else None, n, root=2)
    out["bcast"] = eg.decrypt_ints(SECRET, b)
    ki = ec.KeyIndex([f"dp{i}" for i in range(world)])
    got = ec.route(comm, [((rank + 1) % world, f"dp{rank}", cv)], ki)
    out["route"] = {k: eg.decrypt_ints(SECRET, v) for k, v in got.items()}
    with open(os.path.join(outdir, f"out{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


def test_ec_collectives_gloo_world3():
    W, n = 3, 7
    outdir = tempfile.mkdtemp()
    mp.spawn(_worker, args=(W, _free_port(), outdir), nprocs=W, join=True)
    outs = [json.load(open(os.path.join(outdir, f"out{r}.json"))) for r in range(W)]
    vals = [[(r + 1) * (i + 1) - 3 for i in range(n)] for r in range(W)]
    total = [sum(v[i] for v in vals) for i in range(n)]
    for r, o in enumerate(outs):
        assert o["all_reduce"] == total
        assert o["direct"] == (total if r == 1 else None)
        assert o["sharded"] == ([2 * t for t in total] if r == 0 else None)
        assert o["bcast"] == vals[2]
        src = (r - 1) % W
        assert o["route"] == {f"dp{src}": vals[src]}
