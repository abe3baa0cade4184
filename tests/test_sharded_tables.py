"""Sharded prover-table setup: with every rank proving,
each of W ranks builds 1/W of the GLS-2 signed 8-bit G2 / GT tables of a
signature set and the slices are broadcast into every rank's full table;
the result is bit-identical to a single-rank build (gloo, world 3)."""
import hashlib
import os
import socket
import sys
import tempfile

import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _digest(tabs) -> str:
    h = hashlib.sha256()
    for t in tabs[:2]:
        h.update(t.contiguous().numpy().tobytes())
    h.update(tabs[2].numpy().tobytes())
    return h.hexdigest()


def _worker(rank, world, port, outdir, sigs_path):
    import json

    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DRYNX_PROVER_TABLE_BITS="7")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drynx_amd.parallel.comm import DistComm, bytes_to_obj
    from drynx_amd.proofs import range_proof as rp
    from drynx_amd.query import PublishSignatureBytes

    raw = bytes_to_obj(open(sigs_path, "rb").read())
    sigs = [[PublishSignatureBytes(p, s) for p, s in row] for row in raw]
    comm = DistComm("cpu")
    sm = rp.SigMaterial(sigs, "cpu")
    sm.attach_shard(comm, True)
    shared = sm._prover_tables4(torch.device("cpu"), 7)
    out = {"shared": _digest(shared), "bytes_sent": comm.bytes_sent, "bytes_recv": comm.bytes_recv}
    if rank == 0:
        solo = rp.SigMaterial(sigs, "cpu")
        out["solo"] = _digest(solo._prover_tables4(torch.device("cpu"), 7))
    json.dump(out, open(os.path.join(outdir, f"r{rank}.json"), "w"))
    dist.destroy_process_group()


def test_sharded_gls8_tables_match_single_rank_build():
    import json

    from drynx_amd.parallel.comm import obj_to_bytes
    from drynx_amd.proofs import range_proof as rp

    sigs = rp.init_range_proof_signatures([4, 4, 3, 4, 4, 3], "cpu")  # 2 CNs x 3 columns
    rows = [[(s.Public, s.Signature) for s in sigs[i * 3:(i + 1) * 3]] for i in range(2)]
    outdir = tempfile.mkdtemp()
    path = os.path.join(outdir, "sigs.bin")
    open(path, "wb").write(obj_to_bytes(rows))
    mp.spawn(_worker, args=(3, _free_port(), outdir, path), nprocs=3, join=True)
    res = [json.load(open(os.path.join(outdir, f"r{r}.json"))) for r in range(3)]
    assert res[0]["shared"] == res[0]["solo"]
    assert res[1]["shared"] == res[0]["solo"] and res[2]["shared"] == res[0]["solo"]
    # each rank sent its own slice and received the other two
    assert all(r["bytes_sent"] > 0 and r["bytes_recv"] > r["bytes_sent"] for r in res)
