"""The data plane's ``exchange`` runs ONE ``all_to_all_single`` on every
backend (RCCL on the GPU node, the same call on host-staged buffers under
gloo), so these multi-process gloo tests exercise the exact split / size
logic of the RCCL path: unknown sizes (one size round), known sizes (no size
round), empty and self sends, uneven per-peer payloads, world 2 / 3 / 4."""
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


def _payload(src: int, dst: int, rnd: int):
    import torch

    n = (src * 7 + dst * 3 + rnd) % 5  # 0..4 words: some pairs send nothing
    return torch.arange(n, dtype=torch.int32) + 1000 * src + 100 * dst + 10 * rnd


def _worker(rank, world, port, outdir):
    import json

    import torch
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drynx_amd.parallel.comm import DistComm

    comm = DistComm("cpu")
    errors = []
    for rnd in range(3):
        out = {d: _payload(rank, d, rnd) for d in range(world) if _payload(rank, d, rnd).numel()}
        known = {s: _payload(s, rank, rnd).numel() for s in range(world)} if rnd % 2 else None
        got = comm.exchange(out, recv_sizes=known)
        for s in range(world):
            exp = _payload(s, rank, rnd)
            if exp.numel() == 0:
                if s in got:
                    errors.append(f"r{rnd}: unexpected payload from {s}")
            elif s not in got or not torch.equal(got[s], exp):
                errors.append(f"r{rnd}: wrong payload from {s}: {got.get(s)} vs {exp}")
    # empty exchange (every rank sends nothing)
    if comm.exchange({}):
        errors.append("empty exchange returned data")
    # point-to-point ring (the DRO chain)
    if world > 1:
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        if rank % 2 == 0:
            comm.send(torch.full((6,), rank, dtype=torch.int32), nxt)
            t = comm.recv(6, prv)
        else:
            t = comm.recv(6, prv)
            comm.send(torch.full((6,), rank, dtype=torch.int32), nxt)
        if not bool((t == prv).all()):
            errors.append(f"ring recv {t.tolist()} from {prv}")
    res = {"errors": errors, "sent": comm.bytes_sent, "recv": comm.bytes_recv}
    with open(os.path.join(outdir, f"x{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_exchange_all_to_all_gloo(world):
    import json

    outdir = tempfile.mkdtemp()
    mp.spawn(_worker, args=(world, _free_port(), outdir), nprocs=world, join=True)
    tot_s = tot_r = 0
    for r in range(world):
        d = json.load(open(os.path.join(outdir, f"x{r}.json")))
        assert d["errors"] == [], d["errors"]
        tot_s += d["sent"]
        tot_r += d["recv"]
    assert tot_s == tot_r > 0  # every byte sent to a peer is received by it


def _ctrl_worker(rank, world, port, outdir):
    import json

    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drynx_amd.parallel import comm as cm
    from drynx_amd.utils import timers

    comm = cm.DistComm("cpu")
    errors = []
    # payload sizes around the one-round frame: empty, small, exactly the frame's
    # payload, one byte over, and ~40 KB (two rounds); ranks differ in size
    sizes = [0, 5, cm._CTRL_FIX - 8 - 12, cm._CTRL_FIX - 8, cm._CTRL_FIX - 7, 40_000]
    for k, n in enumerate(sizes):
        mine = {"r": rank, "k": k, "blob": bytes((rank + i) % 251 for i in range(n + rank))}
        got = comm.all_gather_object(mine)
        for r in range(world):
            exp = {"r": r, "k": k, "blob": bytes((r + i) % 251 for i in range(n + r))}
            if got[r] != exp:
                errors.append(f"gather size {n}: rank {r} differs")
        src = k % world
        b = comm.broadcast_object({"src": src, "blob": bytes(i % 7 for i in range(n))} if rank == src else None,
                                  src=src)
        if b != {"src": src, "blob": bytes(i % 7 for i in range(n))}:
            errors.append(f"broadcast size {n} from {src} differs")
    with open(os.path.join(outdir, f"c{rank}.json"), "w") as f:
        json.dump({"errors": errors, "ctrl": timers.counters().get("comm.ctrl_collectives", 0)}, f)
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_control_objects_one_round_framing(world):
    """Control objects travel in one fixed-size round (length + first bytes),
    with a second round only for longer messages; every size on both sides of
    the frame boundary arrives intact on every rank."""
    import json

    outdir = tempfile.mkdtemp()
    mp.spawn(_ctrl_worker, args=(world, _free_port(), outdir), nprocs=world, join=True)
    for r in range(world):
        d = json.load(open(os.path.join(outdir, f"c{r}.json")))
        assert d["errors"] == [], d["errors"]
