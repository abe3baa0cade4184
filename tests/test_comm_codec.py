"""Control-plane codec (parallel/comm.py): msgpack with extension types for
big ints, tuples, sets, tensors and arrays; no pickle crosses a rank boundary
(the reference's onet messages are protobuf, never executable payloads).
Round trip, refusal of non-data objects, and the gloo world-3 object
collectives built on it."""
import json
import os
import socket
import sys
import tempfile

import msgpack
import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from drynx_amd.parallel.comm import bytes_to_obj, obj_to_bytes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_codec_round_trip():
    msg = {("vn0", 3): [1 << 254, -(1 << 70), (1, (2, "x")), {4, 5}, b"\x00\xff", bytearray(b"z"), None, 2.5,
                        False, np.int64(9)],
           7: {"t": torch.arange(6, dtype=torch.int32).reshape(2, 3), "e": torch.zeros(0, dtype=torch.bfloat16),
               "a": np.arange(5, dtype=np.uint64)}}
    got = bytes_to_obj(obj_to_bytes(msg))
    lst = got[("vn0", 3)]
    assert lst[:5] == [1 << 254, -(1 << 70), (1, (2, "x")), {4, 5}, b"\x00\xff"]
    assert lst[5:] == [b"z", None, 2.5, False, 9]
    assert torch.equal(got[7]["t"], msg[7]["t"]) and got[7]["e"].dtype == torch.bfloat16
    assert got[7]["a"].dtype == np.uint64 and got[7]["a"].tolist() == list(range(5))


def test_codec_refuses_objects_and_unknown_extensions():
    class Thing:
        pass

    with pytest.raises(TypeError):
        obj_to_bytes({"x": Thing()})
    with pytest.raises(TypeError):
        obj_to_bytes(lambda: 0)
    with pytest.raises(ValueError):
        bytes_to_obj(msgpack.packb(msgpack.ExtType(99, b"")))
    with pytest.raises(ValueError):  # a dtype outside the whitelist
        bytes_to_obj(msgpack.packb(msgpack.ExtType(5, obj_to_bytes(["|O", [1], b"\x00" * 8]))))


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
    from drynx_amd.parallel.comm import DistComm

    comm = DistComm("cpu")
    b = comm.broadcast_object({"cmd": ("run", 1 << 100), "pad": b"x" * 1000} if rank == 1 else None, src=1)
    g = comm.all_gather_object({f"vn{rank}": [rank] * (rank * 50 + 1)})
    out = {"bcast": [b["cmd"][0], str(b["cmd"][1]), len(b["pad"])],
           "gather": [sorted(d.items()) for d in g]}
    with open(os.path.join(outdir, f"out{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.destroy_process_group()


def test_object_collectives_gloo_world3():
    W = 3
    outdir = tempfile.mkdtemp()
    mp.spawn(_worker, args=(W, _free_port(), outdir), nprocs=W, join=True)
    for r in range(W):
        o = json.load(open(os.path.join(outdir, f"out{r}.json")))
        assert o["bcast"] == ["run", str(1 << 100), 1000]
        assert o["gather"] == [[[f"vn{s}", [s] * (s * 50 + 1)]] for s in range(W)]
