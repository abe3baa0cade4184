"""Communication planes for the party runtime.

The reference moves every protocol message over onet (TCP/protobuf between
separate server processes).  Here parties are logical
entities hosted by ranks (one rank per GPU) and the data plane is
torch.distributed:

* device tensors (ciphertext vectors, proof blobs) go over the ``nccl``
  backend, which on ROCm is RCCL over xGMI;
* small control messages (the SurveyQuery, bitmaps, acks) are msgpack-coded
  (``obj_to_bytes``: plain data only -- no pickle, nothing executable crosses a
  rank boundary) and broadcast / all-gathered as byte tensors on a gloo group.

Point-to-point patterns used by the protocols:
  - ``exchange``: personalised all-to-all (star gathers DP->CN, CN->root, proof
    fan-out to VNs): ONE ``all_to_all_single`` whose per-peer splits go
    straight over the 7 xGMI links on RCCL (no ring hops).  gloo runs the very
    same call on host-staged buffers, so every CPU multi-process test
    exercises the split / size logic of the RCCL path.
  - ``send/recv``: the DRO shuffle chain CN_i -> CN_{i+1}.
RCCL cannot add BN254 points, so EC reductions are exchange + HIP reduce
kernels (parallel/ec_collectives.py).
"""
from __future__ import annotations

import os

import msgpack
import numpy as np
import torch
import torch.distributed as dist

from ..utils import timers


class Comm:
    rank: int = 0
    world: int = 1
    device: torch.device = torch.device("cpu")
    bytes_sent: int = 0  # data-plane bytes to / from other ranks (traffic accounting)
    bytes_recv: int = 0

    def barrier(self):
        pass

    def broadcast_object(self, obj, src: int = 0):
        return obj

    def all_gather_object(self, obj) -> list:
        return [obj]

    def exchange(self, outgoing: dict, recv_sizes: dict | None = None, abort: str | None = None) -> dict:
        """outgoing: dst_rank -> int32 tensor (any shape, on self.device).
        Returns src_rank -> flat int32 tensor received (only non-empty ones).
        ``recv_sizes`` (src -> numel), when the protocol already knows them,
        saves the size round (and its host synchronisation).  ``abort``: this
        rank cannot take part (e.g. its DPs' answers do not fit the query); it
        announces a negative size to every rank in the size round, so EVERY
        rank raises instead of the others waiting in a later collective."""
        if abort is not None:
            raise ExchangeAborted(f"rank {self.rank}: {abort}")
        return {self.rank: outgoing[self.rank].reshape(-1)} if self.rank in outgoing else {}

    def plane(self, name: str) -> "Comm":
        """A communicator for a second thread of collectives (e.g. the pooled
        range verification running beside the CN phases): its control
        collectives use their own process group, so the two threads never
        interleave operations on one group.  It carries no data plane."""
        return self

    def send(self, t: torch.Tensor, dst: int):
        raise RuntimeError("single-process comm has no peers")

    def recv(self, numel: int, src: int) -> torch.Tensor:
        raise RuntimeError("single-process comm has no peers")

    def broadcast_into(self, t: torch.Tensor, src: int):
        """Fill contiguous ``t`` on every rank with ``src``'s content, in place
        (sharded setup: each rank builds a slice of a large table, then every
        slice is broadcast into the same view of the full table)."""
        return t

    def exchange_bytes(self, outgoing: dict) -> dict:
        """Like exchange but for python bytes payloads (proof blobs)."""
        tens = {d: _bytes_to_i32(b, self.device) for d, b in outgoing.items()}
        got = self.exchange(tens)
        return {s: _i32_to_bytes(t) for s, t in got.items()}


class ExchangeAborted(RuntimeError):
    """A rank aborted a data-plane exchange (``Comm.exchange(abort=...)``)."""


def _bytes_to_i32(b: bytes, device) -> torch.Tensor:
    n = len(b)
    pad = (-(n + 8)) % 4
    raw = n.to_bytes(8, "little") + b + b"\x00" * pad
    return torch.from_numpy(np.frombuffer(raw, dtype=np.int32).copy()).to(device)


def _i32_to_bytes(t: torch.Tensor) -> bytes:
    raw = t.detach().cpu().numpy().tobytes()
    n = int.from_bytes(raw[:8], "little")
    return raw[8: 8 + n]


class LocalComm(Comm):
    """World of one rank: every logical party lives in this process."""

    def __init__(self, device="cpu"):
        self.rank, self.world = 0, 1
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())


class DistComm(Comm):
    """torch.distributed world; one rank per GPU (RCCL) or per CPU process (gloo)."""

    def __init__(self, device=None):
        assert dist.is_initialized(), "init_process_group first (see parallel.launch)"
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.backend = dist.get_backend()
        if device is None:
            if self.backend == "nccl":
                device = torch.device("cuda", torch.cuda.current_device())
            else:
                device = torch.device("cpu")
        self.device = torch.device(device)
        # control plane: gloo group (CPU objects) even when the data plane is RCCL
        self._ctrl = dist.new_group(backend="gloo") if self.backend == "nccl" else None
        # where the data plane's all_to_all_single buffers live: HBM for RCCL,
        # host memory for gloo (whose all-to-all is CPU only)
        self._stage = self.device if self.backend == "nccl" else torch.device("cpu")
        # control groups of the side planes (created by every rank, in this order)
        # ("pool2": the second stage of a staged range plane, proof_collection.extend_range_plane)
        self._planes = {name: _CtrlPlane(self, dist.new_group(backend="gloo")) for name in ("pool", "pool2")}

    def plane(self, name: str) -> "Comm":
        return self._planes[name]

    def barrier(self):
        if self.backend == "nccl":
            dist.barrier(group=self._ctrl)
        else:
            dist.barrier()

    def broadcast_object(self, obj, src: int = 0):
        return _bcast_obj(self.rank, obj, src, self._ctrl)

    def all_gather_object(self, obj) -> list:
        return _gather_obj(self.rank, self.world, obj, self._ctrl)

    def exchange(self, outgoing: dict, recv_sizes: dict | None = None, abort: str | None = None) -> dict:
        """ONE ``all_to_all_single`` whatever the backend: on RCCL the per-peer
        splits go straight over the xGMI links from HBM; on gloo (CPU tests,
        one-GPU rehearsals) the same call runs on host-staged buffers.  Unknown
        receive sizes cost one size round (a W-element all-to-all), which also
        carries an ``abort`` (negative sizes) to every rank."""
        W = self.world
        stage = self._stage
        timers.count("comm.data_exchanges")
        flat = {d: t.reshape(-1).to(torch.int32) for d, t in outgoing.items()} if abort is None else {}
        send_sizes = [0] * W
        for d, t in flat.items():
            send_sizes[d] = t.numel()
        if recv_sizes is None:
            ss = torch.tensor([-1] * W if abort is not None else send_sizes, dtype=torch.int64, device=stage)
            rs = torch.empty_like(ss)
            dist.all_to_all_single(rs, ss)
            recv = [int(v) for v in rs.tolist()]
            if abort is not None:
                raise ExchangeAborted(f"rank {self.rank}: {abort}")
            bad = [s for s, v in enumerate(recv) if v < 0]
            if bad:
                raise ExchangeAborted(f"rank {self.rank}: exchange aborted by rank(s) {bad}")
        elif abort is not None:
            raise ValueError("exchange(abort=...) needs the size round (recv_sizes=None)")
        else:
            recv = [int(recv_sizes.get(s, 0)) for s in range(W)]
        parts = [flat[d].to(stage) for d in range(W) if send_sizes[d]]
        send = torch.cat(parts) if parts else torch.empty(0, dtype=torch.int32, device=stage)
        buf = torch.empty(sum(recv), dtype=torch.int32, device=stage)
        dist.all_to_all_single(buf, send, output_split_sizes=recv, input_split_sizes=send_sizes)
        self.bytes_sent += 4 * (sum(send_sizes) - send_sizes[self.rank])
        self.bytes_recv += 4 * (sum(recv) - recv[self.rank])
        if buf.device != self.device:
            buf = buf.to(self.device, non_blocking=True)
        out, off = {}, 0
        for s in range(W):
            if recv[s]:
                out[s] = buf[off: off + recv[s]]
            off += recv[s]
        return out

    _BCAST_CHUNK = 1 << 28  # elements per collective (1 GiB of int32)

    def broadcast_into(self, t: torch.Tensor, src: int):
        """``Comm.broadcast_into`` over the data plane: RCCL broadcasts straight
        into the HBM view (chunked to 1 GiB per call, no staging copy, no
        gathered temporary); gloo stages each chunk through host memory."""
        assert t.is_contiguous()
        flat = t.view(-1)
        n = flat.numel()
        for a in range(0, n, self._BCAST_CHUNK):
            part = flat[a: a + self._BCAST_CHUNK]
            if part.device == self._stage:
                dist.broadcast(part, src)
            else:
                st = part.to(self._stage) if self.rank == src else torch.empty(part.shape, dtype=part.dtype,
                                                                                 device=self._stage)
                dist.broadcast(st, src)
                if self.rank != src:
                    part.copy_(st)
            if self.rank == src:
                self.bytes_sent += part.numel() * part.element_size()
            else:
                self.bytes_recv += part.numel() * part.element_size()
        return t

    def send(self, t: torch.Tensor, dst: int):
        t = t.contiguous().to(self._stage)
        self.bytes_sent += t.numel() * t.element_size()
        dist.send(t, dst)

    def recv(self, numel: int, src: int) -> torch.Tensor:
        t = torch.empty(numel, dtype=torch.int32, device=self._stage)
        dist.recv(t, src)
        self.bytes_recv += 4 * numel
        return t.to(self.device)


_CTRL_FIX = 8192  # bytes per rank in a control message's first (usually only) round


def _frame(b: bytes) -> torch.Tensor:
    """[8-byte length | first _CTRL_FIX - 8 bytes of the message], zero padded."""
    t = torch.zeros(_CTRL_FIX, dtype=torch.uint8)
    t[:8] = torch.frombuffer(bytearray(len(b).to_bytes(8, "little")), dtype=torch.uint8)
    head = b[: _CTRL_FIX - 8]
    if head:
        t[8: 8 + len(head)] = torch.frombuffer(bytearray(head), dtype=torch.uint8)
    return t


def _unframe(t: torch.Tensor) -> tuple:
    raw = t.numpy().tobytes()
    n = int.from_bytes(raw[:8], "little")
    return n, raw[8: 8 + min(n, _CTRL_FIX - 8)]


def _bcast_obj(rank: int, obj, src: int, group):
    """Control message from ``src`` to every rank (msgpack, no pickle): ONE
    fixed-size broadcast carrying the length and the first bytes (a second
    one only for the tail of a message over ~8 KB) -- each control collective
    is a latency-bound round over the host TCP plane."""
    timers.count("comm.ctrl_collectives")
    b = obj_to_bytes(obj) if rank == src else b""
    t = _frame(b) if rank == src else torch.zeros(_CTRL_FIX, dtype=torch.uint8)
    dist.broadcast(t, src, group=group)
    n, head = _unframe(t)
    if n > _CTRL_FIX - 8:
        rest = n - (_CTRL_FIX - 8)
        tail = torch.frombuffer(bytearray(b[_CTRL_FIX - 8:]), dtype=torch.uint8) if rank == src \
            else torch.empty(rest, dtype=torch.uint8)
        dist.broadcast(tail, src, group=group)
        head = head + tail.numpy().tobytes()
    return obj if rank == src else bytes_to_obj(head)


def _gather_obj(rank: int, world: int, obj, group) -> list:
    """All-gather of control objects: one fixed-size round (lengths + first
    bytes of every rank's message), a second only when some message is
    longer than it (every rank sees every length, so all agree)."""
    timers.count("comm.ctrl_collectives")
    b = obj_to_bytes(obj)
    frames = [torch.empty(_CTRL_FIX, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(frames, _frame(b), group=group)
    got = [_unframe(f) for f in frames]
    m = max(n for n, _ in got) - (_CTRL_FIX - 8)
    if m > 0:
        mine = torch.zeros(m, dtype=torch.uint8)
        tail = b[_CTRL_FIX - 8:]
        if tail:
            mine[: len(tail)] = torch.frombuffer(bytearray(tail), dtype=torch.uint8)
        bufs = [torch.empty(m, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(bufs, mine, group=group)
        got = [(n, h + (bufs[r].numpy().tobytes()[: n - (_CTRL_FIX - 8)] if n > _CTRL_FIX - 8 else b""))
               for r, (n, h) in enumerate(got)]
    return [obj if r == rank else bytes_to_obj(got[r][1]) for r in range(world)]


class _CtrlPlane(Comm):
    """Control collectives of a side plane on their own gloo group (see
    ``Comm.plane``); data-plane exchanges stay on the main thread's comm."""

    def __init__(self, parent: "DistComm", group):
        self.rank, self.world, self.device = parent.rank, parent.world, parent.device
        self._group = group

    def barrier(self):
        dist.barrier(group=self._group)

    def broadcast_object(self, obj, src: int = 0):
        return _bcast_obj(self.rank, obj, src, self._group)

    def all_gather_object(self, obj) -> list:
        return _gather_obj(self.rank, self.world, obj, self._group)

    def exchange(self, outgoing: dict, recv_sizes: dict | None = None) -> dict:
        raise RuntimeError("a control plane carries no data-plane exchanges (use the main comm)")


def _force_dist() -> bool:
    """DRYNX_FORCE_DIST=1: a world of ONE rank still runs torch.distributed and
    the DistComm planes (RCCL data plane + gloo control groups), so a one-GPU
    box exercises the exact multi-GPU code path (init with a device id, the
    all_to_all_single splits on HBM tensors, side-plane groups)."""
    return os.environ.get("DRYNX_FORCE_DIST") == "1"


def make_comm(device=None) -> Comm:
    if dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or _force_dist()):
        return DistComm(device)
    if device is None:
        device = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0"))) if torch.cuda.is_available() else "cpu"
    device = torch.device(device)
    if device.type == "cuda" and device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    return LocalComm(device)


def init_distributed(backend: str | None = None):
    """Initialise torch.distributed from the torchrun env (RANK/WORLD_SIZE/MASTER_*)."""
    if dist.is_initialized():
        return
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1 and not (_force_dist() and "MASTER_ADDR" in os.environ):
        return
    if backend is None:
        # DRYNX_DIST_BACKEND=gloo rehearses the multi-rank GPU path with several
        # ranks sharing one GPU (RCCL needs one GPU per rank)
        backend = os.environ.get("DRYNX_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group("gloo")


# ---------------------------------------------------------------- control codec
# msgpack plus four extension types; anything else is refused when encoding.
# Decoding builds only ints, floats, str, bytes, lists, dicts, tuples, sets,
# numpy arrays and CPU tensors of whitelisted dtypes: a peer's message cannot
# name code to run (the reference's onet messages are protobuf for the same
# reason).
_X_INT, _X_TUPLE, _X_SET, _X_TENSOR, _X_NDARRAY = 1, 2, 3, 4, 5
_TORCH_DTYPES = {str(d).removeprefix("torch."): d for d in (
    torch.uint8, torch.int8, torch.int16, torch.int32, torch.int64, torch.bool, torch.float16, torch.bfloat16,
    torch.float32, torch.float64)}
_NP_DTYPES = {np.dtype(t).str for t in (np.uint8, np.int8, np.int16, np.int32, np.int64, np.uint16, np.uint32,
                                        np.uint64, np.bool_, np.float16, np.float32, np.float64)}


def _pack_default(o):
    if isinstance(o, bool):
        return bool(o)
    if isinstance(o, int):  # beyond 64 bits (BN254 scalars, coordinates)
        return msgpack.ExtType(_X_INT, int(o).to_bytes(int(o).bit_length() // 8 + 1, "little", signed=True))
    if isinstance(o, tuple):
        return msgpack.ExtType(_X_TUPLE, obj_to_bytes(list(o)))
    if isinstance(o, (set, frozenset)):
        return msgpack.ExtType(_X_SET, obj_to_bytes(list(o)))
    if isinstance(o, (bytearray, memoryview)):
        return bytes(o)
    if isinstance(o, np.generic):
        return o.item()
    for base in (dict, list, str, float, bytes):  # subclasses (OrderedDict, IntEnum-like str, ...)
        if isinstance(o, base):
            return base(o)
    if isinstance(o, torch.Tensor):
        t = o.detach().cpu().contiguous()
        name = str(t.dtype).removeprefix("torch.")
        if name not in _TORCH_DTYPES:
            raise TypeError(f"control message: tensor dtype {t.dtype} not supported")
        raw = t.reshape(-1).view(torch.uint8).numpy().tobytes() if t.numel() else b""
        return msgpack.ExtType(_X_TENSOR, obj_to_bytes([name, list(t.shape), raw]))
    if isinstance(o, np.ndarray):
        a = np.ascontiguousarray(o)
        if a.dtype.str not in _NP_DTYPES:
            raise TypeError(f"control message: array dtype {a.dtype} not supported")
        return msgpack.ExtType(_X_NDARRAY, obj_to_bytes([a.dtype.str, list(a.shape), a.tobytes()]))
    raise TypeError(f"control message: {type(o).__name__} is not plain data")


def _ext_hook(code, data):
    if code == _X_INT:
        return int.from_bytes(data, "little", signed=True)
    if code == _X_TUPLE:
        return tuple(bytes_to_obj(data))
    if code == _X_SET:
        return set(bytes_to_obj(data))
    if code == _X_TENSOR:
        name, shape, raw = bytes_to_obj(data)
        dt = _TORCH_DTYPES[name]
        flat = torch.frombuffer(bytearray(raw), dtype=torch.uint8) if raw else torch.zeros(0, dtype=torch.uint8)
        return flat.view(dt).reshape(shape)
    if code == _X_NDARRAY:
        dts, shape, raw = bytes_to_obj(data)
        if dts not in _NP_DTYPES:
            raise ValueError(f"control message: array dtype {dts} not supported")
        return np.frombuffer(raw, dtype=np.dtype(dts)).reshape(shape).copy()
    raise ValueError(f"control message: unknown extension type {code}")


def obj_to_bytes(obj) -> bytes:
    return msgpack.packb(obj, default=_pack_default, strict_types=True, use_bin_type=True)


def bytes_to_obj(b: bytes):
    return msgpack.unpackb(b, ext_hook=_ext_hook, raw=False, strict_map_key=False)
