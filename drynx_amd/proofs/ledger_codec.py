"""Compact ledger form of range-proof payloads.

A VN stores every signed range bundle it received (storeProof,
proof_collection_protocol.go:318-331; bbolt keeps them all).  ~68% of a
bundle is GT elements -- the A_j commitments, 384 bytes each -- and a GT
element is unitary, so the ledger keeps each as its torus (T2) image c =
(1 + g) / h, 192 bytes (``native.gt_t2_compress``, csrc/kernels/dx_gt_t2.hip):
a query's ~560 MB of range payloads become ~370 MB to copy off the GPU and
fdatasync (verdict r4 weak #4: the W = 8 ledger is disk-bound).

Reading a value back rebuilds the signed payload bit for bit
(``decompress_bytes``; ``ledger.store.Store`` does it for every blob it
returns), so GetProofs, digests and audits see exactly what was signed.  A
list whose GT elements do not all round-trip exactly (non-canonical limbs,
not unitary: a malformed or malicious proof) makes the whole bundle fall back
to the raw bytes.

Blob layout (int32 words): MAGIC, ok flag (written on the device: 1 when
every element round-trips), raw payload words (int64), region count, then
(word offset int64, element count int64) per region, then the payload with
each region's A block replaced by its T2 image.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import native as nt

MAGIC = 0x32435052  # b"RPC2" little-endian
_HEAD = 5


def is_compressed(b) -> bool:
    """A blob in this layout: the magic, the ok flag and a header whose sizes
    account for every byte (a stored payload of another kind that happens to
    start with the magic is not mistaken for one)."""
    if len(b) < 4 * _HEAD or len(b) % 4 or int.from_bytes(bytes(b[:4]), "little") != MAGIC:
        return False
    w = np.frombuffer(bytes(b[:4 * _HEAD]), dtype=np.int32)
    k = int(w[4])
    if int(w[1]) != 1 or k < 0 or 4 * (_HEAD + 4 * k) > len(b):
        return False
    total = int(w[2:4].view(np.int64)[0])
    regs = np.frombuffer(bytes(b[4 * _HEAD: 4 * (_HEAD + 4 * k)]), dtype=np.int64).reshape(k, 2)
    return bool(len(b) // 4 == _HEAD + 4 * k + total - 48 * int(regs[:, 1].sum())) if k else False


class Pending:
    """A range bundle to store compressed.  ``produce`` (the ledger thread, on
    the ledger stream) locates the GT blocks (from the VN's decoded views, or
    from the bundle's own header words when the payload is stored before the
    VN decoded it), builds the device image (``launch``), copies it to the
    host and returns the bytes to store (``finish``): the image when every
    element round-trips, else the raw payload."""

    def __init__(self, tensor: torch.Tensor, regions: list | None):
        self.tensor = tensor.contiguous().reshape(-1)  # int32 words
        self.regions = regions  # [(word offset, n elements)], sorted; None: from the header
        self.image = None

    def produce(self, stream):
        with torch.cuda.stream(stream):
            if self.regions is None:
                self.regions = regions_from_header(self.tensor)
            if not self.regions:
                return memoryview(self.tensor.cpu().numpy()).cast("B")
            img = self.launch()
            host = torch.empty((img.numel(),), dtype=torch.uint8, pin_memory=True)
            nt.copy_to_host([(img, host)], host)
            ev = torch.cuda.Event()
            ev.record(stream)
        ev.synchronize()
        return self.finish(memoryview(host.numpy()))

    def launch(self) -> torch.Tensor:
        t = self.tensor
        dev = t.device
        if dev.type == "cuda":
            t.record_stream(torch.cuda.current_stream(dev))
        head = [MAGIC, 0] + list(np.array([t.numel()], dtype=np.int64).view(np.int32)) + [len(self.regions)]
        for off, m in self.regions:
            head += list(np.array([off, m], dtype=np.int64).view(np.int32))
        n_img = len(head) + t.numel() - sum(48 * m for _, m in self.regions)
        img = torch.empty((n_img,), dtype=torch.int32, device=dev)
        hdr = torch.tensor(head, dtype=torch.int32)
        if dev.type == "cuda":
            hdr = hdr.pin_memory().to(dev, non_blocking=True)
        pairs, oks, pos, q = [(hdr, img[:len(head)])], [], 0, len(head)
        for off, m in self.regions:
            pairs.append((t[pos:off], img[q: q + off - pos]))
            q += off - pos
            c = img[q: q + 48 * m].view(m, 48)
            oks.append(nt.gt_t2_compress(t[off: off + 96 * m].view(m, 96), out=c))
            q += 48 * m
            pos = off + 96 * m
        pairs.append((t[pos:], img[q:]))
        nt.batched_copy(pairs)  # the header and every raw segment in one launch
        okall = torch.cat(oks).all() if len(oks) > 1 else oks[0].all()
        img[1:2].copy_(okall.to(torch.int32).view(1))
        self.image = img
        return img.view(torch.uint8)

    def finish(self, mv: memoryview):
        """The bytes to store: the compressed image when every element
        round-trips, else the raw payload (a synchronous copy, rare)."""
        if int.from_bytes(bytes(mv[4:8]), "little") == 1:
            return mv
        return memoryview(self.tensor.cpu().numpy()).cast("B")


def regions_from_header(t: torch.Tensor) -> list:
    """The GT blocks of a packed bundle (``requests.range_bundle_pack``) from
    its header words: [count, len_i...] then per list 'RPR1', n, u, l, S,
    offsets, cols, commitments, challenge, zr, D, zphi, zv, V, A (A last).
    A few small host reads (the ledger thread); a layout that does not add up
    yields no regions (the payload is stored raw)."""
    W = t.numel()
    if W < 2:
        return []
    k = int(t[0])
    if k < 1 or 1 + k > W:
        return []
    lens = t[1: 1 + k].cpu().tolist()
    pos, regions = 1 + k, []
    for ln in lens:
        if ln < 5 or pos + ln > W:
            return []
        magic, n, u, l, S = t[pos: pos + 5].cpu().tolist()
        if magic != 0x52505231:
            return []
        if n > 0 and not (u == 0 and l == 0):
            m = n * S * l
            off = pos + 5 + 3 * n + 48 * n + 40 * n + 8 * n * l + 8 * m + 32 * m
            if off + 96 * m != pos + ln:
                return []
            if m:
                regions.append((off, m))
        pos += ln
    return regions if pos == W else []


def regions_from_shape(words: int, S: int, l: int) -> list | None:
    """The GT block of a one-list bundle of ``words`` int32 words whose proofs
    have S servers and l digits (the query's shape): 2 + 5 + n (91 + 8 l +
    136 S l) words for n proofs.  No device read; a wrong guess only costs the
    compact form (its elements fail the round-trip check)."""
    per = 91 + 8 * l + 136 * S * l
    if S < 1 or l < 1 or words < 7 + per or (words - 7) % per:
        return None
    n = (words - 7) // per
    m = n * S * l
    return [(words - 96 * m, m)]


def prepare(req, shape: tuple | None = None) -> Pending | None:
    """A ``Pending`` for a range request on the GPU: the GT blocks from the
    VN's decoded views into its signed tensor when it has them, else from the
    query's proof shape (S, l) when given, else from the bundle header at write
    time; None when the payload cannot take the form."""
    t, lists = req.tensor, req.decoded
    if t is None or t.dtype != torch.int32 or not t.is_contiguous():
        return None
    if not isinstance(lists, list) or not lists:
        return Pending(t, regions_from_shape(t.numel(), *shape) if shape else None)
    base = t.data_ptr()
    end = base + 4 * t.numel()
    regions = []
    for r in lists:
        A = getattr(r, "A", None)
        if A is None or A.numel() == 0:
            continue
        if not A.is_contiguous() or A.dtype != torch.int32 or not (base <= A.data_ptr() < end):
            return None
        regions.append(((A.data_ptr() - base) // 4, A.shape[0]))
    if not regions:
        return None
    regions.sort()
    return Pending(t, regions)


def decompress_bytes(b, device=None) -> bytes:
    """The signed payload bytes of a compressed blob (GPU when there is one)."""
    if not is_compressed(b):
        raise ValueError("not a valid compressed range payload")
    w = np.frombuffer(bytes(b), dtype=np.int32)
    total = int(w[2:4].view(np.int64)[0])
    k = int(w[4])
    regs = w[_HEAD: _HEAD + 4 * k].view(np.int64).reshape(k, 2) if k else np.zeros((0, 2), np.int64)
    body = w[_HEAD + 4 * k:]
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    out = torch.empty((total,), dtype=torch.int32, device=device)
    src = torch.from_numpy(body.copy()).to(device)
    pos = bp = 0
    for off, m in regs.tolist():
        n_raw = off - pos
        out[pos:off].copy_(src[bp: bp + n_raw])
        bp += n_raw
        nt.gt_t2_decompress(src[bp: bp + 48 * m].view(m, 48), out=out[off: off + 96 * m].view(m, 96))
        bp += 48 * m
        pos = off + 96 * m
    out[pos:].copy_(src[bp:])
    return out.cpu().numpy().tobytes()
