"""Compact ledger form of range-proof payloads.

A VN stores every signed range bundle it received (storeProof,
proof_collection_protocol.go:318-331; bbolt keeps them all).  ~68% of a
bundle is GT elements -- the A_j commitments, 384 bytes each -- and a GT
element is unitary, so the ledger keeps each as its torus (T2) image c =
(1 + g) / h, 192 bytes (``native.gt_t2_compress``, csrc/kernels/dx_gt_t2.hip):
so fewer bytes to copy off the GPU and fdatasync per query (verdict r4 weak
#4: the W = 8 ledger is disk-bound).

Reading a value back rebuilds the signed payload bit for bit
(``decompress_bytes``; ``ledger.store.Store`` does it for every blob
its writer tagged compact: ``Pending.compact`` after ``finish``), so
GetProofs, digests and audits see exactly what was signed.  A list whose
GT elements do not all round-trip exactly (non-canonical limbs, not unitary:
a malformed or malicious proof) makes the whole bundle fall back to the raw
bytes.

The V_j (G2 points, 23% of a bundle) are kept as x plus one flag word (y's
parity, infinity; ``native.g2_x_compress``): 32 -> 17 words each.  Together
a query's ~567 MB of range payloads become ~313 MB.

Blob layout (int32 words): MAGIC, ok flag (written on the device: 1 when
every element round-trips), raw payload words (int64), region count, then
(word offset int64, element count int64, kind) per region -- kind 0: GT block
(96 -> 48 words per element), 1: G2 block (32 -> 17: x block, then flags) --
then the payload with each region replaced by its compact image.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import native as nt

MAGIC = 0x32435052  # b"RPC2" little-endian
_HEAD = 5
_RW = 5  # header words per region
_GT, _G2 = 0, 1
_FULL = {_GT: 96, _G2: 32}
_SMALL = {_GT: 48, _G2: 17}


def _regions(b, k: int) -> np.ndarray:
    return np.frombuffer(bytes(b[4 * _HEAD: 4 * (_HEAD + _RW * k)]), dtype=np.int32).reshape(k, _RW)


def is_compressed(b) -> bool:
    """A blob in this layout: the magic, the ok flag and a header whose sizes
    account for every byte (a stored payload of another kind that happens to
    start with the magic is not mistaken for one)."""
    if len(b) < 4 * _HEAD or len(b) % 4 or int.from_bytes(bytes(b[:4]), "little") != MAGIC:
        return False
    w = np.frombuffer(bytes(b[:4 * _HEAD]), dtype=np.int32)
    k = int(w[4])
    if int(w[1]) != 1 or k < 1 or 4 * (_HEAD + _RW * k) > len(b):
        return False
    total = int(w[2:4].view(np.int64)[0])
    r = _regions(b, k)
    if not np.isin(r[:, 4], (_GT, _G2)).all():
        return False
    m = r[:, 2:4].copy().view(np.int64).reshape(-1)
    saved = sum(int(mi) * (_FULL[int(kd)] - _SMALL[int(kd)]) for mi, kd in zip(m, r[:, 4]))
    return len(b) // 4 == _HEAD + _RW * k + total - saved


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
        self.compact = False  # set by ``finish``: the stored bytes are the compact image

    def produce(self, stream):
        with torch.cuda.stream(stream):
            if self.regions is None:
                self.regions = regions_from_header(self.tensor)
            if not self.regions:
                self.compact = False
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
        for off, m, kind in self.regions:
            head += list(np.array([off, m], dtype=np.int64).view(np.int32)) + [kind]
        n_img = len(head) + t.numel() - sum(m * (_FULL[kd] - _SMALL[kd]) for _, m, kd in self.regions)
        img = torch.empty((n_img,), dtype=torch.int32, device=dev)
        hdr = torch.tensor(head, dtype=torch.int32)
        if dev.type == "cuda":
            hdr = hdr.pin_memory().to(dev, non_blocking=True)
        pairs, oks, pos, q = [(hdr, img[:len(head)])], [], 0, len(head)
        for off, m, kind in self.regions:
            pairs.append((t[pos:off], img[q: q + off - pos]))
            q += off - pos
            src = t[off: off + _FULL[kind] * m].view(m, _FULL[kind])
            if kind == _GT:
                oks.append(nt.gt_t2_compress(src, out=img[q: q + 48 * m].view(m, 48)))
            else:
                oks.append(nt.g2_x_compress(src, x_out=img[q: q + 16 * m].view(m, 16),
                                            flag_out=img[q + 16 * m: q + 17 * m])[2])
            q += _SMALL[kind] * m
            pos = off + _FULL[kind] * m
        pairs.append((t[pos:], img[q:]))
        nt.batched_copy(pairs)  # the header and every raw segment in one launch
        okall = torch.cat(oks).all() if len(oks) > 1 else oks[0].all()
        img[1:2].copy_(okall.to(torch.int32).view(1))
        self.image = img
        return img.view(torch.uint8)

    def finish(self, mv: memoryview):
        """The bytes to store: the compressed image when every element
        round-trips, else the raw payload (a synchronous copy, rare)."""
        self.compact = int.from_bytes(bytes(mv[4:8]), "little") == 1
        if self.compact:
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
                regions += [(off - 32 * m, m, _G2), (off, m, _GT)]
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
    return [(words - 128 * m, m, _G2), (words - 96 * m, m, _GT)] if m else None


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
        for F, kind in ((getattr(r, "V", None), _G2), (getattr(r, "A", None), _GT)):
            if F is None or F.numel() == 0:
                continue
            if not F.is_contiguous() or F.dtype != torch.int32 or not (base <= F.data_ptr() < end):
                return None
            regions.append(((F.data_ptr() - base) // 4, F.shape[0], kind))
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
    r = _regions(b, k)
    body = w[_HEAD + _RW * k:]
    if device is None:
        device = "cuda" if torch.cuda.is_available() else "cpu"
    out = torch.empty((total,), dtype=torch.int32, device=device)
    src = torch.from_numpy(body.copy()).to(device)
    pos = bp = 0
    for row in r:
        off, m = (int(v) for v in row[:4].copy().view(np.int64))
        kind = int(row[4])
        out[pos:off].copy_(src[bp: bp + off - pos])
        bp += off - pos
        dst = out[off: off + _FULL[kind] * m].view(m, _FULL[kind])
        if kind == _GT:
            nt.gt_t2_decompress(src[bp: bp + 48 * m].view(m, 48), out=dst)
        else:
            _, bad = nt.g2_x_decompress(src[bp: bp + 16 * m].view(m, 16), src[bp + 16 * m: bp + 17 * m], out=dst)
            if bool(bad.any()):
                raise ValueError("compressed range payload holds an x with no G2 point")
        bp += _SMALL[kind] * m
        pos = off + _FULL[kind] * m
    out[pos:].copy_(src[bp:])
    return out.cpu().numpy().tobytes()
