"""Payload digests for signed proof envelopes.

Reference: lib/proof/structs_proofs.go — every ``New*ProofRequest`` marshals
its proof and Schnorr-signs the bytes (:117, :143, ...); ``VerifyProofSignature``
re-checks them (:498-505).  A range-proof bundle of a wide query is tens of MB
(per value ``256 + 32 l + 544 S l`` B), so the digest that is
signed is a chunked SHA-256 whose slices hash in parallel where the bytes
live (HBM on a GPU, dx_sha256_chunks):

    digest(b) = SHA-256("DXTH1" || le64(len b) || le64(CHUNK) || H(s_0) || ... || H(s_k-1))

with s_i the CHUNK-byte slices of b (the last may be short; an empty payload
has one empty slice).  ``digest_bytes`` (hashlib) and ``digest_tensor`` (HIP
kernel over a tensor's raw bytes) are bit-identical; tests pin that.
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np
import torch

from .. import native as nt

CHUNK = 4096
_TAG = b"DXTH1"


def _finish(nbytes: int, slice_digests: bytes) -> bytes:
    h = hashlib.sha256()
    h.update(_TAG + struct.pack("<QQ", nbytes, CHUNK))
    h.update(slice_digests)
    return h.digest()


def digest_bytes(b: bytes) -> bytes:
    mv = memoryview(b)
    n = len(mv)
    parts = [hashlib.sha256(mv[o: o + CHUNK]).digest() for o in range(0, n, CHUNK)] or [hashlib.sha256(b"").digest()]
    return _finish(n, b"".join(parts))


def digest_tensor(t: torch.Tensor) -> bytes:
    """Digest of the raw (little-endian) bytes of a contiguous tensor."""
    t = t.contiguous()
    words = nt.sha256_chunks(t, CHUNK)
    be = words.cpu().numpy().view(np.uint32).astype(">u4").tobytes()
    return _finish(t.numel() * t.element_size(), be)


def digest_rows(t: torch.Tensor) -> list:
    """``digest_tensor`` of every row of a contiguous 2-D tensor, in one launch
    and one device-to-host copy (the envelopes of a batch of DPs)."""
    t = t.contiguous()
    words = nt.sha256_rows(t, CHUNK)
    be = words.cpu().numpy().view(np.uint32).astype(">u4")
    row_bytes = t.shape[1] * t.element_size()
    return [_finish(row_bytes, be[r].tobytes()) for r in range(t.shape[0])]


def digest_many(tensors: list, flags: list | None = None):
    """``digest_tensor`` of many tensors of one device: one segmented launch
    and ONE device-to-host copy for all of them (a VN inbox's envelopes).
    ``flags``: device bools (validity checks of the same payloads) read back
    in that same copy -> (digests, [bool]) instead of the digests alone."""
    if not tensors:
        return ([], [bool(f) for f in flags]) if flags is not None else []
    dev = tensors[0].device
    same = all(t.device == dev for t in tensors)
    if not same:
        dg = [digest_tensor(t) for t in tensors]
        return (dg, [bool(f) for f in flags]) if flags is not None else dg
    parts = nt.sha256_segments(tensors, CHUNK)
    nf = len(flags) if flags else 0
    if nf:
        parts_f = parts + [torch.stack([f.reshape(()).to(dev) for f in flags]).to(parts[0].dtype).reshape(1, -1)]
    else:
        parts_f = parts
    flat = torch.cat([p.reshape(-1) for p in parts_f]) if len(parts_f) > 1 else parts_f[0].reshape(-1)
    host = flat.cpu().numpy()
    be = host.view(np.uint32).astype(">u4")
    out, o = [], 0
    for t, p in zip(tensors, parts):
        k = p.numel()
        out.append(_finish(t.numel() * t.element_size(), be[o: o + k].tobytes()))
        o += k
    if flags is None:
        return out
    return out, [bool(v) for v in host[o: o + nf]]
