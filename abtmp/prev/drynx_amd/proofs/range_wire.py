"""The reference's wire/ledger layout of range-proof lists.

Reference: a DP's range-proof request carries ``network.Marshal(&proofBytes)``
with ``proofBytes = RangeProofList.ToBytes()`` (lib/proof/structs_proofs.go:
110-131), and every VN stores exactly those bytes in its bbolt bucket
``surveyID/range`` (protocols/proof_collection_protocol.go:318-331), which
``GetProofs`` serves (services/service_skipchain.go:240-320).  Per proof
(lib/range/range_proof.go:72-155):

  RangeProofBytes{Commit: K||C (2 x 64 B),
                  RP: RangeProofDataBytes{Challenge 32 B, Zr 32 B, D 64 B,
                      Zv[i] = l scalars (32 l B) per server i, Zphi = l scalars,
                      V[i] = l G2 points (128 l B), A[i] = l GT values (384 l B)}}

This framework moves proofs between GPUs as raw Montgomery limbs
(``RangeProofList.pack``); this module turns a bundle into the reference
layout (canonical big-endian kyber encodings, dedis/protobuf framing, onet
type-id envelope) for the ledger and ``GetProofs``, and back for verification.
The framing of a list whose proofs share (u, l, S) is a constant template, so
it is assembled with numpy block copies instead of per-field Python encoding.
Parity of the dedis/protobuf framing and of the type id is re-derived, not
pinned against the Go encoder (drynx_amd/wire/onet.py).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import native as nt
from ..crypto import bn254 as bn
from ..crypto.elgamal import CipherVector
from ..wire import onet
from ..wire import protobuf as pb
from . import range_proof as rp

LIST_TYPE = "libdrynxrange.RangeProofListBytes"


def _uvarint(n: int) -> bytes:
    out = bytearray()
    pb.put_uvarint(out, n)
    return bytes(out)


def _hdr(num: int, length: int) -> bytes:
    return _uvarint((num << 3) | 2) + _uvarint(length)


def _block(h: bytes, n: int, *shape, device="cpu") -> torch.Tensor:
    return torch.frombuffer(bytearray(h), dtype=torch.uint8).to(device).expand(n, *shape, len(h))


def _be(t: torch.Tensor, mont: bool) -> torch.Tensor:
    """8-limb rows -> canonical 32-byte big-endian rows (on the tensor's device):
    out of Montgomery form for field elements, then the little-endian limb
    string reversed."""
    rows = t.reshape(-1, 8).contiguous()
    if mont:
        rows = nt.fp_from_mont(rows)
    return rows.view(torch.uint8).view(-1, 32).flip(1)


def list_fields(r: rp.RangeProofList) -> dict:
    """Canonical kyber encodings of a list's fields as uint8 tensors on the
    list's device (G1 = x||y, G2 = x.c1||x.c0||y.c1||y.c0, GT = the 12 Fp
    coefficients in reverse tower order, scalars 32 B big-endian)."""
    n, l, S = len(r), r.l, r.S
    both = torch.stack([r.commit.K, r.commit.C], dim=1).reshape(-1, 24)
    f = {"commit": _be(nt.g1_to_affine(both), True).reshape(n, 128)}
    if r.has_rp and n:
        f["challenge"] = _be(r.challenge, False).reshape(n, 32)
        f["zr"] = _be(r.zr, False).reshape(n, 32)
        f["D"] = _be(nt.g1_to_affine(r.D.contiguous()), True).reshape(n, 64)
        f["zv"] = _be(r.zv, False).reshape(n, S, 32 * l)
        f["zphi"] = _be(r.zphi, False).reshape(n, 32 * l)
        f["V"] = _be(r.V, True).reshape(-1, 2, 32).flip(1).reshape(n, S, 128 * l)      # (imag, real) per Fp2
        f["A"] = _be(r.A, True).reshape(-1, 12, 32).flip(1).reshape(n, S, 384 * l)     # reversed coefficients
    return f


def _proof_messages(r: rp.RangeProofList, f: dict) -> torch.Tensor:
    """[n, k] uint8: every proof's RangeProofBytes message with its field-1
    header of the Data slice (all proofs of a list have the same length)."""
    n, l, S = len(r), r.l, r.S
    dev = f["commit"].device
    B = lambda h, *shape: _block(h, n, *shape, device=dev)  # noqa: E731
    commit = [B(_hdr(1, 128)), f["commit"]]
    if not (r.has_rp and n):
        body = torch.cat(commit + [B(_hdr(2, 0))], dim=1)
    else:
        rp_parts = [B(_hdr(1, 32)), f["challenge"], B(_hdr(2, 32)), f["zr"], B(_hdr(3, 64)), f["D"],
                    torch.cat([B(_hdr(4, 32 * l), S), f["zv"]], dim=2).reshape(n, -1),
                    B(_hdr(5, 32 * l)), f["zphi"],
                    torch.cat([B(_hdr(6, 128 * l), S), f["V"]], dim=2).reshape(n, -1),
                    torch.cat([B(_hdr(7, 384 * l), S), f["A"]], dim=2).reshape(n, -1)]
        rp_len = sum(p.shape[1] for p in rp_parts)
        body = torch.cat(commit + [B(_hdr(2, rp_len))] + rp_parts, dim=1)
    return torch.cat([B(_hdr(1, body.shape[1])), body], dim=1)


def is_raw_bundle(b: bytes) -> bool:
    """A raw-limb range bundle (``requests.range_bundle_pack``: [count, sizes...,
    'RPR1' list...]) rather than reference-layout bytes."""
    if len(b) < 12 or len(b) % 4:
        return False
    k = int.from_bytes(b[:4], "little")
    if k < 1 or 4 * (2 + k) > len(b):
        return False
    return int.from_bytes(b[4 * (1 + k): 4 * (2 + k)], "little") == 0x52505231


def encode_bundle(rpls: list, fields: list | None = None) -> bytes:
    """network.Marshal(&RangeProofListBytes) of all proofs of a DP's bundle,
    in output-column order.  Assembled on the proofs' device; one copy of the
    finished bytes to the host."""
    fields = fields if fields is not None else [list_fields(r) for r in rpls]
    msgs = [_proof_messages(r, f) for r, f in zip(rpls, fields)]
    cols = [c for r in rpls for c in r.cols]
    if not msgs:
        return onet.message_type_id(LIST_TYPE)
    allm = msgs[0] if len(msgs) == 1 else None
    if allm is None or cols != sorted(cols):
        rows = [m[i] for m in msgs for i in range(m.shape[0])]
        inner = b"".join(rows[i].cpu().numpy().tobytes() for i in sorted(range(len(rows)), key=lambda i: cols[i]))
    else:
        inner = allm.contiguous().cpu().numpy().tobytes()
    return onet.message_type_id(LIST_TYPE) + (_hdr(1, len(inner)) + inner if inner else b"")


def decode_bundle(b: bytes, ranges, device="cpu") -> list:
    """Parse reference-layout bytes back into RangeProofLists (one per (u, l)
    group, proofs in column order).  The layout carries no (u, l): like
    RangeProofVerification they come from the query's ``Ranges`` (column p of
    the list <-> output p)."""
    name, d = onet.unmarshal(b)
    if name != LIST_TYPE:
        raise ValueError(f"expected {LIST_TYPE}, got {name}")
    proofs = d["Data"]
    groups: dict = {}
    for p, pr in enumerate(proofs):
        rg = ranges[p] if ranges is not None and p < len(ranges) else (0, 0)
        u, l = int(rg[0]), int(rg[1])
        off = int(rg[2]) if len(rg) > 2 else 0
        groups.setdefault((u, l), []).append((p, off, pr))
    out = []
    for (u, l), items in groups.items():
        cols = [p for p, _, _ in items]
        offs = [o for _, o, _ in items]
        commit = CipherVector.from_bytes(b"".join(pr["Commit"] for _, _, pr in items), device)
        has_rp = not (u == 0 and l == 0)
        if not has_rp:
            out.append(rp.RangeProofList(u, l, 0, offs, cols, commit))
            continue
        S = len(items[0][2]["RP"]["V"])
        r = rp.RangeProofList(u, l, S, offs, cols, commit)
        rps = [pr["RP"] for _, _, pr in items]
        cat = lambda key: b"".join(x[key] for x in rps)  # noqa: E731
        catn = lambda key: b"".join(b"".join(x[key]) for x in rps)  # noqa: E731
        for x in rps:
            if len(x["V"]) != S or len(x["A"]) != S or len(x["Zv"]) != S or len(x["Zphi"]) != 32 * l \
                    or any(len(v) != 128 * l for v in x["V"]) or any(len(a) != 384 * l for a in x["A"]) \
                    or any(len(z) != 32 * l for z in x["Zv"]):
                raise ValueError("range proof fields do not match (u, l, S)")
        r.challenge = _scalars(cat("Challenge"), device)
        r.zr = _scalars(cat("Zr"), device)
        r.D = nt.g1_from_affine(bn.g1_aff_from_bytes(cat("D"), device))
        r.zv = _scalars(catn("Zv"), device)
        r.zphi = _scalars(cat("Zphi"), device)
        r.V = bn.g2_aff_from_bytes(catn("V"), device)
        r.A = bn.gt_from_bytes(catn("A"), device)
        out.append(r)
    return out


def _scalars(b: bytes, device) -> torch.Tensor:
    """Scalars as transmitted (no reduction: a non-canonical value must fail
    the verifier's decode check, as kyber's UnmarshalBinary would refuse it)."""
    arr = np.frombuffer(b, dtype=np.uint8).reshape(-1, 32)
    limbs = arr.view(">u4").astype("<u4")[:, ::-1].copy()
    return bn.to_tensor(limbs, device)
