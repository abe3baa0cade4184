"""Σ-protocol proofs on device tensors: Schnorr signatures, obfuscation DLEQ
(Chaum–Pedersen) and key-switching proofs.

Reference:
  * Schnorr envelopes: kyber sign/schnorr, lib/proof/structs_proofs.go:117,
    :498-505 (signature = R (64 B) || s (32 B)).
  * Obfuscation: lib/obfuscation/obfuscation_proof.go:36-114 — prove knowledge
    of s with Co.K = s*C.K and Co.C = s*C.C (kyber proof.Rep/And + HashProve).
  * Key switching: unlynx KeySwitchListProofCreation/Verification (external,
    used at services/service.go:566-616) — each CN share (v B, v Q - x K) is
    consistent with its public key X = x B.

Wire/transcript deviation (documented): kyber's proof framework hashes a
blake2xb transcript per element; here one SHA-256 Fiat–Shamir challenge binds
the whole list (context string, all statement points, all commitments) and
each element gets its own response.  The verification equations are the
standard ones and run batched on the device.
"""
from __future__ import annotations

import hashlib
import math
import os
from dataclasses import dataclass

import numpy as np
import torch

from .. import native as nt
from ..crypto import bn254 as bn
from ..crypto import oracle as O
from ..crypto.elgamal import CipherVector
from ..utils import timers


def _aff_bytes(jac: torch.Tensor) -> bytes:
    if jac.numel() == 0:
        return b""
    return bn.g1_aff_to_bytes(nt.g1_to_affine(jac.contiguous().view(-1, 24))).tobytes()


def pts_be(jac: torch.Tensor) -> torch.Tensor:
    """[m, 24] Jacobian -> [m, 64] uint8 kyber encodings (affine x || y, big
    endian, infinity = zeros) computed where the points live (HBM on a GPU)."""
    aff = nt.g1_to_affine(jac.contiguous().view(-1, 24))
    xy = nt.fp_from_mont(aff.reshape(-1, 8))
    return xy.view(torch.uint8).view(-1, 32).flip(1).reshape(-1, 64)


def points_digests(groups: list, flags: list | None = None):
    """Per group (a list of Jacobian point tensors / CipherVectors) the chunked
    digest (crypto/digest.py) of the kyber encodings of all its points, in
    order: ONE normalisation launch, one encoding pass, one segmented SHA-256
    launch and ONE device-to-host copy for every group together (a
    transcript is 3-6 vectors of thousands of points).  ``flags``: device
    bools read back in the same copy -> (digests, [bool])."""
    from ..crypto import digest as dg

    flat, sizes = [], []
    for grp in groups:
        m = 0
        for p in grp:
            ts = (p.K, p.C) if isinstance(p, CipherVector) else (p,)
            for t in ts:
                t = t.contiguous().view(-1, 24)
                flat.append(t)
                m += t.shape[0]
        sizes.append(m)
    if not flat:
        out = [dg.digest_bytes(b"") for _ in groups]
        return (out, [bool(f) for f in flags]) if flags is not None else out
    be = pts_be(torch.cat(flat) if len(flat) > 1 else flat[0])
    views, o = [], 0
    for m in sizes:
        views.append(be[o: o + m])
        o += m
    return dg.digest_many(views, flags)


def fs_hash(context: str, raw: tuple, pts_digest: bytes) -> int:
    """Fiat-Shamir challenge: SHA-256(context || raw parts || digest of the
    point encodings) mod r."""
    h = hashlib.sha256(context.encode())
    for r in raw:
        h.update(r)
    h.update(pts_digest)
    return int.from_bytes(h.digest(), "big") % O.R


def fs_challenge(context: str, *parts) -> int:
    """Challenge of one transcript: raw (bytes) parts in order, then the digest
    of every point part (tensors / CipherVectors) in order."""
    return fs_challenges([(context, parts)])[0]


def fs_challenges(specs) -> list:
    """Challenges of several transcripts [(context, parts), ...]; the point
    parts of all of them are encoded and digested on the device together."""
    groups, raws = [], []
    for context, parts in specs:
        pts = [p for p in parts if isinstance(p, (torch.Tensor, CipherVector))]
        raw = tuple(p if isinstance(p, (bytes, bytearray)) else str(p).encode()
                    for p in parts if not isinstance(p, (torch.Tensor, CipherVector)))
        groups.append(pts)
        raws.append((context, raw))
    dgs = points_digests(groups)
    return [fs_hash(ctx, raw, d) for (ctx, raw), d in zip(raws, dgs)]


def _rand64(n: int, device, coins=None) -> torch.Tensor:
    """Random nonzero 64-bit batch weights, unknown to provers: the verifier's
    own ``coins`` (crypto/coins.py) or fresh device CSPRNG output."""
    if coins is not None:
        return coins.bits(n, device, 64, odd=True)
    r = bn.random_scalars(n, device)
    r[:, 2:] = 0
    r[:, 0] |= 1
    return r


def _points_ok(tensors: list) -> torch.Tensor:
    """Device bool: every row of every [m, 24] Jacobian tensor has canonical
    limbs and is on the curve (a received raw payload is untrusted)."""
    flat = torch.cat([t.reshape(-1, 24) for t in tensors]) if len(tensors) > 1 else tensors[0].reshape(-1, 24)
    if flat.shape[0] == 0:
        return torch.ones((), dtype=torch.bool, device=flat.device)
    return nt.limbs_canonical(flat.reshape(-1, 8)).bool().all() & nt.g1j_on_curve(flat).bool().all()


def _scalars_ok(t: torch.Tensor) -> torch.Tensor:
    if t.numel() == 0:
        return torch.ones((), dtype=torch.bool, device=t.device)
    return nt.limbs_canonical(t.reshape(-1, 8), fr=True).bool().all()


def _digest_checked(proofs: list, groups_of) -> None:
    """Decoded data of received proofs, computed once per proof and shared by
    co-hosted VNs: the transcript's point digest and the host verdict of the
    payload's lazy well-formedness flag (every point row canonical and on the
    curve, every response scalar canonical), read back in the digest's copy."""
    todo = [pr for pr in proofs if not pr.pts_digest]
    if not todo:
        return
    fl = [pr for pr in todo if isinstance(pr.wellformed, torch.Tensor)]
    dgs, oks = points_digests([groups_of(pr) for pr in todo], [pr.wellformed for pr in fl])
    for pr, d in zip(todo, dgs):
        pr.pts_digest = d
    for pr, ok in zip(fl, oks):
        pr.wellformed = bool(ok)


def _head_words(tensors: list, width: int) -> list:
    """The first ``width`` words of every packed payload, ONE device-to-host copy."""
    if not tensors:
        return []
    return torch.nn.utils.rnn.pad_sequence([t[:width] for t in tensors], batch_first=True).cpu().tolist()


def _msm_is_zero(points: list, scalars: list) -> bool:
    """sum_i k_i P_i == O over the concatenated lists (one Pippenger MSM)."""
    res = nt.g1_msm(torch.cat(points).contiguous(), torch.cat(scalars).contiguous())
    return not bool(res[0, 16:24].any())


def _sc(vals, device):
    return bn.scalars_tensor(vals, device)


def _first(n: int, threshold: float) -> int:
    return int(math.ceil(threshold * n))


# ----------------------------------------------------------------------------- Schnorr
def schnorr_sign(secret: int, msg: bytes) -> bytes:
    k = O.random_scalar()
    R = bn.g1_mul_point(k)
    X = bn.g1_mul_point(secret)
    e = int.from_bytes(hashlib.sha256(O.g1_to_bytes(R) + O.g1_to_bytes(X) + msg).digest(), "big") % O.R
    s = (k + e * secret) % O.R
    return O.g1_to_bytes(R) + O.scalar_to_bytes(s)


def schnorr_sign_batch(secrets: list, msgs: list, device="cpu") -> list:
    """``schnorr_sign`` of many (secret, message) pairs (the envelopes of every
    DP of a rank): the nonce points R_i = k_i B and the public keys X_i = x_i B
    come from one fixed-base launch, their encodings from one conversion; the
    challenges and responses are host hashing and scalar arithmetic."""
    n = len(secrets)
    if n == 0:
        return []
    ks = [O.random_scalar() for _ in range(n)]
    # signing stays on the device even for a handful of envelopes: host
    # fixed-base products compete with the query's host threads (same-box
    # A/B, profiles/r4/ab_bisect.txt: host signing of the per-CN proofs cost
    # ~9 ms of a ~200 ms query); DRYNX_SIGN_DEVICE_MIN=k signs below k on the host
    dev = torch.device(device) if n >= int(os.environ.get("DRYNX_SIGN_DEVICE_MIN", "1")) \
        else torch.device("cpu")
    pts = nt.g1_fb_mul(bn.base_table(dev), bn.scalars_tensor(ks + [int(x) for x in secrets], dev))
    enc = bn.g1_aff_to_bytes(nt.g1_to_affine(pts))
    out = []
    for i in range(n):
        Rb, Xb = enc[i].tobytes(), enc[n + i].tobytes()
        x = int(secrets[i]) % O.R
        e = int.from_bytes(hashlib.sha256(Rb + Xb + msgs[i]).digest(), "big") % O.R
        out.append(Rb + O.scalar_to_bytes((ks[i] + e * x) % O.R))
    return out


def schnorr_verify(public, msg: bytes, sig: bytes) -> bool:
    if len(sig) != 96 or public is None:
        return False
    try:
        R = O.g1_from_bytes(sig[:64])
    except ValueError:
        return False
    s = int.from_bytes(sig[64:], "big")
    # same acceptance rule as schnorr_verify_batch: R at infinity or a
    # non-canonical s is rejected, whatever the size of the VN's inbox
    if R is None or s >= O.R:
        return False
    e = int.from_bytes(hashlib.sha256(sig[:64] + O.g1_to_bytes(public) + msg).digest(), "big") % O.R
    lhs = bn.g1_mul_point(s)
    return lhs == O.g1_add(R, bn.g1_mul_point(e, public))


_SIG_DEVICE_MIN = 256


def schnorr_verify_batch(items: list, device="cpu") -> list:
    """schnorr_verify over many (public, msg, sig) at once: s_i B by one
    fixed-base launch, e_i X_i by one variable-base launch, one addition and
    one equality launch.  A VN inbox holds one envelope per DP and per CN
    proof; one host scalar multiplication per envelope made 6000-DP surveys
    host-bound (structs_proofs.go:498-505 verifies each in its own goroutine)."""
    out = [False] * len(items)
    idx, R, X, s, e = [], [], [], [], []
    for i, (public, msg, sig) in enumerate(items):
        if len(sig) != 96 or public is None:
            continue
        try:
            Ri = O.g1_from_bytes(sig[:64])
        except ValueError:
            continue
        si = int.from_bytes(sig[64:], "big")
        if Ri is None or si >= O.R:
            continue
        idx.append(i)
        R.append(Ri)
        X.append(public)
        s.append(si)
        e.append(int.from_bytes(hashlib.sha256(sig[:64] + O.g1_to_bytes(public) + msg).digest(), "big") % O.R)
    if not idx:
        return out
    # a VN inbox of a few dozen envelopes verifies on the host pool: a GPU
    # launch chain plus its read-back costs more than the products themselves
    dev = torch.device(device) if len(idx) >= int(os.environ.get("DRYNX_SIG_DEVICE_MIN", _SIG_DEVICE_MIN)) \
        else torch.device("cpu")
    with timers.span(f"sig.products[{len(idx)}]"):
        lhs = nt.g1_fb_mul(bn.base_table(dev), _sc(s, dev))
        rhs = nt.g1_add(bn.g1_jac_tensor(R, dev), nt.g1_mul(bn.g1_jac_tensor(X, dev), _sc(e, dev)))
        ok = nt.g1_eq(lhs, rhs).cpu().tolist()
    for i, v in zip(idx, ok):
        out[i] = bool(v)
    return out


# Fiat-Shamir context strings carry the transcript version: v2 = SHA-256 over
# context || raw parts || chunked digest of the point encodings (crypto/digest.py).
# Proofs made with another transcript layout fail the challenge check.
OBF_CONTEXT = "proofTest/obfuscation/v2"
KS_CONTEXT = "proofTest/keyswitch/v2"

# ----------------------------------------------------------------------------- obfuscation (DLEQ)
OBF_MAGIC = 0x4F425031  # "OBP1"
_OBF_HEAD = 10          # magic, n, c (8 limbs)


@dataclass
class ObfuscationProof:
    C: CipherVector     # before
    Co: CipherVector    # after (s_i * C_i)
    T: CipherVector     # commitments (a_i K_i, a_i C_i)
    c: int
    z: torch.Tensor     # [n, 8]
    pts_digest: bytes = b""  # decoded data: digest of the transcript's point encodings
    # received payloads: device bool (every point canonical + on the curve, z
    # canonical), a host bool once read back; None = built locally / decoded from bytes
    wellformed: object = None

    # reference-style export (kyber affine encodings): ledger / GetProofs
    def to_bytes(self) -> bytes:
        return b"".join([len(self.C).to_bytes(8, "little"), self.C.to_bytes(), self.Co.to_bytes(), self.T.to_bytes(),
                         O.scalar_to_bytes(self.c), bn.scalars_to_bytes(self.z).tobytes()])

    @staticmethod
    def from_bytes(b: bytes, device="cpu") -> "ObfuscationProof":
        n = int.from_bytes(b[:8], "little")
        if len(b) != 8 + 3 * 128 * n + 32 + 32 * n:
            raise ValueError("obfuscation proof length does not match its header")
        o = 8
        cvs = []
        for _ in range(3):
            cvs.append(CipherVector.from_bytes(b[o: o + 128 * n], device))
            o += 128 * n
        c = int.from_bytes(b[o: o + 32], "big")
        o += 32
        z = bn.scalars_from_bytes(np.frombuffer(b[o: o + 32 * n], dtype=np.uint8), device)
        return ObfuscationProof(cvs[0], cvs[1], cvs[2], c, z)

    # intra-cluster payload: raw Montgomery limbs, no host marshalling
    def pack(self) -> torch.Tensor:
        dev = self.C.device
        n = len(self.C)
        head = torch.cat([torch.tensor([OBF_MAGIC, n], dtype=torch.int32),
                          bn.scalars_tensor([self.c], "cpu").reshape(-1)])
        pts = [t.reshape(-1) for cv in (self.C, self.Co, self.T) for t in (cv.K, cv.C)]
        return torch.cat([bn.h2d(head, dev)] + pts + [self.z.reshape(-1)])

    @staticmethod
    def unpack(t: torch.Tensor, head: list | None = None) -> "ObfuscationProof":
        if head is None:
            head = t[:_OBF_HEAD].cpu().tolist()
        if head[0] != OBF_MAGIC or head[1] < 0:
            raise ValueError("not a packed obfuscation proof")
        n = head[1]
        if t.numel() != _OBF_HEAD + 6 * 24 * n + 8 * n:
            raise ValueError("packed obfuscation proof length does not match its header")
        c = bn.scalars_from_tensor(torch.tensor(head[2:10], dtype=torch.int32).view(1, 8))[0]
        o = _OBF_HEAD
        parts = []
        for _ in range(6):
            parts.append(t[o: o + 24 * n].view(n, 24))
            o += 24 * n
        z = t[o: o + 8 * n].view(n, 8)
        if c >= O.R:
            raise ValueError("non-canonical challenge in an obfuscation proof")
        return ObfuscationProof(CipherVector(parts[0], parts[1]), CipherVector(parts[2], parts[3]),
                                CipherVector(parts[4], parts[5]), c, z, wellformed=_points_ok(parts) & _scalars_ok(z))


def obfuscation_list_proof_creation(C: CipherVector, Co: CipherVector, s: torch.Tensor) -> ObfuscationProof:
    """ObfuscationListProofCreation: per element DLEQ log_{K}(Ko) == log_{C}(Co) == s_i."""
    dev = C.device
    a = bn.random_scalars(len(C), dev)
    T = C.mul_scalars(a)
    c = fs_challenge(OBF_CONTEXT, C, Co, T)
    z = nt.fr_arith(nt.FR_ADD, a, nt.fr_arith(nt.FR_MUL, s, _sc([c], dev)))
    return ObfuscationProof(C, Co, T, c, z)


def _obf_fs_ok(proofs: list) -> list:
    """Each proof's Fiat-Shamir check: the challenge recomputed from the
    transcript's point digest (decoded data, computed once per proof), and
    the payload's well-formedness."""
    _digest_checked(proofs, lambda pr: [pr.C, pr.Co, pr.T])
    return [pr.wellformed is not False and fs_hash(OBF_CONTEXT, (), pr.pts_digest) == pr.c for pr in proofs]


def obfuscation_list_proof_verification(pr: ObfuscationProof, threshold: float = 1.0) -> bool:
    """ObfuscationListProofVerification(percent): z K == T1 + c Ko and z C == T2 + c Co
    for the first ceil(threshold * n) elements (reference sampling)."""
    n = len(pr.C)
    k = _first(n, threshold)
    if k == 0:
        return True
    if not _obf_fs_ok([pr])[0]:
        return False
    dev = pr.C.device
    c = _sc([pr.c], dev)
    Cs, Cos, Ts, z = pr.C[:k], pr.Co[:k], pr.T[:k], pr.z[:k].contiguous()
    lhs = Cs.mul_scalars(z)
    rhs = Ts.add(Cos.mul_scalars(c))
    return bool(nt.g1_eq(lhs.K, rhs.K).all()) and bool(nt.g1_eq(lhs.C, rhs.C).all())


# ----------------------------------------------------------------------------- key switching
KS_MAGIC = 0x4B535031   # "KSP1"
_KS_HEAD = 2 + 3 * 16 + 2 * 8  # magic, n, X / Q / T3 affine, c, zb


@dataclass
class KeySwitchProof:
    X: tuple                 # CN public key
    Q: tuple                 # target (querier) public key
    K: torch.Tensor          # [n, 24] original K values
    share: CipherVector      # (v B, v Q - x K)
    T1: torch.Tensor         # a_i B
    T2: torch.Tensor         # a_i Q - b K_i
    T3: bytes                # b B (one point)
    c: int
    za: torch.Tensor         # [n, 8]
    zb: int
    pts_digest: bytes = b""  # decoded data: digest of the transcript's point encodings
    wellformed: object = None  # as ObfuscationProof.wellformed (K, share, T1, T2 rows; za)

    # reference-style export (kyber affine encodings): ledger / GetProofs
    def to_bytes(self) -> bytes:
        n = self.K.shape[0]
        return b"".join([n.to_bytes(8, "little"), O.g1_to_bytes(self.X), O.g1_to_bytes(self.Q), _aff_bytes(self.K),
                         self.share.to_bytes(), _aff_bytes(self.T1), _aff_bytes(self.T2), self.T3,
                         O.scalar_to_bytes(self.c), bn.scalars_to_bytes(self.za).tobytes(),
                         O.scalar_to_bytes(self.zb)])

    @staticmethod
    def from_bytes(b: bytes, device="cpu") -> "KeySwitchProof":
        n = int.from_bytes(b[:8], "little")
        if len(b) != 8 + 128 + 64 * n + 128 * n + 128 * n + 64 + 32 + 32 * n + 32:
            raise ValueError("key-switch proof length does not match its header")
        o = 8
        X = O.g1_from_bytes(b[o: o + 64]); o += 64
        Q = O.g1_from_bytes(b[o: o + 64]); o += 64

        def pts(cnt):
            nonlocal o
            t = nt.g1_from_affine(bn.g1_aff_from_bytes(np.frombuffer(b[o: o + 64 * cnt], dtype=np.uint8), device))
            o += 64 * cnt
            return t
        K = pts(n)
        share = CipherVector.from_bytes(b[o: o + 128 * n], device); o += 128 * n
        T1 = pts(n)
        T2 = pts(n)
        T3 = b[o: o + 64]; o += 64
        c = int.from_bytes(b[o: o + 32], "big"); o += 32
        za = bn.scalars_from_bytes(np.frombuffer(b[o: o + 32 * n], dtype=np.uint8), device); o += 32 * n
        zb = int.from_bytes(b[o: o + 32], "big")
        if c >= O.R or zb >= O.R:
            raise ValueError("non-canonical scalar in a key-switch proof")
        return KeySwitchProof(X, Q, K, share, T1, T2, T3, c, za, zb)

    # intra-cluster payload: raw Montgomery limbs, no host marshalling
    def pack(self) -> torch.Tensor:
        dev = self.K.device
        n = self.K.shape[0]
        head = torch.cat([torch.tensor([KS_MAGIC, n], dtype=torch.int32),
                          bn.g1_aff_tensor([self.X, self.Q, O.g1_from_bytes(self.T3)], "cpu").reshape(-1),
                          bn.scalars_tensor([self.c, self.zb], "cpu").reshape(-1)])
        body = [t.reshape(-1) for t in (self.K, self.share.K, self.share.C, self.T1, self.T2, self.za)]
        return torch.cat([bn.h2d(head, dev)] + body)

    @staticmethod
    def unpack(t: torch.Tensor, head: list | None = None) -> "KeySwitchProof":
        if head is None:
            head = t[:_KS_HEAD].cpu().tolist()
        if head[0] != KS_MAGIC or head[1] < 0:
            raise ValueError("not a packed key-switch proof")
        n = head[1]
        if t.numel() != _KS_HEAD + 5 * 24 * n + 8 * n:
            raise ValueError("packed key-switch proof length does not match its header")
        hp = torch.tensor(head[2:50], dtype=torch.int32).view(3, 16)
        lim = bn.limbs_to_ints(hp.numpy().reshape(-1, 8))
        if any(v >= O.P for v in lim):
            raise ValueError("non-canonical coordinate in a key-switch proof header")
        X, Q, T3 = bn.g1_points_from_aff(hp)
        for pt in (X, Q, T3):
            if not O.g1_on_curve(pt):
                raise ValueError("key-switch proof header point not on the curve")
        c, zb = bn.scalars_from_tensor(torch.tensor(head[50:66], dtype=torch.int32).view(2, 8))
        o = _KS_HEAD
        rows = []
        for _ in range(5):
            rows.append(t[o: o + 24 * n].view(n, 24))
            o += 24 * n
        za = t[o: o + 8 * n].view(n, 8)
        if c >= O.R or zb >= O.R:
            raise ValueError("non-canonical scalar in a key-switch proof header")
        return KeySwitchProof(X, Q, rows[0], CipherVector(rows[1], rows[2]), rows[3], rows[4], O.g1_to_bytes(T3),
                              c, za, zb, wellformed=_points_ok(rows) & _scalars_ok(za))


def unpack_many(kind: str, tensors: list) -> list:
    """Unpack many packed proofs of one kind with ONE header copy; an entry is
    the proof or the exception that rejects it."""
    cls, width = {"keyswitch": (KeySwitchProof, _KS_HEAD), "obfuscation": (ObfuscationProof, _OBF_HEAD)}[kind]
    heads = _head_words(tensors, width)
    out = []
    for t, h in zip(tensors, heads):
        try:
            out.append(cls.unpack(t, h[: min(width, t.numel())] if t.numel() >= width else t.cpu().tolist()))
        except Exception as e:  # noqa: BLE001 -- a malformed payload is a rejected proof
            out.append(e)
    return out


def key_switch_share(x: int, K: torch.Tensor, Q_point, v: torch.Tensor | None = None):
    """One CN's key-switching share: (v_i B, v_i Q - x K_i)."""
    from ..crypto.elgamal import pk_table

    dev = K.device
    n = K.shape[0]
    if v is None:
        v = bn.random_scalars(n, dev)
    tabB = bn.base_table(dev)
    tabQ = pk_table(Q_point, dev).tabP
    xK = nt.g1_mul(K.contiguous(), _sc([x], dev))
    share = CipherVector(nt.g1_fb_mul(tabB, v), nt.g1_add(nt.g1_fb_mul(tabQ, v), xK, subtract=True))
    return share, v


@dataclass
class KeySwitchPending:
    """What a batch of co-located CNs needs to finish their key-switch proofs
    (challenge + responses) off the query's critical path."""
    secrets: list
    publics: list
    Q: tuple
    K: torch.Tensor
    shares: CipherVector
    T1: torch.Tensor
    T2: torch.Tensor
    a: torch.Tensor
    v: torch.Tensor
    bs: list


def key_switch_shares_batch(secrets: list, publics: list, K: torch.Tensor, Q_point, with_proofs: bool):
    """Key-switching shares of several co-located CNs over the same K vector
    in a handful of launches sized (#CNs x n) instead of per CN.  -> (list of
    shares, KeySwitchPending or None): the shares need no host round trip;
    ``finish_keyswitch_proofs`` completes the proofs (one device-to-host copy
    for the challenges of every CN)."""
    from ..crypto.elgamal import pk_table

    dev = K.device
    n, c = K.shape[0], len(secrets)
    tabB = bn.base_table(dev)
    tabQ = pk_table(Q_point, dev).tabP
    Kt = K.repeat(c, 1).contiguous()
    x_rep = torch.cat([_sc([x], dev).expand(n, 8) for x in secrets]).contiguous()
    v = bn.random_scalars(c * n, dev)
    scal = [x_rep]
    bs = None
    if with_proofs:
        bs = [O.random_scalar() for _ in secrets]
        scal.append(torch.cat([_sc([b], dev).expand(n, 8) for b in bs]).contiguous())
    with timers.span("ks.varmul"):
        prods = nt.g1_mul(torch.cat([Kt] * len(scal)).contiguous(), torch.cat(scal).contiguous())
    xK = prods[: c * n].contiguous()
    with timers.span("ks.fixedbase"):
        vB = nt.g1_fb_mul(tabB, v)
        vQ = nt.g1_fb_mul(tabQ, v)
        shares_all = CipherVector(vB, nt.g1_add(vQ, xK, subtract=True))
    shares = [shares_all[j * n:(j + 1) * n] for j in range(c)]
    if not with_proofs:
        return shares, None
    with timers.span("ks.commit"):
        a = bn.random_scalars(c * n, dev)
        T1 = nt.g1_fb_mul(tabB, a)
        T2 = nt.g1_add(nt.g1_fb_mul(tabQ, a), prods[c * n:].contiguous(), subtract=True)
    return shares, KeySwitchPending(list(secrets), list(publics), Q_point, K, shares_all, T1, T2, a, v, bs)


def finish_keyswitch_proofs(p: KeySwitchPending) -> list:
    """Challenges (every CN's transcript digested on the device, ONE copy to
    the host) and responses za = a + c v (one launch) of a pending batch."""
    dev = p.K.device
    c_n = len(p.secrets)
    n = p.K.shape[0]
    T3s = [O.g1_to_bytes(bn.g1_mul_point(b)) for b in p.bs]
    Qb = O.g1_to_bytes(p.Q)
    groups = [[p.K, p.shares[j * n:(j + 1) * n], p.T1[j * n:(j + 1) * n], p.T2[j * n:(j + 1) * n]]
              for j in range(c_n)]
    with timers.span("ks.transcript"):
        dgs = points_digests(groups)
    chs = [fs_hash(KS_CONTEXT, (O.g1_to_bytes(p.publics[j]), Qb, T3s[j]), dgs[j]) for j in range(c_n)]
    c_rep = torch.cat([_sc([ch], dev).expand(n, 8) for ch in chs]).contiguous()
    za = nt.fr_arith(nt.FR_ADD, p.a, nt.fr_arith(nt.FR_MUL, p.v, c_rep))
    out = []
    for j in range(c_n):
        sl = slice(j * n, (j + 1) * n)
        out.append(KeySwitchProof(p.publics[j], p.Q, p.K, p.shares[sl], p.T1[sl].contiguous(), p.T2[sl].contiguous(),
                                  T3s[j], chs[j], za[sl].contiguous(), (p.bs[j] + chs[j] * p.secrets[j]) % O.R,
                                  dgs[j]))
    return out


def key_switch_list_proof_creation(x: int, X, Q_point, K: torch.Tensor, share: CipherVector,
                                   v: torch.Tensor) -> KeySwitchProof:
    from ..crypto.elgamal import pk_table

    dev = K.device
    n = K.shape[0]
    a = bn.random_scalars(n, dev)
    b = O.random_scalar()
    tabB = bn.base_table(dev)
    tabQ = pk_table(Q_point, dev).tabP
    T1 = nt.g1_fb_mul(tabB, a)
    T2 = nt.g1_add(nt.g1_fb_mul(tabQ, a), nt.g1_mul(K.contiguous(), _sc([b], dev)), subtract=True)
    T3 = O.g1_to_bytes(bn.g1_mul_point(b))
    c = fs_challenge(KS_CONTEXT, O.g1_to_bytes(X), O.g1_to_bytes(Q_point), T3, K, share, T1, T2)
    za = nt.fr_arith(nt.FR_ADD, a, nt.fr_arith(nt.FR_MUL, v, _sc([c], dev)))
    zb = (b + c * x) % O.R
    return KeySwitchProof(X, Q_point, K, share, T1, T2, T3, c, za, zb)


def _ks_fs_ok(proofs: list, copies: int = 1):
    """Each proof's weight-free checks, done by the verifier itself: the
    challenge recomputed from the transcript (point digests are decoded data,
    computed once per proof) and zb B == T3 + c X.  ``copies`` verifying
    nodes of one rank run their own checks in ONE native batch (zb B by one
    fixed-base call, c X by one variable-base call) -> one list per copy
    (copies > 1) or the list itself."""
    with timers.span("ks.verify.transcripts"):
        _digest_checked(proofs, lambda pr: [pr.K, pr.share, pr.T1, pr.T2])
    rows, chs, idx = [], [], []
    res = [[False] * len(proofs) for _ in range(copies)]
    for cp in range(copies):
        for i, pr in enumerate(proofs):
            c = fs_hash(KS_CONTEXT, (O.g1_to_bytes(pr.X), O.g1_to_bytes(pr.Q), pr.T3), pr.pts_digest)
            if c != pr.c or pr.wellformed is False or pr.zb >= O.R:
                continue
            try:
                T3 = O.g1_from_bytes(pr.T3)
            except ValueError:
                continue
            rows.append((pr, T3))
            chs.append(c)
            idx.append((cp, i))
    if rows:
        zb = bn.scalars_tensor([pr.zb % O.R for pr, _ in rows], "cpu")
        lhs = nt.g1_fb_mul(bn.base_table("cpu"), zb)
        cX = nt.g1_mul(bn.g1_jac_tensor([pr.X for pr, _ in rows], "cpu"), bn.scalars_tensor(chs, "cpu"))
        rhs = nt.g1_add(bn.g1_jac_tensor([T3 for _, T3 in rows], "cpu"), cX)
        for (cp, i), ok in zip(idx, nt.g1_eq(lhs, rhs).tolist()):
            res[cp][i] = bool(ok)
    return res if copies > 1 else res[0]


def key_switch_batch_verification(proofs: list, threshold: float = 1.0, combine: bool = True, coins=None) -> list:
    """Verify several CNs' key-switch proofs (same querier key) as ONE random
    linear combination: with 64-bit weights rho_i, sig_i per element drawn
    from the verifier's ``coins``,
      (sum rho za) B + (sum sig za) Q - sum rho T1 - sum c rho (vB)
        - sum zb sig K - sum sig T2 - sum c sig (vQ - xK) == O
    is one Pippenger MSM (no per-element 256-step chains; soundness error
    2^-64).  If the combined check fails, each proof is re-checked alone so the
    bitmap blames exactly the bad ones."""
    if not proofs:
        return []
    ok = _ks_fs_ok(proofs)
    live = [(i, pr, _first(pr.K.shape[0], threshold)) for i, pr in enumerate(proofs)]
    live = [(i, pr, k) for i, pr, k in live if ok[i] and k > 0]
    if not live or not combine:
        return ok
    with timers.span("ks.verify.msm"):
        if _ks_combined(live, 1, [coins])[0]:
            return ok
    for idx, pr, k in live:
        ok[idx] = _ks_combined([(idx, pr, k)], 1, [coins])[0]
    return ok


def key_switch_batch_verification_multi(proofs: list, threshold: float, coins_list: list) -> list:
    """``key_switch_batch_verification`` for several verifying nodes hosted on
    one rank: every VN runs its own Fiat-Shamir / T3 checks and its own random
    combination (weights from its own coins); the combinations share ONE
    grouped MSM launch.  -> [per-VN list of bools]."""
    n_vn = len(coins_list)
    if not proofs:
        return [[] for _ in range(n_vn)]
    oks = _ks_fs_ok(proofs, n_vn) if n_vn > 1 else [_ks_fs_ok(proofs)]
    lives = [[(i, pr, _first(pr.K.shape[0], threshold)) for i, pr in enumerate(proofs) if ok[i]] for ok in oks]
    lives = [[x for x in lv if x[2] > 0] for lv in lives]
    out = [list(ok) for ok in oks]
    if all(lv == lives[0] for lv in lives) and lives[0]:
        with timers.span("ks.verify.msm_multi"):
            verdicts = _ks_combined(lives[0], n_vn, coins_list)
    else:
        verdicts = [(_ks_combined(lv, 1, [c])[0] if lv else True) for lv, c in zip(lives, coins_list)]
    for v in range(n_vn):
        if not verdicts[v]:  # this VN's own per-proof re-check blames the bad ones
            for idx, pr, k in lives[v]:
                out[v][idx] = _ks_combined([(idx, pr, k)], 1, [coins_list[v]])[0]
    return out


def _ks_combined(live, n_vn: int = 1, coins=None):
    """Grouped MSM: every per-element weight stays 64 bit (8 bucket additions
    per point instead of 32); the per-proof challenges c, zb multiply the five
    group sums of each proof on the host.  -> [bool] (``n_vn`` independent
    combinations, fresh weights each, sharing the one MSM launch).  Each VN's
    weights are ONE draw from its coins ([rho | sig] over every live proof);
    the points, the weight selection and the groups are built once."""
    dev = live[0][1].K.device
    nl = len(live)
    cl = coins if isinstance(coins, (list, tuple)) else [coins] * n_vn
    ks = [k for _, _, k in live]
    kt = sum(ks)
    offs = np.cumsum([0] + ks)
    # rows in (proof j, role gi) order -- gi 0: rho T1, 1: rho vB, 2: sig K (x zb), 3: sig T2,
    # 4: sig (vQ - xK) (x c) -- each row's weight index in [rho | sig] and its group
    pts = torch.cat([pt[:k] for _, pr, k in live for pt in (pr.T1, pr.share.K, pr.K, pr.T2, pr.share.C)])
    sel = np.concatenate([(0 if gi < 2 else kt) + offs[j] + np.arange(k) for j, k in enumerate(ks) for gi in range(5)])
    grp1 = np.concatenate([np.full(k, 5 * j + gi) for j, k in enumerate(ks) for gi in range(5)])
    za = torch.cat([pr.za[:k] for _, pr, k in live]).contiguous()
    sel_t = torch.from_numpy(sel).to(dev)
    glv = dev.type == "cuda" and len(set(ks)) == 1
    if glv:
        # GLV weights rho = a + b lambda (a, b 32-bit: 2^64 distinct residues,
        # the same 2^-64 soundness as uniform 64-bit weights): the weighted
        # points take a 32-doubling joint ladder over (P, phi(P))
        pairs = [c.glv(2 * kt, dev) if c is not None else nt.glv_weights(2 * kt, dev) for c in cl]
        AB = torch.cat([p_[0] for p_ in pairs])                               # [n_vn * 2kt, 2]
        W = torch.cat([p_[1] for p_ in pairs])                                # [n_vn * 2kt, 8]
    else:
        W = torch.cat([_rand64(2 * kt, dev, c) for c in cl])                  # [n_vn * 2kt, 8]
        scs = W.view(n_vn, 2 * kt, 8).index_select(1, sel_t).reshape(-1, 8).contiguous()
    full = nt.fr_dot_rows(W, za, 2 * n_vn, b_periodic=True)                  # [sum rho za, sum sig za] per VN
    if glv:
        # equal-length proofs (the CNs switch the same K): every weighted point
        # by one GLV variable-base launch and the 5 nl n_vn group sums by a
        # chunked tree -- no bucket plan and its host sync; group sums and za
        # dots come back in ONE copy
        k0, ng = ks[0], 5 * nl
        # item-major [k0, n_vn * ng] layout: the group sums are g1_sum's axis-0
        # reduction of the products as launched (no transposed copy of them)
        pts_t = pts.view(ng, k0, 24).transpose(0, 1).unsqueeze(1).expand(k0, n_vn, ng, 24).reshape(-1, 24)
        abs_ = AB.view(n_vn, 2 * kt, 2).index_select(1, sel_t).view(n_vn, ng, k0, 2)
        abs_t = abs_.permute(2, 0, 1, 3).reshape(-1, 2).contiguous()
        prod = nt.g1_mul_glv(pts_t.contiguous(), abs_t).view(k0, n_vn * ng, 24)
        sums = nt.g1_sum(prod)
        both = torch.cat([sums.reshape(-1), full.reshape(-1)]).cpu()
        G = both[: sums.numel()].view(-1, 24)
        full = both[sums.numel():].view(-1, 8)
    else:
        grp = (np.arange(n_vn).reshape(-1, 1) * (5 * nl) + grp1.reshape(1, -1)).reshape(-1)
        G = nt.g1_msm_grouped(pts.contiguous().repeat(n_vn, 1), scs, torch.from_numpy(grp.astype(np.int32)).to(dev),
                              5 * nl * n_vn, bits=64)
        full = full.cpu()
    Q = live[0][1].Q
    facs = _sc([f for _, pr, _ in live for f in (1, pr.c, pr.zb, 1, pr.c)], "cpu")
    BQ = bn.g1_jac_tensor([O.G1_GEN, Q], "cpu")
    out = []
    for v in range(n_vn):
        # lhs = (sum rho za) B + (sum sig za) Q; rhs = sum_j G0 + c G1 + zb G2 + G3 + c G4
        lhs = nt.g1_add(*nt.g1_mul(BQ, full[2 * v: 2 * v + 2].contiguous()).split(1))
        g = G[5 * nl * v: 5 * nl * (v + 1)].contiguous()
        rhs = nt.g1_sum(nt.g1_mul(g, facs).view(-1, 1, 24))
        out.append(bool(nt.g1_eq(lhs, rhs)[0]))
    return out


def obfuscation_batch_verification(proofs: list, threshold: float = 1.0, coins=None) -> list:
    """Several CNs' obfuscation proofs as one random linear combination:
      sum rho (z K - T1 - c Ko) + sum sig (z C - T2 - c Co) == O
    (one MSM; per-proof re-check only if the combination fails)."""
    if not proofs:
        return []
    ok = _obf_fs_ok(proofs)
    live = [(i, pr, _first(len(pr.C), threshold)) for i, pr in enumerate(proofs)]
    live = [(i, pr, k) for i, pr, k in live if ok[i] and k > 0]
    if not live:
        return ok
    if _obf_combined(live, coins):
        return ok
    for idx, pr, k in live:
        ok[idx] = _obf_combined([(idx, pr, k)], coins)
    return ok


def _obf_combined(live, coins=None) -> bool:
    """Grouped MSM: rho z K + sig z C (full-size weights), rho T1 + sig T2
    and rho Ko + sig Co (64-bit weights, the latter times c on the host)."""
    dev = live[0][1].C.device
    pts, scs, grp = [], [], []
    for j, (_, pr, k) in enumerate(live):
        rho, sig = _rand64(k, dev, coins), _rand64(k, dev, coins)
        z = pr.z[:k].contiguous()
        terms = ((pr.C.K, nt.fr_arith(nt.FR_MUL, rho, z), 0), (pr.C.C, nt.fr_arith(nt.FR_MUL, sig, z), 0),
                 (pr.T.K, rho, 1), (pr.T.C, sig, 1), (pr.Co.K, rho, 2), (pr.Co.C, sig, 2))
        for pt, w, gi in terms:
            pts.append(pt[:k])
            scs.append(w)
            grp.append(torch.full((k,), 3 * j + gi, dtype=torch.int32, device=dev))
    pts, scs, grp = torch.cat(pts).contiguous(), torch.cat(scs).contiguous(), torch.cat(grp)
    full = grp % 3 == 0
    Gf = nt.g1_msm_grouped(pts[full].contiguous(), scs[full].contiguous(), grp[full] // 3, len(live))
    Gs = nt.g1_msm_grouped(pts[~full].contiguous(), scs[~full].contiguous(), grp[~full] - grp[~full] // 3 - 1,
                           2 * len(live), bits=64)
    # sum_j A_j == sum_j B_j + c_j C_j
    lhs = nt.g1_sum(Gf.view(-1, 1, 24))
    facs = []
    for _, pr, _ in live:
        facs += [1, pr.c]
    rhs = nt.g1_sum(nt.g1_mul(Gs.contiguous(), _sc(facs, "cpu")).view(-1, 1, 24))
    return bool(nt.g1_eq(lhs, rhs)[0])


def key_switch_list_proof_verification(pr: KeySwitchProof, threshold: float = 1.0) -> bool:
    from ..crypto.elgamal import pk_table

    n = pr.K.shape[0]
    k = _first(n, threshold)
    if k == 0:
        return True
    if not _ks_fs_ok([pr])[0]:
        return False
    dev = pr.K.device
    tabB = bn.base_table(dev)
    tabQ = pk_table(pr.Q, dev).tabP
    cs = _sc([pr.c], dev)
    za = pr.za[:k].contiguous()
    # za B == T1 + c (vB)
    ok1 = nt.g1_eq(nt.g1_fb_mul(tabB, za),
                   nt.g1_add(pr.T1[:k].contiguous(), nt.g1_mul(pr.share.K[:k].contiguous(), cs)))
    # za Q - zb K == T2 + c (vQ - xK)
    lhs = nt.g1_add(nt.g1_fb_mul(tabQ, za), nt.g1_mul(pr.K[:k].contiguous(), _sc([pr.zb], dev)), subtract=True)
    rhs = nt.g1_add(pr.T2[:k].contiguous(), nt.g1_mul(pr.share.C[:k].contiguous(), cs))
    ok2 = nt.g1_eq(lhs, rhs)
    return bool(ok1.all()) and bool(ok2.all())
