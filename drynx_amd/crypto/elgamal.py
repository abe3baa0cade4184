"""Additively homomorphic EC-ElGamal over BN254 G1 on device tensors.

Re-supplies unlynx's ``lib`` ElGamal (external to the reference, used at e.g.
lib/encoding/sum.go:24, lib/structs.go:290-353):

* Enc(m) = (K = r*B, C = m*B + r*P)            -> ``encrypt_ints``
* Add    = component-wise point addition        -> ``CipherVector.add``
* Dec    = dlog(C - x*K) with a bounded BSGS     -> ``DecryptionTable``
* CheckZero: C - x*K == identity                 -> ``decrypt_check_zero``

A CipherVector is two [n, 24] int32 Jacobian tensors (K, C) living on the
party's device; the wire form is kyber's K||C (2 x 64 B per ciphertext).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from .. import native as nt
from . import bn254 as bn
from . import oracle as O


# ----------------------------------------------------------------------------- keys
@dataclass
class KeyPair:
    secret: int
    public: tuple  # oracle affine point

    @staticmethod
    def generate() -> "KeyPair":
        x = O.random_scalar()
        return KeyPair(x, bn.g1_mul_point(x))

    @staticmethod
    def from_secret(x: int) -> "KeyPair":
        return KeyPair(x % O.R, bn.g1_mul_point(x % O.R))

    def public_jac(self, device="cpu") -> torch.Tensor:
        return bn.g1_jac_tensor([self.public], device)

    def secret_tensor(self, device="cpu") -> torch.Tensor:
        return bn.scalars_tensor([self.secret], device)


def aggregate_keys(points) -> tuple:
    """Collective key P = sum of the CNs' public keys (onet Roster.Aggregate)."""
    acc = None
    for p in points:
        acc = O.g1_add(acc, p)
    return acc


# ----------------------------------------------------------------------------- ciphertext vectors
class CipherVector:
    __slots__ = ("K", "C")

    def __init__(self, K: torch.Tensor, C: torch.Tensor):
        assert K.shape == C.shape and K.shape[-1] == 24
        self.K = K.contiguous()
        self.C = C.contiguous()

    def __len__(self):
        return self.K.shape[0]

    @property
    def device(self):
        return self.K.device

    def to(self, device) -> "CipherVector":
        return CipherVector(self.K.to(device), self.C.to(device))

    @staticmethod
    def zeros(n: int, device="cpu") -> "CipherVector":
        inf = bn.g1_infinity_jac(n, device)
        return CipherVector(inf, inf.clone())

    def clone(self) -> "CipherVector":
        return CipherVector(self.K.clone(), self.C.clone())

    def add(self, other: "CipherVector") -> "CipherVector":
        return CipherVector(nt.g1_add(self.K, other.K), nt.g1_add(self.C, other.C))

    def sub(self, other: "CipherVector") -> "CipherVector":
        return CipherVector(nt.g1_add(self.K, other.K, True), nt.g1_add(self.C, other.C, True))

    def mul_scalars(self, s: torch.Tensor) -> "CipherVector":
        """Component-wise (s_i*K_i, s_i*C_i); s may be one broadcast scalar."""
        return CipherVector(nt.g1_mul(self.K, s), nt.g1_mul(self.C, s))

    def __getitem__(self, idx) -> "CipherVector":
        return CipherVector(self.K[idx].reshape(-1, 24), self.C[idx].reshape(-1, 24))

    @staticmethod
    def cat(cvs) -> "CipherVector":
        cvs = list(cvs)
        return CipherVector(torch.cat([c.K for c in cvs]), torch.cat([c.C for c in cvs]))

    @staticmethod
    def sum(cvs) -> "CipherVector":
        """Homomorphic sum of equally-long vectors (K5 reduction over axis 0)."""
        cvs = list(cvs)
        if len(cvs) == 1:
            return cvs[0].clone()
        K = nt.g1_sum(torch.stack([c.K for c in cvs]))
        C = nt.g1_sum(torch.stack([c.C for c in cvs]))
        return CipherVector(K, C)

    # wire: kyber CipherText = K || C, 64 B each (affine, big endian)
    def to_bytes(self) -> bytes:
        if len(self) == 0:
            return b""
        both = torch.cat([self.K, self.C], dim=1).view(-1, 24)
        aff = nt.g1_to_affine(both)
        b = bn.g1_aff_to_bytes(aff).reshape(-1, 128)
        return b.tobytes()

    @staticmethod
    def from_bytes(data: bytes, device="cpu") -> "CipherVector":
        if len(data) == 0:
            return CipherVector(torch.empty((0, 24), dtype=torch.int32, device=device),
                                torch.empty((0, 24), dtype=torch.int32, device=device))
        arr = np.frombuffer(data, dtype=np.uint8).reshape(-1, 2, 64)
        aff = bn.g1_aff_from_bytes(arr.reshape(-1), device)
        jac = nt.g1_from_affine(aff).view(-1, 2, 24)
        return CipherVector(jac[:, 0].contiguous(), jac[:, 1].contiguous())

    def points(self):
        """(K, C) as oracle affine points (tests / debugging)."""
        return bn.g1_points_from_jac(self.K), bn.g1_points_from_jac(self.C)


# ----------------------------------------------------------------------------- encryption
class PublicKeyTable:
    """Comb tables for (B, P): every encryption is two fixed-base mults (K2/K3)."""

    def __init__(self, public_point, device="cpu"):
        self.point = public_point
        self.device = torch.device(device)
        self.tabB = bn.base_table(device)
        self.tabP = nt.g1_fb_table(bn.g1_aff_tensor([public_point], device))

    @property
    def public_jac(self) -> torch.Tensor:
        return bn.g1_jac_tensor([self.point], self.device)


_pk_cache: dict = {}


def pk_table(public_point, device="cpu") -> PublicKeyTable:
    key = (O.g1_to_bytes(public_point), str(torch.device(device)))
    t = _pk_cache.get(key)
    if t is None:
        if len(_pk_cache) > 64:
            # tables of other keys may still be read by queued kernels of any
            # stream: the device drains before their memory goes back
            if torch.cuda.is_available() and torch.cuda.is_initialized():
                torch.cuda.synchronize()
            _pk_cache.clear()
        t = _pk_cache[key] = bn.publish(PublicKeyTable(public_point, device))
    return t


def encrypt_ints(pk: PublicKeyTable, values, r: torch.Tensor | None = None):
    """EncryptIntVectorGetRs: returns (CipherVector, r)."""
    m = values if isinstance(values, torch.Tensor) else torch.tensor(list(values), dtype=torch.int64)
    m = m.to(device=pk.device, dtype=torch.int64).reshape(-1).contiguous()
    if r is None:
        r = bn.random_scalars(m.numel(), pk.device)
    K, C = nt.elgamal_encrypt(pk.tabB, pk.tabP, m, r)
    return CipherVector(K, C), r


def encrypt_scalars(pk: PublicKeyTable, s: torch.Tensor, r: torch.Tensor | None = None):
    """EncryptScalar: (r*B, s*B + r*P) for arbitrary scalars s (OR/AND encodings)."""
    n = s.shape[0]
    if r is None:
        r = bn.random_scalars(n, pk.device)
    K = nt.g1_fb_mul(pk.tabB, r)
    C = nt.g1_add(nt.g1_fb_mul(pk.tabB, s), nt.g1_fb_mul(pk.tabP, r))
    return CipherVector(K, C), r


def decrypt_points(secret: int, cv: CipherVector) -> torch.Tensor:
    """M_i = C_i - x*K_i (Jacobian)."""
    x = bn.scalars_tensor([secret], cv.device)
    xK = nt.g1_mul(cv.K, x)
    return nt.g1_add(cv.C, xK, subtract=True)


def decrypt_check_zero(secret: int, cv: CipherVector) -> torch.Tensor:
    """unlynx DecryptCheckZero: 0 where the plaintext point is the identity, else 1."""
    M = decrypt_points(secret, cv)
    inf = bn.g1_infinity_jac(len(cv), cv.device)
    return (1 - nt.g1_eq(M, inf).to(torch.int64))


class DecryptionTable:
    """Baby-step/giant-step dlog for |m| <= bound (unlynx CreateDecryptionTable
    + DecryptIntWithNeg; the reference's client uses bound 10000,
    services/api.go:49-50).  The baby-step hash table lives on the device; on a
    GPU it can be sized to hundreds of MB of HBM so 1e6-record aggregates decode
    with few giant steps."""

    def __init__(self, bound: int = 10000, device="cpu", max_baby: int | None = None):
        self.device = torch.device(device)
        self.bound = int(bound)
        span = 2 * self.bound + 1
        if self.device.type == "cuda":
            # HBM is plentiful: a baby table of up to 2^24 entries (~400 MB hash
            # table, built once and cached) leaves few serial giant steps per value
            self.m_baby = max(2, min(span + 1, max_baby or (1 << 24)))
        else:
            self.m_baby = max(2, min(int(math.isqrt(span)) + 1, max_baby or (1 << 15)))
        self.n_giant = (span + self.m_baby - 1) // self.m_baby + 1
        cap = 1
        while cap < 2 * self.m_baby:
            cap <<= 1
        tabB = bn.base_table(self.device)
        self.keys, self.vals = nt.bsgs_build(tabB, self.m_baby, cap)
        self.giant = nt.g1_to_affine(nt.g1_fb_mul_i64(tabB, torch.tensor([self.m_baby], dtype=torch.int64,
                                                                             device=self.device)))
        self.offset_pt = nt.g1_fb_mul_i64(tabB, torch.tensor([self.bound], dtype=torch.int64, device=self.device))

    def solve(self, M_jac: torch.Tensor, strict: bool = True) -> torch.Tensor:
        T = nt.g1_add(M_jac.contiguous(), self.offset_pt)
        out, found = nt.bsgs_solve(T, self.giant, self.keys, self.vals, self.m_baby, self.n_giant, self.bound)
        if strict and not bool(found.all()):
            bad = int((found == 0).sum())
            raise ValueError(f"{bad} plaintexts outside the decryption table range [-{self.bound}, {self.bound}]")
        return out

    def decrypt(self, secret: int, cv: CipherVector, strict: bool = True) -> torch.Tensor:
        return self.solve(decrypt_points(secret, cv), strict)


_dt_cache: dict = {}


def decryption_table(bound: int = 10000, device="cpu") -> DecryptionTable:
    key = (int(bound), str(torch.device(device)))
    t = _dt_cache.get(key)
    if t is None:
        t = _dt_cache[key] = bn.publish(DecryptionTable(bound, device))
    return t


def decrypt_auto(secret: int, cv: CipherVector, bound: int = 10000, max_bound: int = 1 << 44) -> torch.Tensor:
    """Decrypt with a table that grows (x256) until every plaintext is found:
    aggregates of 1e6-record logistic regressions exceed the reference's fixed
    10000-entry table."""
    M = decrypt_points(secret, cv)
    out = torch.zeros(len(cv), dtype=torch.int64, device=cv.device)
    todo = torch.arange(len(cv), device=cv.device)
    b = max(1, int(bound))
    while todo.numel():
        t = decryption_table(b, cv.device)
        T = nt.g1_add(M.index_select(0, todo).contiguous(), t.offset_pt)
        vals, found = nt.bsgs_solve(T, t.giant, t.keys, t.vals, t.m_baby, t.n_giant, t.bound)
        ok = found.bool()
        out[todo[ok]] = vals[ok]
        todo = todo[~ok]
        if b >= max_bound and todo.numel():
            raise ValueError(f"{todo.numel()} plaintexts beyond +/-{max_bound}")
        b = min(b * 256, max_bound)
    return out


def decrypt_ints(secret: int, cv: CipherVector, bound: int = 10000) -> list[int]:
    return [int(v) for v in decryption_table(bound, cv.device).decrypt(secret, cv).cpu().tolist()]
