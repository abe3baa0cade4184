"""Aggregation proofs and verifiable-shuffle proofs.

Aggregation — unlynx AggregationListProofCreation/Verification (external; used
by the CollectiveAggregation ProofFunc, services/service.go:515-560): the CN
publishes the ciphertext vectors it received and its claimed sum; a VN
recomputes the sum (K5 kernel) and compares the first ceil(threshold * n)
elements.

Shuffle (DRO, differential-privacy noise list) — unlynx ShuffleProofCreation /
ShuffleProofVerification (a Neff proof, external; services/service.go:632-665).
Here a Sako–Kilian cut-and-choose shuffle proof: the prover commits to k
shadow shuffles Z_t of the input; Fiat–Shamir bits decide, per shadow,
whether to open input->shadow or shadow->output (permutation + re-encryption
randomness).  Soundness 2^-k; every opening check is a batched re-encryption
on the device (2 fixed-base mults per element).  The Neff argument itself is
not reproduced (documented deviation; same statement proven).
"""
from __future__ import annotations

import hashlib
import math
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import native as nt
from ..crypto import bn254 as bn
from ..crypto import oracle as O
from ..crypto.elgamal import CipherVector, pk_table


# ----------------------------------------------------------------------------- aggregation
@dataclass
class AggregationProof:
    inputs: list          # list of CipherVector (one per contributor)
    result: CipherVector  # claimed sum

    def to_bytes(self) -> bytes:
        parts = [len(self.inputs).to_bytes(8, "little"), len(self.result).to_bytes(8, "little")]
        for cv in self.inputs:
            parts.append(cv.to_bytes())
        parts.append(self.result.to_bytes())
        return b"".join(parts)

    @staticmethod
    def from_bytes(b: bytes, device="cpu") -> "AggregationProof":
        k = int.from_bytes(b[:8], "little")
        n = int.from_bytes(b[8:16], "little")
        o = 16
        ins = []
        for _ in range(k):
            ins.append(CipherVector.from_bytes(b[o: o + 128 * n], device))
            o += 128 * n
        res = CipherVector.from_bytes(b[o: o + 128 * n], device)
        return AggregationProof(ins, res)


def aggregation_list_proof_creation(inputs: list, result: CipherVector) -> AggregationProof:
    return AggregationProof(list(inputs), result)


def aggregation_list_proof_verification(pr: AggregationProof, threshold: float = 1.0) -> bool:
    n = len(pr.result)
    k = int(math.ceil(threshold * n))
    if k == 0 or not pr.inputs:
        return True
    s = CipherVector.sum([cv[:k] for cv in pr.inputs])
    r = pr.result[:k]
    return bool(nt.g1_eq(s.K, r.K).all()) and bool(nt.g1_eq(s.C, r.C).all())


# ----------------------------------------------------------------------------- shuffle
def rerandomize(cv: CipherVector, rho: torch.Tensor, P_point) -> CipherVector:
    """(K + rho B, C + rho P) — fresh encryption randomness under P."""
    pk = pk_table(P_point, cv.device)
    return CipherVector(nt.g1_add(cv.K, nt.g1_fb_mul(pk.tabB, rho)), nt.g1_add(cv.C, nt.g1_fb_mul(pk.tabP, rho)))


def permute(cv: CipherVector, perm: torch.Tensor) -> CipherVector:
    """(perm X)_i = X_{perm[i]}."""
    p = perm.to(cv.device)
    return CipherVector(cv.K.index_select(0, p).contiguous(), cv.C.index_select(0, p).contiguous())


def shuffle_sequence(cv: CipherVector, P_point):
    """ShuffleSequence: random permutation + re-randomisation; returns (Y, perm, rho)."""
    import os

    n = len(cv)
    perm = torch.from_numpy(np.argsort(np.frombuffer(os.urandom(8 * n), dtype="<u8"), kind="stable"))
    rho = bn.random_scalars(n, cv.device)
    return rerandomize(permute(cv, perm), rho, P_point), perm, rho


@dataclass
class ShuffleProof:
    X: CipherVector
    Y: CipherVector
    Z: list                                   # k shadow lists
    bits: list                                # challenge bits
    perms: list                               # opened permutations (np int64 arrays)
    rhos: list                                # opened randomness tensors [n, 8]

    def to_bytes(self) -> bytes:
        n, k = len(self.X), len(self.Z)
        parts = [n.to_bytes(8, "little"), k.to_bytes(8, "little"), self.X.to_bytes(), self.Y.to_bytes()]
        for t in range(k):
            parts += [self.Z[t].to_bytes(), bytes([self.bits[t]]), np.asarray(self.perms[t], dtype="<i8").tobytes(),
                      bn.scalars_to_bytes(self.rhos[t]).tobytes()]
        return b"".join(parts)

    @staticmethod
    def from_bytes(b: bytes, device="cpu") -> "ShuffleProof":
        n = int.from_bytes(b[:8], "little")
        k = int.from_bytes(b[8:16], "little")
        o = 16
        X = CipherVector.from_bytes(b[o: o + 128 * n], device); o += 128 * n
        Y = CipherVector.from_bytes(b[o: o + 128 * n], device); o += 128 * n
        Z, bits, perms, rhos = [], [], [], []
        for _ in range(k):
            Z.append(CipherVector.from_bytes(b[o: o + 128 * n], device)); o += 128 * n
            bits.append(b[o]); o += 1
            perms.append(np.frombuffer(b[o: o + 8 * n], dtype="<i8").copy()); o += 8 * n
            rhos.append(bn.scalars_from_bytes(np.frombuffer(b[o: o + 32 * n], dtype=np.uint8), device)); o += 32 * n
        return ShuffleProof(X, Y, Z, bits, perms, rhos)


def _bits(X, Y, Z, k) -> list:
    h = hashlib.sha256()
    for cv in [X, Y] + list(Z):
        h.update(cv.to_bytes())
    out, ctr = [], 0
    while len(out) < k:
        d = hashlib.sha256(h.digest() + ctr.to_bytes(4, "little")).digest()
        for byte in d:
            for i in range(8):
                out.append((byte >> i) & 1)
        ctr += 1
    return out[:k]


def shuffle_proof_creation(X: CipherVector, Y: CipherVector, perm: torch.Tensor, rho: torch.Tensor, P_point,
                           k: int = 40) -> ShuffleProof:
    """Y_i = X_{perm[i]} + Enc0(rho_i).  Shadows Z_t,i = X_{sig[i]} + Enc0(tau_i)."""
    import os

    n = len(X)
    dev = X.device
    sigs, taus, Z = [], [], []
    for _ in range(k):
        sig = np.argsort(np.frombuffer(os.urandom(8 * n), dtype="<u8"), kind="stable")
        tau = bn.random_scalars(n, dev)
        sigs.append(sig)
        taus.append(tau)
        Z.append(rerandomize(permute(X, torch.from_numpy(sig)), tau, P_point))
    bits = _bits(X, Y, Z, k)
    perm_np = perm.cpu().numpy()
    perms, rhos = [], []
    for t in range(k):
        if bits[t] == 0:
            perms.append(sigs[t])
            rhos.append(taus[t])
        else:
            # Y_i = Z_{lam(i)} + Enc0(rho_i - tau_{lam(i)}),  lam = sig^-1 o perm
            inv = np.empty(n, dtype=np.int64)
            inv[sigs[t]] = np.arange(n)
            lam = inv[perm_np]
            lam_t = torch.from_numpy(lam).to(dev)
            d = nt.fr_arith(nt.FR_SUB, rho, taus[t].index_select(0, lam_t).contiguous())
            perms.append(lam)
            rhos.append(d)
    return ShuffleProof(X, Y, Z, bits, perms, rhos)


def shuffle_proof_verification(pr: ShuffleProof, P_point) -> bool:
    k = len(pr.Z)
    if _bits(pr.X, pr.Y, pr.Z, k) != list(pr.bits):
        return False
    for t in range(k):
        perm = pr.perms[t]
        if sorted(perm.tolist()) != list(range(len(pr.X))):
            return False
        src, dst = (pr.X, pr.Z[t]) if pr.bits[t] == 0 else (pr.Z[t], pr.Y)
        exp = rerandomize(permute(src, torch.from_numpy(perm)), pr.rhos[t].to(src.device), P_point)
        if not (bool(nt.g1_eq(exp.K, dst.K).all()) and bool(nt.g1_eq(exp.C, dst.C).all())):
            return False
    return True


# ----------------------------------------------------------------------------- DP noise
def generate_noise_values_scale(n: int, mean: float, b: float, quanta: float, scale: float, limit: float) -> list:
    """Discretised, clipped Laplace noise list (unlynx GenerateNoiseValuesScale,
    external; called at services/service.go:657).  Values k*quanta in
    [-limit, limit] appear with multiplicity proportional to the Laplace(mean, b)
    density; the list is scaled, then padded/trimmed to n.  Parity unpinned
    (the unlynx source is not available)."""
    if n <= 0:
        return []
    if quanta <= 0:
        quanta = 1.0
    if limit <= 0:
        limit = quanta * max(1, n)
    ks = np.arange(-limit, limit + quanta / 2, quanta)
    pdf = np.exp(-np.abs(ks - mean) / max(b, 1e-12)) / (2 * max(b, 1e-12)) * quanta
    counts = np.round(pdf / pdf.sum() * n).astype(np.int64)
    vals = np.repeat(ks, counts) * scale
    if vals.size < n:
        vals = np.concatenate([vals, np.full(n - vals.size, mean * scale)])
    return [int(round(v)) for v in vals[:n]]
