"""Aggregation proofs and verifiable-shuffle proofs.

Aggregation — unlynx AggregationListProofCreation/Verification (external; used
by the CollectiveAggregation ProofFunc, services/service.go:515-560): the CN
publishes the ciphertext vectors it received and its claimed sum; a VN
recomputes the sum (K5 kernel) and compares the first ceil(threshold * n)
elements.

Shuffle (DRO, differential-privacy noise list) — unlynx ShuffleSequence
(permutation + re-randomisation, here on the device); the shuffle proof is
proofs/shuffle.py (commitment-consistent proof of a shuffle, one MSM to verify).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

from .. import native as nt
from ..crypto import bn254 as bn
from ..crypto.elgamal import CipherVector, pk_table


# ----------------------------------------------------------------------------- aggregation
AGG_MAGIC = 0x41475031  # "AGP1"
_AGG_HEAD = 3           # magic, contributors k, rows n


@dataclass
class AggregationProof:
    inputs: list          # list of CipherVector (one per contributor)
    result: CipherVector  # claimed sum
    stacked: object = None  # decoded proofs: (K, C) [contributors, n, 24] behind ``inputs``

    # reference-style export (kyber affine encodings): ledger / GetProofs
    def to_bytes(self) -> bytes:
        parts = [len(self.inputs).to_bytes(8, "little"), len(self.result).to_bytes(8, "little")]
        if self.inputs and all(len(cv) == len(self.result) for cv in self.inputs):
            # one normalisation + one device-to-host copy for every contributor
            # (a CN with thousands of DPs would otherwise pay one sync per DP)
            parts.append(CipherVector.cat(list(self.inputs) + [self.result]).to_bytes())
            return b"".join(parts)
        for cv in self.inputs:
            parts.append(cv.to_bytes())
        parts.append(self.result.to_bytes())
        return b"".join(parts)

    @staticmethod
    def from_bytes(b: bytes, device="cpu") -> "AggregationProof":
        k = int.from_bytes(b[:8], "little")
        n = int.from_bytes(b[8:16], "little")
        if len(b) != 16 + 128 * n * (k + 1):
            raise ValueError("aggregation proof length does not match its header")
        # every contributor and the result in one decode (a CN with thousands of
        # DPs would otherwise pay one decode launch sequence per DP)
        allcv = CipherVector.from_bytes(b[16:], device)
        K = allcv.K.view(k + 1, n, 24)
        C = allcv.C.view(k + 1, n, 24)
        ins = [CipherVector(K[i], C[i]) for i in range(k)]
        return AggregationProof(ins, CipherVector(K[k], C[k]), (K[:k], C[:k]))

    # intra-cluster payload: raw Jacobian limbs of [K inputs..., K result] and
    # [C inputs..., C result], assembled on the device with no host marshalling
    def pack(self) -> torch.Tensor:
        dev = self.result.device
        k, n = len(self.inputs), len(self.result)
        if any(len(cv) != n for cv in self.inputs):
            raise ValueError("aggregation proof inputs differ in length from the result")
        head = bn.h2d(torch.tensor([AGG_MAGIC, k, n], dtype=torch.int32), dev)
        Ks = [cv.K.reshape(-1) for cv in self.inputs] + [self.result.K.reshape(-1)]
        Cs = [cv.C.reshape(-1) for cv in self.inputs] + [self.result.C.reshape(-1)]
        return torch.cat([head] + Ks + Cs)

    @staticmethod
    def unpack(t: torch.Tensor, head: list | None = None) -> "AggregationProof":
        if head is None:
            head = t[:_AGG_HEAD].cpu().tolist()
        magic, k, n = head[:3]
        if magic != AGG_MAGIC or k < 0 or n < 0 or t.numel() != _AGG_HEAD + 2 * (k + 1) * n * 24:
            raise ValueError("malformed packed aggregation proof")
        K = t[_AGG_HEAD: _AGG_HEAD + (k + 1) * n * 24].view(k + 1, n, 24)
        C = t[_AGG_HEAD + (k + 1) * n * 24:].view(k + 1, n, 24)
        ins = [CipherVector(K[i], C[i]) for i in range(k)]
        return AggregationProof(ins, CipherVector(K[k], C[k]), (K[:k], C[:k]))


def unpack_many(tensors: list) -> list:
    """Unpack many packed aggregation proofs with ONE header copy (an entry is
    the proof or the exception that rejects it)."""
    if not tensors:
        return []
    heads = torch.nn.utils.rnn.pad_sequence([t[:_AGG_HEAD] for t in tensors], batch_first=True).cpu().tolist()
    out = []
    for t, h in zip(tensors, heads):
        try:
            out.append(AggregationProof.unpack(t, h))
        except Exception as e:  # noqa: BLE001 -- a malformed payload is a rejected proof
            out.append(e)
    return out


def aggregation_list_proof_creation(inputs: list, result: CipherVector) -> AggregationProof:
    return AggregationProof(list(inputs), result)


def aggregation_check(pr: AggregationProof, threshold: float = 1.0) -> torch.Tensor:
    """Device bool (no host sync): the inputs' canonical, on-curve limbs sum to
    the claimed result on the first ceil(threshold * n) rows (K5 reduction +
    projective comparison)."""
    n = len(pr.result)
    k = int(math.ceil(threshold * n))
    dev = pr.result.device
    if k == 0 or not pr.inputs:
        return torch.ones((), dtype=torch.bool, device=dev)
    if pr.stacked is not None:
        Ks, Cs = pr.stacked[0][:, :k], pr.stacked[1][:, :k]
    else:
        Ks = torch.stack([cv.K[:k] for cv in pr.inputs])
        Cs = torch.stack([cv.C[:k] for cv in pr.inputs])
    pts = torch.cat([Ks.reshape(-1, 24), Cs.reshape(-1, 24), pr.result.K[:k], pr.result.C[:k]])
    valid = nt.limbs_canonical(pts.reshape(-1, 8)).bool().all() & nt.g1j_on_curve(pts).bool().all()
    sK, sC = nt.g1_sum(Ks.contiguous()), nt.g1_sum(Cs.contiguous())
    eq = nt.g1_eq(torch.cat([sK, sC]), torch.cat([pr.result.K[:k], pr.result.C[:k]]).contiguous())
    return valid & eq.bool().all()


def aggregation_list_proof_verification(pr: AggregationProof, threshold: float = 1.0) -> bool:
    return bool(aggregation_check(pr, threshold))


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
