"""Verifiable shuffle of ElGamal lists: commitment-consistent proof of a
shuffle (Terelius–Wikström permutation-matrix argument), batched on the GPU.

Reference: the DRO noise list is shuffled and re-randomised by every CN with a
verifiable-shuffle proof (unlynx ShuffleSequence + ShuffleProofCreation /
ShuffleProofVerification -- kyber's Neff PairShuffle; used at
services/service.go:619-665, data/data.go:61-71).  Same statement, different
(offline-derivable) argument, whose work is MSM-shaped instead of a sequential
interactive chain:

Statement.  Y_j = X_{pi(j)} + Enc0(s_j) for a secret permutation pi and
re-encryption randomness s (Enc0(s) = (s B, s P)).

Prover.
  1. u_j = r_j B + h_{pi(j)}: commitments to the columns of the permutation
     matrix under independent generators h_0..h_N (hash-to-G1, no known logs).
  2. e = PRG(H(P, X, Y, u)) (128-bit components), e'_i = e_{pi^-1(i)}.
  3. Product chain: B_i = beta_i B + (prod_{k<=i} e'_k) h_0 with fresh beta_i --
     a parallel prefix product instead of the sequential chain, satisfying
     B_i = b_i B + e'_i B_{i-1} with b_i = beta_i - e'_i beta_{i-1} (B_0 = h_0).
  4. Sigma protocol for, with the SAME responses k_E for e' in all equations,
       A  = rho B + sum e'_i h_i              (A = sum e_j u_j)
       B_i = b_i B + e'_i B_{i-1}             (product of e' == product of e)
       C  = c B                               (C = sum u_j - sum h_i: unit column sums)
       D  = d B                               (D = B_N - (prod e) h_0)
       F  = sum e'_i X_i + Enc0(sigma)        (F = sum e_j Y_j)
     commitments A', B'_i, C', D', F'; challenge v = H(...); responses
     k = witness_nonce + v * witness.
Verifier.  Every check, including the recomputation of A, C, D and F, is
folded with random 64-bit weights into ONE Pippenger MSM over ~8N points
(native g1_msm); soundness error ~ 2^-64 + N/2^128.

Parity: the reference's Neff proof bytes (kyber PairShuffle) are not
reproducible offline; the statement, its use (DRO chain, one proof per CN) and
the VN verification / bitmap semantics are the reference ones.
"""
from __future__ import annotations

import hashlib
import struct
from dataclasses import dataclass

import numpy as np
import torch

from .. import native as nt
from ..crypto import bn254 as bn
from ..crypto import digest as dg
from ..crypto import oracle as O
from ..crypto.elgamal import CipherVector, pk_table

SEED = hashlib.sha256(b"drynx-amd/shuffle/generators/v1").digest()
_TAG = b"drynx-amd/shuffle/v1"

_gen_cache: dict = {}
_h0_tab: dict = {}


def generators(n: int, device) -> torch.Tensor:
    """Jacobian [n+1, 24]: h_0 .. h_n (cached per device, grown by doubling)."""
    dev = torch.device(device)
    key = str(dev)
    cur = _gen_cache.get(key)
    if cur is None or cur.shape[0] < n + 1:
        m = max(n + 1, 2 * (cur.shape[0] if cur is not None else 0), 64)
        _gen_cache[key] = cur = bn.publish(nt.g1_from_affine(nt.hash_to_g1(SEED, 0, m, dev)))
    return cur[: n + 1]


def _h0_table(device):
    key = str(torch.device(device))
    if key not in _h0_tab:
        _h0_tab[key] = nt.g1_fb_table(nt.g1_to_affine(generators(0, device)[:1].contiguous()))
    return _h0_tab[key]


# ----------------------------------------------------------------------------- Fr helpers (device)
def _mul(a, b):
    return nt.fr_arith(nt.FR_MUL, a.contiguous(), b.contiguous())


def _add(a, b):
    return nt.fr_arith(nt.FR_ADD, a.contiguous(), b.contiguous())


def _sub(a, b):
    return nt.fr_arith(nt.FR_SUB, a.contiguous(), b.contiguous())


def _neg(a):
    return nt.fr_arith(nt.FR_NEG, a.contiguous())


def _sc(x: int, device):
    return bn.scalars_tensor([x % O.R], device)


def _sum(x: torch.Tensor) -> torch.Tensor:
    cur = x.contiguous()
    while cur.shape[0] > 1:
        if cur.shape[0] % 2:
            cur = torch.cat([cur, torch.zeros((1, 8), dtype=torch.int32, device=cur.device)])
        cur = _add(cur[0::2], cur[1::2])
    return cur


def _prefix_products(x: torch.Tensor) -> torch.Tensor:
    """P_i = prod_{k<=i} x_k (Hillis-Steele scan: log2(N) wide Fr launches)."""
    cur = x.contiguous()
    shift = 1
    while shift < cur.shape[0]:
        cur = torch.cat([cur[:shift], _mul(cur[shift:], cur[:-shift])])
        shift *= 2
    return cur


def _to_int(t: torch.Tensor) -> int:
    return bn.scalars_from_tensor(t.reshape(1, 8))[0]


def _rand64(n: int, device) -> torch.Tensor:
    r = bn.random_scalars(n, device)
    r[:, 2:] = 0
    r[:, 0] |= 1
    return r


# ----------------------------------------------------------------------------- transcript
def _pts_digest(jac: torch.Tensor) -> bytes:
    return dg.digest_tensor(nt.g1_to_affine(jac.contiguous().view(-1, 24)))


def _challenge_e(P_point, X: CipherVector, Y: CipherVector, u: torch.Tensor):
    h = hashlib.sha256(_TAG)
    h.update(O.g1_to_bytes(P_point) + struct.pack("<Q", len(X)))
    h.update(_pts_digest(torch.cat([X.K, X.C, Y.K, Y.C, u])))
    t1 = h.digest()
    e = nt.prg_scalars(t1, len(X), X.device)
    e[:, 4:] = 0  # 128-bit challenge components
    return t1, e


def _challenge_v(t1: bytes, B, Bp, singles) -> int:
    h = hashlib.sha256(t1)
    h.update(_pts_digest(torch.cat([B, Bp] + singles)))
    return int.from_bytes(h.digest(), "big") % O.R


@dataclass
class ShuffleProof:
    X: CipherVector
    Y: CipherVector
    u: torch.Tensor          # [N, 24] permutation commitments
    B: torch.Tensor          # [N, 24] product chain
    Ap: torch.Tensor         # [1, 24]
    Bp: torch.Tensor         # [N, 24]
    Cp: torch.Tensor
    Dp: torch.Tensor
    FpK: torch.Tensor
    FpC: torch.Tensor
    kA: int
    kB: torch.Tensor         # [N, 8]
    kC: int
    kD: int
    kE: torch.Tensor         # [N, 8]
    kF: int

    def to_bytes(self) -> bytes:
        n = len(self.X)
        pts = torch.cat([self.u, self.B, self.Bp, self.Ap, self.Cp, self.Dp, self.FpK, self.FpC])
        return b"".join([n.to_bytes(8, "little"), self.X.to_bytes(), self.Y.to_bytes(),
                         bn.g1_aff_to_bytes(nt.g1_to_affine(pts.contiguous())).tobytes(),
                         bn.scalars_to_bytes(torch.cat([self.kB, self.kE])).tobytes(),
                         b"".join(O.scalar_to_bytes(x) for x in (self.kA, self.kC, self.kD, self.kF))])

    @staticmethod
    def from_bytes(b: bytes, device="cpu") -> "ShuffleProof":
        n = int.from_bytes(b[:8], "little")
        o = 8
        X = CipherVector.from_bytes(b[o: o + 128 * n], device); o += 128 * n
        Y = CipherVector.from_bytes(b[o: o + 128 * n], device); o += 128 * n
        m = 3 * n + 5
        pts = nt.g1_from_affine(bn.g1_aff_from_bytes(np.frombuffer(b[o: o + 64 * m], dtype=np.uint8), device))
        o += 64 * m
        sc = bn.scalars_from_bytes(np.frombuffer(b[o: o + 64 * n], dtype=np.uint8), device)
        o += 64 * n
        kA, kC, kD, kF = (int.from_bytes(b[o + 32 * i: o + 32 * i + 32], "big") for i in range(4))
        u, B, Bp = pts[:n], pts[n:2 * n], pts[2 * n:3 * n]
        s5 = [pts[3 * n + i: 3 * n + i + 1] for i in range(5)]
        return ShuffleProof(X, Y, u, B, s5[0], Bp, s5[1], s5[2], s5[3], s5[4], kA, sc[:n], kC, kD, sc[n:], kF)


# ----------------------------------------------------------------------------- prover / verifier
def prove(X: CipherVector, Y: CipherVector, perm: torch.Tensor, s: torch.Tensor, P_point) -> ShuffleProof:
    """Y_j = X_{perm[j]} + Enc0(s_j)."""
    dev = X.device
    N = len(X)
    h = generators(N, dev)
    pk = pk_table(P_point, dev)
    tabB, tabP = pk.tabB, pk.tabP
    perm = perm.to(dev).long()
    r = bn.random_scalars(N, dev)
    u = nt.g1_add(nt.g1_fb_mul(tabB, r), h.index_select(0, perm + 1).contiguous())
    t1, e = _challenge_e(P_point, X, Y, u)
    ep = torch.empty_like(e)
    ep[perm] = e                                       # e'_i = e_{pi^-1(i)}
    rho, c, sigma = _sum(_mul(e, r)), _sum(r), _sum(_mul(e, s))
    pref = _prefix_products(ep)
    beta = bn.random_scalars(N, dev)
    B = nt.g1_add(nt.g1_fb_mul(tabB, beta), nt.g1_fb_mul(_h0_table(dev), pref))
    beta_prev = torch.cat([torch.zeros((1, 8), dtype=torch.int32, device=dev), beta[:-1]])
    b = _sub(beta, _mul(ep, beta_prev))
    d = beta[N - 1: N]
    alpha, gamma, delta, phi = (bn.random_scalars(1, dev) for _ in range(4))
    eps = bn.random_scalars(N, dev)
    betap = bn.random_scalars(N, dev)

    def msm(pts, ks):  # -> [1, 24] on dev
        return nt.g1_msm(pts.contiguous(), ks.contiguous()).to(dev)

    Ap = nt.g1_add(msm(h[1:], eps), nt.g1_fb_mul(tabB, alpha))
    Bprev = torch.cat([h[:1], B[:-1]])
    Bp = nt.g1_add(nt.g1_fb_mul(tabB, betap), nt.g1_mul(Bprev.contiguous(), eps))
    Cp = nt.g1_fb_mul(tabB, gamma)
    Dp = nt.g1_fb_mul(tabB, delta)
    FpK = nt.g1_add(msm(X.K, eps), nt.g1_fb_mul(tabB, phi))
    FpC = nt.g1_add(msm(X.C, eps), nt.g1_fb_mul(tabP, phi))
    v = _challenge_v(t1, B, Bp, [Ap, Cp, Dp, FpK, FpC])
    vt = _sc(v, dev)
    kA = _to_int(_add(alpha, _mul(vt, rho)))
    kE = _add(eps, _mul(ep, vt.expand(N, 8)))
    kB = _add(betap, _mul(b, vt.expand(N, 8)))
    kC = _to_int(_add(gamma, _mul(vt, c)))
    kD = _to_int(_add(delta, _mul(vt, d)))
    kF = _to_int(_add(phi, _mul(vt, sigma)))
    return ShuffleProof(X, Y, u, B, Ap, Bp, Cp, Dp, FpK, FpC, kA, kB, kC, kD, kE, kF)


def verify(pr: ShuffleProof, P_point) -> bool:
    X, Y = pr.X, pr.Y
    N = len(X)
    dev = X.device
    if N == 0 or len(Y) != N or pr.u.shape[0] != N or pr.B.shape[0] != N or pr.Bp.shape[0] != N \
            or pr.kE.shape[0] != N or pr.kB.shape[0] != N:
        return False
    h = generators(N, dev)
    t1, e = _challenge_e(P_point, X, Y, pr.u)
    v = _challenge_v(t1, pr.B, pr.Bp, [pr.Ap, pr.Cp, pr.Dp, pr.FpK, pr.FpC])
    vt = _sc(v, dev)
    lam = _rand64(5, dev)
    l1, l3, l4, l5, l6 = (lam[i: i + 1] for i in range(5))
    mu = _rand64(N, dev)
    kE, kB = pr.kE.to(dev), pr.kB.to(dev)
    ve = lambda t: t.expand(N, 8)  # noqa: E731
    prod_e = _prefix_products(e)[N - 1: N]
    v_l3 = _mul(vt, l3)
    # scalars of every point of the combined equation (see module docstring)
    s_g = _add(_add(_add(_mul(l1, _sc(pr.kA, dev)), _sum(_mul(mu, kB))),
                    _add(_mul(l3, _sc(pr.kC, dev)), _mul(l4, _sc(pr.kD, dev)))), _mul(l5, _sc(pr.kF, dev)))
    s_P = _mul(l6, _sc(pr.kF, dev))
    s_h0 = _add(_mul(mu[:1], kE[:1]), _mul(_mul(vt, l4), prod_e))
    s_h = _add(_mul(ve(l1), kE), ve(v_l3))
    mu_next_kE = _mul(mu[1:], kE[1:])
    s_B = _neg(_mul(ve(vt), mu))
    s_B = torch.cat([_add(s_B[:-1], mu_next_kE), _sub(s_B[-1:], _mul(vt, l4))])
    s_Bp = _neg(mu)
    s_u = _neg(_add(_mul(ve(_mul(vt, l1)), e), ve(v_l3)))
    s_XK, s_XC = _mul(ve(l5), kE), _mul(ve(l6), kE)
    s_YK, s_YC = _neg(_mul(ve(_mul(vt, l5)), e)), _neg(_mul(ve(_mul(vt, l6)), e))
    singles = [_neg(l1), _neg(l3), _neg(l4), _neg(l5), _neg(l6)]
    pts = torch.cat([bn.g1_jac_tensor([O.G1_GEN, P_point], dev), h, pr.B, pr.Bp, pr.u, X.K, X.C, Y.K, Y.C,
                     pr.Ap, pr.Cp, pr.Dp, pr.FpK, pr.FpC])
    ks = torch.cat([s_g, s_P, s_h0, s_h, s_B, s_Bp, s_u, s_XK, s_XC, s_YK, s_YC] + singles)
    res = nt.g1_msm(pts.contiguous(), ks.contiguous())
    return not bool(res[0, 16:24].any())
