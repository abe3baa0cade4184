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


def fs_challenge(context: str, *parts) -> int:
    """SHA-256 Fiat–Shamir challenge over the context and the affine encodings
    of every point: all point tensors are normalised in ONE batched launch
    (a transcript is 4-7 vectors of thousands of points)."""
    return fs_challenges([(context, parts)])[0]


def fs_challenges(specs) -> list:
    """Challenges of several transcripts [(context, parts), ...] with ONE
    to_affine launch for all their points (short vectors are latency-bound)."""
    jacs, layouts = [], []
    for context, parts in specs:
        layout = [("raw", context.encode())]
        for p in parts:
            if isinstance(p, torch.Tensor):
                jacs.append(p.contiguous().view(-1, 24))
                layout.append(("pts", jacs[-1].shape[0]))
            elif isinstance(p, CipherVector):
                for t in (p.K, p.C):
                    jacs.append(t.contiguous().view(-1, 24))
                    layout.append(("pts", jacs[-1].shape[0]))
            else:
                layout.append(("raw", p if isinstance(p, (bytes, bytearray)) else str(p).encode()))
        layouts.append(layout)
    allb = _aff_bytes(torch.cat(jacs)) if jacs else b""
    out, o = [], 0
    for layout in layouts:
        h = hashlib.sha256()
        for kind, v in layout:
            if kind == "pts":
                h.update(allb[o: o + 64 * v])
                o += 64 * v
            else:
                h.update(v)
        out.append(int.from_bytes(h.digest(), "big") % O.R)
    return out


def _rand64(n: int, device) -> torch.Tensor:
    """Random nonzero 64-bit batch weights (device CSPRNG), unknown to provers."""
    r = bn.random_scalars(n, device)
    r[:, 2:] = 0
    r[:, 0] |= 1
    return r


def _msm_is_zero(points: list, scalars: list) -> bool:
    """sum_i k_i P_i == O over the concatenated lists (one Pippenger MSM)."""
    res = nt.g1_msm(torch.cat(points).contiguous(), torch.cat(scalars).contiguous())
    return not bool(res[0, 16:24].any())


def _fr_sum(x: torch.Tensor) -> torch.Tensor:
    """[m, 8] -> [1, 8] Fr sum (pairwise tree on the device)."""
    cur = x
    while cur.shape[0] > 1:
        if cur.shape[0] % 2:
            cur = torch.cat([cur, torch.zeros((1, 8), dtype=torch.int32, device=cur.device)])
        cur = nt.fr_arith(nt.FR_ADD, cur[0::2].contiguous(), cur[1::2].contiguous())
    return cur


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
    dev = torch.device(device)
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
    dev = torch.device(device)
    lhs = nt.g1_fb_mul(bn.base_table(dev), _sc(s, dev))
    rhs = nt.g1_add(bn.g1_jac_tensor(R, dev), nt.g1_mul(bn.g1_jac_tensor(X, dev), _sc(e, dev)))
    ok = nt.g1_eq(lhs, rhs).cpu().tolist()
    for i, v in zip(idx, ok):
        out[i] = bool(v)
    return out


# ----------------------------------------------------------------------------- obfuscation (DLEQ)
@dataclass
class ObfuscationProof:
    C: CipherVector     # before
    Co: CipherVector    # after (s_i * C_i)
    T: CipherVector     # commitments (a_i K_i, a_i C_i)
    c: int
    z: torch.Tensor     # [n, 8]

    def to_bytes(self) -> bytes:
        return b"".join([len(self.C).to_bytes(8, "little"), self.C.to_bytes(), self.Co.to_bytes(), self.T.to_bytes(),
                         O.scalar_to_bytes(self.c), bn.scalars_to_bytes(self.z).tobytes()])

    @staticmethod
    def from_bytes(b: bytes, device="cpu") -> "ObfuscationProof":
        n = int.from_bytes(b[:8], "little")
        o = 8
        cvs = []
        for _ in range(3):
            cvs.append(CipherVector.from_bytes(b[o: o + 128 * n], device))
            o += 128 * n
        c = int.from_bytes(b[o: o + 32], "big")
        o += 32
        z = bn.scalars_from_bytes(np.frombuffer(b[o: o + 32 * n], dtype=np.uint8), device)
        return ObfuscationProof(cvs[0], cvs[1], cvs[2], c, z)


def obfuscation_list_proof_creation(C: CipherVector, Co: CipherVector, s: torch.Tensor) -> ObfuscationProof:
    """ObfuscationListProofCreation: per element DLEQ log_{K}(Ko) == log_{C}(Co) == s_i."""
    dev = C.device
    a = bn.random_scalars(len(C), dev)
    T = C.mul_scalars(a)
    c = fs_challenge("proofTest/obfuscation", C, Co, T)
    z = nt.fr_arith(nt.FR_ADD, a, nt.fr_arith(nt.FR_MUL, s, _sc([c], dev)))
    return ObfuscationProof(C, Co, T, c, z)


def obfuscation_list_proof_verification(pr: ObfuscationProof, threshold: float = 1.0) -> bool:
    """ObfuscationListProofVerification(percent): z K == T1 + c Ko and z C == T2 + c Co
    for the first ceil(threshold * n) elements (reference sampling)."""
    n = len(pr.C)
    k = _first(n, threshold)
    if k == 0:
        return True
    if fs_challenge("proofTest/obfuscation", pr.C, pr.Co, pr.T) != pr.c:
        return False
    dev = pr.C.device
    c = _sc([pr.c], dev)
    Cs, Cos, Ts, z = pr.C[:k], pr.Co[:k], pr.T[:k], pr.z[:k].contiguous()
    lhs = Cs.mul_scalars(z)
    rhs = Ts.add(Cos.mul_scalars(c))
    return bool(nt.g1_eq(lhs.K, rhs.K).all()) and bool(nt.g1_eq(lhs.C, rhs.C).all())


# ----------------------------------------------------------------------------- key switching
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

    def to_bytes(self) -> bytes:
        n = self.K.shape[0]
        cached = getattr(self, "_aff", None)  # affine encodings kept from the prover's transcript
        Kb, shb, t1b, t2b = cached if cached is not None else (
            _aff_bytes(self.K), self.share.to_bytes(), _aff_bytes(self.T1), _aff_bytes(self.T2))
        return b"".join([n.to_bytes(8, "little"), O.g1_to_bytes(self.X), O.g1_to_bytes(self.Q), Kb, shb, t1b, t2b,
                         self.T3,
                         O.scalar_to_bytes(self.c), bn.scalars_to_bytes(self.za).tobytes(),
                         O.scalar_to_bytes(self.zb)])

    @staticmethod
    def from_bytes(b: bytes, device="cpu") -> "KeySwitchProof":
        n = int.from_bytes(b[:8], "little")
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
        return KeySwitchProof(X, Q, K, share, T1, T2, T3, c, za, zb)


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


def key_switch_shares_batch(secrets: list, publics: list, K: torch.Tensor, Q_point, with_proofs: bool):
    """Key-switching shares (and proofs) of several co-located CNs over the same
    K vector in a handful of launches sized (#CNs x n) instead of per CN."""
    from ..crypto.elgamal import pk_table

    dev = K.device
    n, c = K.shape[0], len(secrets)
    tabB = bn.base_table(dev)
    tabQ = pk_table(Q_point, dev).tabP
    Kt = K.repeat(c, 1).contiguous()
    x_rep = torch.cat([_sc([x], dev).expand(n, 8) for x in secrets]).contiguous()
    v = bn.random_scalars(c * n, dev)
    scal = [x_rep]
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
    out = []
    if with_proofs:
        with timers.span("ks.commit"):
            a = bn.random_scalars(c * n, dev)
            T1 = nt.g1_fb_mul(tabB, a)
            T2 = nt.g1_add(nt.g1_fb_mul(tabQ, a), prods[c * n:].contiguous(), subtract=True)
    if not with_proofs:
        return [(shares_all[j * n:(j + 1) * n], None) for j in range(c)]
    # every CN's transcript in ONE normalisation launch; the affine encodings are
    # kept on the proofs so marshalling them later needs no further launch
    T3s = [O.g1_to_bytes(bn.g1_mul_point(b)) for b in bs]
    with timers.span("ks.affine"):
        aff = _aff_bytes(torch.cat([K, shares_all.K, shares_all.C, T1, T2]))
    seg = 64 * n
    Kb = aff[:seg]

    def part(block, j):
        o = seg * (1 + block * c + j)
        return aff[o: o + seg]

    Qb = O.g1_to_bytes(Q_point)
    for j in range(c):
        sl = slice(j * n, (j + 1) * n)
        share = shares_all[sl]
        t1, t2 = T1[sl].contiguous(), T2[sl].contiguous()
        sKb, sCb, t1b, t2b = part(0, j), part(1, j), part(2, j), part(3, j)
        with timers.span("ks.hash"):
            h = hashlib.sha256()
            for piece in (b"proofTest/keyswitch", O.g1_to_bytes(publics[j]), Qb, Kb, sKb, sCb, t1b, t2b, T3s[j]):
                h.update(piece)
        ch = int.from_bytes(h.digest(), "big") % O.R
        za = nt.fr_arith(nt.FR_ADD, a[sl].contiguous(), nt.fr_arith(nt.FR_MUL, v[sl].contiguous(), _sc([ch], dev)))
        pr = KeySwitchProof(publics[j], Q_point, K, share, t1, t2, T3s[j], ch, za, (bs[j] + ch * secrets[j]) % O.R)
        shb = np.concatenate([np.frombuffer(sKb, np.uint8).reshape(n, 64),
                              np.frombuffer(sCb, np.uint8).reshape(n, 64)], axis=1).tobytes()
        pr._aff = (Kb, shb, t1b, t2b)
        out.append((share, pr))
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
    c = fs_challenge("proofTest/keyswitch", O.g1_to_bytes(X), O.g1_to_bytes(Q_point), K, share, T1, T2, T3)
    za = nt.fr_arith(nt.FR_ADD, a, nt.fr_arith(nt.FR_MUL, v, _sc([c], dev)))
    zb = (b + c * x) % O.R
    return KeySwitchProof(X, Q_point, K, share, T1, T2, T3, c, za, zb)


def key_switch_batch_verification(proofs: list, threshold: float = 1.0, combine: bool = True) -> list:
    """Verify several CNs' key-switch proofs (same querier key) as ONE random
    linear combination: with fresh 64-bit weights rho_i, sig_i per element,
      (sum rho za) B + (sum sig za) Q - sum rho T1 - sum c rho (vB)
        - sum zb sig K - sum sig T2 - sum c sig (vQ - xK) == O
    is one Pippenger MSM (no per-element 256-step chains; soundness error
    2^-64).  If the combined check fails, each proof is re-checked alone so the
    bitmap blames exactly the bad ones."""
    if not proofs:
        return []
    # weight-free part (recomputed challenge, the x-part T3 check): a property
    # of the proof data, computed once per decoded proof and shared by the
    # verifying nodes co-hosted on this rank (each keeps its own random weights)
    todo = [pr for pr in proofs if getattr(pr, "_fs_ok", None) is None]
    if todo:
        with timers.span("ks.verify.challenges"):
            cs = fs_challenges([("proofTest/keyswitch", (O.g1_to_bytes(pr.X), O.g1_to_bytes(pr.Q), pr.K, pr.share,
                                                         pr.T1, pr.T2, pr.T3)) for pr in todo])
            for pr, c in zip(todo, cs):
                pr._fs_ok = c == pr.c and bn.g1_mul_point(pr.zb) == O.g1_add(O.g1_from_bytes(pr.T3),
                                                                             bn.g1_mul_point(c, pr.X))
    ok, live = [], []
    for pr in proofs:
        k = _first(pr.K.shape[0], threshold)
        ok.append(pr._fs_ok)
        if pr._fs_ok and k > 0:
            live.append((len(ok) - 1, pr, k))
    if not live or not combine:
        return ok
    with timers.span("ks.verify.msm"):
        if _ks_combined(live)[0]:
            return ok
    for idx, pr, k in live:
        ok[idx] = _ks_combined([(idx, pr, k)])[0]
    return ok


def key_switch_batch_verification_multi(proofs: list, threshold: float, n_vn: int) -> list:
    """``key_switch_batch_verification`` for ``n_vn`` verifying nodes hosted on
    one rank: the weight-free part once, every VN's random combination in ONE
    grouped MSM (one bucket plan and host sync instead of one per VN), each
    VN's verdict from its own weights.  -> [per-VN list of bools]."""
    if not proofs:
        return [[] for _ in range(n_vn)]
    ok = key_switch_batch_verification(proofs, threshold, combine=False)
    live = [(i, pr, _first(pr.K.shape[0], threshold)) for i, pr in enumerate(proofs)]
    live = [(i, pr, k) for i, pr, k in live if ok[i] and k > 0]
    if not live:
        return [list(ok) for _ in range(n_vn)]
    with timers.span("ks.verify.msm_multi"):
        verdicts = _ks_combined(live, n_vn)
    out = []
    for v in range(n_vn):
        res = list(ok)
        if not verdicts[v]:  # this VN's own per-proof re-check blames the bad ones
            for idx, pr, k in live:
                res[idx] = _ks_combined([(idx, pr, k)])[0]
        out.append(res)
    return out


def _ks_combined(live, n_vn: int = 1):
    """Grouped MSM: every per-element weight stays 64 bit (8 bucket additions
    per point instead of 32); the per-proof challenges c, zb multiply the five
    group sums of each proof on the host.  ``n_vn`` independent combinations
    (fresh weights each) share the one MSM launch -> [bool] per combination."""
    dev = live[0][1].K.device
    nl = len(live)
    pts, scs, grp = [], [], []
    sB, sQ = [], []
    for v in range(n_vn):
        for j, (_, pr, k) in enumerate(live):
            rho, sig = _rand64(k, dev), _rand64(k, dev)
            za = pr.za[:k].contiguous()
            # group 5j+0: rho T1, +1: rho vB, +2: sig K (x zb), +3: sig T2, +4: sig (vQ - xK) (x c)
            for gi, (pt, w) in enumerate(((pr.T1, rho), (pr.share.K, rho), (pr.K, sig), (pr.T2, sig),
                                          (pr.share.C, sig))):
                pts.append(pt[:k])
                scs.append(w)
                grp.append(torch.full((k,), (v * nl + j) * 5 + gi, dtype=torch.int32, device=dev))
            sB.append(_fr_sum(nt.fr_arith(nt.FR_MUL, rho, za)))
            sQ.append(_fr_sum(nt.fr_arith(nt.FR_MUL, sig, za)))
    G = nt.g1_msm_grouped(torch.cat(pts).contiguous(), torch.cat(scs).contiguous(), torch.cat(grp),
                          5 * nl * n_vn, bits=64)
    Q = live[0][1].Q
    out = []
    for v in range(n_vn):
        full = torch.cat([_fr_sum(torch.cat(sB[v * nl:(v + 1) * nl])),
                          _fr_sum(torch.cat(sQ[v * nl:(v + 1) * nl]))]).cpu()
        # lhs = (sum rho za) B + (sum sig za) Q; rhs = sum_j G0 + c G1 + zb G2 + G3 + c G4
        lhs = nt.g1_add(*nt.g1_mul(bn.g1_jac_tensor([O.G1_GEN, Q], "cpu"), full).split(1))
        facs, fpts = [], []
        for j, (_, pr, _) in enumerate(live):
            g = G[5 * (v * nl + j): 5 * (v * nl + j) + 5]
            facs += [1, pr.c, pr.zb, 1, pr.c]
            fpts.append(g)
        rhs = nt.g1_sum(nt.g1_mul(torch.cat(fpts).contiguous(), _sc(facs, "cpu")).view(-1, 1, 24))
        out.append(bool(nt.g1_eq(lhs, rhs)[0]))
    return out


def obfuscation_batch_verification(proofs: list, threshold: float = 1.0) -> list:
    """Several CNs' obfuscation proofs as one random linear combination:
      sum rho (z K - T1 - c Ko) + sum sig (z C - T2 - c Co) == O
    (one MSM; per-proof re-check only if the combination fails)."""
    if not proofs:
        return []
    todo = [pr for pr in proofs if getattr(pr, "_fs_ok", None) is None]   # shared by co-hosted VNs
    if todo:
        for pr, c in zip(todo, fs_challenges([("proofTest/obfuscation", (pr.C, pr.Co, pr.T)) for pr in todo])):
            pr._fs_ok = c == pr.c
    ok, live = [], []
    for pr in proofs:
        k = _first(len(pr.C), threshold)
        good = pr._fs_ok
        ok.append(good)
        if good and k > 0:
            live.append((len(ok) - 1, pr, k))
    if not live:
        return ok
    if _obf_combined(live):
        return ok
    for idx, pr, k in live:
        ok[idx] = _obf_combined([(idx, pr, k)])
    return ok


def _obf_combined(live) -> bool:
    """Grouped MSM: rho z K + sig z C (full-size weights), rho T1 + sig T2
    and rho Ko + sig Co (64-bit weights, the latter times c on the host)."""
    dev = live[0][1].C.device
    pts, scs, grp = [], [], []
    for j, (_, pr, k) in enumerate(live):
        rho, sig = _rand64(k, dev), _rand64(k, dev)
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
    c = fs_challenge("proofTest/keyswitch", O.g1_to_bytes(pr.X), O.g1_to_bytes(pr.Q), pr.K, pr.share, pr.T1, pr.T2,
                     pr.T3)
    if c != pr.c:
        return False
    # zb B == T3 + c X
    T3 = O.g1_from_bytes(pr.T3)
    if bn.g1_mul_point(pr.zb) != O.g1_add(T3, bn.g1_mul_point(c, pr.X)):
        return False
    dev = pr.K.device
    tabB = bn.base_table(dev)
    tabQ = pk_table(pr.Q, dev).tabP
    cs = _sc([c], dev)
    za = pr.za[:k].contiguous()
    # za B == T1 + c (vB)
    ok1 = nt.g1_eq(nt.g1_fb_mul(tabB, za),
                   nt.g1_add(pr.T1[:k].contiguous(), nt.g1_mul(pr.share.K[:k].contiguous(), cs)))
    # za Q - zb K == T2 + c (vQ - xK)
    lhs = nt.g1_add(nt.g1_fb_mul(tabQ, za), nt.g1_mul(pr.K[:k].contiguous(), _sc([pr.zb], dev)), subtract=True)
    rhs = nt.g1_add(pr.T2[:k].contiguous(), nt.g1_mul(pr.share.C[:k].contiguous(), cs))
    ok2 = nt.g1_eq(lhs, rhs)
    return bool(ok1.all()) and bool(ok2.all())
