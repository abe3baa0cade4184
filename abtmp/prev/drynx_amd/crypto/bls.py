"""BLS multi-signatures over BN254 with BDN rogue-key-safe aggregation — the
collective signature on skipchain forward links.

Reference: the VNs' skipchain (cothority skipchain, ``CreateGenesis`` /
``StoreSkipBlock`` at services/service_skipchain.go:498-525) is collectively
signed by the roster with BLS/BDN CoSi over bn256.  Here:

  * keys      x in Fr, public X2 = x B2 in G2 (each VN derives it from its
              node secret);
  * sign      sigma = x H(m), H a try-and-increment hash onto G1 (BN254 G1 has
              cofactor 1, so every curve point is in the group);
  * aggregate BDN coefficients t_i = H'(i, X2_0 .. X2_{n-1}) (128 bits):
              sigma = sum t_i sigma_i, apk = sum t_i X2_i over the signers of a
              participation mask — a forged "rogue" key cannot cancel honest
              keys because the coefficients bind the whole roster;
  * verify    e(sigma, -B2) * e(H(m), apk) == 1: one two-term Miller product and
              one final exponentiation (native pairing ops, host or device).

Parity: the hash-to-curve and coefficient hashes are this framework's own
(kyber's bn256 hash-to-G1 and BDN coefficient derivation are not available
offline); the algebra and the security notion are the cothority ones.
"""
from __future__ import annotations

import hashlib

import torch

from .. import native as nt
from . import bn254 as bn
from . import oracle as O

_H2C_TAG = b"DXBLS1-H2G1"
_COEF_TAG = b"DXBLS1-BDN"
_SQRT_EXP = (O.P + 1) // 4  # p = 3 mod 4


def hash_to_g1(msg: bytes) -> tuple:
    """Try-and-increment map to G1: x = H(tag || ctr || msg) mod p until
    x^3 + 3 is a square; the parity of y is fixed by one more hash bit."""
    ctr = 0
    while True:
        d = hashlib.sha512(_H2C_TAG + ctr.to_bytes(4, "big") + msg).digest()
        x = int.from_bytes(d[:48], "big") % O.P
        rhs = (x * x * x + O.B1) % O.P
        y = pow(rhs, _SQRT_EXP, O.P)
        if y * y % O.P == rhs:
            if (y & 1) != (d[48] & 1):
                y = (O.P - y) % O.P
            return (x, y)
        ctr += 1


def public_key(secret: int) -> tuple:
    """X2 = x B2 (G2, oracle affine form) on the native host path."""
    aff = nt.g2_fb_mul(bn.base2_table("cpu"), bn.scalars_tensor([secret % O.R], "cpu"))
    return bn.g2_points_from_aff(aff)[0]


def sign(secret: int, msg: bytes) -> tuple:
    return bn.g1_mul_point(secret % O.R, hash_to_g1(msg))


def hash_to_g1_many(msgs: list, tries: int = 4) -> list:
    """``hash_to_g1`` of several messages: the first ``tries`` candidates of
    every message get their square roots in ONE native host batch (the map
    needs ~2 on average); a message whose candidates all fail continues on
    the scalar path.  Same points as ``hash_to_g1``."""
    cand = []
    for m in msgs:
        for ctr in range(tries):
            d = hashlib.sha512(_H2C_TAG + ctr.to_bytes(4, "big") + m).digest()
            x = int.from_bytes(d[:48], "big") % O.P
            cand.append((x, d[48] & 1))
    roots = nt.fp_sqrt_host([(x * x * x + O.B1) % O.P for x, _ in cand])
    out = []
    for i, m in enumerate(msgs):
        pt = None
        for ctr in range(tries):
            (x, bit), y = cand[i * tries + ctr], roots[i * tries + ctr]
            if y is not None:
                pt = (x, y if (y & 1) == bit else (O.P - y) % O.P)
                break
        out.append(pt if pt is not None else hash_to_g1(m))
    return out


def sign_many(items: list) -> list:
    """[(secret, msg)] -> signatures, all scalar multiplications in ONE native
    batch (the VNs co-hosted on a rank sign a block and a forward link each)."""
    if not items:
        return []
    pts = bn.g1_jac_tensor(hash_to_g1_many([m for _, m in items]), "cpu")
    ks = bn.scalars_tensor([sk % O.R for sk, _ in items], "cpu")
    return bn.g1_points_from_jac(nt.g1_mul(pts, ks))


def bdn_coefficients(publics: list) -> list:
    """t_i = first 128 bits of SHA-256(tag || i || X2_0 || ... || X2_{n-1})."""
    h = hashlib.sha256(_COEF_TAG)
    for p in publics:
        h.update(O.g2_to_bytes(p))
    base = h.digest()
    return [int.from_bytes(hashlib.sha256(base + i.to_bytes(4, "big")).digest()[:16], "big") | 1
            for i in range(len(publics))]


def aggregate(publics: list, partials: dict) -> tuple:
    """Aggregate signature of the signers in ``partials`` (index -> sigma_i)."""
    t = bdn_coefficients(publics)
    items = sorted(partials.items())
    if not items:
        return None
    # every t_i sigma_i in one native batch, then one sum
    prods = nt.g1_mul(bn.g1_jac_tensor([s for _, s in items], "cpu"),
                      bn.scalars_tensor([t[i] for i, _ in items], "cpu"))
    return bn.g1_points_from_jac(nt.g1_sum(prods.view(-1, 1, 24)))[0]


_subgroup_ok: dict = {}


def in_g2(pk) -> bool:
    """Prime-order subgroup check r * X2 == O (G2 has a large cofactor), cached per key."""
    if pk is None:
        return False
    k = O.g2_to_bytes(pk)
    if k not in _subgroup_ok:
        r_limbs = bn.to_tensor(bn.ints_to_limbs([O.R]), "cpu")  # r itself (not reduced mod r)
        out = nt.g2_mul(bn.g2_aff_tensor([pk], "cpu"), r_limbs)
        _subgroup_ok[k] = not bool(out.any())
    return _subgroup_ok[k]


def aggregate_public(publics: list, mask: list):
    """sum t_i X2_i over the mask; None if any key is outside the G2 subgroup."""
    t = bdn_coefficients(publics)
    acc = None
    for i, on in enumerate(mask):
        if on:
            if not in_g2(publics[i]):
                return None
            acc = O.g2_add(acc, _g2_mul(t[i], publics[i]))
    return acc


def _g2_mul(k: int, pt):
    out = nt.g2_mul(bn.g2_aff_tensor([pt], "cpu"), bn.scalars_tensor([k], "cpu"))
    return bn.g2_points_from_aff(out)[0]


def verify(apk, msg: bytes, sig) -> bool:
    """e(sig, -B2) e(H(m), apk) == 1 (one Miller product, one final exp)."""
    if apk is None or sig is None or not O.g1_on_curve(sig):
        return False
    P = bn.g1_aff_tensor([sig, hash_to_g1(msg)], "cpu")
    Q = bn.g2_aff_tensor([O.g2_neg(O.G2_GEN), apk], "cpu")
    f = nt.miller_loop(P, Q)
    e = nt.final_exp(nt.gt_mul(f[0:1].contiguous(), f[1:2].contiguous()))
    return bool(torch.equal(e, nt.gt_one("cpu")))


def verify_multi(publics: list, mask: list, msg: bytes, sig) -> bool:
    return verify(aggregate_public(publics, mask), msg, sig)


def mask_to_hex(mask: list) -> str:
    v = 0
    for i, on in enumerate(mask):
        if on:
            v |= 1 << i
    return f"{len(mask)}:{v:x}"


def mask_from_hex(s: str) -> list:
    n, v = s.split(":")
    v = int(v, 16)
    return [bool((v >> i) & 1) for i in range(int(n))]
