"""Pure-Python BN254 golden model (slow, exact).

This is the ground truth every native (host C++ / HIP gfx950) kernel is tested
against.  It re-derives, from first principles, the group the reference uses:
``lib/suite.go:10`` sets ``bn256.NewSuiteG1()`` (kyber's cloudflare-derived
BN256 = BN254 / alt_bn128), and ``lib/range/range_proof.go:8,540-544`` needs
the optimal-ate pairing.

Tower (identical to the native code, so intermediate values compare 1:1):
    Fp2  = Fp[i]  / (i^2 + 1)
    Fp6  = Fp2[v] / (v^3 - xi),  xi = 9 + i
    Fp12 = Fp6[w] / (w^2 - v)
G1: y^2 = x^3 + 3 over Fp, generator (1, -2) (cloudflare ``curveGen``).
G2: y^2 = x^3 + 3/xi over Fp2 (D-type twist), EIP-197 generator.

The pairing here is the textbook definition (affine Miller loop on the
untwisted curve over Fp12, final exponentiation by (p^12-1)/r using Python
``pow``).  The fast final-exponentiation chain used natively is also provided
(``final_exp_fast``) and checked against the textbook one in the tests.
"""
from __future__ import annotations

import hashlib
import secrets

U = 4965661367192848881
P = 36 * U**4 + 36 * U**3 + 24 * U**2 + 6 * U + 1
R = 36 * U**4 + 36 * U**3 + 18 * U**2 + 6 * U + 1
assert P == 21888242871839275222246405745257275088696311157297823662689037894645226208583
assert R == 21888242871839275222246405745257275088548364400416034343698204186575808495617


def inv_mod(a: int, m: int) -> int:
    return pow(a % m, -1, m)


# ----------------------------------------------------------------------------- Fp2
class Fp2:
    __slots__ = ("c0", "c1")

    def __init__(self, c0: int = 0, c1: int = 0):
        self.c0 = c0 % P
        self.c1 = c1 % P

    @staticmethod
    def zero():
        return Fp2(0, 0)

    @staticmethod
    def one():
        return Fp2(1, 0)

    def __add__(self, o):
        return Fp2(self.c0 + o.c0, self.c1 + o.c1)

    def __sub__(self, o):
        return Fp2(self.c0 - o.c0, self.c1 - o.c1)

    def __neg__(self):
        return Fp2(-self.c0, -self.c1)

    def __mul__(self, o):
        if isinstance(o, int):
            return Fp2(self.c0 * o, self.c1 * o)
        return Fp2(self.c0 * o.c0 - self.c1 * o.c1, self.c0 * o.c1 + self.c1 * o.c0)

    __rmul__ = __mul__

    def __eq__(self, o):
        return self.c0 == o.c0 and self.c1 == o.c1

    def __hash__(self):
        return hash((self.c0, self.c1))

    def is_zero(self):
        return self.c0 == 0 and self.c1 == 0

    def conj(self):
        return Fp2(self.c0, -self.c1)

    def inv(self):
        t = inv_mod(self.c0 * self.c0 + self.c1 * self.c1, P)
        return Fp2(self.c0 * t, -self.c1 * t)

    def mul_xi(self):  # * (9 + i)
        return Fp2(9 * self.c0 - self.c1, 9 * self.c1 + self.c0)

    def __pow__(self, e: int):
        res, b = Fp2.one(), self
        while e:
            if e & 1:
                res = res * b
            b = b * b
            e >>= 1
        return res

    def __repr__(self):
        return f"Fp2({hex(self.c0)}, {hex(self.c1)})"


XI = Fp2(9, 1)


# ----------------------------------------------------------------------------- Fp6
class Fp6:
    __slots__ = ("c0", "c1", "c2")

    def __init__(self, c0: Fp2, c1: Fp2, c2: Fp2):
        self.c0, self.c1, self.c2 = c0, c1, c2

    @staticmethod
    def zero():
        return Fp6(Fp2.zero(), Fp2.zero(), Fp2.zero())

    @staticmethod
    def one():
        return Fp6(Fp2.one(), Fp2.zero(), Fp2.zero())

    def __add__(self, o):
        return Fp6(self.c0 + o.c0, self.c1 + o.c1, self.c2 + o.c2)

    def __sub__(self, o):
        return Fp6(self.c0 - o.c0, self.c1 - o.c1, self.c2 - o.c2)

    def __neg__(self):
        return Fp6(-self.c0, -self.c1, -self.c2)

    def __mul__(self, o):
        if isinstance(o, Fp2):
            return Fp6(self.c0 * o, self.c1 * o, self.c2 * o)
        a0, a1, a2 = self.c0, self.c1, self.c2
        b0, b1, b2 = o.c0, o.c1, o.c2
        t0, t1, t2 = a0 * b0, a1 * b1, a2 * b2
        c0 = t0 + ((a1 * b2) + (a2 * b1)).mul_xi()
        c1 = (a0 * b1) + (a1 * b0) + t2.mul_xi()
        c2 = (a0 * b2) + (a2 * b0) + t1
        return Fp6(c0, c1, c2)

    def mul_v(self):  # * v
        return Fp6(self.c2.mul_xi(), self.c0, self.c1)

    def __eq__(self, o):
        return self.c0 == o.c0 and self.c1 == o.c1 and self.c2 == o.c2

    def is_zero(self):
        return self.c0.is_zero() and self.c1.is_zero() and self.c2.is_zero()

    def inv(self):
        a0, a1, a2 = self.c0, self.c1, self.c2
        A = a0 * a0 - (a1 * a2).mul_xi()
        B = (a2 * a2).mul_xi() - a0 * a1
        C = a1 * a1 - a0 * a2
        F = a0 * A + ((a2 * B) + (a1 * C)).mul_xi()
        Fi = F.inv()
        return Fp6(A * Fi, B * Fi, C * Fi)


# ----------------------------------------------------------------------------- Fp12
class Fp12:
    __slots__ = ("c0", "c1")

    def __init__(self, c0: Fp6, c1: Fp6):
        self.c0, self.c1 = c0, c1

    @staticmethod
    def zero():
        return Fp12(Fp6.zero(), Fp6.zero())

    @staticmethod
    def one():
        return Fp12(Fp6.one(), Fp6.zero())

    def __add__(self, o):
        return Fp12(self.c0 + o.c0, self.c1 + o.c1)

    def __sub__(self, o):
        return Fp12(self.c0 - o.c0, self.c1 - o.c1)

    def __neg__(self):
        return Fp12(-self.c0, -self.c1)

    def __mul__(self, o):
        a0, a1, b0, b1 = self.c0, self.c1, o.c0, o.c1
        t0, t1 = a0 * b0, a1 * b1
        return Fp12(t0 + t1.mul_v(), (a0 + a1) * (b0 + b1) - t0 - t1)

    def __eq__(self, o):
        return self.c0 == o.c0 and self.c1 == o.c1

    def is_one(self):
        return self == Fp12.one()

    def conj(self):
        return Fp12(self.c0, -self.c1)

    def inv(self):
        t = (self.c0 * self.c0 - (self.c1 * self.c1).mul_v()).inv()
        return Fp12(self.c0 * t, -(self.c1 * t))

    def __pow__(self, e: int):
        if e < 0:
            return self.inv() ** (-e)
        res, b = Fp12.one(), self
        while e:
            if e & 1:
                res = res * b
            b = b * b
            e >>= 1
        return res

    def frob(self, k: int = 1):
        """x -> x^(p^k) (coefficient-wise Frobenius with precomputed gammas)."""
        out = self
        for _ in range(k):
            out = _frob1(out)
        return out

    def coeffs(self):
        """12 Fp2 -> 24 ints in native storage order (c0.c0.c0, c0.c0.c1, ...)."""
        out = []
        for f6 in (self.c0, self.c1):
            for f2 in (f6.c0, f6.c1, f6.c2):
                out += [f2.c0, f2.c1]
        return out

    @staticmethod
    def from_coeffs(c):
        f2 = [Fp2(c[2 * k], c[2 * k + 1]) for k in range(6)]
        return Fp12(Fp6(f2[0], f2[1], f2[2]), Fp6(f2[3], f2[4], f2[5]))


# Frobenius: element = sum_{k} a_k * W^k basis with w^k; for tower coefficient of
# v^j w^h (j in 0..2, h in 0..1) the exponent of w is e = 2j + h and
# (a w^e)^p = conj(a) * w^e * gamma_e, gamma_e = xi^{e (p-1)/6}.
GAMMA1 = [XI ** (e * (P - 1) // 6) for e in range(6)]


def _frob1(x: Fp12) -> Fp12:
    c = [x.c0.c0, x.c0.c1, x.c0.c2, x.c1.c0, x.c1.c1, x.c1.c2]
    # index k -> (j, h): k<3 -> (k,0) ; k>=3 -> (k-3,1); e = 2j+h
    out = []
    for k, a in enumerate(c):
        j, h = (k, 0) if k < 3 else (k - 3, 1)
        out.append(a.conj() * GAMMA1[2 * j + h])
    return Fp12(Fp6(out[0], out[1], out[2]), Fp6(out[3], out[4], out[5]))


# ----------------------------------------------------------------------------- curves
B1 = 3
B2 = Fp2(3, 0) * XI.inv()

G1_GEN = (1, P - 2)  # cloudflare/kyber curveGen = (1, -2)
G2_GEN = (
    Fp2(10857046999023057135944570762232829481370756359578518086990519993285655852781,
        11559732032986387107991004021392285783925812861821192530917403151452391805634),
    Fp2(8495653923123431417604973247489272438418190587263600148770280649306958101930,
        4082367875863433681332203403145435568316851327593401208105741076214120093531),
)


def g1_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B1) % P == 0


def g1_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        if (y1 + y2) % P == 0:
            return None
        lam = 3 * x1 * x1 * inv_mod(2 * y1, P) % P
    else:
        lam = (y2 - y1) * inv_mod(x2 - x1, P) % P
    x3 = (lam * lam - x1 - x2) % P
    return (x3, (lam * (x1 - x3) - y1) % P)


def g1_neg(a):
    return None if a is None else (a[0], (-a[1]) % P)


def g1_mul(k: int, pt):
    k %= R
    res, add = None, pt
    while k:
        if k & 1:
            res = g1_add(res, add)
        add = g1_add(add, add)
        k >>= 1
    return res


def g1_mul_signed(k: int, pt):
    """k may be negative (used for IntToPoint of negative ints)."""
    return g1_neg(g1_mul(-k, pt)) if k < 0 else g1_mul(k, pt)


def g2_on_curve(pt):
    if pt is None:
        return True
    x, y = pt
    return y * y - x * x * x - B2 == Fp2.zero()


def g2_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        if (y1 + y2).is_zero():
            return None
        lam = (x1 * x1 * 3) * (y1 * 2).inv()
    else:
        lam = (y2 - y1) * (x2 - x1).inv()
    x3 = lam * lam - x1 - x2
    return (x3, lam * (x1 - x3) - y1)


def g2_neg(a):
    return None if a is None else (a[0], -a[1])


def g2_mul(k: int, pt):
    k %= R
    res, add = None, pt
    while k:
        if k & 1:
            res = g2_add(res, add)
        add = g2_add(add, add)
        k >>= 1
    return res


assert g1_on_curve(G1_GEN) and g2_on_curve(G2_GEN)


# ----------------------------------------------------------------------------- pairing
def _fp12_from_fp(a: int) -> Fp12:
    return Fp12(Fp6(Fp2(a, 0), Fp2.zero(), Fp2.zero()), Fp6.zero())


def _fp12_from_fp2(a: Fp2) -> Fp12:
    return Fp12(Fp6(a, Fp2.zero(), Fp2.zero()), Fp6.zero())


W = Fp12(Fp6.zero(), Fp6.one())          # w
W2 = W * W                                # w^2 = v
W3 = W2 * W


def untwist(q):
    """psi: E'(Fp2) -> E(Fp12), (x, y) -> (x w^2, y w^3)."""
    x, y = q
    return (_fp12_from_fp2(x) * W2, _fp12_from_fp2(y) * W3)


def _e12_add(a, b):
    x1, y1 = a
    x2, y2 = b
    if x1 == x2:
        lam = (x1 * x1 * _fp12_from_fp(3)) * (y1 * _fp12_from_fp(2)).inv()
    else:
        lam = (y2 - y1) * (x2 - x1).inv()
    x3 = lam * lam - x1 - x2
    return (x3, lam * (x1 - x3) - y1), lam


def _line(t, lam, pxy):
    xt, yt = t
    px, py = pxy
    return (py - yt) - lam * (px - xt)


ATE_LOOP = 6 * U + 2


def miller_loop(p1, q2) -> Fp12:
    if p1 is None or q2 is None:
        return Fp12.one()
    Pp = (_fp12_from_fp(p1[0]), _fp12_from_fp(p1[1]))
    Q = untwist(q2)
    T = Q
    f = Fp12.one()
    bits = bin(ATE_LOOP)[3:]
    for bit in bits:
        T2, lam = _e12_add(T, T)
        f = f * f * _line(T, lam, Pp)
        T = T2
        if bit == "1":
            T3, lam = _e12_add(T, Q)
            f = f * _line(T, lam, Pp)
            T = T3
    Q1 = (Q[0].frob(1), Q[1].frob(1))
    Q2 = (Q[0].frob(2), -Q[1].frob(2))
    T3, lam = _e12_add(T, Q1)
    f = f * _line(T, lam, Pp)
    T = T3
    T3, lam = _e12_add(T, Q2)
    f = f * _line(T, lam, Pp)
    return f


FINAL_EXP = (P**12 - 1) // R


def final_exp(f: Fp12) -> Fp12:
    return f ** FINAL_EXP


def pairing(p1, q2) -> Fp12:
    return final_exp(miller_loop(p1, q2))


def _cyc_pow_u(f: Fp12) -> Fp12:
    return f ** U


def final_exp_fast(f: Fp12) -> Fp12:
    """Easy part + Scott et al. hard part (exact exponent (p^4-p^2+1)/r).

    Mirrors the native chain in csrc/bn254/pairing.h step for step.
    """
    t = f.conj() * f.inv()          # f^(p^6-1)
    t = t.frob(2) * t               # ^(p^2+1)
    fu = _cyc_pow_u(t)
    fu2 = _cyc_pow_u(fu)
    fu3 = _cyc_pow_u(fu2)
    y3 = fu.frob(1).conj()
    fu2p = fu2.frob(1)
    fu3p = fu3.frob(1)
    y2 = fu2.frob(2)
    y0 = t.frob(1) * t.frob(2) * t.frob(3)
    y1 = t.conj()
    y5 = fu2.conj()
    y4 = (fu * fu2p).conj()
    y6 = (fu3 * fu3p).conj()
    t0 = y6 * y6 * y4 * y5
    t1 = y3 * y5 * t0
    t0 = t0 * y2
    t1 = t1 * t1 * t0
    t1 = t1 * t1
    t0 = t1 * y1
    t1 = t1 * y0
    t0 = t0 * t0 * t1
    return t0


# ----------------------------------------------------------------------------- codecs (kyber layout)
def fp_to_bytes(a: int) -> bytes:
    return (a % P).to_bytes(32, "big")


def g1_to_bytes(pt) -> bytes:
    if pt is None:
        return b"\x00" * 64
    return fp_to_bytes(pt[0]) + fp_to_bytes(pt[1])


def g1_from_bytes(b: bytes):
    x, y = int.from_bytes(b[:32], "big"), int.from_bytes(b[32:64], "big")
    if x == 0 and y == 0:
        return None
    pt = (x, y)
    if not g1_on_curve(pt):
        raise ValueError("G1 point not on curve")
    return pt


def fp2_to_bytes(a: Fp2) -> bytes:  # cloudflare gfP2{x,y} = x*i + y: imaginary first
    return fp_to_bytes(a.c1) + fp_to_bytes(a.c0)


def g2_to_bytes(pt) -> bytes:
    if pt is None:
        return b"\x00" * 128
    return fp2_to_bytes(pt[0]) + fp2_to_bytes(pt[1])


def fp2_from_bytes(b: bytes) -> Fp2:
    return Fp2(int.from_bytes(b[32:64], "big"), int.from_bytes(b[:32], "big"))


def g2_from_bytes(b: bytes):
    if b == b"\x00" * 128:
        return None
    pt = (fp2_from_bytes(b[:64]), fp2_from_bytes(b[64:128]))
    if not g2_on_curve(pt):
        raise ValueError("G2 point not on curve")
    return pt


def gt_to_bytes(f: Fp12) -> bytes:
    # gfP12{x,y} = x*w + y ; gfP6{x,y,z} = x v^2 + y v + z: highest coefficient first
    out = b""
    for f6 in (f.c1, f.c0):
        for f2 in (f6.c2, f6.c1, f6.c0):
            out += fp2_to_bytes(f2)
    return out


def scalar_to_bytes(s: int) -> bytes:
    return (s % R).to_bytes(32, "big")


def scalar_from_hash(digest: bytes) -> int:
    """kyber mod.Int.SetBytes: big-endian integer reduced mod the group order."""
    return int.from_bytes(digest, "big") % R


def random_scalar() -> int:
    return secrets.randbelow(R - 1) + 1


def sha3_512(*parts: bytes) -> bytes:
    h = hashlib.sha3_512()
    for p_ in parts:
        h.update(p_)
    return h.digest()
