"""Native (host path of the HIP library) vs the Python oracle, bit-exact."""
import random

import pytest
import torch

from drynx_amd import native as nt
from drynx_amd.crypto import bn254 as bn
from drynx_amd.crypto import oracle as O

RNG = random.Random(7)
SCALARS = [0, 1, 2, 3, 255, 256, 2**64 - 1, 2**64 + 5, O.R - 1, O.R - 2] + [RNG.randrange(O.R) for _ in range(6)]


def test_fp_mont_roundtrip():
    vals = [0, 1, O.P - 1, 123456789] + [RNG.randrange(O.P) for _ in range(4)]
    t = bn.to_tensor(bn.ints_to_limbs(vals), "cpu")
    m = nt.fp_to_mont(t)
    assert bn.limbs_to_ints(bn.to_numpy(m)) == [bn.mont(v) for v in vals]
    assert bn.limbs_to_ints(bn.to_numpy(nt.fp_from_mont(m))) == vals


@pytest.mark.parametrize("op", ["add", "sub", "mul", "neg", "inv"])
def test_fr_arith(op):
    a = [RNG.randrange(1, O.R) for _ in range(8)]
    b = [RNG.randrange(O.R) for _ in range(8)]
    ta, tb = bn.scalars_tensor(a), bn.scalars_tensor(b)
    code = {"add": nt.FR_ADD, "sub": nt.FR_SUB, "mul": nt.FR_MUL, "neg": nt.FR_NEG, "inv": nt.FR_INV}[op]
    out = bn.scalars_from_tensor(nt.fr_arith(code, ta, tb if op in ("add", "sub", "mul") else None))
    f = {"add": lambda x, y: (x + y) % O.R, "sub": lambda x, y: (x - y) % O.R, "mul": lambda x, y: x * y % O.R,
         "neg": lambda x, y: (-x) % O.R, "inv": lambda x, y: pow(x, -1, O.R)}[op]
    assert out == [f(x, y) for x, y in zip(a, b)]


def test_g1_fixed_and_variable_base():
    tab = bn.base_table()
    fb = bn.g1_points_from_jac(nt.g1_fb_mul(tab, bn.scalars_tensor(SCALARS)))
    vb = bn.g1_points_from_jac(nt.g1_mul(bn.g1_jac_tensor([O.G1_GEN]), bn.scalars_tensor(SCALARS)))
    exp = [O.g1_mul(k, O.G1_GEN) for k in SCALARS]
    assert fb == exp and vb == exp


def test_g1_signed_and_group_law():
    m = torch.tensor([0, 1, -1, 5, -5, 2**40], dtype=torch.int64)
    got = bn.g1_points_from_jac(nt.g1_fb_mul_i64(bn.base_table(), m))
    assert got == [O.g1_mul_signed(int(v), O.G1_GEN) for v in m]
    a = bn.g1_jac_tensor([O.g1_mul(3, O.G1_GEN), O.G1_GEN, None, O.G1_GEN])
    b = bn.g1_jac_tensor([O.g1_mul(4, O.G1_GEN), O.G1_GEN, O.G1_GEN, O.g1_neg(O.G1_GEN)])
    s = bn.g1_points_from_jac(nt.g1_add(a, b))
    assert s == [O.g1_mul(7, O.G1_GEN), O.g1_mul(2, O.G1_GEN), O.G1_GEN, None]
    assert nt.g1_eq(a, a).all()


def test_g1_sum_reduction():
    pts = [O.g1_mul(k + 1, O.G1_GEN) for k in range(3 * 5)]
    x = bn.g1_jac_tensor(pts).view(5, 3, 24)
    got = bn.g1_points_from_jac(nt.g1_sum(x))
    exp = [O.g1_mul(sum(k * 3 + g + 1 for k in range(5)), O.G1_GEN) for g in range(3)]
    assert got == exp


def test_g2_mults():
    ks = SCALARS[:6]
    fb = bn.g2_points_from_aff(nt.g2_fb_mul(bn.base2_table(), bn.scalars_tensor(ks)))
    vb = bn.g2_points_from_aff(nt.g2_mul(bn.g2_generator_aff(), bn.scalars_tensor(ks)))
    exp = [O.g2_mul(k, O.G2_GEN) for k in ks]
    assert fb == exp and vb == exp


def test_pairing_matches_oracle():
    P = [O.G1_GEN, O.g1_mul(5, O.G1_GEN), None]
    Q = [O.G2_GEN, O.g2_mul(3, O.G2_GEN), O.G2_GEN]
    e = bn.gt_from_tensor(nt.pairing(bn.g1_aff_tensor(P), bn.g2_aff_tensor(Q)))
    e0 = O.pairing(O.G1_GEN, O.G2_GEN)
    assert e[0] == e0 and e[1] == e0 ** 15 and e[2] == O.Fp12.one()
    ml = nt.miller_loop(bn.g1_aff_tensor(P[:1]), bn.g2_aff_tensor(Q[:1]))
    assert bn.gt_from_tensor(nt.final_exp(ml))[0] == e0


def test_gt_ops():
    e0 = O.pairing(O.G1_GEN, O.G2_GEN)
    t = bn.gt_tensor([e0])
    ks = [0, 1, 7, 2**70 + 3, O.R - 1]
    got = bn.gt_from_tensor(nt.gt_pow(t, bn.scalars_tensor(ks)))
    assert got == [e0 ** k for k in ks]
    tab = nt.gt_fb_table(t)
    assert bn.gt_from_tensor(nt.gt_fb_pow(tab, bn.scalars_tensor(ks))) == got
    sq = nt.gt_mul(t, t)
    assert bn.gt_from_tensor(sq)[0] == e0 * e0
    prod = nt.gt_prod(torch.stack([t, sq, t]).view(3, 1, 96))
    assert bn.gt_from_tensor(prod)[0] == e0 ** 4


def test_wire_codecs_match_oracle():
    p = O.g1_mul(99, O.G1_GEN)
    q = O.g2_mul(99, O.G2_GEN)
    e = O.pairing(p, q)
    assert bytes(bn.g1_aff_to_bytes(bn.g1_aff_tensor([p]))[0]) == O.g1_to_bytes(p)
    assert bytes(bn.g2_aff_to_bytes(bn.g2_aff_tensor([q]))[0]) == O.g2_to_bytes(q)
    assert bytes(bn.gt_to_bytes(bn.gt_tensor([e]))[0]) == O.gt_to_bytes(e)
    assert bn.g1_points_from_aff(bn.g1_aff_from_bytes(O.g1_to_bytes(p))) == [p]
    assert bn.g2_points_from_aff(bn.g2_aff_from_bytes(O.g2_to_bytes(q))) == [q]
    with pytest.raises(ValueError):
        bn.g1_aff_from_bytes(b"\x00" * 63 + b"\x05")


def test_random_scalars_in_range():
    s = bn.scalars_from_tensor(bn.random_scalars(500))
    assert all(0 < v < O.R for v in s) and len(set(s)) == 500


def test_gt_bucket_multi_exp64_matches_direct():
    """prod a_i^{rho_i} (64-bit rho) through the bucket plan == per-item powers."""
    import os

    import numpy as np

    x = nt.pairing(bn.g1_generator_aff("cpu"), bn.g2_generator_aff("cpu"))
    n = 200
    a = nt.gt_pow(x, bn.random_scalars(n))
    rho = torch.zeros((n, 8), dtype=torch.int32)
    rho[:, :2] = torch.from_numpy(np.frombuffer(os.urandom(8 * n), dtype="<i4").reshape(n, 2).copy())
    rho[:7, :2] = 0  # all-zero digits: items contribute nothing
    got = nt._multi_exp64_run(a, nt._multi_exp64_plan(rho))
    ref = nt.gt_prod(nt.gt_pow(a, rho).view(-1, 1, 96), chunk=4).view(1, 96)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("bits", [64, 256])
def test_g1_msm_grouped_matches_oracle(bits):
    """Grouped Pippenger MSM (one bucket pass, G independent sums) vs oracle."""
    n, G = 40, 3
    ks = [RNG.randrange(1 << bits) % O.R for _ in range(n)]
    ks[3] = 0
    es = [RNG.randrange(1, O.R) for _ in range(n)]
    grp = [RNG.randrange(G) for _ in range(n)]
    grp[:G] = list(range(G))
    pts = [O.g1_mul(e, O.G1_GEN) for e in es]
    out = bn.g1_points_from_jac(nt.g1_msm_grouped(bn.g1_jac_tensor(pts), bn.scalars_tensor(ks),
                                                  torch.tensor(grp, dtype=torch.int32), G + 1, bits=bits))
    for g in range(G + 1):
        exp = O.g1_mul(sum(k * e for k, e, gg in zip(ks, es, grp) if gg == g) % O.R, O.G1_GEN)
        assert out[g] == exp
    one = bn.g1_points_from_jac(nt.g1_msm(bn.g1_jac_tensor(pts), bn.scalars_tensor(ks)))
    assert one[0] == O.g1_mul(sum(k * e for k, e in zip(ks, es)) % O.R, O.G1_GEN)


def test_glv_weight_constants_match_oracle():
    """GLV batch weights (csrc/kernels/dx_glv.hip): phi(x, y) = (beta x, y) is
    [lambda] on G1 and x^lambda = x^(p^8) on GT; rho = a + b lambda."""
    from drynx_amd import native as nt
    from drynx_amd.crypto import bn254 as bn
    from drynx_amd.crypto import oracle as O

    x = O.g1_mul(987654321, O.G1_GEN)
    assert O.g1_mul(nt.GLV_LAMBDA, x) == (nt.GLV_BETA * x[0] % O.P, x[1])
    assert pow(O.P, 8, O.R) == nt.GLV_LAMBDA
    e = O.pairing(O.G1_GEN, O.G2_GEN) ** 12345
    got = bn.gt_from_tensor(nt.gt_frob8(bn.gt_tensor([e])))[0]
    assert got == e ** nt.GLV_LAMBDA
    ab, rho = nt.glv_weights(64, "cpu")
    for (a, b), r in zip(ab.tolist(), bn.scalars_from_tensor(rho)):
        a, b = a & 0xFFFFFFFF, b & 0xFFFFFFFF
        assert r == a + b * nt.GLV_LAMBDA  # < r: no reduction, all 2^64 (a, b) distinct


def test_gls6_tables_match_oracle():
    """GLS-2 6-bit tables (prover mode 6): k A = k0 A + psi(k1 A) and
    E^k = E^k0 frob(E^k1) with k = k0 + k1 * 6u^2 -- against the oracle."""
    import random

    from drynx_amd import native as nt
    from drynx_amd.crypto import bn254 as bn
    from drynx_amd.crypto import oracle as O

    rng = random.Random(3)
    A = O.g2_mul(rng.randrange(1, O.R), O.G2_GEN)
    E = O.pairing(O.g1_mul(5, O.G1_GEN), A)
    ks = [rng.randrange(O.R) for _ in range(5)] + [0, 1, O.R - 1, 6 * O.U * O.U, 6 * O.U * O.U - 1]
    kt = bn.scalars_tensor(ks)
    g2 = nt.g2_gls6_mul(nt.g2_gls6_table(bn.g2_aff_tensor([A])), kt)
    assert bn.g2_points_from_aff(g2) == [None if k % O.R == 0 else O.g2_mul(k, A) for k in ks]
    gt = nt.gt_gls6_pow(nt.gt_gls6_table(bn.gt_tensor([E])), kt)
    assert bn.gt_from_tensor(gt) == [E ** k for k in ks]
