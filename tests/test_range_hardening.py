"""Range-proof verification hardening (VERDICT r1 'What's weak' 2, ADVICE):
non-GT a_ij values, V outside G2, chosen challenges, the v2 transcript and
the decoding checks of raw-limb payloads.  Mode 0 keeps the reference's
semantics (it trusts the proof's challenge, range_proof.go:504-565)."""
import pytest
import torch

from drynx_amd import native as nt
from drynx_amd.crypto import bn254 as bn
from drynx_amd.crypto import elgamal as eg
from drynx_amd.crypto import oracle as O
from drynx_amd.ops.encoding import CreateProofBatch
from drynx_amd.proofs import range_proof as rp


@pytest.fixture(scope="module")
def setup():
    S, u, l = 2, 4, 3
    sigs = [rp.init_range_proof_signatures([u] * 3) for _ in range(S)]
    kps = [eg.KeyPair.generate() for _ in range(S)]
    P = eg.aggregate_keys([k.public for k in kps])
    return S, u, l, sigs, rp.SigMaterial(sigs), P, eg.pk_table(P)


def _prove(setup, vals, mode=0):
    S, u, l, sigs, sm, P, pk = setup
    cv, r = eg.encrypt_ints(pk, vals)
    n = len(vals)
    return rp.create_range_proofs(CreateProofBatch(vals, r, cv, [u] * n, [l] * n, list(range(n)), [0] * n), sm, P,
                                  mode=mode)[0]


def _order_q_element():
    """An element of the cyclotomic subgroup of prime order q = 493356762637
    (a factor of (p^4 - p^2 + 1) / r): outside GT, invisible to a cyclotomic
    membership test."""
    q = 493356762637
    h2 = (O.P ** 4 - O.P ** 2 + 1) // O.R
    assert h2 % q == 0
    x = O.Fp12.from_coeffs(list(range(3, 15)))
    y = x.conj() * x.inv()            # x^(p^6 - 1)
    y = y.frob(2) * y                  # ^(p^2 + 1): cyclotomic
    h = y ** (O.R * (h2 // q))
    assert not h.is_one() and (h ** q).is_one()
    return h


def test_negated_pair_of_a_values_rejected(setup):
    """two a_ij multiplied by -1 cancel in a product with odd
    weights; -1 is outside the cyclotomic subgroup, so the decode check rejects."""
    rpl = _prove(setup, [5, 6])
    sm, P = setup[4], setup[5]
    assert rp.verify_range_proof_list(rpl, sm, P)
    one = torch.zeros(96, dtype=torch.int32)
    one[:8] = bn.to_tensor(bn.ints_to_limbs([bn.mont(O.P - 1)]), "cpu")[0]  # -1 in Fp12
    for k in (0, 1):
        rpl.A[k] = nt.gt_mul(rpl.A[k: k + 1].contiguous(), one.view(1, 96))[0]
    assert not rp.verify_range_proof_list(rpl, sm, P)


def test_non_gt_component_rejected(setup):
    rpl = _prove(setup, [5, 6])
    sm, P = setup[4], setup[5]
    h = bn.gt_tensor([_order_q_element()], "cpu")
    assert bool(nt.gt_cyclotomic(h).all())          # passes the cheap per-element test ...
    rpl.A[3] = nt.gt_mul(rpl.A[3:4].contiguous(), h)[0]
    assert not rp.verify_range_proof_list(rpl, sm, P)  # ... but not the batch equation + GT combination
    # the same component in two entries, inverse in the second: a product with
    # weights rho_1 = rho_2 would cancel; the independent combination does not
    rpl2 = _prove(setup, [5, 6])
    hinv = bn.gt_tensor([_order_q_element().inv()], "cpu")
    rpl2.A[0] = nt.gt_mul(rpl2.A[0:1].contiguous(), h)[0]
    rpl2.A[1] = nt.gt_mul(rpl2.A[1:2].contiguous(), hinv)[0]
    assert not rp.verify_range_proof_list(rpl2, sm, P)


def test_chosen_challenge_accepted_by_reference_mode_only(setup, monkeypatch):
    """A prover that picks its own challenge (c = 1) instead of the hash:
    the reference verifier trusts it (inherited gap), strict mode recomputes it."""
    orig = rp.challenges
    monkeypatch.setattr(rp, "challenges", lambda C, *a, **k: bn.scalars_tensor([1] * C.shape[0], C.device))
    rpl = _prove(setup, [7, 8])
    monkeypatch.setattr(rp, "challenges", orig)
    sm, P = setup[4], setup[5]
    assert rp.verify_range_proof_list(rpl, sm, P, mode=0)
    assert not rp.verify_range_proof_list(rpl, sm, P, mode=1)


def test_v2_transcript(setup):
    sm, P = setup[4], setup[5]
    rpl = _prove(setup, [0, 9, 63], mode=2)
    assert rp.verify_range_proof_list(rpl, sm, P, mode=2)
    assert rp.verify_range_proof_list(rpl, sm, P, mode=0)       # the reference check does not look at c
    assert not rp.verify_range_proof_list(rpl, sm, P, mode=1)   # v1 challenge differs
    rpl1 = _prove(setup, [0, 9, 63], mode=1)
    assert rp.verify_range_proof_list(rpl1, sm, P, mode=1)
    assert not rp.verify_range_proof_list(rpl1, sm, P, mode=2)


def _fp2_sqrt(a: O.Fp2):
    p = O.P
    n = (a.c0 * a.c0 + a.c1 * a.c1) % p
    g = pow(n, (p + 1) // 4, p)
    if g * g % p != n:
        return None
    for sgn in (1, -1):
        d = (a.c0 + sgn * g) * pow(2, -1, p) % p
        x0 = pow(d, (p + 1) // 4, p)
        if x0 * x0 % p == d and x0:
            x1 = a.c1 * pow(2 * x0, -1, p) % p
            r = O.Fp2(x0, x1)
            if r * r == a:
                return r
    return None


def test_v_outside_g2_rejected_in_strict_mode(setup):
    sm, P = setup[4], setup[5]
    rpl = _prove(setup, [3])
    for k in range(2, 200):  # a twist point with a cofactor component
        x = O.Fp2(k, 1)
        y = _fp2_sqrt(x * x * x + O.B2)
        if y is not None:
            break
    pt = (x, y)
    assert O.g2_on_curve(pt) and O.g2_add(O.g2_mul(O.R - 1, pt), pt) is not None  # not in G2
    V = bn.g2_aff_tensor([pt])
    assert bool(nt.g2_on_curve(V).all()) and not bool(nt.g2_subgroup(V).any())
    G = bn.g2_aff_tensor([O.g2_mul(5, O.G2_GEN)])
    assert bool(nt.g2_subgroup(G).all())
    rpl.V[1] = V[0]
    assert not rp.validate_list(rpl, mode=1)
    assert rp.validate_list(rpl, mode=0)  # on the curve: only the equation rejects it in mode 0
    assert not rp.verify_range_proof_list(rpl, sm, P, mode=0)


def test_raw_limb_payload_checks(setup):
    sm, P = setup[4], setup[5]
    rpl = _prove(setup, [2, 3])
    back = rp.RangeProofList.unpack(rpl.pack())
    assert rp.validate_list(back)
    for field, row, val in [("zv", 0, -1), ("V", 2, -1), ("D", 0, 12345)]:
        bad = rp.RangeProofList.unpack(rpl.pack().clone())
        t = getattr(bad, field)
        if val == -1:
            t[row, :] = -1          # all-ones limbs: >= p / >= r
        else:
            t[row, 3] ^= val        # off the curve
        assert not rp.validate_list(bad), field
        assert not rp.verify_range_proof_list(bad, sm, P)


def _g2_mul_full(k: int, Q):
    """k * Q on the whole twist group (the oracle's g2_mul reduces k mod r)."""
    acc, add = None, Q
    while k:
        if k & 1:
            acc = O.g2_add(acc, add)
        add = O.g2_add(add, add)
        k >>= 1
    return acc


def test_g2_subgroup_rejects_every_torsion_order():
    """The fast membership test [u+1]Q + psi([u]Q) + psi^2([u]Q) == psi^3([2u]Q)
    (dx_g2_subgroup) against adversarial V = G + T, T of each prime order
    dividing the twist cofactor 2p - r: every such V is rejected, every G2
    point accepted (the msm verifier's regrouping requires V in G2)."""
    import random

    h = 2 * O.P - O.R
    primes = [10069, 5864401, 1875725156269, 197620364512881247228717050342013327560683201906968909]
    assert h == primes[0] * primes[1] * primes[2] * primes[3]
    rnd = random.Random(11)
    G = O.g2_mul(123456789, O.G2_GEN)
    pts, want = [G, O.G2_GEN], [1, 1]
    for q in primes:
        while True:
            x = O.Fp2(rnd.randrange(O.P), rnd.randrange(O.P))
            y = _fp2_sqrt(x * x * x + O.B2)
            if y is None:
                continue
            T = _g2_mul_full(h // q * O.R, (x, y))
            if T is not None:
                break
        assert _g2_mul_full(q, T) is None
        pts += [T, O.g2_add(G, T)]
        want += [0, 0]
    got = nt.g2_subgroup(bn.g2_aff_tensor(pts)).tolist()
    assert got == want


def test_v_with_small_torsion_rejected_by_regrouped_verifier(setup, monkeypatch):
    """V_it = G_it + T with T of order 10069 (the smallest cofactor prime):
    the bilinearity-regrouped verifier ("msm", mode 0) rejects it through the
    exact G2 membership of its U combinations (a torsion component survives
    a random combination unless the weights cancel it mod 10069)."""
    import random

    sm, P = setup[4], setup[5]
    rpl = _prove(setup, [3, 5])
    assert rp.verify_range_proof_list(rpl, sm, P, mode=0)
    h = 2 * O.P - O.R
    rnd = random.Random(5)
    while True:
        x = O.Fp2(rnd.randrange(O.P), rnd.randrange(O.P))
        y = _fp2_sqrt(x * x * x + O.B2)
        if y is not None:
            T = _g2_mul_full(h // 10069 * O.R, (x, y))
            if T is not None:
                break
    G = bn.g2_points_from_aff(rpl.V[2:3].cpu())[0]
    rpl.V = rpl.V.clone()
    rpl.V[2] = bn.g2_aff_tensor([O.g2_add(G, T)])[0].to(rpl.V.device)
    assert bool(nt.g2_on_curve(rpl.V[2:3]).all())
    assert not rp.verify_range_proof_list(rpl, sm, P, mode=0)



def test_gt_membership_matches_generic_pow():
    """dx_gt_membership (x^p by Frobenius vs two cyclotomic u-ladders) agrees
    with x^p == x^(6u^2) computed by the oracle with exact exponents, on GT
    elements and on cyclotomic elements outside GT (the easy part of the final
    exponentiation of random Fp12 values) -- which it must reject."""
    import random

    rng = random.Random(5)
    g = O.pairing(O.G1_GEN, O.G2_GEN)
    inside_vals = [g ** rng.randrange(O.R) for _ in range(3)]
    inside = bn.gt_tensor(inside_vals, "cpu")
    outside_vals = []
    for _ in range(3):
        e = O.Fp12.from_coeffs([rng.randrange(O.P) for _ in range(12)])
        c = e.conj() * e.inv()
        outside_vals.append(c.frob(2) * c)
    outside = bn.gt_tensor(outside_vals, "cpu")
    assert all(nt.gt_cyclotomic(outside).tolist())
    # reference with the oracle's exact exponents (a scalar tensor would
    # reduce p mod r = 6u^2 and make the comparison vacuous)
    for vals, t in ((inside_vals, inside), (outside_vals, outside)):
        ref = [x ** O.P == x ** (6 * O.U * O.U) for x in vals]
        assert [bool(v) for v in nt.gt_membership(t).tolist()] == ref
    assert all(nt.gt_membership(inside).tolist())
    assert not any(nt.gt_membership(outside).tolist())
