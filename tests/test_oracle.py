"""Golden-model sanity: the pure-Python BN254 oracle is itself correct."""
from drynx_amd.crypto import oracle as O


def test_curve_params():
    assert O.g1_on_curve(O.G1_GEN) and O.g2_on_curve(O.G2_GEN)
    assert O.g1_mul(O.R, O.G1_GEN) is None
    assert O.g2_mul(O.R, O.G2_GEN) is None


def test_pairing_bilinear_and_order():
    e = O.pairing(O.G1_GEN, O.G2_GEN)
    assert not e.is_one() and (e ** O.R).is_one()
    assert O.pairing(O.g1_mul(6, O.G1_GEN), O.g2_mul(7, O.G2_GEN)) == e ** 42


def test_fast_final_exp_matches_textbook():
    f = O.miller_loop(O.g1_mul(3, O.G1_GEN), O.G2_GEN)
    assert O.final_exp_fast(f) == O.final_exp(f)


def test_frobenius():
    f = O.miller_loop(O.G1_GEN, O.G2_GEN)
    assert f.frob(1) == f ** O.P


def test_codecs_roundtrip():
    p = O.g1_mul(12345, O.G1_GEN)
    assert O.g1_from_bytes(O.g1_to_bytes(p)) == p
    q = O.g2_mul(777, O.G2_GEN)
    assert O.g2_from_bytes(O.g2_to_bytes(q)) == q
    assert O.g1_to_bytes(None) == b"\x00" * 64
