"""BLS/BDN collective signatures (skipchain forward links, cothority CoSi role)."""
from drynx_amd.crypto import bls
from drynx_amd.crypto import oracle as O
from drynx_amd.ledger import skipchain as skc
from drynx_amd.query import ServerIdentity


def _keys(n):
    xs = [O.random_scalar() for _ in range(n)]
    return xs, [bls.public_key(x) for x in xs]


def test_hash_to_g1_on_curve_and_deterministic():
    for m in (b"", b"a", b"block" * 20):
        p = bls.hash_to_g1(m)
        assert O.g1_on_curve(p) and p == bls.hash_to_g1(m)
    assert bls.hash_to_g1(b"a") != bls.hash_to_g1(b"b")


def test_public_key_matches_oracle_and_subgroup():
    x = O.random_scalar()
    pk = bls.public_key(x)
    assert pk == O.g2_mul(x, O.G2_GEN)
    assert bls.in_g2(pk)


def test_multisig_masks_and_tampering():
    xs, pks = _keys(4)
    m = b"\x01" * 32
    parts = {i: bls.sign(x, m) for i, x in enumerate(xs)}
    agg = bls.aggregate(pks, parts)
    assert bls.verify_multi(pks, [1, 1, 1, 1], m, agg)
    assert not bls.verify_multi(pks, [1, 1, 1, 0], m, agg)
    assert not bls.verify_multi(pks, [1, 1, 1, 1], b"\x02" * 32, agg)
    sub = bls.aggregate(pks, {1: parts[1], 3: parts[3]})
    assert bls.verify_multi(pks, [0, 1, 0, 1], m, sub)
    # a plain (non-BDN) sum does not verify: coefficients bind the roster
    plain = None
    for s in parts.values():
        plain = O.g1_add(plain, s)
    assert not bls.verify_multi(pks, [1, 1, 1, 1], m, plain)


def test_skipchain_block_cosig():
    xs, pks = _keys(3)
    ids = [ServerIdentity(f"vn{i}", O.g1_mul(x, O.G1_GEN), bls=pk) for i, (x, pk) in enumerate(zip(xs, pks))]
    data = skc.new_data_block("s1", {"s1/range/dp0//vn0": 1}, ids)
    b = skc.make_block(None, data, ids)
    for i, x in enumerate(xs):
        skc.sign_block(b, f"vn{i}", x)
    skc.finalize_cosig(b)
    assert b.verify_signatures()
    b2 = skc.SkipBlock.from_bytes(b.to_bytes())
    assert b2.verify_signatures()
    # a missing signer fails the default (all-VN) policy but passes a 2/3 threshold
    b3 = skc.SkipBlock.from_bytes(b.to_bytes())
    del b3.ForwardSignatures["vn2"]
    skc.finalize_cosig(b3)
    assert not b3.verify_signatures()
    assert b3.verify_signatures(threshold=2 / 3)
    # tampered data breaks the hash
    b4 = skc.SkipBlock.from_bytes(b.to_bytes())
    assert b"\x12\x02s1" in b4.Data                      # DataBlock.SurveyID (protobuf field 2)
    b4.Data = b4.Data.replace(b"\x12\x02s1", b"\x12\x02s2")
    assert not b4.verify_signatures()
