"""unlynx ElGamal equivalents: encrypt/decrypt (negatives), homomorphism, CheckZero, bytes."""
from drynx_amd.crypto import elgamal as eg
from drynx_amd.crypto import oracle as O


def test_encrypt_decrypt_roundtrip_and_negatives():
    kp = eg.KeyPair.generate()
    pk = eg.pk_table(kp.public)
    vals = [0, 1, -1, 9999, -10000, 42]
    cv, r = eg.encrypt_ints(pk, vals)
    assert eg.decrypt_ints(kp.secret, cv) == vals
    K, C = cv.points()
    rs = __import__("drynx_amd.crypto.bn254", fromlist=["x"]).scalars_from_tensor(r)
    assert K[3] == O.g1_mul(rs[3], O.G1_GEN)
    assert C[3] == O.g1_add(O.g1_mul(9999, O.G1_GEN), O.g1_mul(rs[3], kp.public))


def test_homomorphic_sum_and_scalar():
    kp = eg.KeyPair.generate()
    pk = eg.pk_table(kp.public)
    a, _ = eg.encrypt_ints(pk, [1, 2, 3])
    b, _ = eg.encrypt_ints(pk, [10, -20, 30])
    assert eg.decrypt_ints(kp.secret, a.add(b)) == [11, -18, 33]
    assert eg.decrypt_ints(kp.secret, b.sub(a)) == [9, -22, 27]
    assert eg.decrypt_ints(kp.secret, eg.CipherVector.sum([a, a, b])) == [12, -16, 36]
    from drynx_amd.crypto import bn254 as bn

    assert eg.decrypt_ints(kp.secret, a.mul_scalars(bn.scalars_tensor([3]))) == [3, 6, 9]


def test_check_zero_and_bytes():
    kp = eg.KeyPair.generate()
    pk = eg.pk_table(kp.public)
    cv, _ = eg.encrypt_ints(pk, [0, 5, 0])
    assert eg.decrypt_check_zero(kp.secret, cv).tolist() == [0, 1, 0]
    b = cv.to_bytes()
    assert len(b) == 3 * 128
    assert eg.decrypt_ints(kp.secret, eg.CipherVector.from_bytes(b)) == [0, 5, 0]


def test_decrypt_auto_large_values():
    kp = eg.KeyPair.generate()
    pk = eg.pk_table(kp.public)
    vals = [3_000_000, -2_500_000, 7]
    cv, _ = eg.encrypt_ints(pk, vals)
    assert eg.decrypt_auto(kp.secret, cv, 10000).tolist() == vals


def test_collective_key_decrypts_with_sum_of_secrets():
    kps = [eg.KeyPair.generate() for _ in range(3)]
    P = eg.aggregate_keys([k.public for k in kps])
    cv, _ = eg.encrypt_ints(eg.pk_table(P), [77])
    assert eg.decrypt_ints(sum(k.secret for k in kps) % O.R, cv) == [77]
