"""Obfuscation (incl. the negative test of obfuscation_proof_test.go:30-31),
key-switch, Schnorr, aggregation and shuffle proofs."""

from drynx_amd.crypto import bn254 as bn
from drynx_amd.crypto import elgamal as eg
from drynx_amd.crypto import oracle as O
from drynx_amd.proofs import aggregation_shuffle as ags
from drynx_amd.proofs import sigma


def _cv(vals):
    kp = eg.KeyPair.generate()
    pk = eg.pk_table(kp.public)
    return kp, pk, eg.encrypt_ints(pk, vals)[0]


def test_schnorr():
    x = O.random_scalar()
    X = O.g1_mul(x, O.G1_GEN)
    sig = sigma.schnorr_sign(x, b"msg")
    assert len(sig) == 96 and sigma.schnorr_verify(X, b"msg", sig)
    assert not sigma.schnorr_verify(X, b"msh", sig)
    assert not sigma.schnorr_verify(O.g1_mul(2, X), b"msg", sig)


def test_obfuscation_proof_positive_and_negative():
    kp, pk, C = _cv([0, 3, 0, 9])
    s = bn.random_scalars(4)
    Co = C.mul_scalars(s)
    pr = sigma.obfuscation_list_proof_creation(C, Co, s)
    assert sigma.obfuscation_list_proof_verification(pr)
    back = sigma.ObfuscationProof.from_bytes(pr.to_bytes())
    assert sigma.obfuscation_list_proof_verification(back)
    wrong = sigma.obfuscation_list_proof_creation(C, Co, bn.random_scalars(4))  # wrong scalar -> false
    assert not sigma.obfuscation_list_proof_verification(wrong)
    assert eg.decrypt_check_zero(kp.secret, Co).tolist() == [0, 1, 0, 1]


def test_key_switch_share_and_proof():
    xs = [O.random_scalar() for _ in range(3)]
    P = eg.aggregate_keys([O.g1_mul(x, O.G1_GEN) for x in xs])
    cv, _ = eg.encrypt_ints(eg.pk_table(P), [5, -7])
    q = eg.KeyPair.generate()
    Ks, Cs = [], []
    for x in xs:
        share, v = sigma.key_switch_share(x, cv.K, q.public)
        pr = sigma.key_switch_list_proof_creation(x, O.g1_mul(x, O.G1_GEN), q.public, cv.K, share, v)
        assert sigma.key_switch_list_proof_verification(pr)
        assert sigma.key_switch_list_proof_verification(sigma.KeySwitchProof.from_bytes(pr.to_bytes()))
        Ks.append(share)
    tot = eg.CipherVector.sum(Ks)
    switched = eg.CipherVector(tot.K, __import__("drynx_amd").native.g1_add(cv.C, tot.C))
    assert eg.decrypt_ints(q.secret, switched) == [5, -7]
    # a share computed with the wrong secret does not verify
    share, v = sigma.key_switch_share(xs[0] + 1, cv.K, q.public)
    bad = sigma.key_switch_list_proof_creation(xs[0], O.g1_mul(xs[0], O.G1_GEN), q.public, cv.K, share, v)
    assert not sigma.key_switch_list_proof_verification(bad)


def test_aggregation_proof():
    kp, pk, a = _cv([1, 2])
    b, _ = eg.encrypt_ints(pk, [3, 4])
    pr = ags.aggregation_list_proof_creation([a, b], a.add(b))
    assert ags.aggregation_list_proof_verification(pr)
    assert ags.aggregation_list_proof_verification(ags.AggregationProof.from_bytes(pr.to_bytes()))
    assert not ags.aggregation_list_proof_verification(ags.aggregation_list_proof_creation([a, b], a.add(a)))


def test_shuffle_proof():
    from drynx_amd.proofs import shuffle as sh

    kp, pk, X = _cv([1, 2, 3, 4, 5, 0, 7, 7])
    Y, perm, rho = ags.shuffle_sequence(X, kp.public)
    pr = sh.prove(X, Y, perm, rho, kp.public)
    assert sh.verify(pr, kp.public)
    assert sh.verify(sh.ShuffleProof.from_bytes(pr.to_bytes()), kp.public)
    assert sorted(eg.decrypt_ints(kp.secret, Y)) == sorted(eg.decrypt_ints(kp.secret, X))
    Z, _ = eg.encrypt_ints(pk, [1, 2, 3, 4, 6, 0, 7, 7])  # not a shuffle of X
    assert not sh.verify(sh.prove(X, Z, perm, rho, kp.public), kp.public)
    wrong = perm.clone()
    wrong[[0, 1]] = wrong[[1, 0]]  # claimed permutation does not match Y
    assert not sh.verify(sh.prove(X, Y, wrong, rho, kp.public), kp.public)
    for field in ("kE", "kB"):
        bad = sh.ShuffleProof.from_bytes(pr.to_bytes())
        t = getattr(bad, field).clone()
        t[2, 0] ^= 1
        setattr(bad, field, t)
        assert not sh.verify(bad, kp.public)
    bad = sh.ShuffleProof.from_bytes(pr.to_bytes())
    bad.kA ^= 1
    assert not sh.verify(bad, kp.public)


def test_shuffle_generators_match_host_hash():
    import hashlib

    from drynx_amd import native as nt
    from drynx_amd.proofs import shuffle as sh

    def h2g(i):
        for ctr in range(128):
            d = hashlib.sha256(sh.SEED + i.to_bytes(8, "little") + ctr.to_bytes(4, "little")).digest()
            x = int.from_bytes(d, "big") % O.P
            rhs = (x * x * x + 3) % O.P
            y = pow(rhs, (O.P + 1) // 4, O.P)
            if y * y % O.P == rhs:
                return (x, O.P - y if y & 1 else y)

    got = bn.g1_points_from_jac(sh.generators(9, "cpu"))
    assert got == [h2g(i) for i in range(10)]
    assert len(set(got)) == 10 and all(O.g1_on_curve(p) for p in got)
    assert nt.hash_to_g1(sh.SEED, 3, 2, "cpu").shape == (2, 16)


def test_noise_generation():
    v = ags.generate_noise_values_scale(100, 0.0, 2.0, 1.0, 1.0, 10)
    assert len(v) == 100 and max(abs(x) for x in v) <= 10 and v.count(0) > v.count(5)


def test_batched_keyswitch_and_obfuscation_verification():
    xs = [O.random_scalar() for _ in range(3)]
    X = [O.g1_mul(x, O.G1_GEN) for x in xs]
    P = eg.aggregate_keys(X)
    cv, _ = eg.encrypt_ints(eg.pk_table(P), [4, -9, 16])
    q = eg.KeyPair.generate()
    shares, pend = sigma.key_switch_shares_batch(xs, X, cv.K, q.public, True)
    prs = sigma.finish_keyswitch_proofs(pend)
    assert sigma.key_switch_batch_verification(prs) == [True, True, True]
    # the packed (raw-limb) payload round trip verifies too, with fresh decoded digests
    back = [sigma.KeySwitchProof.unpack(pr.pack()) for pr in prs]
    assert sigma.key_switch_batch_verification(back) == [True, True, True]
    tot = eg.CipherVector.sum(shares)
    out = eg.CipherVector(tot.K, __import__("drynx_amd").native.g1_add(cv.C, tot.C))
    assert eg.decrypt_ints(q.secret, out) == [4, -9, 16]
    prs[1].za[0, 0] ^= 1  # break one element of one proof
    assert sigma.key_switch_batch_verification(prs) == [True, False, True]
    s = [bn.random_scalars(3) for _ in range(2)]
    obf = [sigma.obfuscation_list_proof_creation(cv, cv.mul_scalars(si), si) for si in s]
    obf.append(sigma.obfuscation_list_proof_creation(cv, cv.mul_scalars(s[0]), s[1]))
    assert sigma.obfuscation_batch_verification(obf) == [True, True, False]


def test_batch_verification_blames_only_the_bad_proof():
    """Random-linear-combination (MSM) batch checks: one tampered proof among
    good ones is pinned individually."""
    kps = [eg.KeyPair.generate() for _ in range(3)]
    q = eg.KeyPair.generate()
    P = eg.aggregate_keys([k.public for k in kps])
    pk = eg.pk_table(P)
    cv, _ = eg.encrypt_ints(pk, [1, 2, 3, 4])
    ks = []
    for kp in kps:
        share, v = sigma.key_switch_share(kp.secret, cv.K, q.public)
        ks.append(sigma.key_switch_list_proof_creation(kp.secret, kp.public, q.public, cv.K, share, v))
    assert sigma.key_switch_batch_verification(ks) == [True, True, True]
    ks[1].za = ks[1].za.clone()
    ks[1].za[2, 0] ^= 1
    assert sigma.key_switch_batch_verification(ks) == [True, False, True]
    obs = []
    for _ in range(3):
        s = bn.random_scalars(4)
        obs.append(sigma.obfuscation_list_proof_creation(cv, cv.mul_scalars(s), s))
    assert sigma.obfuscation_batch_verification(obs) == [True, True, True]
    obs[2].z = obs[2].z.clone()
    obs[2].z[0, 0] ^= 1
    assert sigma.obfuscation_batch_verification(obs) == [True, True, False]


def test_schnorr_verify_batch_matches_single():
    from drynx_amd.crypto import oracle as O
    from drynx_amd.proofs import sigma

    keys = [O.random_scalar() for _ in range(5)]
    pubs = [O.g1_mul(k, O.G1_GEN) for k in keys]
    items = []
    for i, k in enumerate(keys):
        msg = f"digest {i}".encode()
        items.append((pubs[i], msg, sigma.schnorr_sign(k, msg)))
    good_sig = items[0][2]
    items.append((pubs[1], b"digest 0", good_sig))                      # wrong key
    items.append((pubs[0], b"other", good_sig))                         # wrong message
    items.append((pubs[0], b"digest 0", good_sig[:64] + (1).to_bytes(32, "big")))  # wrong s
    items.append((None, b"digest 0", good_sig))                          # unknown sender
    items.append((pubs[0], b"digest 0", good_sig[:90]))                  # truncated
    items.append((pubs[0], b"digest 0", b"\x01" * 64 + good_sig[64:]))  # R off the curve
    # R at infinity, which the key holder can produce (s B = e X): rejected by both paths
    import hashlib

    e = int.from_bytes(hashlib.sha256(bytes(64) + O.g1_to_bytes(pubs[0]) + b"inf").digest(), "big") % O.R
    items.append((pubs[0], b"inf", bytes(64) + O.scalar_to_bytes(e * keys[0] % O.R)))
    # a non-canonical s (s + r: the same group element)
    s0 = int.from_bytes(good_sig[64:], "big")
    items.append((pubs[0], b"digest 0", good_sig[:64] + (s0 + O.R).to_bytes(32, "big")))
    want = [sigma.schnorr_verify(p, m, s) for p, m, s in items]
    assert want == [True] * 5 + [False] * 8
    assert sigma.schnorr_verify_batch(items) == want


def test_multi_vn_keyswitch_verification_matches_single():
    """Co-hosted VNs' key-switch checks in one grouped MSM (each with its own
    weights) give every VN the single-VN verdicts, including the blame."""
    kps = [eg.KeyPair.generate() for _ in range(3)]
    q = eg.KeyPair.generate()
    cv, _ = eg.encrypt_ints(eg.pk_table(eg.aggregate_keys([k.public for k in kps])), [5, 6, 7])
    ks = []
    for kp in kps:
        share, v = sigma.key_switch_share(kp.secret, cv.K, q.public)
        ks.append(sigma.key_switch_list_proof_creation(kp.secret, kp.public, q.public, cv.K, share, v))
    from drynx_amd.crypto.coins import Coins

    assert sigma.key_switch_batch_verification_multi(ks, 1.0, [Coins() for _ in range(3)]) == [[True] * 3] * 3
    ks[2].za = ks[2].za.clone()
    ks[2].za[1, 0] ^= 1
    assert sigma.key_switch_batch_verification_multi(ks, 1.0, [Coins(), Coins()]) == [[True, True, False]] * 2
    assert sigma.key_switch_batch_verification_multi([], 1.0, [Coins(), Coins()]) == [[], []]


class _ZeroCoins:
    """Sabotaged coins: every batch weight is 0 (a verifier with these coins
    accepts any combination).  Used to show that one VN's coins cannot change
    another VN's verdicts."""

    def bits(self, n, device, bits=64, odd=False):
        import torch

        return torch.zeros((n, 8), dtype=torch.int32, device=device)

    def random(self):
        return 0.0


def test_one_vns_coins_cannot_change_anothers_keyswitch_verdict():
    from drynx_amd.crypto.coins import Coins

    kps = [eg.KeyPair.generate() for _ in range(2)]
    q = eg.KeyPair.generate()
    cv, _ = eg.encrypt_ints(eg.pk_table(eg.aggregate_keys([k.public for k in kps])), [1, 2])
    ks = []
    for kp in kps:
        share, v = sigma.key_switch_share(kp.secret, cv.K, q.public)
        ks.append(sigma.key_switch_list_proof_creation(kp.secret, kp.public, q.public, cv.K, share, v))
    ks[0].za = ks[0].za.clone()
    ks[0].za[0, 0] ^= 1  # forged response
    res = sigma.key_switch_batch_verification_multi(ks, 1.0, [Coins(), _ZeroCoins()])
    assert res[0] == [False, True]  # the honest VN blames the forged proof, whatever VN 1's coins are


def test_packed_payloads_round_trip():
    """Raw-limb payloads (the intra-cluster format) of the per-CN proofs."""
    kp, pk, a = _cv([1, 2, 3])
    b, _ = eg.encrypt_ints(pk, [4, 5, 6])
    agg = ags.aggregation_list_proof_creation([a, b], a.add(b))
    back = ags.AggregationProof.unpack(agg.pack())
    assert ags.aggregation_list_proof_verification(back)
    assert ags.AggregationProof.from_bytes(back.to_bytes()).result.to_bytes() == agg.result.to_bytes()
    bad = agg.pack().clone()
    bad[-1] ^= 1  # corrupt a limb of the claimed sum
    assert not ags.aggregation_list_proof_verification(ags.AggregationProof.unpack(bad))
    s = bn.random_scalars(3)
    ob = sigma.obfuscation_list_proof_creation(a, a.mul_scalars(s), s)
    ob2 = sigma.ObfuscationProof.unpack(ob.pack())
    assert sigma.obfuscation_batch_verification([ob2]) == [True]
    assert sigma.obfuscation_list_proof_verification(sigma.ObfuscationProof.from_bytes(ob2.to_bytes()))
    import pytest

    with pytest.raises(ValueError):
        sigma.ObfuscationProof.unpack(ob.pack()[:-1])



def _add_p_to_x(t, row: int):
    """Row ``row`` of a packed Jacobian tensor with its X limbs replaced by
    X + p: the same field element, non-canonical limbs."""
    import numpy as np
    import torch

    lim = t[row, :8].numpy().reshape(1, 8)
    x = bn.limbs_to_ints(lim)[0] + O.P
    assert x < 2 ** 256
    t[row, :8] = torch.from_numpy(np.asarray(bn.ints_to_limbs([x]), dtype=np.uint32).view(np.int32).reshape(8))


def _ks_proofs(n_vals=3):
    xs = [O.random_scalar() for _ in range(2)]
    X = [O.g1_mul(x, O.G1_GEN) for x in xs]
    cv, _ = eg.encrypt_ints(eg.pk_table(eg.aggregate_keys(X)), list(range(n_vals)))
    q = eg.KeyPair.generate()
    _, pend = sigma.key_switch_shares_batch(xs, X, cv.K, q.public, True)
    return sigma.finish_keyswitch_proofs(pend)


def test_packed_keyswitch_rejects_non_canonical_and_off_curve_rows():
    """every point row and response scalar of a received
    packed key-switch payload is checked (canonical limbs, on the curve).  A
    non-canonical X limb encodes the same point, so the Fiat-Shamir challenge
    and the equations would still hold: only the well-formedness check
    rejects it."""
    prs = _ks_proofs()
    good = [sigma.KeySwitchProof.unpack(pr.pack()) for pr in prs]
    assert sigma.key_switch_batch_verification(good) == [True, True]
    for field in ("T1", "share.K", "K"):
        prs = _ks_proofs()
        back = [sigma.KeySwitchProof.unpack(pr.pack()) for pr in prs]
        tgt = back[1].share.K if field == "share.K" else getattr(back[1], field)
        tgt = tgt.clone()
        _add_p_to_x(tgt, 0)
        if field == "share.K":
            back[1].share = eg.CipherVector(tgt, back[1].share.C)
        else:
            setattr(back[1], field, tgt)
        back[1].wellformed = sigma._points_ok([back[1].K, back[1].share.K, back[1].share.C, back[1].T1, back[1].T2])
        assert sigma.key_switch_batch_verification(back) == [True, False], field
    # off-curve row straight in the packed payload
    prs = _ks_proofs()
    t = prs[0].pack().clone()
    n = prs[0].K.shape[0]
    off = sigma._KS_HEAD + 3 * 24 * n  # T1 row 0
    t[off: off + 24] = bn.g1_jac_tensor([(1, 1)]).reshape(-1)  # y^2 = 1 != x^3 + 3
    bad = sigma.KeySwitchProof.unpack(t)
    assert not bool(bad.wellformed)
    assert sigma.key_switch_batch_verification([bad]) == [False]
    assert not sigma.key_switch_list_proof_verification(sigma.KeySwitchProof.unpack(t))
    # non-canonical response scalar za (za + r)
    t = prs[0].pack().clone()
    zo = sigma._KS_HEAD + 5 * 24 * n
    import numpy as np
    import torch

    z0 = bn.limbs_to_ints(t[zo: zo + 8].numpy().reshape(1, 8))[0] + O.R
    t[zo: zo + 8] = torch.from_numpy(np.asarray(bn.ints_to_limbs([z0]), dtype=np.uint32).view(np.int32).reshape(8))
    assert sigma.key_switch_batch_verification([sigma.KeySwitchProof.unpack(t)]) == [False]


def test_packed_keyswitch_rejects_non_canonical_zb_and_c():
    import numpy as np
    import pytest
    import torch

    pr = _ks_proofs()[0]
    t = pr.pack().clone()
    for pos, v in ((58, pr.zb + O.R), (50, pr.c + O.R)):  # header words of zb and c
        b = t.clone()
        b[pos: pos + 8] = torch.from_numpy(np.asarray(bn.ints_to_limbs([v]), dtype=np.uint32).view(np.int32).reshape(8))
        with pytest.raises(ValueError):
            sigma.KeySwitchProof.unpack(b)


def test_packed_obfuscation_rejects_non_canonical_rows():
    kp, pk, a = _cv([1, 2, 3])
    s = bn.random_scalars(3)
    ob = sigma.obfuscation_list_proof_creation(a, a.mul_scalars(s), s)
    t = ob.pack().clone()
    assert sigma.obfuscation_batch_verification([sigma.ObfuscationProof.unpack(t)]) == [True]
    rows = t[sigma._OBF_HEAD: sigma._OBF_HEAD + 24 * 3].view(3, 24).clone()  # C.K
    _add_p_to_x(rows, 1)
    t[sigma._OBF_HEAD: sigma._OBF_HEAD + 24 * 3] = rows.reshape(-1)
    bad = sigma.ObfuscationProof.unpack(t)
    assert sigma.obfuscation_batch_verification([bad]) == [False]
    assert not sigma.obfuscation_list_proof_verification(sigma.ObfuscationProof.unpack(t))


def test_coins_bits_keep_exactly_the_requested_width():
    """40-bit weights have bits 32-39 set (somewhere) and
    nothing at or above bit 40."""
    from drynx_amd.crypto.coins import Coins

    r = Coins().bits(4096, "cpu", 40)
    assert int((r[:, 2:] != 0).sum()) == 0
    w1 = r[:, 1]
    assert int((w1 & ~0xFF).abs().sum()) == 0 and int((w1 != 0).sum()) > 4000
    r64 = Coins().bits(64, "cpu", 64)
    assert int((r64[:, 2:] != 0).sum()) == 0 and int((r64[:, 1] != 0).sum()) > 60
    from drynx_amd.proofs import range_proof as rp

    g = rp._rand64(4096, "cpu", 40)
    assert int((g[:, 2:] != 0).sum()) == 0 and int((g[:, 1] & ~0xFF).abs().sum()) == 0
    assert int((g[:, 1] != 0).sum()) > 4000
