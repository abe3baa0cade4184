"""lib/range/range_proof_test.go equivalents + batched-vs-reference checks."""
import pytest

from drynx_amd.crypto import elgamal as eg
from drynx_amd.ops.encoding import CreateProofBatch
from drynx_amd.proofs import range_proof as rp


@pytest.fixture(scope="module")
def setup():
    S, u, l = 2, 4, 3
    sigs = [[rp.init_range_proof_signature(u) for _ in range(3)] for _ in range(S)]
    kps = [eg.KeyPair.generate() for _ in range(S)]
    P = eg.aggregate_keys([k.public for k in kps])
    return S, u, l, sigs, rp.SigMaterial(sigs), P, eg.pk_table(P)


def _prove(setup, vals, offs=None):
    S, u, l, sigs, sm, P, pk = setup
    cv, r = eg.encrypt_ints(pk, vals)
    n = len(vals)
    b = CreateProofBatch(vals, r, cv, [u] * n, [l] * n, list(range(n)), offs or [0] * n)
    return rp.create_range_proofs(b, sm, P)[0]


def test_valid_proofs_verify_batched_and_reference(setup):
    rpl = _prove(setup, [0, 17, 63])
    sm, P = setup[4], setup[5]
    assert rp.verify_range_proof_list(rpl, sm, P)
    assert all(rp.verify_range_proof_single_reference(rpl, p, sm, P) for p in range(3))


def test_out_of_range_fails(setup):
    rpl = _prove(setup, [64])  # 4^3 = 64 is out of range
    assert not rp.verify_range_proof_list(rpl, setup[4], setup[5])
    assert not rp.verify_range_proof_single_reference(rpl, 0, setup[4], setup[5])


@pytest.mark.parametrize("field", ["A", "V", "zv", "zphi", "zr", "challenge"])
def test_tampering_detected(setup, field):
    rpl = _prove(setup, [5, 6])
    t = getattr(rpl, field)
    t[-1, 3] ^= 4
    assert not rp.verify_range_proof_list(rpl, setup[4], setup[5])


def test_bytes_roundtrip_and_no_proof_case(setup):
    rpl = _prove(setup, [1, 2])
    back = rp.RangeProofList.from_bytes(rpl.to_bytes())
    assert rp.verify_range_proof_list(back, setup[4], setup[5])
    empty = rp.RangeProofList(0, 0, 0, [0], [0], rpl.commit[:1])
    assert rp.verify_range_proof_list(empty, setup[4], setup[5])  # u = l = 0 -> true (range_proof.go:508)


def test_threshold_checks_only_prefix(setup):
    rpl = _prove(setup, [1, 64])  # second proof is bad
    sm, P = setup[4], setup[5]
    assert rp.verify_range_proof_list(rpl, sm, P, threshold=0.5)  # only the first ceil(0.5*2)=1
    assert not rp.verify_range_proof_list(rpl, sm, P, threshold=1.0)


def test_signed_offset_extension(setup):
    rpl = _prove(setup, [-30, 31], offs=[32, 32])
    assert rp.verify_range_proof_list(rpl, setup[4], setup[5])


def test_to_base():
    assert rp.to_base(13, 2, 6) == [1, 0, 1, 1, 0, 0]
    assert rp.to_base(-5, 16, 3) == [0, 0, 0]  # reference: non-positive -> zeros


def test_deterministic_signature():
    a = rp.init_range_proof_signature_deterministic(3)
    b = rp.init_range_proof_signature_deterministic(3)
    assert a == b and len(a.Signature) == 3 * 128


def test_device_challenge_hash_matches_sha3_512():
    """dx_rp_challenges (Keccak on the device/host path) == hashlib SHA3-512 mod r."""
    import numpy as np
    import torch

    from drynx_amd import native as nt
    from drynx_amd.crypto import bn254 as bn
    from drynx_amd.crypto import oracle as O
    from drynx_amd.proofs import range_proof as rp

    pts = [O.g1_mul(k, O.G1_GEN) for k in (1, 2, 3, 12345, O.R - 1)] + [None]
    aff = bn.g1_aff_tensor(pts, "cpu")
    ys = [O.g1_to_bytes(O.g1_mul(k, O.G1_GEN)) for k in (7, 11)]
    cols = [0, 1, 1, 0, 1, 0]
    bw = torch.from_numpy(np.frombuffer(O.g1_to_bytes(O.G1_GEN), dtype="<i4").copy())
    yw = torch.from_numpy(np.frombuffer(b"".join(ys), dtype="<i4").reshape(-1, 16).copy())
    got = bn.scalars_from_tensor(nt.rp_challenges(aff, bw, yw, torch.tensor(cols, dtype=torch.int32)))
    exp = rp._challenge_hash(bn.g1_aff_to_bytes(aff), [ys[c] for c in cols])
    assert got == exp


@pytest.mark.parametrize("bits", ["8", "7", "6", "4", "0"])
def test_prover_table_layouts_agree(setup, bits, monkeypatch):
    """8-bit combs, 4-bit (HBM-sized, random per-CN per-column keys) and the
    table-free prover all produce proofs the batched and the per-equation
    reference verifiers accept."""
    S, u, l, sigs, _, P, pk = setup
    monkeypatch.setenv("DRYNX_PROVER_TABLE_BITS", bits)
    sm = rp.SigMaterial(sigs)  # fresh: the layout is chosen once per signature set
    assert sm.table_mode("cpu") == int(bits)
    cv, r = eg.encrypt_ints(pk, [3, 40, 63])
    b = CreateProofBatch([3, 40, 63], r, cv, [u] * 3, [l] * 3, [0, 1, 2], [0] * 3)
    rpl = rp.create_range_proofs(b, sm, P)[0]
    assert rp.verify_range_proof_list(rpl, sm, P)
    assert all(rp.verify_range_proof_single_reference(rpl, p, sm, P) for p in range(3))


def test_device_digits_match_host_digits():
    """The prover's device digit decomposition (int64, low l digits of
    m + offset) equals the host one, and declines values outside its range."""
    import random

    import torch

    for u, l in [(16, 16), (4, 3), (2, 5), (10, 6)]:
        off = min(u ** l // 2, 1 << 62)
        vals = [random.randint(-off, min(u ** l - off - 1, (1 << 62) - 1)) for _ in range(200)]
        got = rp._digits_dev(torch.tensor(vals), [off] * 200, u, l, "cpu", vals)
        assert (got.numpy() == rp._digits(vals, [off] * 200, u, l)).all()
    assert rp._digits_dev(torch.tensor([1 << 62]), [0], 16, 16, "cpu", [1 << 62]) is None
