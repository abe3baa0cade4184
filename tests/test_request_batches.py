"""Batched envelopes for many DPs (ScaleDPs: thousands of one-proof DPs per
rank): packing, digests and Schnorr signatures of all bundles at once, and the
VN's batched decode, against the one-bundle paths
(lib/proof/structs_proofs.go:110-182 marshal + sign / unmarshal)."""
import pytest
import torch

from drynx_amd.crypto import digest as dg
from drynx_amd.crypto import elgamal as eg
from drynx_amd.crypto import oracle as O
from drynx_amd.ops.encoding import CreateProofBatch
from drynx_amd.proofs import range_proof as rp
from drynx_amd.proofs import requests as prq
from drynx_amd.proofs import sigma


@pytest.fixture(scope="module")
def bundles():
    S, u, l = 2, 4, 3
    sigs = [rp.init_range_proof_signatures([u] * 2) for _ in range(S)]
    kps = [eg.KeyPair.generate() for _ in range(S)]
    P = eg.aggregate_keys([k.public for k in kps])
    pk = eg.pk_table(P)
    vals = [1, 5, 7, 2, 9, 3, 0, 4]
    cv, r = eg.encrypt_ints(pk, vals)
    n = len(vals)
    big = rp.create_range_proofs(CreateProofBatch(vals, r, cv, [u] * n, [l] * n, [0, 1] * (n // 2), [0] * n),
                                 rp.SigMaterial(sigs), P)[0]
    # four DPs with two proofs each: consecutive slices of one prover batch
    return [[rp.rpl_range(big, 2 * g, 2 * g + 2)] for g in range(4)], rp.SigMaterial(sigs), P


def test_pack_many_matches_single(bundles):
    bs, _, _ = bundles
    ts, packed = prq.range_bundle_pack_many(bs)
    assert packed is not None and packed.shape[0] == 4
    for b, t in zip(bs, ts):
        assert torch.equal(t, prq.range_bundle_pack(b))
    # non-consecutive inputs take the stacking path, same bytes
    ts2, packed2 = prq.range_bundle_pack_many([bs[2], bs[0]])
    assert torch.equal(ts2[0], prq.range_bundle_pack(bs[2])) and torch.equal(ts2[1], prq.range_bundle_pack(bs[0]))
    # mixed shapes: bundle by bundle
    ts3, packed3 = prq.range_bundle_pack_many([bs[0], bs[1] + bs[2]])
    assert packed3 is None and torch.equal(ts3[1], prq.range_bundle_pack(bs[1] + bs[2]))


def test_digest_rows_matches_digest_tensor(bundles):
    ts, packed = prq.range_bundle_pack_many(bundles[0])
    assert dg.digest_rows(packed) == [dg.digest_tensor(t) for t in ts]
    assert dg.digest_rows(packed) == [dg.digest_bytes(t.numpy().tobytes()) for t in ts]


def test_schnorr_sign_batch_verifies():
    secrets = [O.random_scalar() for _ in range(5)]
    msgs = [bytes([i]) * (i + 1) for i in range(5)]
    sigs = sigma.schnorr_sign_batch(secrets, msgs)
    for x, m, s in zip(secrets, msgs, sigs):
        X = O.g1_mul(x, O.G1_GEN)
        assert sigma.schnorr_verify(X, m, s)
        assert not sigma.schnorr_verify(X, m + b"!", s)


def test_new_range_requests_and_unpack_many(bundles):
    bs, sm, P = bundles
    secrets = [O.random_scalar() for _ in bs]
    reqs = prq.new_range_requests([(f"dp{i}", b) for i, b in enumerate(bs)], "s1", secrets, "cpu")
    for req, x in zip(reqs, secrets):
        assert prq.verify_signature(req, O.g1_mul(x, O.G1_GEN))
        fresh = prq.ProofRequest("range", "s1", req.sender_id, "", None, b"", tensor=req.tensor)
        assert fresh.digest() == req.digest()
    dec = prq.range_bundle_unpack_many([r.tensor for r in reqs])
    for d, b in zip(dec, bs):
        assert len(d) == 1 and d[0].cols == b[0].cols and d[0].offset == b[0].offset
        assert torch.equal(d[0].A, b[0].A) and torch.equal(d[0].commit.K, b[0].commit.K)
        assert rp.verify_range_proof_list(d[0], sm, P)


def test_unpack_many_rejects_malformed(bundles):
    ts, _ = prq.range_bundle_pack_many(bundles[0])
    bad_len = ts[0][:-5].clone()                   # truncated payload
    bad_size = ts[1].clone()
    bad_size[1] += 1                               # size word does not match
    bad_n = ts[2].clone()
    bad_n[3] = 3                                   # proof count does not match the fields
    tiny = torch.tensor([1, 2, 3], dtype=torch.int32)
    out = prq.range_bundle_unpack_many([bad_len, bad_size, bad_n, tiny, ts[3]])
    assert all(isinstance(o, Exception) for o in out[:4])
    assert isinstance(out[4], list)


def test_unpack_many_wide_lists():
    """Bundles of ONE list with more than 64 proofs (a wide query's DP list:
    2070 proofs for SPECTF LR) decode through the batched header path, equal to
    the one-bundle decode, and a truncated one is rejected alone."""
    vals = list(range(70))
    pk = eg.pk_table(eg.KeyPair.generate().public)
    cv, _ = eg.encrypt_ints(pk, vals)
    cols = [i % 5 for i in range(70)]
    lists = [rp.RangeProofList(0, 0, 0, [7 * i for i in range(70)], cols, cv)]
    t = prq.range_bundle_pack(lists)
    short = t[:-24]
    out = prq.range_bundle_unpack_many([t, t.clone(), short])
    ref = prq.range_bundle_unpack(t)
    for got in out[:2]:
        assert got[0].offset == ref[0].offset and got[0].cols == ref[0].cols
        assert torch.equal(got[0].commit.K, ref[0].commit.K) and torch.equal(got[0].commit.C, ref[0].commit.C)
    assert isinstance(out[2], Exception)


def test_cat_rows_strided_blocks_match_cat():
    """native.cat_rows: >= 256 equally shaped blocks at a constant stride in one
    storage take one strided copy; the result equals torch.cat and owns its
    memory (also when the blocks are adjacent)."""
    from drynx_amd import native as nt

    base = torch.arange(300 * 37, dtype=torch.int32).view(300, 37)
    for blocks in ([base[i, 5:17].view(3, 4) for i in range(300)],
                   [base.view(-1)[12 * i: 12 * (i + 1)].view(3, 4) for i in range(300)]):
        out = nt.cat_rows([blocks])[0]
        assert torch.equal(out, torch.cat(blocks)) and out.untyped_storage().data_ptr() != base.data_ptr()
    few = [base[i, 5:17].view(3, 4) for i in range(10)]
    assert torch.equal(nt.cat_rows([few])[0], torch.cat(few))


def test_unpack_many_packed_rows_fast_path(bundles):
    """>= 64 one-list bundles packed as rows of one tensor take the unbind fast
    path; every list equals the per-bundle unpack (fields, offsets, columns)."""
    bs, _, _ = bundles
    many = [bs[g % 4] for g in range(80)]
    ts, packed = prq.range_bundle_pack_many(many)
    assert packed is not None
    fast = prq.range_bundle_unpack_many(ts)
    for t, f in zip(ts, fast):
        ref = prq.range_bundle_unpack(t)
        assert len(f) == len(ref) == 1
        a, b = f[0], ref[0]
        assert (a.u, a.l, a.S, a.offset, a.cols) == (b.u, b.l, b.S, b.offset, b.cols)
        for fld in ("challenge", "zr", "D", "zphi", "zv", "V", "A"):
            assert torch.equal(getattr(a, fld), getattr(b, fld)), fld
        assert torch.equal(a.commit.K, b.commit.K) and torch.equal(a.commit.C, b.commit.C)
    # a malformed row (wrong magic) makes the batch take the per-bundle path: that bundle alone is rejected
    bad = packed.clone()
    bad[5, 2] = 0
    rows = list(bad.unbind(0))
    res = prq.range_bundle_unpack_many(rows)
    assert isinstance(res[5], Exception) and all(isinstance(x, list) for i, x in enumerate(res) if i != 5)
