"""Compact ledger form of range payloads (proofs/ledger_codec.py): GT elements
stored as torus (T2) images and rebuilt bit for bit, on the host build here
and on the GPU in the marked test; a bundle whose GT elements do not round-trip
falls back to its raw bytes; the store returns the signed bytes either way."""
import os

import pytest
import torch

from drynx_amd import native as nt
from drynx_amd.crypto import elgamal as eg
from drynx_amd.ledger.store import Store
from drynx_amd.ops.encoding import CreateProofBatch
from drynx_amd.proofs import ledger_codec as lc
from drynx_amd.proofs import range_proof as rp
from drynx_amd.proofs import requests as prq


@pytest.fixture(scope="module")
def bundle():
    S, u, l = 2, 4, 3
    sigs = [rp.init_range_proof_signatures([u] * 2) for _ in range(S)]
    kps = [eg.KeyPair.generate() for _ in range(S)]
    P = eg.aggregate_keys([k.public for k in kps])
    vals = [1, 5, 7, 2, 9, 3]
    cv, r = eg.encrypt_ints(eg.pk_table(P), vals)
    n = len(vals)
    lists = rp.create_range_proofs(CreateProofBatch(vals, r, cv, [u] * n, [l] * n, [0, 1] * (n // 2), [0] * n),
                                   rp.SigMaterial(sigs), P)
    return prq.range_bundle_pack(lists)


def _roundtrip(t: torch.Tensor):
    req = prq.ProofRequest("range", "s", "dp", "", None, b"", tensor=t)
    req.decoded = prq.range_bundle_unpack(t)
    pend = lc.prepare(req)
    assert pend is not None
    img = pend.launch()
    if img.is_cuda:
        torch.cuda.synchronize()
    host = img.cpu().numpy()
    return pend.finish(memoryview(host).cast("B"))


def _check(t: torch.Tensor):
    raw = t.cpu().numpy().tobytes()
    stored = bytes(_roundtrip(t))
    assert lc.is_compressed(stored) and len(stored) < 0.6 * len(raw)
    assert lc.decompress_bytes(stored, device=t.device) == raw
    bad = t.clone()
    bad[-7] ^= 1  # one limb of the last GT element: no longer unitary
    stored_bad = bytes(_roundtrip(bad))
    assert not lc.is_compressed(stored_bad) and stored_bad == bad.cpu().numpy().tobytes()


def test_t2_roundtrip_and_fallback_host(bundle):
    _check(bundle)


def test_gt_t2_rejects_non_unitary():
    from drynx_amd.crypto import bn254 as bn

    z = torch.zeros((2, 96), dtype=torch.int32)
    _, ok = nt.gt_t2_compress(z)
    assert ok.tolist() == [0, 0]
    one = torch.zeros((1, 96), dtype=torch.int32)  # 1 = 1 + 0 w: h = 0, no torus image
    one[0, :8] = bn.to_tensor(bn.ints_to_limbs([bn.mont(1)]), "cpu").reshape(-1)
    _, ok1 = nt.gt_t2_compress(one)
    assert ok1.tolist() == [0]


def test_store_returns_signed_bytes(tmp_path, bundle):
    """A compact image the writer TAGGED (``ledger.store.Compact``: a rank's
    blob segment or a node-shared file) reads back as the signed bytes; the
    same image stored untagged, or any value that merely looks like one, is
    returned as stored (nothing is decompressed by sniffing)."""
    from drynx_amd.ledger.store import BlobSegment, Compact, NodeBlobs

    stored = bytes(_roundtrip(bundle))
    signed = bundle.cpu().numpy().tobytes()
    st = Store(str(tmp_path / "db.sqlite"))
    seg = BlobSegment(str(tmp_path / "ledger_r0.blobs"))
    ref_c, ref_r = seg.put_many(["c", "r"], lambda: [Compact(memoryview(stored)), memoryview(stored)])
    st.update("s/range", "tagged", ref_c)
    st.update("s/range", "untagged", ref_r)
    st.update("s/range", "inline", stored)
    assert st.get("s/range", "tagged") == signed
    assert st.get("s/range", "untagged") == stored and st.get("s/range", "inline") == stored
    # node-shared: the claimant writes the compact image, another rank's whole-file reference reads it
    root = str(tmp_path / "node")
    w, r = NodeBlobs(root), NodeBlobs(root)
    assert w.claim(["d"]) == [True] and r.claim(["d"]) == [False]
    w.put_many(["d"], lambda: [Compact(memoryview(stored))])
    w.flush()
    st.update("s/range", "node", r.put_refs(["d"])[0])
    assert st.get("s/range", "node") == signed
    st.update("s/other", "k", b"RPC2" + b"\0" * 40)
    assert st.get("s/other", "k") == b"RPC2" + b"\0" * 40
    st.close()
    seg.close(remove=True)
    w.close(remove=True)
    assert os.path.exists(root)  # another user (r) still has the node directory open
    r.close(remove=True)
    assert not os.path.exists(root)


@pytest.mark.gpu
def test_t2_roundtrip_gpu(bundle):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _check(bundle.cuda())
    # device compress == host compress, device decompress == host decompress
    A = prq.range_bundle_unpack(bundle)[0].A
    c_h, ok_h = nt.gt_t2_compress(A)
    c_d, ok_d = nt.gt_t2_compress(A.cuda())
    assert torch.equal(c_h, c_d.cpu()) and torch.equal(ok_h, ok_d.cpu()) and bool(ok_h.all())
    assert torch.equal(nt.gt_t2_decompress(c_d).cpu(), A)


def test_regions_from_header_match_decoded_views(bundle):
    req = prq.ProofRequest("range", "s", "dp", "", None, b"", tensor=bundle)
    req.decoded = prq.range_bundle_unpack(bundle)
    assert lc.regions_from_header(bundle) == lc.prepare(req).regions
    two = prq.range_bundle_pack(prq.range_bundle_unpack(bundle) * 2)  # a two-list bundle
    req2 = prq.ProofRequest("range", "s", "dp", "", None, b"", tensor=two)
    req2.decoded = prq.range_bundle_unpack(two)
    regs = lc.regions_from_header(two)
    assert len(regs) == 4 and regs == lc.prepare(req2).regions
    assert lc.regions_from_header(two[:-1]) == []  # a layout that does not add up: stored raw
    assert lc.prepare(prq.ProofRequest("range", "s", "dp", "", None, b"", tensor=two)).regions is None


def test_regions_from_shape(bundle):
    assert lc.regions_from_shape(bundle.numel(), 2, 3) == lc.regions_from_header(bundle)
    assert lc.regions_from_shape(bundle.numel(), 3, 3) is None  # a shape that does not divide: header path


def test_g2_block_fallback(bundle):
    """A V_j off the twist makes the bundle fall back to raw bytes too."""
    req = prq.ProofRequest("range", "s", "dp", "", None, b"", tensor=bundle)
    req.decoded = prq.range_bundle_unpack(bundle)
    off, m, kind = lc.prepare(req).regions[0]
    assert kind == 1
    bad = bundle.clone()
    bad[off + 3] ^= 1  # x of the first V: (almost surely) no longer on the twist
    stored = bytes(_roundtrip(bad))
    assert not lc.is_compressed(stored) and stored == bad.cpu().numpy().tobytes()


def test_coalesce_adjacent_blob_buffers():
    """ledger.store._coalesce: slices of one host buffer that sit back to back
    merge into one write; other buffers break the run; bytes unchanged."""
    import numpy as np

    from drynx_amd.ledger.store import _coalesce

    mv = memoryview(np.arange(10000, dtype=np.uint8))
    bufs = [mv[i * 100:(i + 1) * 100] for i in range(100)]
    assert [b.nbytes for b in _coalesce(bufs)] == [10000]
    mixed = bufs[:50] + [memoryview(b"x" * 100)] + bufs[60:]
    out = _coalesce(mixed)
    assert [b.nbytes for b in out] == [5000, 100, 4000]
    assert b"".join(bytes(b) for b in out) == b"".join(bytes(b) for b in mixed)
