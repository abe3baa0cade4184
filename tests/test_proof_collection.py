"""ProofCollection protocol with the good-proof factory (reference:
protocols/proof_collection_protocol_test.go:43-294 — one prover, 3 VNs,
nbrProofs of each kind, every bitmap entry must be ProofTrue) plus a
tampered-envelope case."""

from drynx_amd.proofs import requests as prq
from drynx_amd.protocols import proof_collection as pcp
from drynx_amd.services.api import DrynxClient
from drynx_amd.services.local import local_cluster, make_survey
from drynx_amd.utils.test_data import create_random_good_test_data

def _setup(tmp_path):
    cl, node = local_cluster(3, 1, 3, device="cpu", workdir=str(tmp_path))
    client = DrynxClient(node)
    sq = make_survey(client, cl, "mean", query_min=0, query_max=10, rows=4, proofs=1, ranges=[16, 16])
    return cl, node, sq


def _requests(cl, sq, data):
    cn = cl.cns[0]
    reqs = []
    for kind, proofs in data.items():
        sender = cl.dps[0] if kind == "range" else cn
        for i, pr in enumerate(proofs):
            reqs.append(prq.new_proof_request(kind, pr, sq.SurveyID, sender.id, str(i), sender.keypair.secret))
    return reqs


def test_all_good_proofs_recorded_true(tmp_path):
    cl, node, sq = _setup(tmp_path)
    data = create_random_good_test_data(sq.RosterServers.aggregate(), sq.ClientPubKey,
                                        sq.Query.IVSigs.InputValidationSigs, 2, entity=cl.cns[0].keypair)
    block = pcp.proof_collection(node, sq, _requests(cl, sq, data))
    codes = block.data_block().Proofs
    assert len(codes) == 3 * 2 * 5  # every VN records every request
    assert set(codes.values()) == {prq.PROOF_TRUE}
    assert block.verify_signatures()
    # every VN stored every non-shuffle proof (storeProof skips shuffles)
    stored = node.get_proofs("vn1", sq.SurveyID)
    assert len(stored) == 2 * 4
    node.close(remove=True)


def test_tampered_payload_is_a_bad_signature(tmp_path):
    cl, node, sq = _setup(tmp_path)
    data = create_random_good_test_data(sq.RosterServers.aggregate(), sq.ClientPubKey,
                                        sq.Query.IVSigs.InputValidationSigs, 1, entity=cl.cns[0].keypair)
    reqs = _requests(cl, sq, data)
    for r in reqs:
        if r.kind == "aggregation":
            b = bytearray(r.data)
            b[-1] ^= 1
            r.data = bytes(b)
            r.obj = None
    codes = pcp.proof_collection(node, sq, reqs).data_block().Proofs
    assert {v for k, v in codes.items() if "/aggregation/" in k} == {prq.PROOF_FALSE_SIGN}
    assert {v for k, v in codes.items() if "/aggregation/" not in k} == {prq.PROOF_TRUE}
    node.close(remove=True)


def test_early_range_plane_only_with_range_proofs(tmp_path, monkeypatch):
    """The range plane starts before the CN phases only when there are range
    proofs to verify: with ranges (0, 0) the DPs ship commitments only and
    their signing / fan-out stays off the CN phases' thread
    (``early_plane_ok``); the pool itself is used either way."""
    cl, node, sq = _setup(tmp_path)
    assert pcp.early_plane_ok(node, sq)
    client = DrynxClient(node)
    sq0 = make_survey(client, cl, "mean", query_min=0, query_max=10, rows=4, proofs=1, ranges=[0, 0])
    assert not pcp.early_plane_ok(node, sq0)
    monkeypatch.setenv("DRYNX_RANGE_PLANE", "0")
    assert not pcp.early_plane_ok(node, sq)
    node.close(remove=True)


def test_commitment_only_lists_are_not_decoded(tmp_path, monkeypatch):
    """With every query range (0, 0) the verification is true whatever the
    list holds (range_proof.go:508-510): the VN neither decodes nor checks the
    commitment-only bundles (the serial path's rp.verify.unpack_many)."""
    cl, node, sq = _setup(tmp_path)
    client = DrynxClient(node)
    sq0 = make_survey(client, cl, "mean", query_min=0, query_max=10, rows=4, proofs=1, ranges=[0, 0])
    calls = []
    monkeypatch.setattr(prq, "range_bundle_unpack_many", lambda ts: calls.append(len(ts)) or [])
    monkeypatch.setattr(prq, "range_bundle_unpack", lambda t: calls.append(1))
    req = prq.ProofRequest("range", sq0.SurveyID, cl.dps[0].id, "", b"\x00" * 64, b"")
    base, parts = prq._range_parts([req, req], [0, 1], sq0, "cpu", None)
    assert base == {0: True, 1: True} and parts == {0: [], 1: []} and not calls
    # a query with range proofs still decodes (and rejects the garbage)
    base, _ = prq._range_parts([req], [0], sq, "cpu", None)
    assert base == {0: False}
    node.close(remove=True)
