"""In-process multi-party surveys (the onet LocalTest analogue): every
operation end to end, proofs + VNs + skipchain, getters, malicious parties."""
import pytest
import torch

from drynx_amd.ops import encoding as enc
from drynx_amd.proofs import requests as prq
from drynx_amd.query import QueryDiffP
from drynx_amd.services.api import DrynxClient
from drynx_amd.services.local import local_cluster, make_survey


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    cl, node = local_cluster(3, 5, 3, device="cpu", workdir=str(tmp_path_factory.mktemp("db")))
    yield cl, node, DrynxClient(node)
    node.close(remove=True)


def _sum_clear(res, n):
    return [sum(v[0][i] for v in res.clear_dp.values()) for i in range(n)]


@pytest.mark.parametrize("op", ["sum", "mean", "variance", "cosim", "frequencyCount", "lin_reg", "MLeval"])
def test_numeric_ops_match_clear(env, op):
    cl, node, client = env
    sq = make_survey(client, cl, op, query_min=0, query_max=6, rows=12, d=2)
    _, vals, res = client.send_survey_query(sq)
    n = sq.Query.Operation.NbrOutput
    tot = _sum_clear(res, n)
    exp = enc.decode_values(op, tot, sq.Query.Operation)
    assert vals[0] == pytest.approx(exp, rel=1e-9, abs=1e-9)


@pytest.mark.parametrize("op", ["min", "max", "bool_OR", "bool_AND", "union", "inter"])
def test_boolean_ops(env, op):
    cl, node, client = env
    dp_data = {}
    rows = [[2, 3, 5], [4, 5, 6], [3, 4, 5], [1, 5, 5], [5, 5, 2]]
    for i, dp in enumerate(cl.dps):
        dp_data[dp.id] = [torch.tensor(rows[i], dtype=torch.int64)]
    node.dp_data = dp_data
    try:
        sq = make_survey(client, cl, op, query_min=0, query_max=6, rows=3)
        _, vals, _ = client.send_survey_query(sq)
    finally:
        node.dp_data = {}
    sets = [set(r) for r in rows]
    exp = {"min": [1.0], "max": [6.0], "bool_OR": [1.0], "bool_AND": [0.0],
           "union": [float(any(i in s for s in sets)) for i in range(7)],
           "inter": [float(all(i in s for s in sets)) for i in range(7)]}[op]
    assert vals[0] == exp


def test_group_by_and_cutting_factor(env):
    cl, node, client = env
    sq = make_survey(client, cl, "mean", query_min=0, query_max=9, rows=10, group_by=(3, 2))
    groups, vals, res = client.send_survey_query(sq)
    assert len(groups) == 6 and all(v == vals[0] for v in vals)
    sq = make_survey(client, cl, "sum", query_min=0, query_max=9, rows=10, cutting_factor=3)
    _, vals, res = client.send_survey_query(sq)
    assert vals[0][0] == sum(v[0][0] for v in res.clear_dp.values())


def test_proofs_skipchain_and_getters(env):
    cl, node, client = env
    sq = make_survey(client, cl, "frequencyCount", query_min=0, query_max=3, rows=6, proofs=1, ranges=[2, 4])
    _, vals, res = client.send_survey_query(sq)
    assert vals[0] == [float(x) for x in _sum_clear(res, 4)]
    b = res.block
    codes = b.data_block().Proofs
    assert set(codes.values()) == {prq.PROOF_TRUE}
    assert len(codes) == 3 * (5 + 3 + 3)  # VNs x (range per DP + aggregation per CN + keyswitch per CN)
    assert b.verify_signatures({p.id: p.public for p in cl.parties})
    assert client.send_get_block("vn2", sq.SurveyID).Hash == b.Hash
    assert client.send_get_latest_block("vn0").Hash == b.Hash
    assert client.send_get_genesis("vn1") is not None
    proofs = client.send_get_proofs("vn0", sq.SurveyID)
    assert len(proofs) == 5 + 3 + 3 and all(k.endswith("/vn0") for k in proofs)
    assert node.get_bitmap("vn1", sq.SurveyID) == {k: v for k, v in codes.items() if k.endswith("/vn1")}
    # second survey appends a linked block
    sq2 = make_survey(client, cl, "sum", query_min=0, query_max=3, rows=6, proofs=1, ranges=[2, 4])
    _, _, res2 = client.send_survey_query(sq2)
    assert res2.block.BackLink == b.Hash and res2.block.Index == b.Index + 1


def test_obfuscation_and_diffp_with_proofs(env):
    cl, node, client = env
    sq = make_survey(client, cl, "union", query_min=0, query_max=4, rows=4, proofs=1, ranges=[2, 1],
                     obfuscation=True)
    _, vals, res = client.send_survey_query(sq)
    assert set(res.block.data_block().Proofs.values()) == {1}
    dp = QueryDiffP(LapMean=0.0, LapScale=1.0, NoiseListSize=8, Quanta=1.0, Scale=1.0, Limit=3)
    sq = make_survey(client, cl, "sum", query_min=0, query_max=4, rows=4, proofs=1, ranges=[16, 4], diffp=dp)
    _, vals, res = client.send_survey_query(sq)
    assert abs(vals[0][0] - sum(v[0][0] for v in res.clear_dp.values())) <= 3
    kinds = {k.split("/")[1] for k in res.block.data_block().Proofs}
    assert kinds == {"range", "aggregation", "keyswitch", "shuffle"}


def test_malicious_dp_and_bad_signature_recorded(env, monkeypatch):
    """Fault injection: a DP lying about its range and a forged
    envelope signature show up as bitmap codes 0 and 4."""
    cl, node, client = env
    orig = node._range_proofs

    def evil(sq, dp_results, proofs):
        orig(sq, dp_results, proofs)
        for r in proofs:
            if r.kind == "range" and r.sender_id == "dp0":
                r.obj[0].zv[0, 1] ^= 1  # corrupt after signing -> content false
                r.data = prq.range_bundle_to_bytes(r.obj)
                r.signature = __import__("drynx_amd.proofs.sigma", fromlist=["x"]).schnorr_sign(
                    cl.by_id("dp0").keypair.secret, r.digest())
            if r.kind == "range" and r.sender_id == "dp1":
                r.signature = b"\x00" * 96
    monkeypatch.setattr(node, "_range_proofs", evil)
    sq = make_survey(client, cl, "sum", query_min=0, query_max=3, rows=4, proofs=1, ranges=[16, 2])
    _, _, res = client.send_survey_query(sq)
    codes = res.block.data_block().Proofs
    assert {v for k, v in codes.items() if "/range/dp0/" in k} == {prq.PROOF_FALSE}
    assert {v for k, v in codes.items() if "/range/dp1/" in k} == {prq.PROOF_FALSE_SIGN}
    assert {v for k, v in codes.items() if "/range/dp2/" in k} == {prq.PROOF_TRUE}


def test_sampled_verification_codes(env):
    cl, node, client = env
    sq = make_survey(client, cl, "sum", query_min=0, query_max=3, rows=4, proofs=1, ranges=[16, 2],
                     verification_sharding=1)
    _, _, res = client.send_survey_query(sq)
    codes = res.block.data_block().Proofs
    by_req = {}
    for k, v in codes.items():
        by_req.setdefault(k.rsplit("/", 1)[0], []).append(v)
    for v in by_req.values():
        assert sorted(v) == [1, 2, 2]  # exactly one VN verified each request


def test_close_db(env, tmp_path):
    cl, node = local_cluster(2, 2, 1, device="cpu", workdir=str(tmp_path))
    client = DrynxClient(node)
    sq = make_survey(client, cl, "sum", query_min=0, query_max=3, rows=4, proofs=1, ranges=[16, 2])
    client.send_survey_query(sq)
    import os

    path = os.path.join(str(tmp_path), "db_vn0.sqlite")
    assert os.path.exists(path)
    client.send_close_db("vn0", remove=True)
    assert not os.path.exists(path)


def test_chain_resumes_after_restart(tmp_path):
    """Checkpoint/resume: a node restarted over the same workdir appends to the
    persisted skipchain (back link to the last block) instead of a new genesis."""
    cl, node = local_cluster(2, 2, 1, device="cpu", workdir=str(tmp_path), deterministic_keys=True)
    client = DrynxClient(node)
    sq = make_survey(client, cl, "sum", query_min=0, query_max=3, rows=4, proofs=1, ranges=[16, 2])
    _, _, res1 = client.send_survey_query(sq)
    node.close()
    cl2, node2 = local_cluster(2, 2, 1, device="cpu", workdir=str(tmp_path), deterministic_keys=True)
    client2 = DrynxClient(node2)
    sq2 = make_survey(client2, cl2, "sum", query_min=0, query_max=3, rows=4, proofs=1, ranges=[16, 2])
    _, _, res2 = client2.send_survey_query(sq2)
    assert res2.block.Index == res1.block.Index + 1
    assert res2.block.BackLink == res1.block.Hash
    assert res2.block.GenesisID == res1.block.GenesisID
    assert node2.get_genesis("vn0").Hash == res1.block.GenesisID
    node2.close(remove=True)


def test_fault_plan_marks_malicious_parties(tmp_path):
    """FaultPlan: a DP with a corrupted range proof -> 0, a CN with a
    forged key-switch envelope -> 4, an honest CN's aggregation proof -> 1."""
    from drynx_amd.utils.faults import FaultPlan

    cl, node = local_cluster(3, 3, 2, device="cpu", workdir=str(tmp_path))
    client = DrynxClient(node)
    node.fault_plan = FaultPlan({("dp1", "range"): "corrupt_proof", ("cn2", "keyswitch"): "bad_signature",
                                 ("cn0", "aggregation"): "corrupt_proof"})
    sq = make_survey(client, cl, "sum", query_min=0, query_max=3, rows=4, proofs=1, ranges=[16, 2])
    _, _, res = client.send_survey_query(sq)
    codes = res.block.data_block().Proofs
    by = lambda frag: {v for k, v in codes.items() if frag in k}  # noqa: E731
    assert by("/range/dp1/") == {prq.PROOF_FALSE}
    assert by("/range/dp0/") == by("/range/dp2/") == {prq.PROOF_TRUE}
    assert by("/keyswitch/cn2/") == {prq.PROOF_FALSE_SIGN}
    assert by("/keyswitch/cn0/") == {prq.PROOF_TRUE}
    assert by("/aggregation/cn0/") == {prq.PROOF_FALSE}
    node.close(remove=True)


@pytest.mark.parametrize("mode", [1, 2])
def test_strict_range_modes_end_to_end(env, mode):
    """SurveyQuery.RangeProofMode: the DPs prove (v2 transcript for mode 2),
    every VN recomputes the challenge and checks V in G2 -> all codes 1."""
    cl, node, client = env
    sq = make_survey(client, cl, "sum", query_min=0, query_max=9, rows=6, proofs=1, ranges=[16, 2],
                     range_proof_mode=mode)
    _, vals, res = client.send_survey_query(sq)
    assert vals[0][0] == sum(v[0][0] for v in res.clear_dp.values())
    assert set(res.block.data_block().Proofs.values()) == {prq.PROOF_TRUE}


def test_vn_api_registration_and_blocking_end_verification(env):
    """SendSurveyQueryToVNs then a SendEndVerification issued BEFORE the survey
    runs: it blocks until the root VN appended the survey's block."""
    import threading

    cl, node, client = env
    sq = make_survey(client, cl, "sum", query_min=0, query_max=9, rows=6, proofs=1, ranges=[16, 2])
    client.send_survey_query_to_vns(sq)
    assert sq.SurveyID in node.vn_surveys
    got = {}
    t = threading.Thread(target=lambda: got.setdefault("b", client.send_end_verification("vn0", sq.SurveyID, 120)))
    t.start()
    _, _, res = client.send_survey_query(sq)
    t.join(120)
    assert got["b"] is not None and got["b"].Hash == res.block.Hash
    assert client.send_end_verification("vn0", "no-such-survey", 0.05) is None


def test_get_proofs_reference_layout_roundtrip(env):
    """GetProofs serves range proofs as network.Marshal(&RangeProofListBytes)
    (range_proof.go:72-155, proof_collection_protocol.go:318-331): decode the
    bytes with the query's ranges and verify them again."""
    from drynx_amd.proofs import range_proof as rp
    from drynx_amd.proofs import range_wire as rw

    cl, node, client = env
    sq = make_survey(client, cl, "mean", query_min=0, query_max=9, rows=6, proofs=1, ranges=[16, 3])
    _, _, res = client.send_survey_query(sq)
    proofs = client.send_get_proofs("vn1", sq.SurveyID)
    rng = {k: v for k, v in proofs.items() if "/range/" in k}
    assert len(rng) == 5
    sm = node.verifier_cache.sigmat(sq, "cpu")
    P = sq.RosterServers.aggregate()
    for k, b in rng.items():
        assert b[:16] == rw.onet.message_type_id(rw.LIST_TYPE)
        lists = rw.decode_bundle(b, sq.Query.Ranges)
        assert len(lists) == 1 and len(lists[0]) == 2  # mean: 2 outputs, one proof each
        assert rp.verify_range_proof_list(lists[0], sm, P)
    # a flipped byte inside one proof's A values breaks exactly that list
    k0 = next(iter(rng))
    bad = bytearray(rng[k0])
    bad[-5] ^= 1
    assert not rp.verify_range_proof_list(rw.decode_bundle(bytes(bad), sq.Query.Ranges)[0], sm, P)


def test_skipchain_forward_links_and_update_chain(env):
    """Genesis -> latest through verified forward links (GetUpdateChain /
    GetLatestBlock from a known block); VerifyBase and forward-link checks
    reject a block with a bad back link or a forged forward link."""
    import dataclasses

    from drynx_amd.ledger import skipchain as skc

    cl, node, client = env
    for _ in range(2):
        sq = make_survey(client, cl, "sum", query_min=0, query_max=3, rows=4, proofs=1, ranges=[16, 2])
        client.send_survey_query(sq)
    head = client.send_get_latest_block("vn0")
    genesis = client.send_get_genesis("vn0")
    chain = node.get_update_chain("vn0", genesis)
    assert chain[0].Hash == genesis.Hash and chain[-1].Hash == head.Hash
    assert [b.Index for b in chain] == list(range(head.Index + 1))
    assert all(skc.verify_base(a, b) for a, b in zip(chain, chain[1:]))
    assert client.send_get_latest_block("vn2", genesis).Hash == head.Hash
    # structural checks
    bad = dataclasses.replace(head, BackLink="00" * 32)
    bad.Hash = bad.compute_hash()
    assert not skc.verify_base(chain[-2], bad)
    assert not skc.verify_base(chain[-2], dataclasses.replace(head, Index=head.Index + 5))
    # a forward link whose signature does not cover the target is rejected
    prev = chain[-2]
    forged = dict(prev.ForwardLinks[-1], To=genesis.Hash)
    assert skc.verify_forward_link(prev, prev.ForwardLinks[-1])
    assert not skc.verify_forward_link(prev, forged)
    import pytest as _pt
    tampered = dataclasses.replace(prev, ForwardLinks=[forged])
    with _pt.raises(ValueError):
        skc.update_chain(lambda h: {b.Hash: b for b in chain}.get(h), tampered)


def test_malformed_queries_give_bitmap_codes(env):
    """Queries whose range proofs cannot verify end with a block of 0 codes,
    not an exception: (a) Ranges too narrow for the DPs' values (u^l = 2:
    every DP's sum is >= 2), (b) input-validation signatures for a smaller
    base than the query's Ranges announce (u = 4 keys, Ranges u = 16) as seen
    by the VNs; a DP asked to prove against such a query refuses up front."""
    cl, node, client = env
    sq = make_survey(client, cl, "sum", query_min=1, query_max=3, rows=4, proofs=1, ranges=[2, 1])
    _, vals, res = client.send_survey_query(sq)
    codes = res.block.data_block().Proofs
    rng = {v for k, v in codes.items() if "/range/" in k}
    assert rng == {prq.PROOF_FALSE}
    assert {v for k, v in codes.items() if "/aggregation/" in k or "/keyswitch/" in k} == {prq.PROOF_TRUE}
    assert vals[0][0] == float(sum(v[0][0] for v in res.clear_dp.values()))  # the query result itself is unaffected

    orig = node._range_proofs

    def then_widen(sq, dp_results, proofs):  # proofs made for u = 4; the VNs' query says u = 16
        orig(sq, dp_results, proofs)
        sq.Query.Ranges = [[16, 2]]

    sq = make_survey(client, cl, "sum", query_min=0, query_max=3, rows=4, proofs=1, ranges=[4, 2])
    node._range_proofs = then_widen
    try:
        _, _, res = client.send_survey_query(sq)
    finally:
        del node._range_proofs
    codes = res.block.data_block().Proofs
    assert {v for k, v in codes.items() if "/range/" in k} == {prq.PROOF_FALSE}

    sq = make_survey(client, cl, "sum", query_min=0, query_max=3, rows=4, proofs=1, ranges=[4, 2])
    sq.Query.Ranges = [[16, 2]]
    with pytest.raises(ValueError, match="signatures"):
        client.send_survey_query(sq)


def test_per_party_timers(env):
    """<dp>_AllProofs spans proving to the VNs' verdicts coming back
    (data_collection_protocol.go:280-345), so it covers this rank's proving
    batch (RangeProving) and ends after every VN's own VerifyRange started;
    every VN of the roster records its own VerifyRange / VerifyKeySwitch."""
    from drynx_amd.utils import timers

    cl, node, client = env
    timers.reset()
    sq = make_survey(client, cl, "sum", query_min=0, query_max=3, rows=6, proofs=1, ranges=[2, 4])
    client.send_survey_query(sq)
    rec = timers.summary()
    assert "RangeProving" in rec
    for dp in cl.dps:
        assert rec[f"{dp.id}_AllProofs"]["sum"] >= rec["RangeProving"]["sum"]
    for vn in cl.vns:
        assert rec[f"{vn.id}_VerifyRange"]["n"] >= 1
        assert f"{vn.id}_VerifyKeySwitch" in rec
    assert not node.take_proof_starts(sq.SurveyID)  # consumed at the feedback point


def test_range_batches_chunked_by_u_cap(tmp_path, monkeypatch):
    """Inboxes above DRYNX_VERIFY_CHUNK_U pairing-side points are verified in
    several batches (a list split across batches by proof ranges): honest
    lists still pass and a forged one is still blamed exactly."""
    from drynx_amd.proofs import requests as prq_mod
    from drynx_amd.utils.faults import FaultPlan

    monkeypatch.setenv("DRYNX_VERIFY_CHUNK_U", "40")  # 2 VNs x 20: lists of 8 proofs x 3 servers split
    seen = []
    orig = prq_mod._item_chunks
    monkeypatch.setattr(prq_mod, "_item_chunks", lambda *a: seen.append(len(orig(*a))) or orig(*a))
    cl, node = local_cluster(3, 3, 2, device="cpu", workdir=str(tmp_path))
    client = DrynxClient(node)
    node.fault_plan = FaultPlan({("dp1", "range"): "corrupt_proof"})
    sq = make_survey(client, cl, "frequencyCount", query_min=0, query_max=7, rows=4, proofs=1, ranges=[4, 2])
    _, _, res = client.send_survey_query(sq)
    codes = res.block.data_block().Proofs
    by = lambda frag: {v for k, v in codes.items() if frag in k}  # noqa: E731
    assert max(seen) > 2
    assert by("/range/dp1/") == {prq.PROOF_FALSE}
    assert by("/range/dp0/") == by("/range/dp2/") == {prq.PROOF_TRUE}
    node.close(remove=True)
