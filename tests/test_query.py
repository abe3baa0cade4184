"""lib/structs.go behaviours: ChooseOperation, CheckParameters, QueryToProofsNbrs, serialisation."""
import pytest

from drynx_amd import query as Q
from drynx_amd.crypto import oracle as O


@pytest.mark.parametrize("name,io", [("sum", (1, 1)), ("mean", (1, 2)), ("variance", (1, 3)), ("cosim", (2, 5)),
                                     ("frequencyCount", (1, 11)), ("min", (1, 11)), ("union", (1, 11)),
                                     ("bool_OR", (1, 1)), ("lin_reg", (4, 14)), ("logistic regression", (0, 0))])
def test_choose_operation(name, io):
    op = Q.choose_operation(name, 0, 10, 3, 0)
    assert (op.NbrInput, op.NbrOutput) == io


def test_choose_operation_cutting_factor_and_unknown():
    assert Q.choose_operation("mean", 0, 0, 0, 4).NbrOutput == 8
    with pytest.raises(ValueError):
        Q.choose_operation("nope", 0, 0, 0, 0)


def _sq(proofs=0, **kw):
    op = Q.choose_operation("sum", 0, 10, 0, 0)
    sq = Q.SurveyQuery(SurveyID="s", Query=Q.Query(Operation=op, Proofs=proofs,
                                                   DPDataGen=Q.QueryDPDataGen([1], 10, 0, 10)))
    for k, v in kw.items():
        setattr(sq, k, v)
    return sq


def test_check_parameters_rules():
    assert Q.check_parameters(_sq(), False)
    bad = _sq(Threshold=0.5)  # no proofs but a threshold
    assert not Q.check_parameters(bad, False)
    p = _sq(proofs=1)
    assert not Q.check_parameters(p, False)  # proofs but no range
    p.Query.Ranges = [[0, 0]]
    assert Q.check_parameters(p, False)
    p.Query.Obfuscation = True  # obfuscation on 'sum' is not accepted
    p.ObfuscationProofThreshold = 1.0
    assert not Q.check_parameters(p, False)
    dp = _sq()
    dp.Query.DiffP = Q.QueryDiffP(LapScale=1.0, NoiseListSize=10, Quanta=1.0, Scale=1.0, Limit=5)
    assert Q.check_parameters(dp, True) and not Q.check_parameters(dp, False)
    mm = _sq()
    mm.Query.DPDataGen.GenerateDataMax = 99
    assert not Q.check_parameters(mm, False)


def test_query_to_proofs_nbrs():
    sq = _sq(proofs=1)
    sq.RosterServers = Q.Roster([Q.ServerIdentity(f"cn{i}", O.G1_GEN) for i in range(3)])
    sq.ServerToDP = {"cn0": [Q.ServerIdentity("a"), Q.ServerIdentity("b")], "cn1": [Q.ServerIdentity("c")],
                     "cn2": None}
    assert Q.query_to_proofs_nbrs(sq) == [3, 0, 3, 0, 3]
    sq.Query.Obfuscation = True
    sq.Query.DiffP = Q.QueryDiffP(NoiseListSize=5)
    assert Q.query_to_proofs_nbrs(sq) == [3, 3, 3, 3, 3]
    sq.Query.Proofs = 0
    assert Q.query_to_proofs_nbrs(sq) == [3, 0, 0, 0, 0]


def test_survey_json_roundtrip():
    sq = _sq(proofs=1)
    sq.RosterServers = Q.Roster([Q.ServerIdentity("cn0", O.G1_GEN, "addr", 2)])
    sq.ClientPubKey = O.g1_mul(5, O.G1_GEN)
    sq.IDtoPublic = {"cn0": O.G1_GEN}
    sq.Query.Ranges = [[16, 5]]
    sq.Query.IVSigs = Q.QueryIVSigs([[Q.PublishSignatureBytes(b"\x01" * 64, b"\x02" * 128)]], 1, 1)
    sq.Query.Operation.LRParameters.Means = [1.5]
    d = sq.to_dict()
    import json

    back = Q.SurveyQuery.from_dict(json.loads(json.dumps(d)))
    assert back.to_dict() == d
    assert back.RosterServers.list[0].rank == 2 and back.ClientPubKey == sq.ClientPubKey
