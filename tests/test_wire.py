"""onet wire format: dedis/protobuf primitives, envelopes, SurveyQuery/DataBlock
round trips.  Byte parity with the Go encoder is unpinned (the onet/protobuf
sources are not in the reference tree): the primitive vectors below are the
protobuf specification's own examples."""
import pytest

from drynx_amd.crypto import oracle as O
from drynx_amd.ledger.skipchain import DataBlock, new_data_block
from drynx_amd.query import LogisticRegressionParameters, QueryDiffP, ServerIdentity
from drynx_amd.services.api import DrynxClient
from drynx_amd.services.local import local_cluster, make_survey
from drynx_amd.wire import messages as M
from drynx_amd.wire import onet
from drynx_amd.wire import protobuf as pb


def test_varint_and_zigzag_spec_vectors():
    out = bytearray()
    pb.put_uvarint(out, 300)
    assert bytes(out) == b"\xac\x02"                      # protobuf encoding guide
    assert [pb.zigzag(v) for v in (0, -1, 1, -2, 2147483647, -2147483648)] == \
        [0, 1, 2, 3, 4294967294, 4294967295]
    for v in (0, 1, -1, 2**62, -(2**63), 2**63 - 1):
        assert pb.unzigzag(pb.zigzag(v)) == v
    # message Test1 { int32 a = 1; } with a = 150 (uint varint) -> 08 96 01
    assert pb.encode((("a", "uint"),), {"a": 150}) == b"\x08\x96\x01"
    # message Test2 { string b = 2; } with b = "testing"
    assert pb.encode((("x", "uint"), ("b", "string")), {"b": "testing"}) == b"\x12\x07testing"


def test_schema_round_trip_all_kinds():
    inner = (("P", "point"), ("N", "sint"))
    schema = (("S", "string"), ("I", "sint"), ("U", "uint"), ("B", "bool"), ("D", "double"), ("Y", "bytes"),
              ("T", "time"), ("M", ("msg", inner)), ("R", ("rep", "sint")), ("RD", ("rep", "double")),
              ("RM", ("rep", ("msg", inner))), ("MP", ("map", "string", "sint")),
              ("PS", ("rep", ("ptrslice", "sint"))), ("RS", ("rep", "string")))
    obj = {"S": "héllo", "I": -5, "U": 7, "B": True, "D": -1.25, "Y": b"\x00\x01", "T": 1_700_000_000_123_456_789,
           "M": {"P": b"\x01" * 64, "N": -(2**63)}, "R": [1, -1, 0, 2**40], "RD": [0.5, -0.0, 3.0],
           "RM": [{"P": b"", "N": 3}, {"P": b"\x02" * 64, "N": 0}], "MP": {"b": 2, "a": -1, "z": 0},
           "PS": [[16, 16], [], [2, 1, -3]], "RS": ["x", ""]}
    enc = pb.encode(schema, obj)
    dec = pb.decode(schema, enc)
    assert dec == obj
    assert pb.encode(schema, dec) == enc                  # deterministic (maps sorted by key)


def test_decoder_rejects_truncation_and_skips_unknown_fields():
    schema = (("A", "sint"), ("B", "string"))
    enc = pb.encode(schema, {"A": 3, "B": "xy"})
    with pytest.raises(ValueError):
        pb.decode(schema, enc[:-1])
    assert pb.decode((("A", "sint"),), enc) == {"A": 3}  # field 2 unknown to this schema


def test_envelope_type_ids():
    a = onet.message_type_id("libdrynx.SurveyQuery")
    assert len(a) == 16 and a != onet.message_type_id("libdrynx.DataBlock")
    assert a[6] >> 4 == 5                                 # UUID version 5
    with pytest.raises(ValueError):
        onet.unmarshal(b"\x00" * 16 + b"")


def test_survey_query_round_trip():
    cl, node = local_cluster(3, 4, 2, device="cpu")
    client = DrynxClient(node, device="cpu")
    lp = LogisticRegressionParameters(NbrRecords=100, NbrFeatures=2, Means=[1.0, 2.0], StandardDeviations=[0.5, 1.5],
                                      Lambda=1.0, Step=0.1, MaxIterations=10, InitialWeights=[0.1] * 3, K=2,
                                      PrecisionApproxCoefficients=100.0)
    sq = make_survey(client, cl, "logistic regression", proofs=1, ranges=[16, 4, 1 << 20], lr_params=lp,
                     thresholds=[1.0, 1.0, 0.5, 0.0, 1.0], verification_sharding=1)
    sq.Query.DiffP = QueryDiffP(LapMean=0.0, LapScale=15.0, NoiseListSize=90, Quanta=1.0, Scale=1.0, Limit=65.0)
    wire = M.survey_query_to_wire(sq)
    assert wire[:16] == onet.message_type_id("libdrynx.SurveyQuery")
    back = M.survey_query_from_wire(wire)
    assert back == sq
    assert M.survey_query_to_wire(back) == wire
    node.close(remove=True)


def test_data_block_is_an_onet_message():
    ids = [ServerIdentity(f"vn{i}", O.g1_mul(i + 2, O.G1_GEN), f"127.0.0.1:{7000 + i}") for i in range(3)]
    db = new_data_block("s1", {"s1/range/dp0/vn0": 1, "s1/keyswitch/cn1/vn1": 4}, ids)
    b = db.to_bytes()
    assert b[:16] == onet.message_type_id("libdrynx.DataBlock")
    back = DataBlock.from_bytes(b)
    assert back.Proofs == db.Proofs and back.Roster == db.Roster and back.SurveyID == "s1"
    assert abs(back.Time - db.Time) < 1e-6 and back.ServerNumber == 3 and back.Sample == db.Sample


def test_range_proof_list_bytes_layout():
    """The device-assembled RangeProofListBytes envelope equals the generic
    dedis/protobuf encoding of the reference structs (range_proof.go:26-57,
    72-155) built from the host codecs, and decodes back to a valid list."""
    from drynx_amd import native as nt
    from drynx_amd.crypto import bn254 as bn
    from drynx_amd.crypto import elgamal as eg
    from drynx_amd.ops.encoding import CreateProofBatch
    from drynx_amd.proofs import range_proof as rp
    from drynx_amd.proofs import range_wire as rw
    from drynx_amd.wire import onet

    S, u, l = 2, 4, 3
    sigs = [rp.init_range_proof_signatures([u] * 3) for _ in range(S)]
    P = eg.aggregate_keys([eg.KeyPair.generate().public for _ in range(S)])
    sm = rp.SigMaterial(sigs)
    cv, r = eg.encrypt_ints(eg.pk_table(P), [1, 5, 9])
    rpl = rp.create_range_proofs(CreateProofBatch([1, 5, 9], r, cv, [u] * 3, [l] * 3, [0, 1, 2], [0] * 3), sm, P)[0]
    b = rw.encode_bundle([rpl])
    commit = [rpl.commit[p:p + 1].to_bytes() for p in range(3)]
    D = bn.g1_aff_to_bytes(nt.g1_to_affine(rpl.D))
    zv = bn.scalars_to_bytes(rpl.zv).reshape(3, S, l * 32)
    V = bn.g2_aff_to_bytes(rpl.V).reshape(3, S, l * 128)
    A = bn.gt_to_bytes(rpl.A).reshape(3, S, l * 384)
    obj = {"Data": [{"Commit": commit[p], "RP": {
        "Challenge": bn.scalars_to_bytes(rpl.challenge)[p].tobytes(), "Zr": bn.scalars_to_bytes(rpl.zr)[p].tobytes(),
        "D": D[p].tobytes(), "Zv": [zv[p, i].tobytes() for i in range(S)],
        "Zphi": bn.scalars_to_bytes(rpl.zphi).reshape(3, l * 32)[p].tobytes(),
        "V": [V[p, i].tobytes() for i in range(S)], "A": [A[p, i].tobytes() for i in range(S)]}} for p in range(3)]}
    assert b == onet.marshal(rw.LIST_TYPE, obj)
    back = rw.decode_bundle(b, [[u, l]] * 3)
    assert len(back) == 1 and rp.verify_range_proof_list(back[0], sm, P)
