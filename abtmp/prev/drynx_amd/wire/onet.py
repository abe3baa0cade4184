"""onet message envelope and the drynx message schemas.

Reference: every drynx message is registered with onet's
``network.RegisterMessage`` (lib/structs.go:610-640 ``init``, services/
service.go:120-160) and travels as ``network.Marshal(msg)`` = a 16-byte
MessageTypeID followed by the dedis/protobuf body.  The type id is a UUIDv5
in the URL namespace over ``NamespaceBodyType + reflect type string``
(e.g. ``libdrynx.SurveyQuery``) [ext, onet v3 network/encoding.go — re-derived,
byte parity unpinned].

Schemas mirror the Go structs field by field (lib/structs.go:18-265 for the
query/response types; onet Roster / network.ServerIdentity [ext];
libunlynx.CipherText [ext]).  Drynx_amd extensions are appended after the
reference fields, so a reference decoder that skips unknown fields still reads
the message.
"""
from __future__ import annotations

import uuid

from . import protobuf as pb

NAMESPACE_URL = "https://dedis.epfl.ch/"
NAMESPACE_BODY_TYPE = NAMESPACE_URL + "/protocolType/"


def message_type_id(go_type: str) -> bytes:
    """onet ``network.MessageType``: UUIDv5(URL namespace, body-type namespace + type string)."""
    return uuid.uuid5(uuid.NAMESPACE_URL, NAMESPACE_BODY_TYPE + go_type).bytes


# ----------------------------------------------------------------------------- schemas
SERVICE_IDENTITY = (("Name", "string"), ("Suite", "string"), ("Public", "point"))
SERVER_IDENTITY = (("Public", "point"), ("ServiceIdentities", ("rep", ("msg", SERVICE_IDENTITY))), ("ID", "bytes"),
                   ("Address", "string"), ("Description", "string"), ("URL", "string"),
                   # drynx_amd extensions: GPU rank, BLS (G2) key of a verifying node
                   ("Rank", "sint"), ("BLS", "point"))
ROSTER = (("ID", "bytes"), ("List", ("rep", ("msg", SERVER_IDENTITY))), ("Aggregate", "point"))

LR_PARAMETERS = (("DatasetName", "string"), ("FilePath", "string"), ("NbrRecords", "sint"), ("NbrFeatures", "sint"),
                 ("Means", ("rep", "double")), ("StandardDeviations", ("rep", "double")), ("Lambda", "double"),
                 ("Step", "double"), ("MaxIterations", "sint"), ("InitialWeights", ("rep", "double")),
                 ("K", "sint"), ("PrecisionApproxCoefficients", "double"))
OPERATION = (("NameOp", "string"), ("NbrInput", "sint"), ("NbrOutput", "sint"), ("QueryMin", "sint"),
             ("QueryMax", "sint"), ("LRParameters", ("msg", LR_PARAMETERS)))
QUERY_DIFFP = (("LapMean", "double"), ("LapScale", "double"), ("NoiseListSize", "sint"), ("Quanta", "double"),
               ("Scale", "double"), ("Limit", "double"))
QUERY_DPDATAGEN = (("GroupByValues", ("rep", "sint")), ("GenerateRows", "sint"), ("GenerateDataMin", "sint"),
                   ("GenerateDataMax", "sint"))
PUBLISH_SIGNATURE_BYTES = (("Public", "point"), ("Signature", "bytes"))
QUERY_IVSIGS = (("InputValidationSigs", ("rep", ("ptrslice", ("msg", PUBLISH_SIGNATURE_BYTES)))),
                ("InputValidationSize1", "sint"), ("InputValidationSize2", "sint"))
WHERE_CLEAR = (("Name", "string"), ("Value", "string"))
QUERY_SQL = (("Select", ("rep", "string")), ("Where", ("rep", ("msg", WHERE_CLEAR))), ("Predicate", "string"),
             ("GroupBy", ("rep", "string")))
QUERY = (("Operation", ("msg", OPERATION)), ("Ranges", ("rep", ("ptrslice", "sint"))), ("Proofs", "sint"),
         ("Obfuscation", "bool"), ("DiffP", ("msg", QUERY_DIFFP)), ("DPDataGen", ("msg", QUERY_DPDATAGEN)),
         ("IVSigs", ("msg", QUERY_IVSIGS)), ("RosterVNs", ("msg", ROSTER)), ("SQL", ("msg", QUERY_SQL)),
         ("CuttingFactor", "sint"))
SURVEY_QUERY = (("SurveyID", "string"), ("RosterServers", ("msg", ROSTER)), ("ClientPubKey", "point"),
                ("IntraMessage", "bool"), ("ServerToDP", ("map", "string", ("ptrslice", ("msg", SERVER_IDENTITY)))),
                ("Query", ("msg", QUERY)), ("IDtoPublic", ("map", "string", "point")), ("Threshold", "double"),
                ("AggregationProofThreshold", "double"), ("ObfuscationProofThreshold", "double"),
                ("RangeProofThreshold", "double"), ("KeySwitchingProofThreshold", "double"),
                # drynx_amd extension (after the reference fields): per-proof VN sharding
                ("VerificationSharding", "sint"), ("RangeProofMode", "sint"))
SURVEY_QUERY_TO_VN = (("SQ", ("msg", SURVEY_QUERY)),)
SURVEY_QUERY_TO_DP = (("SQ", ("msg", SURVEY_QUERY)), ("Root", ("msg", SERVER_IDENTITY)))
# VN requests: the reference sends them to the VN's own server; here one entry
# node hosts many logical VNs, so the VN id is an appended extension field
END_VERIFICATION_REQUEST = (("QueryInfoID", "string"), ("VN", "string"), ("Timeout", "double"))
CIPHERTEXT = (("K", "point"), ("C", "point"))
CIPHERVECTOR = (("Slice", ("rep", ("msg", CIPHERTEXT))),)
RESPONSE_DP = (("Data", ("map", "string", ("ptrslice", ("msg", CIPHERTEXT)))),
               # drynx_amd extensions: survey id, the VN block of the survey (Reply.Latest encoding)
               ("SurveyID", "string"), ("Block", "bytes"))
RESPONSE_DP_BYTES = (("Data", ("map", "string", "bytes")), ("Len", "sint"))
DATA_BLOCK = (("Roster", ("msg", ROSTER)), ("SurveyID", "string"), ("Sample", "double"), ("Time", "time"),
              ("ServerNumber", "sint"), ("Proofs", ("map", "string", "sint")))
BITMAP = (("BitMap", ("map", "string", "sint")),)
GET_PROOFS = (("ID", "string"), ("VN", "string"))
PROOFS_AS_MAP = (("Proofs", ("map", "string", "bytes")),)
CLOSE_DB = (("Close", "sint"), ("VN", "string"))
GET_GENESIS = (("VN", "string"),)
GET_BLOCK = (("Roster", ("msg", ROSTER)), ("ID", "string"), ("VN", "string"))
GET_LATEST_BLOCK = (("Roster", ("msg", ROSTER)), ("Sb", "bytes"), ("VN", "string"))
# Reply{Latest *skipchain.SkipBlock}: Latest carries this framework's block
# encoding (drynx_amd/ledger/skipchain.py), not cothority's SkipBlock
REPLY = (("Latest", "bytes"),)
# control plane of the node servers (drynx_amd-specific)
PING = ()
PING_REPLY = (("Address", "string"), ("Public", "point"))
JOIN = (("World", "sint"), ("Rank", "sint"), ("Master", "string"), ("Backend", "string"), ("Addrs", ("rep", "string")),
        ("Publics", ("rep", "point")), ("Root", "string"), ("Nonce", "bytes"), ("Signature", "bytes"))
JOIN_REPLY = (("Signature", "bytes"),)
ACK = (("OK", "bool"),)
ERROR = (("Message", "string"),)
SHUTDOWN = ()

# lib/range/range_proof.go:26-57 (RangeProofListBytes / RangeProofBytes / RangeProofDataBytes)
RANGE_PROOF_DATA_BYTES = (("Challenge", "bytes"), ("Zr", "bytes"), ("D", "bytes"), ("Zv", ("rep", "bytes")),
                          ("Zphi", "bytes"), ("V", ("rep", "bytes")), ("A", ("rep", "bytes")))
RANGE_PROOF_BYTES = (("Commit", "bytes"), ("RP", ("msg", RANGE_PROOF_DATA_BYTES)))
RANGE_PROOF_LIST_BYTES = (("Data", ("ptrslice", ("msg", RANGE_PROOF_BYTES))),)

MESSAGES = {
    "libdrynxrange.RangeProofListBytes": RANGE_PROOF_LIST_BYTES,
    "libdrynx.SurveyQuery": SURVEY_QUERY,
    "libdrynx.SurveyQueryToVN": SURVEY_QUERY_TO_VN,
    "libdrynx.SurveyQueryToDP": SURVEY_QUERY_TO_DP,
    "libdrynx.EndVerificationRequest": END_VERIFICATION_REQUEST,
    "libdrynx.ResponseDP": RESPONSE_DP,
    "libdrynx.ResponseDPBytes": RESPONSE_DP_BYTES,
    "libdrynx.DataBlock": DATA_BLOCK,
    "libdrynx.BitMap": BITMAP,
    "libdrynx.GetProofs": GET_PROOFS,
    "libdrynx.ProofsAsMap": PROOFS_AS_MAP,
    "libdrynx.CloseDB": CLOSE_DB,
    "libdrynx.GetGenesis": GET_GENESIS,
    "libdrynx.GetBlock": GET_BLOCK,
    "libdrynx.GetLatestBlock": GET_LATEST_BLOCK,
    "libdrynx.Reply": REPLY,
    "drynx_amd.Ping": PING,
    "drynx_amd.PingReply": PING_REPLY,
    "drynx_amd.Join": JOIN,
    "drynx_amd.JoinReply": JOIN_REPLY,
    "drynx_amd.Ack": ACK,
    "drynx_amd.Error": ERROR,
    "drynx_amd.Shutdown": SHUTDOWN,
    "libdrynx.PublishSignatureBytes": PUBLISH_SIGNATURE_BYTES,
    "libdrynx.Query": QUERY,
    "libunlynx.CipherText": CIPHERTEXT,
}
_BY_ID = {message_type_id(name): name for name in MESSAGES}


def marshal(go_type: str, obj: dict) -> bytes:
    """network.Marshal: 16-byte type id || protobuf body."""
    return message_type_id(go_type) + pb.encode(MESSAGES[go_type], obj)


def unmarshal(b: bytes) -> tuple[str, dict]:
    """network.Unmarshal: -> (Go type name, decoded fields)."""
    if len(b) < 16:
        raise ValueError("onet envelope shorter than its type id")
    name = _BY_ID.get(bytes(b[:16]))
    if name is None:
        raise ValueError(f"unregistered message type {bytes(b[:16]).hex()}")
    return name, pb.decode(MESSAGES[name], b[16:])
