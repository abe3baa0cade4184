"""Survey/query data model, validation and planning.

Mirrors the reference's lib/structs.go:
  * QueryDiffP / QueryDPDataGen / QueryIVSigs / Query / Operation /
    LogisticRegressionParameters / SurveyQuery          (structs.go:144-247)
  * add_diff_p            (structs.go:423)
  * check_parameters      (structs.go:446-533)
  * query_to_proofs_nbrs  (structs.go:536-568)
  * choose_operation      (structs.go:591-642)
Everything serialises to plain JSON-able dicts for the control plane.
"""
from __future__ import annotations

import copy
import hashlib
import uuid
from dataclasses import dataclass, field, fields, is_dataclass
from typing import Optional

from .crypto import oracle as O
from .utils.log import get_logger

log = get_logger("query")

OPERATIONS = ("sum", "mean", "variance", "cosim", "frequencyCount", "min", "max", "union", "inter", "bool_OR",
              "bool_AND", "lin_reg", "logistic regression", "MLeval")


# ----------------------------------------------------------------------------- identities
@dataclass
class ServerIdentity:
    """A node of the roster (onet ServerIdentity): id, public key, address, GPU rank."""
    id: str
    public: Optional[tuple] = None  # G1 affine (oracle) point
    address: str = ""
    rank: int = 0
    bls: Optional[tuple] = None     # G2 BLS key (verifying nodes: skipchain collective signature)

    def to_dict(self):
        d = {"id": self.id, "public": O.g1_to_bytes(self.public).hex() if self.public else None,
             "address": self.address, "rank": self.rank}
        if self.bls is not None:
            d["bls"] = O.g2_to_bytes(self.bls).hex()
        return d

    @staticmethod
    def from_dict(d):
        pub = O.g1_from_bytes(bytes.fromhex(d["public"])) if d.get("public") else None
        b = O.g2_from_bytes(bytes.fromhex(d["bls"])) if d.get("bls") else None
        return ServerIdentity(d["id"], pub, d.get("address", ""), d.get("rank", 0), b)

    def __hash__(self):
        return hash(self.id)


@dataclass
class Roster:
    list: list = field(default_factory=list)

    def aggregate(self):
        """Collective public key = sum of member keys (onet Roster.Aggregate)."""
        acc = None
        for si in self.list:
            acc = O.g1_add(acc, si.public)
        return acc

    def ids(self):
        return [s.id for s in self.list]

    def to_dict(self):
        return [s.to_dict() for s in self.list]

    @staticmethod
    def from_dict(d):
        return Roster([ServerIdentity.from_dict(x) for x in (d or [])])


# ----------------------------------------------------------------------------- query structs
@dataclass
class QueryDiffP:
    LapMean: float = 0.0
    LapScale: float = 0.0
    NoiseListSize: int = 0
    Quanta: float = 0.0
    Scale: float = 0.0
    Limit: float = 0.0


@dataclass
class QueryDPDataGen:
    GroupByValues: list = field(default_factory=lambda: [1])
    GenerateRows: int = 0
    GenerateDataMin: int = 0
    GenerateDataMax: int = 0


@dataclass
class PublishSignatureBytes:
    """Per-CN range-proof setup: public y = x*B and BB signatures A_k = (x+k)^-1 B2 (u of them, 128 B each)."""
    Public: bytes = b""
    Signature: bytes = b""

    def to_dict(self):
        return {"Public": self.Public.hex(), "Signature": self.Signature.hex()}

    @staticmethod
    def from_dict(d):
        return PublishSignatureBytes(bytes.fromhex(d["Public"]), bytes.fromhex(d["Signature"]))


@dataclass
class QueryIVSigs:
    # InputValidationSigs[cn][output] -> PublishSignatureBytes
    InputValidationSigs: Optional[list] = None
    InputValidationSize1: int = 0
    InputValidationSize2: int = 0


@dataclass
class LogisticRegressionParameters:
    DatasetName: str = ""
    FilePath: str = ""
    NbrRecords: int = 0
    NbrFeatures: int = 0
    Means: list = field(default_factory=list)
    StandardDeviations: list = field(default_factory=list)
    Lambda: float = 0.0
    Step: float = 0.0
    MaxIterations: int = 0
    InitialWeights: list = field(default_factory=list)
    K: int = 2
    PrecisionApproxCoefficients: float = 1.0


@dataclass
class Operation:
    NameOp: str = ""
    NbrInput: int = 0
    NbrOutput: int = 0
    QueryMin: int = 0
    QueryMax: int = 0
    LRParameters: LogisticRegressionParameters = field(default_factory=LogisticRegressionParameters)


@dataclass
class Query:
    Operation: Operation = field(default_factory=Operation)
    Ranges: Optional[list] = None  # list of [u, l] (optionally [u, l, offset])
    Proofs: int = 0
    Obfuscation: bool = False
    DiffP: QueryDiffP = field(default_factory=QueryDiffP)
    DPDataGen: QueryDPDataGen = field(default_factory=QueryDPDataGen)
    IVSigs: QueryIVSigs = field(default_factory=QueryIVSigs)
    RosterVNs: Optional[Roster] = None
    CuttingFactor: int = 0


@dataclass
class SurveyQuery:
    SurveyID: str = ""
    RosterServers: Roster = field(default_factory=Roster)
    ClientPubKey: Optional[tuple] = None
    IntraMessage: bool = False
    ServerToDP: dict = field(default_factory=dict)  # CN id -> [DP ServerIdentity]
    Query: Query = field(default_factory=Query)
    IDtoPublic: dict = field(default_factory=dict)
    Threshold: float = 0.0
    AggregationProofThreshold: float = 0.0
    ObfuscationProofThreshold: float = 0.0
    RangeProofThreshold: float = 0.0
    KeySwitchingProofThreshold: float = 0.0
    # extension: >0 -> each proof request is verified by exactly this many VNs
    # (deterministic sharding of the verification work across GPUs); 0 -> the
    # reference's random sampling with probability Threshold.
    VerificationSharding: int = 0
    # extension: range-proof verification mode.  0 = the reference
    # (RangeProofVerification trusts the proof's challenge, range_proof.go:
    # 504-565); 1 = strict: the VN recomputes c = SHA3-512(B||C||sum y) and
    # checks every V_ij in G2; 2 = strict with the v2 transcript, whose
    # challenge also binds D and every V_ij, a_ij (range_proof.go:350-374 omits them).
    RangeProofMode: int = 0

    # -------------------------------------------------------------- helpers
    def all_dps(self):
        out = []
        for cn in self.RosterServers.list:
            out += list(self.ServerToDP.get(cn.id) or [])
        return out

    def to_dict(self) -> dict:
        return _to_jsonable(self)

    @staticmethod
    def from_dict(d: dict) -> "SurveyQuery":
        return _survey_from_dict(d)


_digest_memo: dict = {}


def ivsigs_digest(sigs) -> str:
    """sha256 over a signature set (memoised per list object: the same CN
    input-validation keys serve many surveys)."""
    if not sigs:
        return ""
    hit = _digest_memo.get(id(sigs))
    if hit is not None and hit[0] is sigs:
        return hit[1]
    h = hashlib.sha256()
    for row in sigs:
        h.update(len(row).to_bytes(4, "little"))
        for s in row:
            h.update(s.Public)
            h.update(s.Signature)
    d = h.hexdigest()
    if len(_digest_memo) > 16:
        _digest_memo.clear()
    _digest_memo[id(sigs)] = (sigs, d)
    return d


def _to_jsonable(obj):
    if isinstance(obj, (ServerIdentity, Roster, PublishSignatureBytes)):
        return obj.to_dict()
    if is_dataclass(obj):
        out = {}
        for f in fields(obj):
            v = getattr(obj, f.name)
            if f.name == "ClientPubKey":
                out[f.name] = O.g1_to_bytes(v).hex() if v is not None else None
            elif f.name == "IDtoPublic":
                out[f.name] = {k: O.g1_to_bytes(p).hex() for k, p in v.items()}
            elif f.name == "ServerToDP":
                out[f.name] = {k: ([s.to_dict() for s in lst] if lst is not None else None) for k, lst in v.items()}
            elif f.name == "InputValidationSigs":
                out[f.name] = None if v is None else [[s.to_dict() for s in row] for row in v]
            else:
                out[f.name] = _to_jsonable(v)
        return out
    if isinstance(obj, (list, tuple)):
        return [_to_jsonable(x) for x in obj]
    if isinstance(obj, dict):
        return {k: _to_jsonable(v) for k, v in obj.items()}
    return obj


def _survey_from_dict(d: dict) -> SurveyQuery:
    q = d["Query"]
    op = dict(q["Operation"])
    op["LRParameters"] = LogisticRegressionParameters(**op.get("LRParameters", {}))
    ivs = dict(q.get("IVSigs") or {})
    if ivs.get("InputValidationSigs") is not None:
        ivs["InputValidationSigs"] = [[PublishSignatureBytes.from_dict(s) for s in row]
                                      for row in ivs["InputValidationSigs"]]
    query = Query(
        Operation=Operation(**op),
        Ranges=q.get("Ranges"),
        Proofs=q.get("Proofs", 0),
        Obfuscation=q.get("Obfuscation", False),
        DiffP=QueryDiffP(**q.get("DiffP", {})),
        DPDataGen=QueryDPDataGen(**q.get("DPDataGen", {})),
        IVSigs=QueryIVSigs(**ivs),
        RosterVNs=Roster.from_dict(q["RosterVNs"]) if q.get("RosterVNs") is not None else None,
        CuttingFactor=q.get("CuttingFactor", 0),
    )
    return SurveyQuery(
        SurveyID=d.get("SurveyID", ""),
        RosterServers=Roster.from_dict(d.get("RosterServers")),
        ClientPubKey=O.g1_from_bytes(bytes.fromhex(d["ClientPubKey"])) if d.get("ClientPubKey") else None,
        IntraMessage=d.get("IntraMessage", False),
        ServerToDP={k: ([ServerIdentity.from_dict(s) for s in v] if v is not None else None)
                    for k, v in (d.get("ServerToDP") or {}).items()},
        Query=query,
        IDtoPublic={k: O.g1_from_bytes(bytes.fromhex(v)) for k, v in (d.get("IDtoPublic") or {}).items()},
        Threshold=d.get("Threshold", 0.0),
        AggregationProofThreshold=d.get("AggregationProofThreshold", 0.0),
        ObfuscationProofThreshold=d.get("ObfuscationProofThreshold", 0.0),
        RangeProofThreshold=d.get("RangeProofThreshold", 0.0),
        KeySwitchingProofThreshold=d.get("KeySwitchingProofThreshold", 0.0),
        VerificationSharding=d.get("VerificationSharding", 0),
        RangeProofMode=d.get("RangeProofMode", 0),
    )


# ----------------------------------------------------------------------------- planning / validation
def add_diff_p(qdf: QueryDiffP) -> bool:
    """structs.go:423 — differential privacy is requested iff any parameter is set."""
    return not (qdf.LapMean == 0.0 and qdf.LapScale == 0.0 and qdf.NoiseListSize == 0 and qdf.Quanta == 0.0
                and qdf.Scale == 0 and qdf.Limit == 0)


def _ranges_zeros(ranges) -> bool:
    return all(r[0] == 0 and r[1] == 0 for r in ranges)


def _ranges_bits(ranges) -> bool:
    return all(r[0] == 2 and r[1] == 1 for r in ranges)


def check_parameters(sq: SurveyQuery, diffp: bool) -> bool:
    """structs.go:446-533 consistency rules; logs every violated rule."""
    msg = []
    q = sq.Query
    bool_ops = ("bool_AND", "bool_OR", "min", "max", "union", "inter")
    if q.Proofs == 1:
        if q.Obfuscation:
            if sq.ObfuscationProofThreshold == 0:
                msg.append("obfuscation threshold is 0 while obfuscation is true")
            if q.Operation.NameOp not in bool_ops:
                msg.append("obfuscation threshold for a non accepted operation")
            if q.Ranges is None or not _ranges_bits(q.Ranges):
                msg.append("obfuscation and proofs but ranges not for 0,1")
        elif sq.ObfuscationProofThreshold != 0:
            msg.append("obfuscation threshold is set and there is no Obfuscation")
        if q.Ranges is None:
            msg.append("proofs but no range")
        else:
            sigs = q.IVSigs.InputValidationSigs
            if sigs is None and not _ranges_zeros(q.Ranges):
                msg.append("proofs but no signatures")
            if _ranges_zeros(q.Ranges) and sigs is not None:
                msg.append("ranges to 0 but signatures also set")
            if sigs is not None:
                if q.Operation.NbrOutput != len(sigs[0]) or q.Operation.NbrOutput != len(q.Ranges):
                    msg.append("ranges or signatures length do not match with nbr output")
    elif q.Proofs == 0:
        if sq.KeySwitchingProofThreshold != 0 or sq.ObfuscationProofThreshold != 0 or sq.RangeProofThreshold != 0 \
                or sq.Threshold != 0:
            msg.append("no proofs and one of the threshold not 0")
        if q.Ranges is not None or q.IVSigs.InputValidationSigs is not None:
            msg.append("no proofs and some ranges or signatures")
        if q.RosterVNs is not None:
            msg.append("no proofs but VN roster")
    else:
        msg.append("unsupported proof type")
    d = q.DiffP
    if not diffp:
        if add_diff_p(d):
            msg.append("no diffP but parameters not to 0")
    else:
        if (d.Limit == 0.0 and d.Quanta == 0.0) or d.Scale == 0.0 or d.NoiseListSize == 0 or d.LapScale == 0.0:
            msg.append("diffP but parameters are 0")
    if q.Operation.QueryMin != q.DPDataGen.GenerateDataMin or q.Operation.QueryMax != q.DPDataGen.GenerateDataMax:
        msg.append("min or max are inconsistent at DP and operations")
    for m in msg:
        log.warning(m)
    return not msg


def query_to_proofs_nbrs(sq: SurveyQuery) -> list:
    """structs.go:536-568: expected proofs [range, shuffle, aggregation, obfuscation, keyswitch]."""
    nbr_dps = sum(len(v) for v in sq.ServerToDP.values() if v is not None)
    nbr_servers = len(sq.RosterServers.list)
    prf_range = nbr_dps
    if sq.Query.Proofs == 0:
        nbr_servers = 0
    prf_aggr = nbr_servers
    prf_obf = nbr_servers if sq.Query.Obfuscation else 0
    prf_shuffle = nbr_servers if add_diff_p(sq.Query.DiffP) else 0
    prf_ks = nbr_servers
    return [prf_range, prf_shuffle, prf_aggr, prf_obf, prf_ks]


def choose_operation(name: str, query_min: int, query_max: int, d: int, cutting_factor: int) -> Operation:
    """structs.go:591-642."""
    op = Operation(NameOp=name, NbrInput=0, NbrOutput=0, QueryMin=int(query_min), QueryMax=int(query_max))
    if name == "sum":
        op.NbrInput, op.NbrOutput = 1, 1
    elif name == "mean":
        op.NbrInput, op.NbrOutput = 1, 2
    elif name == "variance":
        op.NbrInput, op.NbrOutput = 1, 3
    elif name == "cosim":
        op.NbrInput, op.NbrOutput = 2, 5
    elif name in ("frequencyCount", "min", "max", "union", "inter"):
        op.NbrInput, op.NbrOutput = 1, int(query_max - query_min + 1)
    elif name in ("bool_OR", "bool_AND"):
        op.NbrInput, op.NbrOutput = 1, 1
    elif name == "lin_reg":
        op.NbrInput, op.NbrOutput = d + 1, (d * d + 5 * d + 4) // 2
    elif name == "logistic regression":
        pass
    elif name == "MLeval":
        # reachable here (the reference log.Fatal's, structs.go:633-635): [N, sum y, sum y^2, SSE]
        op.NbrInput, op.NbrOutput = 2, 4
    else:
        raise ValueError(f"Operation: <{name}> does not exist")
    if cutting_factor != 0:
        op.NbrOutput = op.NbrOutput * cutting_factor
    return op


def lr_nbr_outputs(d: int, k: int) -> int:
    """getTotalNumberApproxCoefficients (logistic_regression.go:306): sum_j (d+1)^(j+1)."""
    return sum((d + 1) ** (j + 1) for j in range(k))


def new_survey_id() -> str:
    return str(uuid.uuid4())


def clone(sq: SurveyQuery) -> SurveyQuery:
    return copy.deepcopy(sq)
