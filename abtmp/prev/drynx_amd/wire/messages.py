"""Converters between drynx_amd's Python structs and the onet wire messages.

``survey_query_to_wire`` / ``survey_query_from_wire`` carry a SurveyQuery as
the reference's ``network.Marshal(&SurveyQuery)`` (lib/structs.go:231-247);
``data_block_to_wire`` / ``data_block_from_wire`` give the bytes a skipchain
block stores as its Data (services/service_skipchain.go:498-525 marshals a
``DataBlock``, lib/structs.go:66-73).

Identity mapping: onet identifies a server by a 16-byte UUID; drynx_amd by a
string id.  The UUID is derived from the string id (UUIDv5, URL namespace) and
the string id travels in ``Description`` so the round trip is exact; the GPU
rank and the BLS key of a verifying node are appended as extension fields.
"""
from __future__ import annotations

import uuid

from ..crypto import oracle as O
from ..query import (LogisticRegressionParameters, Operation, PublishSignatureBytes, Query, QueryDiffP,
                     QueryDPDataGen, QueryIVSigs, Roster, ServerIdentity, SurveyQuery)
from . import onet


def _sid_uuid(sid: str) -> bytes:
    return uuid.uuid5(uuid.NAMESPACE_URL, "drynx:" + sid).bytes


def _pt(p) -> bytes:
    return O.g1_to_bytes(p) if p is not None else b""


def _unpt(b: bytes):
    return O.g1_from_bytes(b) if b else None


# ----------------------------------------------------------------------------- identities
def server_identity_to_msg(si: ServerIdentity) -> dict:
    return {"Public": _pt(si.public), "ID": _sid_uuid(si.id), "Address": si.address, "Description": si.id,
            "Rank": si.rank, "BLS": O.g2_to_bytes(si.bls) if si.bls is not None else b""}


def server_identity_from_msg(d: dict) -> ServerIdentity:
    return ServerIdentity(d["Description"], _unpt(d["Public"]), d["Address"], d["Rank"],
                          O.g2_from_bytes(d["BLS"]) if d["BLS"] else None)


def roster_to_msg(r: Roster) -> dict:
    ids = b"".join(_sid_uuid(s.id) for s in r.list)
    return {"ID": uuid.uuid5(uuid.NAMESPACE_URL, ids.hex()).bytes,
            "List": [server_identity_to_msg(s) for s in r.list],
            "Aggregate": _pt(r.aggregate()) if r.list else b""}


def roster_from_msg(d: dict | None) -> Roster:
    return Roster([server_identity_from_msg(x) for x in (d or {}).get("List", [])])


# ----------------------------------------------------------------------------- survey query
def survey_query_to_msg(sq: SurveyQuery) -> dict:
    q = sq.Query
    op = q.Operation
    lr = op.LRParameters
    ivs = q.IVSigs
    return {
        "SurveyID": sq.SurveyID,
        "RosterServers": roster_to_msg(sq.RosterServers),
        "ClientPubKey": _pt(sq.ClientPubKey),
        "IntraMessage": sq.IntraMessage,
        "ServerToDP": {k: ([server_identity_to_msg(s) for s in v] if v is not None else None)
                       for k, v in sq.ServerToDP.items()},
        "Query": {
            "Operation": {"NameOp": op.NameOp, "NbrInput": op.NbrInput, "NbrOutput": op.NbrOutput,
                          "QueryMin": op.QueryMin, "QueryMax": op.QueryMax,
                          "LRParameters": dict(lr.__dict__)},
            "Ranges": [list(r) for r in (q.Ranges or [])],
            "Proofs": q.Proofs,
            "Obfuscation": q.Obfuscation,
            "DiffP": dict(q.DiffP.__dict__),
            "DPDataGen": dict(q.DPDataGen.__dict__),
            "IVSigs": {"InputValidationSigs": [[{"Public": s.Public, "Signature": s.Signature} for s in row]
                                               for row in (ivs.InputValidationSigs or [])],
                       "InputValidationSize1": ivs.InputValidationSize1,
                       "InputValidationSize2": ivs.InputValidationSize2},
            "RosterVNs": roster_to_msg(q.RosterVNs) if q.RosterVNs is not None else None,
            "SQL": {},
            "CuttingFactor": q.CuttingFactor,
        },
        "IDtoPublic": {k: _pt(p) for k, p in sq.IDtoPublic.items()},
        "Threshold": sq.Threshold,
        "AggregationProofThreshold": sq.AggregationProofThreshold,
        "ObfuscationProofThreshold": sq.ObfuscationProofThreshold,
        "RangeProofThreshold": sq.RangeProofThreshold,
        "KeySwitchingProofThreshold": sq.KeySwitchingProofThreshold,
        "VerificationSharding": sq.VerificationSharding,
        "RangeProofMode": sq.RangeProofMode,
    }


def survey_query_from_msg(d: dict) -> SurveyQuery:
    q = d["Query"] or {}
    op = q.get("Operation") or {}
    lr = op.get("LRParameters") or {}
    ivs = q.get("IVSigs") or {}
    sigs = ivs.get("InputValidationSigs") or []
    return SurveyQuery(
        SurveyID=d["SurveyID"],
        RosterServers=roster_from_msg(d["RosterServers"]),
        ClientPubKey=_unpt(d["ClientPubKey"]),
        IntraMessage=d["IntraMessage"],
        ServerToDP={k: [server_identity_from_msg(s) for s in v] for k, v in d["ServerToDP"].items()},
        Query=Query(
            Operation=Operation(op.get("NameOp", ""), op.get("NbrInput", 0), op.get("NbrOutput", 0),
                                op.get("QueryMin", 0), op.get("QueryMax", 0),
                                LogisticRegressionParameters(**lr) if lr else LogisticRegressionParameters()),
            Ranges=[list(r) for r in q.get("Ranges", [])] or None,
            Proofs=q.get("Proofs", 0),
            Obfuscation=q.get("Obfuscation", False),
            DiffP=QueryDiffP(**(q.get("DiffP") or {})),
            DPDataGen=QueryDPDataGen(**(q.get("DPDataGen") or {})),
            IVSigs=QueryIVSigs([[PublishSignatureBytes(s["Public"], s["Signature"]) for s in row] for row in sigs]
                               if sigs else None, ivs.get("InputValidationSize1", 0),
                               ivs.get("InputValidationSize2", 0)),
            RosterVNs=roster_from_msg(q["RosterVNs"]) if q.get("RosterVNs") is not None else None,
            CuttingFactor=q.get("CuttingFactor", 0),
        ),
        IDtoPublic={k: _unpt(v) for k, v in d["IDtoPublic"].items()},
        Threshold=d["Threshold"],
        AggregationProofThreshold=d["AggregationProofThreshold"],
        ObfuscationProofThreshold=d["ObfuscationProofThreshold"],
        RangeProofThreshold=d["RangeProofThreshold"],
        KeySwitchingProofThreshold=d["KeySwitchingProofThreshold"],
        VerificationSharding=d["VerificationSharding"],
        RangeProofMode=d["RangeProofMode"],
    )


def survey_query_to_wire(sq: SurveyQuery) -> bytes:
    return onet.marshal("libdrynx.SurveyQuery", survey_query_to_msg(sq))


def survey_query_from_wire(b: bytes) -> SurveyQuery:
    name, d = onet.unmarshal(b)
    if name != "libdrynx.SurveyQuery":
        raise ValueError(f"expected a SurveyQuery, got {name}")
    return survey_query_from_msg(d)


# ----------------------------------------------------------------------------- data block
def data_block_to_wire(roster: list, survey_id: str, sample: float, t: float, server_number: int,
                       proofs: dict) -> bytes:
    """roster: [{"id", "public" (hex), ["bls" (hex)]}] as the ledger keeps it."""
    lst = [{"Public": bytes.fromhex(e["public"]), "ID": _sid_uuid(e["id"]), "Description": e["id"],
            "BLS": bytes.fromhex(e["bls"]) if e.get("bls") else b""} for e in roster]
    return onet.marshal("libdrynx.DataBlock", {
        "Roster": {"List": lst}, "SurveyID": survey_id, "Sample": sample, "Time": int(round(t * 1e9)),
        "ServerNumber": server_number, "Proofs": {k: int(v) for k, v in proofs.items()}})


def data_block_from_wire(b: bytes) -> dict:
    name, d = onet.unmarshal(b)
    if name != "libdrynx.DataBlock":
        raise ValueError(f"expected a DataBlock, got {name}")
    roster = []
    for e in (d["Roster"] or {}).get("List", []):
        r = {"id": e["Description"], "public": e["Public"].hex()}
        if e["BLS"]:
            r["bls"] = e["BLS"].hex()
        roster.append(r)
    return {"Roster": roster, "SurveyID": d["SurveyID"], "Sample": d["Sample"], "Time": d["Time"] / 1e9,
            "ServerNumber": d["ServerNumber"], "Proofs": d["Proofs"]}
