"""Append-only proof ledger (cothority skipchain equivalent).

Reference: the root VN wraps the merged verification bitmap in a
``DataBlock{Roster, SurveyID, Sample, Time, ServerNumber, Proofs}``
(lib/structs.go:66; services/service_skipchain.go:114-153) and either creates
the genesis block (``CreateGenesis(roster, 1, 1, [VerifyBitmap, VerifyBase],
data)`` :498-505) or appends (:507-525).  Every VN's custom verifier
``verifyFuncBitmap`` (:397-435) accepts a block only if its bitmap matches the
VN's own DB.

Here a block is hash-linked (SHA-256 over index, back link, roster and data)
and carries a forward-link signature from every VN of the roster (Schnorr over
the block hash) — each VN signs only after its bitmap verifier accepted the
block.  (Cothority's BLS collective signature is replaced by the list of
per-VN Schnorr signatures; documented simplification.)
"""
from __future__ import annotations

import hashlib
import json
import time
from dataclasses import dataclass, field

from ..crypto import oracle as O
from ..proofs.sigma import schnorr_sign, schnorr_verify

VERIFY_BITMAP = "VerifyBitmap"
VERIFY_BASE = "VerifyBase"


@dataclass
class DataBlock:
    Roster: list                 # [{"id":..., "public": hex}]
    SurveyID: str
    Sample: float
    Time: float
    ServerNumber: int
    Proofs: dict                 # bitmap key -> code

    def to_bytes(self) -> bytes:
        return json.dumps(self.__dict__, sort_keys=True).encode()

    @staticmethod
    def from_bytes(b: bytes) -> "DataBlock":
        return DataBlock(**json.loads(b.decode()))


@dataclass
class SkipBlock:
    Index: int
    Roster: list
    Data: bytes
    BackLink: str                # hex hash of previous block ("" for genesis)
    VerifierIDs: list
    Hash: str = ""
    ForwardSignatures: dict = field(default_factory=dict)  # vn id -> signature hex
    GenesisID: str = ""

    def compute_hash(self) -> str:
        h = hashlib.sha256()
        h.update(self.Index.to_bytes(8, "little"))
        h.update(self.BackLink.encode())
        h.update(json.dumps(self.Roster, sort_keys=True).encode())
        h.update(json.dumps(self.VerifierIDs).encode())
        h.update(self.Data)
        return h.hexdigest()

    def to_bytes(self) -> bytes:
        d = dict(self.__dict__)
        d["Data"] = self.Data.hex()
        return json.dumps(d, sort_keys=True).encode()

    @staticmethod
    def from_bytes(b: bytes) -> "SkipBlock":
        d = json.loads(b.decode())
        d["Data"] = bytes.fromhex(d["Data"])
        return SkipBlock(**d)

    def data_block(self) -> DataBlock:
        return DataBlock.from_bytes(self.Data)

    def verify_signatures(self, publics: dict) -> bool:
        if self.compute_hash() != self.Hash:
            return False
        for vn in self.Roster:
            sig = self.ForwardSignatures.get(vn["id"])
            if sig is None or not schnorr_verify(publics[vn["id"]], bytes.fromhex(self.Hash), bytes.fromhex(sig)):
                return False
        return True


def roster_json(identities) -> list:
    return [{"id": si.id, "public": O.g1_to_bytes(si.public).hex()} for si in identities]


def new_data_block(survey_id: str, bitmap: dict, vn_identities, sample: float = 0.4) -> DataBlock:
    """DataBlock as built by the root VN (Sample hard-coded to 0.4 in the reference, :115)."""
    return DataBlock(roster_json(vn_identities), survey_id, sample, time.time(), len(vn_identities), dict(bitmap))


def make_block(prev: SkipBlock | None, data: DataBlock, vn_identities) -> SkipBlock:
    sb = SkipBlock(Index=0 if prev is None else prev.Index + 1, Roster=roster_json(vn_identities), Data=data.to_bytes(),
                   BackLink="" if prev is None else prev.Hash, VerifierIDs=[VERIFY_BITMAP, VERIFY_BASE])
    sb.Hash = sb.compute_hash()
    sb.GenesisID = sb.Hash if prev is None else (prev.GenesisID or prev.Hash)
    return sb


def verify_bitmap(sb: SkipBlock, local_bitmap: dict, vn_address: str) -> bool:
    """verifyFuncBitmap: every bitmap entry this VN produced must match the block."""
    proofs = sb.data_block().Proofs
    for k, v in local_bitmap.items():
        if proofs.get(k) != v:
            return False
    return True


def sign_block(sb: SkipBlock, vn_id: str, secret: int):
    sb.ForwardSignatures[vn_id] = schnorr_sign(secret, bytes.fromhex(sb.Hash)).hex()
