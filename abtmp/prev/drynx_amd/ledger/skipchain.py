"""Append-only proof ledger (cothority skipchain equivalent).

Reference: the root VN wraps the merged verification bitmap in a
``DataBlock{Roster, SurveyID, Sample, Time, ServerNumber, Proofs}``
(lib/structs.go:66; services/service_skipchain.go:114-153) and either creates
the genesis block (``CreateGenesis(roster, 1, 1, [VerifyBitmap, VerifyBase],
data)`` :498-505) or appends (:507-525).  Every VN's custom verifier
``verifyFuncBitmap`` (:397-435) accepts a block only if its bitmap matches the
VN's own DB.

Here a block is hash-linked (SHA-256 over index, back link, roster and data)
and carries a BLS collective signature of the VN roster over the block hash
(BDN aggregation, crypto/bls.py, like cothority's BLS CoSi): each VN adds its
partial signature only after its verifiers accepted the block -- the bitmap
check (verifyFuncBitmap) and the structural check ``verify_base`` (cothority
skipchain.VerifyBase: index, back link, genesis id, hash); the aggregate and
the participation mask are stored in ``CoSig`` and checked with one pairing
product.  The chain is created like ``CreateGenesis(roster, 1, 1, ...)``
(service_skipchain.go:500): base 1, height 1, so every block has one back
link and one forward link.  The forward link of block k is signed by block
k's roster over (hash_k, hash_k+1) when block k+1 is appended and is stored
with block k (outside its hash, as in cothority); ``update_chain`` walks and
verifies them from any known block to the latest (GetUpdateChain,
service_skipchain.go:195-205, 498-525).  Roster entries without a BLS key
fall back to per-VN Schnorr signatures.
"""
from __future__ import annotations

import hashlib
import json
import time
from dataclasses import dataclass, field

import math

from ..crypto import bls
from ..crypto import oracle as O
from ..proofs.sigma import schnorr_sign, schnorr_verify
from ..wire.messages import data_block_from_wire, data_block_to_wire

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
        """network.Marshal(&DataBlock): onet envelope + dedis/protobuf body (wire/)."""
        return data_block_to_wire(self.Roster, self.SurveyID, self.Sample, self.Time, self.ServerNumber,
                                  self.Proofs)

    @staticmethod
    def from_bytes(b: bytes) -> "DataBlock":
        return DataBlock(**data_block_from_wire(b))


_DATA_BLOCKS: dict = {}


@dataclass
class SkipBlock:
    Index: int
    Roster: list
    Data: bytes
    BackLink: str                # hex hash of previous block ("" for genesis)
    VerifierIDs: list
    Hash: str = ""
    ForwardSignatures: dict = field(default_factory=dict)  # vn id -> partial signature hex
    GenesisID: str = ""
    CoSig: str = ""              # "<aggregate G1 hex>/<mask>" (BLS collective signature)
    ForwardLinks: list = field(default_factory=list)  # [{"To": hash, "CoSig": ..., "Sigs": {...}}]

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
        """The decoded DataBlock (treat as read-only: decodes are shared by
        content hash, so the VNs of a rank checking the same block decode its
        bitmap -- one entry per proof -- once)."""
        key = hashlib.sha256(self.Data).digest()
        db = _DATA_BLOCKS.get(key)
        if db is None:
            db = DataBlock.from_bytes(self.Data)
            if len(_DATA_BLOCKS) >= 8:
                _DATA_BLOCKS.pop(next(iter(_DATA_BLOCKS)))
            _DATA_BLOCKS[key] = db
        return db

    def bls_keys(self):
        if not self.Roster or not all(vn.get("bls") for vn in self.Roster):
            return None
        return [O.g2_from_bytes(bytes.fromhex(vn["bls"])) for vn in self.Roster]

    def verify_signatures(self, publics: dict | None = None, threshold: float = 1.0) -> bool:
        """Hash check + the roster's collective signature (at least
        ceil(threshold * n) signers; default: every VN of the roster)."""
        if self.compute_hash() != self.Hash:
            return False
        return _verify_cosig(self, self.CoSig, self.ForwardSignatures, bytes.fromhex(self.Hash), publics, threshold)


def _verify_cosig(sb: "SkipBlock", cosig: str, sigs: dict, msg: bytes, publics=None, threshold: float = 1.0) -> bool:
    """A collective signature of ``sb``'s roster over ``msg``: the BLS
    aggregate (at least ceil(threshold * n) signers in the mask), or one
    Schnorr signature per roster member when the roster has no BLS keys."""
    keys = sb.bls_keys()
    if keys is not None:
        if not cosig:
            return False
        agg_hex, mask_hex = cosig.split("/")
        mask = bls.mask_from_hex(mask_hex)
        if len(mask) != len(keys) or sum(mask) < math.ceil(threshold * len(keys)):
            return False
        try:
            sig = O.g1_from_bytes(bytes.fromhex(agg_hex))
        except ValueError:
            return False
        return bls.verify_multi(keys, mask, msg, sig)
    for vn in sb.Roster:
        sig = sigs.get(vn["id"])
        if sig is None or publics is None or not schnorr_verify(publics[vn["id"]], msg, bytes.fromhex(sig)):
            return False
    return True


def roster_json(identities) -> list:
    out = []
    for si in identities:
        e = {"id": si.id, "public": O.g1_to_bytes(si.public).hex()}
        if getattr(si, "bls", None) is not None:
            e["bls"] = O.g2_to_bytes(si.bls).hex()
        out.append(e)
    return out


def new_data_block(survey_id: str, bitmap: dict, vn_identities, sample: float = 0.4,
                   t: float | None = None) -> DataBlock:
    """DataBlock as built by the root VN (Sample hard-coded to 0.4 in the
    reference, :115); ``t``: the root VN's timestamp (every rank builds the
    same block from it)."""
    return DataBlock(roster_json(vn_identities), survey_id, sample, time.time() if t is None else t,
                     len(vn_identities), dict(bitmap))


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
    """A VN's forward-link contribution: BLS partial signature of the block
    hash (Schnorr when the roster carries no BLS keys)."""
    if sb.bls_keys() is not None:
        sb.ForwardSignatures[vn_id] = O.g1_to_bytes(bls.sign(secret, bytes.fromhex(sb.Hash))).hex()
    else:
        sb.ForwardSignatures[vn_id] = schnorr_sign(secret, bytes.fromhex(sb.Hash)).hex()


def finalize_cosig(sb: SkipBlock):
    """Aggregate the partial signatures present into CoSig (BDN coefficients
    over the whole roster; the mask records who signed)."""
    keys = sb.bls_keys()
    if keys is None:
        return
    partials, mask = {}, []
    for i, vn in enumerate(sb.Roster):
        s = sb.ForwardSignatures.get(vn["id"])
        mask.append(s is not None)
        if s is not None:
            partials[i] = O.g1_from_bytes(bytes.fromhex(s))
    agg = bls.aggregate(keys, partials)
    sb.CoSig = (O.g1_to_bytes(agg).hex() if agg is not None else "") + "/" + bls.mask_to_hex(mask)


# ----------------------------------------------------------------------------- structure and forward links
def verify_base(prev: SkipBlock | None, sb: SkipBlock) -> bool:
    """skipchain.VerifyBase: the block is well formed and extends ``prev``
    (index, back link, genesis id, hash, verifier list); ``prev`` None: a
    genesis block."""
    if sb.compute_hash() != sb.Hash or not sb.Roster or VERIFY_BASE not in sb.VerifierIDs:
        return False
    if prev is None:
        return sb.Index == 0 and sb.BackLink == "" and sb.GenesisID == sb.Hash
    return (sb.Index == prev.Index + 1 and sb.BackLink == prev.Hash
            and sb.GenesisID == (prev.GenesisID or prev.Hash))


def forward_link_message(frm: str, to: str) -> bytes:
    return hashlib.sha256(b"drynx_amd/skipchain/forward-link/v1" + bytes.fromhex(frm) + bytes.fromhex(to)).digest()


def sign_forward_link(prev: SkipBlock, to_hash: str, secret: int) -> str:
    """A member of ``prev``'s roster signs the link prev -> to (BLS partial,
    Schnorr when the roster has no BLS keys)."""
    msg = forward_link_message(prev.Hash, to_hash)
    if prev.bls_keys() is not None:
        return O.g1_to_bytes(bls.sign(secret, msg)).hex()
    return schnorr_sign(secret, msg).hex()


def cosign_many(sb: SkipBlock, signers: list) -> tuple:
    """Several VNs of one rank sign ``sb`` (and, when they hold a previous
    block, the forward link prev -> sb) in one batch of BLS scalar
    multiplications.  signers: [(vn_id, secret, prev | None)] ->
    ({vn_id: block partial hex}, {vn_id: link partial hex})."""
    if sb.bls_keys() is None:
        sigs, links = {}, {}
        for vn_id, sk, prev in signers:
            sign_block(sb, vn_id, sk)
            sigs[vn_id] = sb.ForwardSignatures[vn_id]
            if prev is not None:
                links[vn_id] = sign_forward_link(prev, sb.Hash, sk)
        return sigs, links
    items, where = [], []
    for vn_id, sk, prev in signers:
        items.append((sk, bytes.fromhex(sb.Hash)))
        where.append(("b", vn_id))
        if prev is not None:
            items.append((sk, forward_link_message(prev.Hash, sb.Hash)))
            where.append(("l", vn_id))
    sigs, links = {}, {}
    for (kind, vn_id), sig in zip(where, bls.sign_many(items)):
        h = O.g1_to_bytes(sig).hex()
        if kind == "b":
            sb.ForwardSignatures[vn_id] = h
            sigs[vn_id] = h
        else:
            links[vn_id] = h
    return sigs, links


_LINKS: dict = {}  # (prev hash, to hash, partials) -> link: co-hosted VNs each hold a copy of prev


def add_forward_link(prev: SkipBlock, to_hash: str, partials: dict):
    """Aggregate the roster's partial signatures into prev's forward link."""
    memo = (prev.Hash, to_hash, tuple(sorted(partials.items())))
    if memo in _LINKS:
        link = {**_LINKS[memo], "Sigs": dict(_LINKS[memo]["Sigs"])}
        prev.ForwardLinks = [lk for lk in prev.ForwardLinks if lk["To"] != to_hash] + [link]
        return
    link = {"To": to_hash, "CoSig": "", "Sigs": {}}
    keys = prev.bls_keys()
    if keys is None:
        link["Sigs"] = dict(partials)
    else:
        mask, parts = [], {}
        for i, vn in enumerate(prev.Roster):
            p = partials.get(vn["id"])
            mask.append(p is not None)
            if p is not None:
                parts[i] = O.g1_from_bytes(bytes.fromhex(p))
        agg = bls.aggregate(keys, parts)
        link["CoSig"] = (O.g1_to_bytes(agg).hex() if agg is not None else "") + "/" + bls.mask_to_hex(mask)
    if len(_LINKS) > 32:
        _LINKS.clear()
    _LINKS[memo] = {**link, "Sigs": dict(link["Sigs"])}
    prev.ForwardLinks = [lk for lk in prev.ForwardLinks if lk["To"] != to_hash] + [link]


def verify_forward_link(prev: SkipBlock, link: dict, publics: dict | None = None, threshold: float = 1.0) -> bool:
    return _verify_cosig(prev, link.get("CoSig", ""), link.get("Sigs", {}), forward_link_message(prev.Hash, link["To"]),
                         publics, threshold)


def update_chain(get_block, start: SkipBlock, publics: dict | None = None) -> list:
    """GetUpdateChain: from ``start`` follow the (verified) forward links to the
    latest block; every hop checks the link's collective signature, the next
    block's structure (verify_base) and its own collective signature.
    ``get_block(hash)`` -> SkipBlock | None.  Raises ValueError on a bad hop."""
    chain = [start]
    seen = {start.Hash}
    while chain[-1].ForwardLinks:
        cur = chain[-1]
        link = cur.ForwardLinks[-1]
        if not verify_forward_link(cur, link, publics):
            raise ValueError(f"bad forward link from block {cur.Index}")
        nxt = get_block(link["To"])
        if nxt is None or nxt.Hash in seen:
            raise ValueError(f"forward link from block {cur.Index} leads nowhere")
        if not verify_base(cur, nxt) or not nxt.verify_signatures(publics):
            raise ValueError(f"block {nxt.Index} does not extend block {cur.Index}")
        seen.add(nxt.Hash)
        chain.append(nxt)
    return chain
