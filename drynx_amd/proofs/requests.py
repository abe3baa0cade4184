"""Proof request envelopes, signature checks and sampled verification.

Reference: lib/proof/structs_proofs.go — ``ProofRequest`` union of five request
types (:35-104); each ``New*ProofRequest`` marshals the proof and Schnorr-signs
it with the sender's key; ``VerifyProof`` checks the signature in parallel with
a *sampled* verification and returns a bitmap code (:22-27):
0 false, 1 true, 2 received-not-checked, 4 bad signature.

Sampling: reference semantics is ``rand.Float64() <= Threshold`` per VN.
Extension ``SurveyQuery.VerificationSharding = k > 0``: the VNs split the work
deterministically so every request is verified by exactly k VNs (the others
record code 2) — disjoint batched verification across GPUs with guaranteed
coverage.
"""
from __future__ import annotations

import hashlib
import math
import random
from typing import Any

import numpy as np
import torch

from ..crypto import digest as payload_digest
from ..query import ivsigs_digest
from ..utils import timers
from ..utils.log import get_logger
from . import aggregation_shuffle as ags
from . import range_proof as rp
from . import shuffle, sigma

log = get_logger("proofs")

PROOF_FALSE, PROOF_TRUE, PROOF_RECEIVED, PROOF_FALSE_SIGN = 0, 1, 2, 4
# order of QueryToProofsNbrs (structs.go:567) and the VN-side order (service_skipchain.go:57-63)
QUERY_ORDER = ["range", "shuffle", "aggregation", "obfuscation", "keyswitch"]
VN_ORDER = ["range", "aggregation", "obfuscation", "shuffle", "keyswitch"]
TIMER = {"range": "VerifyRange", "aggregation": "VerifyAggregation", "obfuscation": "VerifyObfuscation",
         "shuffle": "VerifyShuffle", "keyswitch": "VerifyKeySwitch"}


class ProofRequest:
    """One signed proof envelope.  The payload is either bytes or, for
    range-proof bundles, the raw limb tensor itself (in HBM on a GPU): its
    digest is computed on the device and its bytes are only materialised when
    something needs them (ledger persistence, control-plane transport)."""

    __slots__ = ("kind", "survey_id", "sender_id", "differ_info", "_data", "signature", "obj", "data_digest",
                 "tensor", "decoded", "sig_ok")

    def __init__(self, kind: str, survey_id: str, sender_id: str, differ_info: str, data: bytes | None,
                 signature: bytes, obj: Any = None, data_digest: bytes = b"", tensor: torch.Tensor | None = None):
        self.kind, self.survey_id, self.sender_id, self.differ_info = kind, survey_id, sender_id, differ_info
        self.sig_ok = None  # ((public, digest, signature), verdict): shared by the VNs of this rank
        self._data = data
        self.signature = signature
        self.obj = obj  # decoded proof (in-process fast path)
        self.data_digest = data_digest  # set for header-only copies (sharded verification)
        self.tensor = tensor
        self.decoded = None  # the VN's own decode of the signed payload (cached across VNs of a rank)

    @property
    def data(self) -> bytes:
        if self._data is None:
            self._data = b"" if self.tensor is None else self.tensor.cpu().numpy().tobytes()
        return self._data

    @data.setter
    def data(self, v: bytes):
        self._data, self.tensor, self.data_digest, self.decoded = v, None, b"", None

    def set_tensor(self, t: torch.Tensor):
        """The payload is (now) this raw tensor; digest recomputed from it."""
        self._data, self.tensor, self.data_digest, self.decoded = None, t, b"", None

    def payload(self):
        """Bytes or the device tensor, whichever is at hand (for the ledger)."""
        return self.tensor if (self._data is None and self.tensor is not None) else self.data

    def base_key(self) -> str:
        return f"{self.survey_id}/{self.kind}/{self.sender_id}/{self.differ_info}"

    def key(self, vn_addr: str) -> str:
        return f"{self.base_key()}/{vn_addr}"

    def digest(self) -> bytes:
        if self.data_digest:
            return self.data_digest
        if self._data is None and self.tensor is not None:
            self.data_digest = payload_digest.digest_tensor(self.tensor)
        else:
            self.data_digest = payload_digest.digest_bytes(self.data)
        return self.data_digest

    @property
    def header_only(self) -> bool:
        return not self._data and self.tensor is None and bool(self.data_digest)

    def header(self) -> "ProofRequest":
        return ProofRequest(self.kind, self.survey_id, self.sender_id, self.differ_info, b"", self.signature,
                            None, self.digest())

    def to_wire(self) -> dict:
        return {"kind": self.kind, "survey_id": self.survey_id, "sender_id": self.sender_id,
                "differ_info": self.differ_info, "data": self.data, "signature": self.signature,
                "digest": self.data_digest if self.header_only else b""}

    @staticmethod
    def from_wire(d: dict) -> "ProofRequest":
        return ProofRequest(d["kind"], d["survey_id"], d["sender_id"], d["differ_info"], d["data"], d["signature"],
                            None, d.get("digest", b""))


def range_bundle_pack(rpls) -> torch.Tensor:
    """All range-proof lists of one DP response as ONE int32 device tensor:
    [count, len_0, ..., len_{k-1}, packed_0, ..., packed_{k-1}]."""
    packed = [r.pack() for r in rpls]
    dev = packed[0].device if packed else torch.device("cpu")
    hdr = torch.tensor([len(packed)] + [p.numel() for p in packed], dtype=torch.int32, device=dev)
    return torch.cat([hdr] + packed)


def _rows_view(ts: list):
    """[G, numel] view of G equally shaped contiguous tensors that sit back to
    back in one storage (slices of one prover batch), else None."""
    t0 = ts[0]
    n = t0.numel()
    if not all(t.is_contiguous() and t.numel() == n for t in ts):
        return None
    step = n * t0.element_size()
    p0 = t0.data_ptr()
    if any(t.data_ptr() != p0 + g * step for g, t in enumerate(ts)):
        return None
    if t0.storage_offset() + len(ts) * n > t0.untyped_storage().nbytes() // t0.element_size():
        return None
    return t0.new_empty(0).set_(t0.untyped_storage(), t0.storage_offset(), (len(ts), n), (n, 1))


def _stack_rows(ts: list) -> torch.Tensor:
    v = _rows_view(ts)
    return v if v is not None else torch.stack([t.reshape(-1) for t in ts])


def range_bundle_pack_many(bundles: list):
    """``range_bundle_pack`` of many DPs' bundles.  When every bundle is one
    list of the same shape (n, u, l, S) -- thousands of one-output DPs -- all
    are packed by one concatenation into a [G, L] tensor whose rows are the
    bundles (returned too, for one-launch digests); otherwise bundle by bundle.
    -> (list of per-bundle tensors, [G, L] tensor or None)"""
    if len(bundles) > 1 and all(len(b) == 1 for b in bundles):
        rs = [b[0] for b in bundles]
        r0 = rs[0]
        shape = (len(r0), r0.u, r0.l, r0.S, r0.has_rp, r0.commit.device)
        if len(r0) and all((len(r), r.u, r.l, r.S, r.has_rp, r.commit.device) == shape for r in rs):
            G, n = len(rs), len(r0)
            fields = [lambda r: r.commit.K, lambda r: r.commit.C]
            if r0.has_rp:
                fields += [lambda r, a=a: getattr(r, a) for a in ("challenge", "zr", "D", "zphi", "zv", "V", "A")]
            per = [_stack_rows([f(r) for r in rs]) for f in fields]
            size = 5 + 3 * n + sum(p.shape[1] for p in per)
            head = np.empty((G, 2 + 5 + 3 * n), dtype=np.int32)
            head[:, :7] = [1, size, 0x52505231, n, r0.u, r0.l, r0.S]
            head[:, 7: 7 + 2 * n] = np.asarray([o for r in rs for o in r.offset], dtype=np.int64).view(np.int32)\
                .reshape(G, 2 * n)
            head[:, 7 + 2 * n:] = np.asarray([c for r in rs for c in r.cols], dtype=np.int32).reshape(G, n)
            ht = torch.from_numpy(head)
            dev = per[0].device
            if dev.type == "cuda":
                ht = ht.pin_memory().to(dev, non_blocking=True)
            packed = torch.cat([ht] + per, dim=1)
            return list(packed.unbind(0)), packed
    return [range_bundle_pack(b) for b in bundles], None


def new_range_requests(items: list, survey_id: str, secrets: list, device) -> list:
    """NewRangeProofRequest for many DPs at once (``items`` = [(dp_id, lists)]):
    one packing concatenation, one digest launch, one signing launch."""
    with timers.span("sign.marshal.range"):
        tensors, packed = range_bundle_pack_many([lists for _, lists in items])
    with timers.span("sign.digest.range"):
        if packed is not None:
            dgs = payload_digest.digest_rows(packed)
        else:
            dgs = [payload_digest.digest_tensor(t) for t in tensors]
    with timers.span("sign.schnorr.range"):
        sigs = sigma.schnorr_sign_batch(secrets, dgs, device)
    return [ProofRequest("range", survey_id, dp_id, "", None, sig, obj=lists, data_digest=dg, tensor=t)
            for (dp_id, lists), t, dg, sig in zip(items, tensors, dgs, sigs)]


_HEAD = 7 + 3 * 64  # header ints fetched per bundle by the batched unpack (lists of <= 64 proofs)


def _unpack_one(t: torch.Tensor, head: list) -> list:
    """One bundle of a single list whose header words (count, size, meta,
    offsets, cols) are already on the host."""
    k, size, magic, n, u, l, S = head[:7]
    if k != 1 or magic != 0x52505231 or size != t.numel() - 2 or n < 0 or 7 + 3 * n > len(head):
        raise ValueError("malformed range bundle header")
    offs = np.asarray(head[7: 7 + 2 * n], dtype=np.int32).view(np.int64).tolist()
    cols = head[7 + 2 * n: 7 + 3 * n]
    return [rp.RangeProofList.unpack(t[2:], (magic, n, u, l, S), offs, cols)]


def range_bundle_unpack_many(ts: list) -> list:
    """``range_bundle_unpack`` of many bundles with one device-to-host copy of
    their headers (instead of a handful of small synchronous copies each);
    bundles with several lists or > 64 proofs take the single path.  An entry
    is the list of RangeProofLists or the exception that rejects the bundle."""
    out: list = [None] * len(ts)
    short = [i for i, t in enumerate(ts) if t.numel() >= 7]
    if short:
        heads = torch.nn.utils.rnn.pad_sequence([ts[i][: _HEAD] for i in short], batch_first=True).cpu().tolist()
    for j, i in enumerate(short):
        h = heads[j]
        try:
            if h[0] == 1 and 0 <= h[3] <= 64:
                out[i] = _unpack_one(ts[i], h[: min(len(h), ts[i].numel())])
        except Exception as e:  # noqa: BLE001 -- a malformed bundle is a rejected proof
            out[i] = e
    for i, t in enumerate(ts):
        if out[i] is None:
            try:
                out[i] = range_bundle_unpack(t)
            except Exception as e:  # noqa: BLE001
                out[i] = e
    return out


def range_bundle_unpack(t: torch.Tensor) -> list:
    k = int(t[0])
    sizes = t[1: 1 + k].cpu().tolist()
    if k < 0 or any(s < 0 for s in sizes) or 1 + k + sum(sizes) != t.numel():
        raise ValueError("malformed range bundle")
    o, out = 1 + k, []
    for s in sizes:
        out.append(rp.RangeProofList.unpack(t[o: o + s]))
        o += s
    return out


def range_bundle_to_bytes(rpls) -> bytes:
    """Marshalled range-proof request payload (raw limb format, see RangeProofList.pack)."""
    return range_bundle_pack(rpls).cpu().numpy().tobytes()


def range_bundle_from_bytes(b: bytes, device="cpu") -> list:
    t = torch.from_numpy(np.frombuffer(b, dtype=np.int32).copy()).to(device)
    return range_bundle_unpack(t)


def range_bundle_export_kyber(rpls) -> bytes:
    """kyber-layout (reference ToBytes field order/sizes) export of a bundle."""
    out = [len(rpls).to_bytes(8, "little")]
    for r in rpls:
        b = r.to_bytes()
        out += [len(b).to_bytes(8, "little"), b]
    return b"".join(out)


def new_proof_request(kind: str, proof, survey_id: str, sender_id: str, differ_info: str, secret: int) -> ProofRequest:
    """New{Range,Aggregation,Obfuscation,Shuffle,KeySwitch}ProofRequest: marshal + Schnorr-sign.
    Range bundles stay a device tensor; their digest is hashed on the device."""
    with timers.span(f"sign.marshal.{kind}"):
        if kind == "range":
            req = ProofRequest(kind, survey_id, sender_id, differ_info, None, b"", obj=proof,
                               tensor=range_bundle_pack(proof))
        else:
            req = ProofRequest(kind, survey_id, sender_id, differ_info, proof.to_bytes(), b"", obj=proof)
    with timers.span(f"sign.digest.{kind}"):
        dg = req.digest()
    with timers.span(f"sign.schnorr.{kind}"):
        req.signature = sigma.schnorr_sign(secret, dg)
    return req


def verify_signature(req: ProofRequest, public) -> bool:
    """VerifyProofSignature (structs_proofs.go:498-505)."""
    return sigma.schnorr_verify(public, req.digest(), req.signature)


def assigned_vns(sq, req: ProofRequest, n_vns: int):
    """Sharded mode: the VN indices that verify this request (None = every VN samples)."""
    shard = int(getattr(sq, "VerificationSharding", 0) or 0)
    if shard <= 0 or n_vns <= 0:
        return None
    if req.kind == "range":
        # the heavy lists are balanced: DP number k -> VNs k+1 .. k+shard
        # (round robin over the survey's DP order, offset by one so a VN placed
        # with its DP on the same rank/GPU never checks that DP's proofs)
        order = _dp_order(sq)
        if req.sender_id in order:
            k = order[req.sender_id]
            return {(k + 1 + j) % n_vns for j in range(min(shard, n_vns))}
    h = int.from_bytes(hashlib.sha256(req.base_key().encode()).digest()[:8], "little")
    return {(h + k) % n_vns for k in range(min(shard, n_vns))}


def _dp_order(sq) -> dict:
    """DP id -> position in the survey's (broadcast, hence rank-consistent) DP roster."""
    cache = getattr(sq, "_dp_order_cache", None)
    if cache is None:
        ids = []
        for dps in (sq.ServerToDP or {}).values():
            ids += [si.id for si in (dps or [])]
        cache = {d: i for i, d in enumerate(ids)}
        try:
            sq._dp_order_cache = cache
        except AttributeError:
            pass
    return cache


def prewarm_keyswitch(reqs: list, sq, vn_ids: list, device, cache: VerifierCache):
    """Key-switch proofs of an inbox verified for SEVERAL co-hosted VNs at once
    (``sigma.key_switch_batch_verification_multi``: one grouped MSM, each VN
    with its own random weights) when every VN verifies every request
    (Threshold 1, no sharding); ``verify_requests`` then reads its VN's
    verdicts from ``cache.ks_pre``."""
    if len(vn_ids) < 2 or sq.Threshold < 1.0 or getattr(sq, "VerificationSharding", 0):
        return
    ks = [i for i, r in enumerate(reqs) if r.kind == "keyswitch" and not r.header_only]
    if len(ks) < 2:
        return
    objs, valid, verdict = [], [], {}
    for i in ks:
        try:
            o = _decode(reqs[i], device)
        except Exception as e:
            log.warning(f"keyswitch proof from {reqs[i].sender_id} rejected: {e}")
            verdict[i] = False
            continue
        if o.X != sq.IDtoPublic.get(reqs[i].sender_id) or o.Q != sq.ClientPubKey:
            verdict[i] = False
            continue
        objs.append(o)
        valid.append(i)
    for vn_id, res in zip(vn_ids, sigma.key_switch_batch_verification_multi(objs, sq.KeySwitchingProofThreshold,
                                                                             len(vn_ids))):
        m = dict(verdict)
        m.update(zip(valid, res))
        cache.ks_pre[(sq.SurveyID, vn_id)] = m
    while len(cache.ks_pre) > 64:
        cache.ks_pre.pop(next(iter(cache.ks_pre)))


def should_verify(sq, req: ProofRequest, vn_index: int, n_vns: int) -> bool:
    a = assigned_vns(sq, req, n_vns)
    if a is not None:
        return vn_index in a
    return random.random() <= sq.Threshold


class VerifierCache:
    """Per-survey device material a VN reuses across requests (signature
    tables, collective key)."""

    def __init__(self):
        self._sig = {}
        self._early: dict = {}  # SurveyID -> {id(lists): (lists, future, index)}
        self.ks_pre: dict = {}  # (SurveyID, vn_id) -> {request index: bool} (prewarm_keyswitch)

    def put_early(self, survey_id: str, objs: list, fut):
        if len(self._early) > 8:
            self._early.clear()
        self._early[survey_id] = {id(o): (o, fut, i) for i, o in enumerate(objs)}

    def take_early(self, survey_id: str, req):
        """The speculative content check started for this exact proof object
        (consumed once: a second VN on the same rank verifies on its own)."""
        m = self._early.get(survey_id)
        if not m or req.obj is None:
            return None
        e = m.get(id(req.obj))
        if e is None or e[0] is not req.obj:
            return None
        del m[id(req.obj)]
        if not m:
            self._early.pop(survey_id, None)
        return e[1], e[2]

    def sigmat(self, sq, device):
        """Keyed by a digest of the signature set, so repeated surveys over the
        same CN input-validation keys reuse the device tables."""
        sigs = sq.Query.IVSigs.InputValidationSigs
        key = (ivsigs_digest(sigs), len(sigs), len(sigs[0]) if sigs else 0, str(device))
        if key not in self._sig:
            if len(self._sig) > 8:
                self._sig.clear()
            self._sig[key] = rp.SigMaterial(sigs, device)
        return self._sig[key]


def _ranges_ok(sq, rpl) -> bool:
    rg = sq.Query.Ranges
    for j, col in enumerate(rpl.cols):
        r = rg[col] if col < len(rg) else None
        if r is None or int(r[0]) != rpl.u or int(r[1]) != rpl.l:
            return False
        if (int(r[2]) if len(r) > 2 else 0) != int(rpl.offset[j]):
            return False
    return True


def verify_content(req: ProofRequest, sq, device, cache: VerifierCache) -> bool:
    P = sq.RosterServers.aggregate()
    if req.kind == "range":
        rpls = _range_lists(req, device)
        sigs = sq.Query.IVSigs.InputValidationSigs
        for r in rpls:
            if not r.has_rp:
                continue
            if sigs is None or not _ranges_ok(sq, r):
                return False
            if not rp.verify_range_proof_list(r, cache.sigmat(sq, device), P, sq.RangeProofThreshold, device,
                                              sq.RangeProofMode):
                return False
        return True
    if req.kind == "aggregation":
        pr = _decode(req, device)
        return ags.aggregation_list_proof_verification(pr, sq.AggregationProofThreshold)
    if req.kind == "obfuscation":
        pr = _decode(req, device)
        return sigma.obfuscation_list_proof_verification(pr, sq.ObfuscationProofThreshold)
    if req.kind == "shuffle":
        pr = _decode(req, device)
        return shuffle.verify(pr, P)
    if req.kind == "keyswitch":
        pr = _decode(req, device)
        if pr.X != sq.IDtoPublic.get(req.sender_id) or pr.Q != sq.ClientPubKey:
            return False
        return sigma.key_switch_list_proof_verification(pr, sq.KeySwitchingProofThreshold)
    raise ValueError(req.kind)


def _prefetch_range_lists(reqs: list, idxs: list, device):
    """Decode the tensor payloads of many range requests at once (see
    ``range_bundle_unpack_many``); a malformed one keeps its exception so
    ``_range_lists`` raises it for that request alone."""
    todo = [i for i in idxs if reqs[i].decoded is None and reqs[i].tensor is not None and reqs[i]._data is None]
    if len(todo) < 2:
        return
    for i, r in zip(todo, range_bundle_unpack_many([reqs[i].tensor.to(device) for i in todo])):
        reqs[i].decoded = r


def _range_lists(req: ProofRequest, device) -> list:
    """The VN's decode of the SIGNED payload (the raw limb tensor, or its bytes),
    never the prover's in-memory object: what is verified is what the
    signature covers (structs_proofs.go:158-182 unmarshals before verifying).
    Decoding a packed tensor is views plus validity checks; the result is
    cached on the request for the other VNs of this rank."""
    if req.decoded is None:
        if req.tensor is not None and req._data is None:
            req.decoded = range_bundle_unpack(req.tensor.to(device))
        else:
            req.decoded = range_bundle_from_bytes(req.data, device)
    if isinstance(req.decoded, Exception):
        raise req.decoded
    return req.decoded


def verify_range_many(reqs: list, idxs: list, sq, device, cache: VerifierCache, part=None) -> dict:
    """Range-proof requests of one VN as ONE batched verification (see
    ``verify_range_many_multi``).  -> {request index: bool}"""
    return verify_range_many_multi(reqs, {"vn": idxs}, sq, device, cache, part)["vn"]


def verify_range_many_multi(reqs: list, vn_idxs: dict, sq, device, cache: VerifierCache, part=None) -> dict:
    """Range-proof requests of several VNs hosted on this rank: the sampled
    prefix of every list (reference RangeProofThreshold semantics) of every
    request, grouped by (u, l), folded into one pairing batch per VN with that
    VN's own random weights; VNs that sample the same requests share the
    decode and the weight-free work (``rp.verify_range_proof_list_multi``).
    If a VN's batch fails, each request is re-checked alone for that VN so the
    bitmap blames exactly the bad ones.  ``part = (k, W)`` checks only the
    k-th of W equal slices of every sampled prefix (the pooled verification of
    a multi-GPU node).  vn_idxs: {vn: [request index]} -> {vn: {index: bool}}"""
    by_set: dict = {}
    for vn, idxs in vn_idxs.items():
        by_set.setdefault(tuple(sorted(idxs)), []).append(vn)
    out = {}
    for idxs, group in by_set.items():
        res = _verify_range_group(reqs, list(idxs), sq, device, cache, part, len(group))
        for vn, rv in zip(group, res):
            out[vn] = rv
    return out


def _verify_range_group(reqs, idxs, sq, device, cache, part, n_vn) -> list:
    P = sq.RosterServers.aggregate()
    sigs = sq.Query.IVSigs.InputValidationSigs
    mode = int(getattr(sq, "RangeProofMode", 0) or 0)
    base, parts = {}, {}
    with timers.span("rp.verify.unpack_many"):
        _prefetch_range_lists(reqs, idxs, device)
    for i in idxs:
        try:
            lists = []
            with timers.span("rp.verify.unpack"):
                unpacked = _range_lists(reqs[i], device)
            for r in unpacked:
                if not r.has_rp:
                    continue
                if sigs is None or not _ranges_ok(sq, r):
                    raise ValueError("ranges / signatures do not match the query")
                k = int(math.ceil(sq.RangeProofThreshold * len(r)))
                lo, hi = 0, k
                if part is not None:
                    lo, hi = (k * part[0]) // part[1], (k * (part[0] + 1)) // part[1]
                if hi > lo:
                    lists.append(r if (lo, hi) == (0, len(r)) else rp.rpl_range(r, lo, hi))
            parts[i] = lists
            base[i] = True
        except Exception as e:
            log.warning(f"range proof from {reqs[i].sender_id} rejected: {e}")
            base[i] = False
    outs = [dict(base) for _ in range(n_vn)]
    live = [i for i in idxs if base[i] and parts[i]]
    if not live:
        return outs
    sigmat = cache.sigmat(sq, device)
    groups: dict = {}
    for i in live:
        for r in parts[i]:
            groups.setdefault((r.u, r.l, r.S), []).append(r)
    oks = [True] * n_vn
    try:
        with timers.span("rp.verify.cat"):
            cats = [rp.rpl_cat(g) for g in groups.values()]
        for c in cats:
            for k, ok in enumerate(rp.verify_range_proof_list_multi(c, sigmat, P, n_vn, device, mode)):
                oks[k] = oks[k] and ok
    except Exception as e:
        log.warning(f"batched range verification failed: {e}")
        oks = [False] * n_vn
    for k in range(n_vn):
        if oks[k] or len(live) == 1:
            for i in live:
                outs[k][i] = oks[k]
            continue
        for i in live:  # attribute the failure (this VN's own re-check, request by request)
            try:
                outs[k][i] = all(rp.verify_range_proof_list(r, sigmat, P, 1.0, device, mode) for r in parts[i])
            except Exception:
                outs[k][i] = False
    return outs


_DECODERS = {"keyswitch": lambda b, d: sigma.KeySwitchProof.from_bytes(b, d),
             "obfuscation": lambda b, d: sigma.ObfuscationProof.from_bytes(b, d),
             "aggregation": lambda b, d: ags.AggregationProof.from_bytes(b, d),
             "shuffle": lambda b, d: shuffle.ShuffleProof.from_bytes(b, d)}


def _decode(req: ProofRequest, device):
    """Unmarshal the signed bytes (cached per request across the VNs of a rank)."""
    if req.decoded is None:
        req.decoded = _DECODERS[req.kind](req.data, device)
    return req.decoded


_SIG_BATCH_MIN = 16  # inboxes at least this long check their envelope signatures in one batch


def verify_requests(reqs: list, sq, vn_id: str, vn_index: int, n_vns: int, device, cache: VerifierCache,
                    range_pooled=None, defer: bool = False):
    """VerifyProof for a VN's whole inbox.  Signatures and sampling per request;
    the content of the short per-CN proofs (key switch, obfuscation) is verified
    in one batched launch per kind; range proofs are already one batch each.
    ``range_pooled``: {base_key: None (not sampled) | bool} -- this VN's range
    results from the pooled verification (``pool_sampling`` decided the
    sampling on this VN's rank beforehand; a dict or a Future of one).
    ``defer``: return a callable that waits for the pooled range results and
    returns the codes (everything else is already checked)."""
    codes = [None] * len(reqs)
    todo: dict = {}
    pooled_idx: list = []
    if len(reqs) >= _SIG_BATCH_MIN:
        # each envelope's Schnorr check is a deterministic function of the signed
        # bytes and the roster key: done once per rank, read by every co-hosted VN
        keys = [(sq.IDtoPublic.get(r.sender_id), r.digest(), r.signature) for r in reqs]
        fresh = [i for i, r in enumerate(reqs) if r.sig_ok is None or r.sig_ok[0] != keys[i]]
        if fresh:
            with timers.span("verify.signature.batch"):
                for i, v in zip(fresh, sigma.schnorr_verify_batch([keys[i] for i in fresh], device)):
                    reqs[i].sig_ok = (keys[i], v)
        sigs_ok = [r.sig_ok[1] for r in reqs]
    else:
        sigs_ok = None
    for i, req in enumerate(reqs):
        if sigs_ok is not None:
            sig_ok = sigs_ok[i]
        else:
            with timers.span(f"verify.signature.{req.kind}"):
                sig_ok = verify_signature(req, sq.IDtoPublic.get(req.sender_id))
        if not sig_ok:
            codes[i] = PROOF_FALSE_SIGN
        elif range_pooled is not None and req.kind == "range" and not req.header_only:
            pooled_idx.append(i)  # resolved below: the pooled batch may still be running
        elif not should_verify(sq, req, vn_index, n_vns):
            codes[i] = PROOF_RECEIVED
        else:
            todo.setdefault(req.kind, []).append(i)
    early = {}
    for i in todo.get("range", []):
        e = cache.take_early(sq.SurveyID, reqs[i])
        if e is not None:
            early[i] = e
    if early:
        todo["range"] = [i for i in todo["range"] if i not in early]
        if not todo["range"]:
            del todo["range"]
    range_future = None
    if "range" in todo and len(todo) > 1 and torch.device(device).type == "cuda":
        # the range lists (the heavy pairing work) verify on a worker thread with
        # their own HIP stream while this thread checks the short per-CN proofs
        idxs = todo.pop("range")
        range_future = _side_pool().submit(_verify_range_side, reqs, idxs, sq, vn_id, device, cache,
                                           torch.cuda.current_stream(torch.device(device)))
    pre = cache.ks_pre.pop((sq.SurveyID, vn_id), None)
    if pre is not None and "keyswitch" in todo and all(i in pre for i in todo["keyswitch"]):
        with timers.timed(f"{vn_id}_{TIMER['keyswitch']}"):
            for i in todo.pop("keyswitch"):
                codes[i] = PROOF_TRUE if pre[i] else PROOF_FALSE
    for kind, idxs in todo.items():
        with timers.timed(f"{vn_id}_{TIMER[kind]}"):
            if kind == "range":
                for i, ok in verify_range_many(reqs, idxs, sq, device, cache).items():
                    codes[i] = PROOF_TRUE if ok else PROOF_FALSE
            elif kind in ("keyswitch", "obfuscation") and len(idxs) > 1:
                objs, valid = [], []
                for i in idxs:
                    try:
                        o = _decode(reqs[i], device)
                        if kind == "keyswitch" and (o.X != sq.IDtoPublic.get(reqs[i].sender_id)
                                                    or o.Q != sq.ClientPubKey):
                            codes[i] = PROOF_FALSE
                            continue
                        objs.append(o)
                        valid.append(i)
                    except Exception as e:
                        log.warning(f"{vn_id}: {kind} proof from {reqs[i].sender_id} rejected: {e}")
                        codes[i] = PROOF_FALSE
                if kind == "keyswitch":
                    res = sigma.key_switch_batch_verification(objs, sq.KeySwitchingProofThreshold)
                else:
                    res = sigma.obfuscation_batch_verification(objs, sq.ObfuscationProofThreshold)
                for i, r in zip(valid, res):
                    codes[i] = PROOF_TRUE if r else PROOF_FALSE
            else:
                for i in idxs:
                    try:
                        ok = verify_content(reqs[i], sq, device, cache)
                    except Exception as e:
                        log.warning(f"{vn_id}: {kind} proof from {reqs[i].sender_id} rejected: {e}")
                        ok = False
                    codes[i] = PROOF_TRUE if ok else PROOF_FALSE
    if range_future is not None:
        for i, code in range_future.result():
            codes[i] = code
    if early:
        with timers.span("rp.verify.early_wait"):
            for i, (fut, j) in early.items():
                codes[i] = PROOF_TRUE if fut.result()[j] else PROOF_FALSE
    def resolve():
        if pooled_idx:
            with timers.span("rp.verify.pooled_wait"):
                pooled = range_pooled.result() if hasattr(range_pooled, "result") else range_pooled
                pooled = pooled.get(vn_id, {}) if vn_id in pooled else pooled
            for i in pooled_idx:
                res = pooled.get(reqs[i].base_key(), False)
                codes[i] = PROOF_RECEIVED if res is None else (PROOF_TRUE if res else PROOF_FALSE)
        return codes

    return resolve if defer else resolve()


class _EarlyReq:
    """The prover's own lists, checked speculatively (opt-in DRYNX_EARLY_RANGE);
    the result is only used for the request whose payload packs these lists."""
    __slots__ = ("obj", "sender_id", "decoded")

    def __init__(self, obj, sender_id):
        self.obj, self.sender_id, self.decoded = obj, sender_id, obj


def start_early_range_verification(items: list, sq, device, cache: VerifierCache, ready_event=None):
    """Speculative content check of range-proof lists produced on THIS rank for
    a VN hosted on this rank: queued on the range worker (own HIP stream) as
    soon as the prover kernels are queued, so the pairing fold overlaps the CN
    phases (aggregation, key switching) instead of starting after them.  The
    reference fires proofs asynchronously and VNs verify on arrival
    (data_collection_protocol.go:278-348, proof_collection_protocol.go:150-200);
    here arrival is the moment the proof tensors exist.  The envelope
    signature and sampling are still checked by ``verify_requests``, which
    takes the result only for the very same proof object.
    items: [(dp_id, lists)] -> future of {index: bool}."""
    reqs = [_EarlyReq(lists, dp_id) for dp_id, lists in items]
    fut = _side_pool().submit(_verify_range_early, reqs, sq, device, cache, ready_event)
    cache.put_early(sq.SurveyID, [r.obj for r in reqs], fut)
    return fut


def _verify_range_early(reqs, sq, device, cache, ready_event) -> dict:
    dev = torch.device(device)
    side = _streams.get(str(dev))
    if side is None:
        side = _streams[str(dev)] = torch.cuda.Stream(dev)
    if ready_event is not None:
        side.wait_event(ready_event)  # the prover's kernels have produced the lists
    with torch.cuda.stream(side), timers.span("rp.verify.early"):
        out = verify_range_many(reqs, list(range(len(reqs))), sq, device, cache)
    side.synchronize()
    return out


_pool = None
_streams: dict = {}


def _side_pool():
    global _pool
    if _pool is None:
        import concurrent.futures as cf

        _pool = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="drynx-vn-range")
    return _pool


def _verify_range_side(reqs, idxs, sq, vn_id, device, cache, main) -> list:
    dev = torch.device(device)
    side = _streams.get(str(dev))
    if side is None:
        side = _streams[str(dev)] = torch.cuda.Stream(dev)
    side.wait_stream(main)  # payloads / decoded lists are ready
    out = []
    with torch.cuda.stream(side), timers.timed(f"{vn_id}_{TIMER['range']}"):
        for i, ok in verify_range_many(reqs, idxs, sq, device, cache).items():
            out.append((i, PROOF_TRUE if ok else PROOF_FALSE))
    side.synchronize()
    return out


def verify_proof(req: ProofRequest, sq, vn_id: str, vn_index: int, n_vns: int, device, cache: VerifierCache) -> int:
    """<Kind>ProofRequest.VerifyProof -> bitmap code."""
    with timers.timed(f"{vn_id}_{TIMER[req.kind]}"):
        if not verify_signature(req, sq.IDtoPublic.get(req.sender_id)):
            return PROOF_FALSE_SIGN
        if not should_verify(sq, req, vn_index, n_vns):
            return PROOF_RECEIVED
        try:
            ok = verify_content(req, sq, device, cache)
        except Exception as e:  # malformed proof bytes => false, never a crash of the VN
            log.warning(f"{vn_id}: {req.kind} proof from {req.sender_id} rejected: {e}")
            ok = False
        return PROOF_TRUE if ok else PROOF_FALSE
