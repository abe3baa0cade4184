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
import os
import random
import time
from typing import Any

import numpy as np
import torch

from ..crypto import bn254 as bn
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
                 "tensor", "decoded", "slice_of")

    def __init__(self, kind: str, survey_id: str, sender_id: str, differ_info: str, data: bytes | None,
                 signature: bytes, obj: Any = None, data_digest: bytes = b"", tensor: torch.Tensor | None = None):
        self.kind, self.survey_id, self.sender_id, self.differ_info = kind, survey_id, sender_id, differ_info
        self.slice_of = None  # pooled helper copy: (lo, hi) bounds per list of the signed bundle (fan_out)
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


def _unpack_rows(ts: list, heads: list, out: list) -> bool:
    """Fast path of ``range_bundle_unpack_many`` for many one-list bundles of
    one shape that are rows of ONE packed tensor (``range_bundle_pack_many``:
    thousands of one-record DPs): every field is cut from the [G, L] view
    once and split into its G per-bundle views by one ``unbind`` (C++), not
    by ~9 Python slicing calls per bundle.  Fills ``out`` and returns True,
    or returns False (nothing filled) when the bundles do not qualify."""
    rows = _rows_view(ts)
    if rows is None:
        return False
    G, W = rows.shape
    h0 = heads[0][:7]
    k, size, magic, n, u, l, S = h0
    if k != 1 or magic != 0x52505231 or size != W - 2 or not 0 <= n <= 64 or min(u, l, S) < 0:
        return False
    if any(h[:7] != h0 for h in heads):
        return False
    has_rp = not (u == 0 and l == 0) and n > 0
    o = 2 + 5 + 3 * n
    widths = [("K", n, 24), ("C", n, 24)]
    if has_rp:
        widths += [("challenge", n, 8), ("zr", n, 8), ("D", n, 24), ("zphi", n * l, 8), ("zv", n * S * l, 8),
                   ("V", n * S * l, 32), ("A", n * S * l, 96)]
    if o + sum(r * w for _, r, w in widths) != W:
        return False
    cols = {}
    for name, r, w in widths:
        cols[name] = rows[:, o: o + r * w].reshape(G, r, w).unbind(0) if r else [rows.new_empty((0, w))] * G
        o += r * w
    fields = ("challenge", "zr", "D", "zphi", "zv", "V", "A")
    for g, h in enumerate(heads):
        offs = np.asarray(h[7: 7 + 2 * n], dtype=np.int32).view(np.int64).tolist()
        rpl = rp.RangeProofList(u, l, S, offs, h[7 + 2 * n: 7 + 3 * n], rp.CipherVector(cols["K"][g], cols["C"][g]))
        if has_rp:
            for f in fields:
                setattr(rpl, f, cols[f][g])
        out[g] = [rpl]
    return True


def range_bundle_unpack_many(ts: list) -> list:
    """``range_bundle_unpack`` of many bundles with one device-to-host copy of
    their headers (instead of a handful of small synchronous copies each);
    bundles with several lists or > 64 proofs take the single path.  An entry
    is the list of RangeProofLists or the exception that rejects the bundle."""
    out: list = [None] * len(ts)
    short = [i for i, t in enumerate(ts) if t.numel() >= 7]
    if short:
        heads = torch.nn.utils.rnn.pad_sequence([ts[i][: _HEAD] for i in short], batch_first=True).cpu().tolist()
        if len(short) == len(ts) and len(ts) >= 64 and _unpack_rows(ts, heads, out):
            return out
    big = []
    for j, i in enumerate(short):
        h = heads[j]
        try:
            if h[0] == 1 and 0 <= h[3] <= 64:
                out[i] = _unpack_one(ts[i], h[: min(len(h), ts[i].numel())])
            elif h[0] == 1 and 64 < h[3] and 7 + 3 * h[3] <= ts[i].numel():
                big.append((i, 7 + 3 * h[3]))
        except Exception as e:  # noqa: BLE001 -- a malformed bundle is a rejected proof
            out[i] = e
    if big:
        # single-list bundles of wide queries (2070 proofs per DP): every full
        # header in ONE more device-to-host copy instead of one sync per bundle
        full = torch.nn.utils.rnn.pad_sequence([ts[i][:w] for i, w in big], batch_first=True).cpu().numpy()
        for (i, w), h in zip(big, full):
            try:
                out[i] = _unpack_one(ts[i], h[:w].tolist())
            except Exception as e:  # noqa: BLE001
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


PACKED_KINDS = ("aggregation", "keyswitch", "obfuscation")


def new_proof_request(kind: str, proof, survey_id: str, sender_id: str, differ_info: str, secret: int) -> ProofRequest:
    """New{Range,Aggregation,Obfuscation,Shuffle,KeySwitch}ProofRequest: marshal + Schnorr-sign."""
    return new_proof_requests([(kind, proof, sender_id, differ_info, secret)], survey_id)[0]


def new_proof_requests(items: list, survey_id: str) -> list:
    """Many envelopes at once (``items`` = [(kind, proof, sender_id,
    differ_info, secret)]).  Range bundles and the per-CN proofs
    (aggregation, key switch, obfuscation) are raw limb tensors assembled
    where the proof lives (no host marshalling); their digests are ONE
    segmented device launch and one copy to the host; the Schnorr signatures
    are one batch.  Shuffle proofs stay bytes (reference-style export)."""
    if not items:
        return []
    reqs = []
    with timers.span("sign.marshal"):
        for kind, proof, sender_id, differ_info, _ in items:
            if kind == "range":
                reqs.append(ProofRequest(kind, survey_id, sender_id, differ_info, None, b"", obj=proof,
                                         tensor=range_bundle_pack(proof)))
            elif kind in PACKED_KINDS:
                reqs.append(ProofRequest(kind, survey_id, sender_id, differ_info, None, b"", obj=proof,
                                         tensor=proof.pack()))
            else:
                reqs.append(ProofRequest(kind, survey_id, sender_id, differ_info, proof.to_bytes(), b"", obj=proof))
    with timers.span("sign.digest"):
        tens = [i for i, r in enumerate(reqs) if r.tensor is not None]
        devs = {reqs[i].tensor.device for i in tens}
        if len(devs) == 1 and len(tens) > 1:
            for i, d in zip(tens, payload_digest.digest_many([reqs[i].tensor for i in tens])):
                reqs[i].data_digest = d
        dgs = [r.digest() for r in reqs]
    with timers.span("sign.schnorr"):
        dev = next(iter(devs)) if devs else "cpu"
        sigs = sigma.schnorr_sign_batch([it[4] for it in items], dgs, dev)
    for r, sig in zip(reqs, sigs):
        r.signature = sig
    return reqs


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


def prewarm_keyswitch(reqs: list, sq, vn_ids: list, device, cache: "VerifierCache", coins: dict | None = None):
    """Key-switch proofs of an inbox verified for SEVERAL co-hosted VNs at once
    when every VN verifies every request (Threshold 1, no sharding): one
    grouped MSM in which every VN's random combination uses that VN's own
    coins, and every VN's own Fiat-Shamir / T3 checks
    (``sigma.key_switch_batch_verification_multi``); ``verify_requests``
    then reads its VN's verdicts from ``cache.ks_pre``."""
    if len(vn_ids) < 2 or sq.Threshold < 1.0 or getattr(sq, "VerificationSharding", 0):
        return
    ks = [i for i, r in enumerate(reqs) if r.kind == "keyswitch" and not r.header_only]
    if len(ks) < 2:
        return
    t0 = time.perf_counter()
    _prefetch_packed(reqs, ks, device)
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
    coins = coins or {}
    for vn_id, res in zip(vn_ids, sigma.key_switch_batch_verification_multi(
            objs, sq.KeySwitchingProofThreshold, [coins.get(v) for v in vn_ids])):
        m = dict(verdict)
        m.update(zip(valid, res))
        m["dt"] = time.perf_counter() - t0  # every VN's verdicts exist once the shared batch is done
        cache.ks_pre[(sq.SurveyID, vn_id)] = m
    while len(cache.ks_pre) > 64:
        cache.ks_pre.pop(next(iter(cache.ks_pre)))


def prewarm_signatures(reqs: list, sq, vn_ids: list, cache: "VerifierCache"):
    """Every co-hosted VN's own Schnorr checks of the inbox's envelopes in ONE
    host-pool batch (each VN's copy of every check is computed; the batch
    only spreads them over the cores together); ``verify_requests`` reads its
    VN's verdicts from ``cache.sig_pre``."""
    if len(vn_ids) < 2 or not reqs:
        return
    with timers.span("verify.digests"):
        prefetch_digests(reqs)
    keys = [(sq.IDtoPublic.get(r.sender_id), r.digest(), r.signature) for r in reqs]
    dev = next((r.tensor.device for r in reqs if r.tensor is not None), "cpu")
    with timers.span(f"verify.signature.multi[{len(vn_ids)}]"):
        ok = sigma.schnorr_verify_batch(keys * len(vn_ids), dev)  # host below DRYNX_SIG_DEVICE_MIN checks
    n = len(reqs)
    tag = _inbox_tag(reqs)
    for j, vn_id in enumerate(vn_ids):
        cache.sig_pre[(sq.SurveyID, vn_id)] = (tag, ok[j * n:(j + 1) * n])
    while len(cache.sig_pre) > 64:
        cache.sig_pre.pop(next(iter(cache.sig_pre)))


def _inbox_tag(reqs: list) -> bytes:
    """Digest of an inbox's (sender, payload digest, signature) tuples:
    cached signature verdicts apply only to exactly the envelopes they were
    computed for (the two-stage flow checks two inboxes of one survey)."""
    import hashlib

    h = hashlib.sha256()
    for r in reqs:
        h.update(r.sender_id.encode() + b"\x00" + bytes(r.digest()) + bytes(r.signature))
    return h.digest()


def should_verify(sq, req: ProofRequest, vn_index: int, n_vns: int, coins=None) -> bool:
    """The VN's sampling decision: ``rand.Float64() <= Threshold`` from the
    VN's own coins (structs_proofs.go:160-161), or the sharding extension."""
    a = assigned_vns(sq, req, n_vns)
    if a is not None:
        return vn_index in a
    return (coins.random() if coins is not None else random.random()) <= sq.Threshold


class VerifierCache:
    """Per-survey device material a VN reuses across requests (signature
    tables, collective key)."""

    def __init__(self):
        self._sig = {}
        self.ks_pre: dict = {}  # (SurveyID, vn_id) -> {request index: bool} (prewarm_keyswitch)
        self.sig_pre: dict = {}  # (SurveyID, vn_id) -> (inbox tag, [bool]) (prewarm_signatures)

    def sigmat(self, sq, device):
        """Keyed by a digest of the signature set, so repeated surveys over the
        same CN input-validation keys reuse the device tables."""
        sigs = sq.Query.IVSigs.InputValidationSigs
        key = (ivsigs_digest(sigs), len(sigs), len(sigs[0]) if sigs else 0, str(device))
        if key not in self._sig:
            if len(self._sig) > 8:
                # another set's tables may still be read by queued kernels of
                # any stream: the device drains before their memory goes back
                if torch.device(device).type == "cuda":
                    torch.cuda.synchronize(device)
                self._sig.clear()
            self._sig[key] = bn.publish(rp.SigMaterial(sigs, device))
        return self._sig[key]


def _range_table(sq):
    """The query's Ranges as int64 columns (u, l, offset) plus a validity
    mask, built once per survey object (a Python loop over 2070 columns per
    DP list cost ~2 ms each on the range plane's critical path)."""
    cached = getattr(sq, "_range_table_cache", None)
    rg = sq.Query.Ranges or []
    if cached is not None and cached[0] is rg:
        return cached[1]
    n = len(rg)
    tab = np.zeros((4, n), dtype=np.int64)
    for c, r in enumerate(rg):
        if r is None or len(r) < 2:
            continue
        off = int(r[2]) if len(r) > 2 else 0
        if not (0 <= off < (1 << 63)):
            continue
        tab[:, c] = (int(r[0]), int(r[1]), off, 1)
    try:
        sq._range_table_cache = (rg, tab)
    except AttributeError:
        pass
    return tab


def _ranges_ok(sq, rpl) -> bool:
    """Every proof of the list claims its column's (u, l, offset) from the query."""
    tab = _range_table(sq)
    cols = np.asarray(rpl.cols, dtype=np.int64)
    if cols.size == 0:
        return True
    if cols.min() < 0 or cols.max() >= tab.shape[1]:
        return False
    try:
        offs = np.asarray(rpl.offset, dtype=np.int64)
    except (OverflowError, TypeError, ValueError):
        return False
    t = tab[:, cols]
    return bool(t[3].all() and (t[0] == rpl.u).all() and (t[1] == rpl.l).all() and (t[2] == offs).all())


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


def verify_range_many(reqs: list, idxs: list, sq, device, cache: VerifierCache, part=None, coins=None) -> dict:
    """Range-proof requests of one VN as ONE batched verification (see
    ``verify_range_many_multi``).  -> {request index: bool}"""
    return verify_range_many_multi(reqs, {"vn": idxs}, sq, device, cache, part, {"vn": coins})["vn"]


def verify_range_many_multi(reqs: list, vn_idxs: dict, sq, device, cache: VerifierCache, part=None,
                            coins: dict | None = None) -> dict:
    """Range-proof requests of several VNs hosted on this rank: the sampled
    prefix of every list (reference RangeProofThreshold semantics) of every
    request, grouped by (u, l), folded into one pairing batch per VN with that
    VN's own random weights (``coins[vn]``); VNs that sample the same requests
    share the decode and the weight-free work (``rp.verify_range_proof_list_multi``).
    If a VN's batch fails, the failing requests are located by bisection over
    that VN's own re-checks (``_blame``) so the bitmap blames exactly the bad
    ones.  ``part = (k, W)`` checks only the k-th of W equal slices of every
    sampled prefix (the pooled verification of a multi-GPU node); a helper
    copy that already holds only its slice (``slice_of``) is checked whole.
    vn_idxs: {vn: [request index]} -> {vn: {index: bool}}"""
    coins = coins or {}
    by_set: dict = {}
    for vn, idxs in vn_idxs.items():
        by_set.setdefault(tuple(sorted(idxs)), []).append(vn)
    out = {}
    for idxs, group in by_set.items():
        res = _verify_range_group(reqs, list(idxs), sq, device, cache, part, [coins.get(vn) for vn in group])
        for vn, rv in zip(group, res):
            out[vn] = rv
    return out


def sampled_bounds(sq, n: int, part=None) -> tuple:
    """[lo, hi) of a list of n proofs that a verifier checks: the sampled
    prefix ceil(RangeProofThreshold * n) (range_proof.go:486), or its k-th of
    W equal slices for ``part = (k, W)``, or of W weighted slices for
    ``part = (k, W, c_0, ..., c_W)`` (cumulative integer weights, c_0 = 0)."""
    k = int(math.ceil(sq.RangeProofThreshold * n))
    if part is None:
        return 0, k
    if len(part) > 2:
        c = part[2:]
        return (k * c[part[0]]) // c[-1], (k * c[part[0] + 1]) // c[-1]
    return (k * part[0]) // part[1], (k * (part[0] + 1)) // part[1]


# extra work of a rank, in units of a plain helper's pool share, that its
# slice is shortened by.  Every rank's part starts at the same moment -- the
# range fan-out is ONE exchange after every rank has signed its proofs, so at
# the slowest rank's proving end -- so a rank proving an extra DP gets NO
# discount (a discount only lengthened the other parts: profiles/r5/it15,
# pool(share) ~ 13 ms + 122 ms x share); a VN rank's part also carries the
# digests of the other slices (a side stream: +2.2 ms of its part at equal
# shares, profiles/r5/it16).  Round 6: 0.22 while the pool stream ran at
# normal priority (the VN ranks' parts ended ~1.5 ms after the others',
# profiles/r6/final/rank_share_w8_vnw014.json); with the pool stream at high
# priority the digests cost less of the part and 0.14 balances again (same-box
# A/B: projection 45.0-45.4 vs 45.8-46.2 ms at 0.22, profiles/r6/vnw_ab/)
_POOL_DP_W, _POOL_VN_W = 0.0, 0.14


def rank_weights(dps: list, vns: list) -> list:
    """Each rank's share weight for the pooled checks: 1 - _POOL_DP_W (per
    extra DP) - _POOL_VN_W (per VN) (floor 0.25); all 1 under
    DRYNX_POOL_BALANCE=0."""
    if os.environ.get("DRYNX_POOL_BALANCE", "1") == "0":
        return [1.0] * len(dps)
    lo = min(dps)
    return [max(0.25, 1.0 - _POOL_DP_W * (dps[k] - lo) - _POOL_VN_W * vns[k]) for k in range(len(dps))]


def balanced_parts(W: int, dps: list, vns: list) -> list:
    """Pool parts for W ranks weighted so every rank's check ends together
    (``rank_weights``), as (k, W, cumulative weights) tuples
    (``sampled_bounds``).  Calibrated from one-GPU measurements of each
    rank's share (tools/rank_share.py)."""
    if W <= 1 or os.environ.get("DRYNX_POOL_BALANCE", "1") == "0":
        return [(k, W) for k in range(W)]
    w = rank_weights(dps, vns)
    iw = [max(1, int(round(1000 * x))) for x in w]
    cum = [0]
    for x in iw:
        cum.append(cum[-1] + x)
    return [(k, W, *cum) for k in range(W)]


def _range_parts(reqs, idxs, sq, device, part):
    """Decode + query-consistency checks of every request's lists, cut to the
    part this rank checks -> (base verdicts {i: bool}, parts {i: [lists]})."""
    sigs = sq.Query.IVSigs.InputValidationSigs
    base, parts = {}, {}
    tab = _range_table(sq)
    if tab.shape[1] and tab[3].all() and not (tab[0] | tab[1]).any():
        # every column commitment-only (u = l = 0): the verification is true
        # whatever the list holds (range_proof.go:508-510), so nothing is decoded
        for i in idxs:
            base[i], parts[i] = reqs[i].tensor is not None or reqs[i]._data is not None, []
        return base, parts
    with timers.span("rp.verify.unpack_many"):
        _prefetch_range_lists(reqs, idxs, device)
    for i in idxs:
        try:
            lists = []
            unpacked = _range_lists(reqs[i], device)
            for r in unpacked:
                if not r.has_rp:
                    continue
                if sigs is None or not _ranges_ok(sq, r):
                    raise ValueError("ranges / signatures do not match the query")
                if reqs[i].slice_of is not None:
                    lo, hi = 0, len(r)  # a helper's copy: already this rank's slice
                else:
                    lo, hi = sampled_bounds(sq, len(r), part)
                if hi > lo:
                    lists.append(r if (lo, hi) == (0, len(r)) else rp.rpl_range(r, lo, hi))
            parts[i] = lists
            base[i] = True
        except Exception as e:
            log.warning(f"range proof from {reqs[i].sender_id} rejected: {e}")
            base[i] = False
    return base, parts


_RPL_FIELDS = ("challenge", "zr", "D", "zphi", "zv", "V", "A")


def lists_digests(entries: list) -> list:
    """Digest of each entry (a list of RangeProofLists, e.g. one request's
    slice for one pooled part) over its header values and the raw limbs of
    every field, computed from VIEWS of the lists (no packing copy): every
    field region of every entry in ONE segmented SHA-256 launch, one copy to
    the host.  A helper rank reports the digest of the slice it verified; the
    VN recomputes it from its own signed payload, so a helper's verdict only
    counts for exactly the bytes the VN received."""
    tens, spans, metas = [], [], []
    for lists in entries:
        a = len(tens)
        meta = []
        for r in lists:
            # (numpy conversions: a VN rank digests ~70 slices of ~260 proofs
            # per part; per-element int() calls cost it ~6 ms of host time)
            meta += [np.array([len(r), r.u, r.l, r.S], dtype="<i8"), np.asarray(r.offset, dtype="<i8"),
                     np.asarray(r.cols, dtype="<i8")]
            tens += [r.commit.K, r.commit.C]
            if r.has_rp and len(r):
                tens += [getattr(r, f) for f in _RPL_FIELDS]
        spans.append((a, len(tens)))
        metas.append(np.concatenate(meta).tobytes() if meta else b"")
    if tens:
        devs = {t.device for t in tens}
        if len(devs) == 1:
            parts = payload_digest.digest_many([t.contiguous() for t in tens])
        else:
            parts = [payload_digest.digest_tensor(t) for t in tens]
    else:
        parts = []
    out = []
    for (a, b), meta in zip(spans, metas):
        h = hashlib.sha256(b"drynx_amd/range-slice" + meta)
        for d in parts[a:b]:
            h.update(d)
        out.append(h.digest())
    return out


def slice_lists(lists: list, sq, part) -> list:
    """The lists of one bundle cut to what rank ``part[0]`` of ``part[1]``
    checks (empty slices dropped)."""
    out = []
    for r in lists:
        if not r.has_rp:
            continue
        lo, hi = sampled_bounds(sq, len(r), part)
        if hi > lo:
            out.append(r if (lo, hi) == (0, len(r)) else rp.rpl_range(r, lo, hi))
    return out


def _verify_range_group(reqs, idxs, sq, device, cache, part, coins_list: list) -> list:
    P = sq.RosterServers.aggregate()
    mode = int(getattr(sq, "RangeProofMode", 0) or 0)
    n_vn = len(coins_list)
    base, parts = _range_parts(reqs, idxs, sq, device, part)
    outs = [dict(base) for _ in range(n_vn)]
    live = [i for i in idxs if base[i] and parts[i]]
    if not live:
        return outs
    sigmat = cache.sigmat(sq, device)
    for k, bad in enumerate(_bad_requests(live, parts, sigmat, P, device, mode, coins_list)):
        for i in live:
            outs[k][i] = i not in bad
    return outs


_dig_streams: dict = {}


def _slice_digests_async(ok_idx: list, entries: list, device):
    """``lists_digests`` of this part's slices as an idle task of the part's
    verifier (run while it waits for its device passes, on a HIP stream of
    its own ordered after the caller's): the digests are needed only for the
    gather after the part, so they no longer delay its start."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return rp.add_idle_task(rp.Deferred(lambda: dict(zip(ok_idx, lists_digests(entries)))))
    st = _dig_streams.get(str(dev))
    if st is None:
        st = _dig_streams[str(dev)] = torch.cuda.Stream(dev)
    st.wait_stream(torch.cuda.current_stream(dev))

    def run():
        with torch.cuda.stream(st), timers.span("rp.verify.slice_digests"):
            return dict(zip(ok_idx, lists_digests(entries)))
    return rp.add_idle_task(rp.Deferred(run))


def verify_range_pool_part(reqs: list, vn_idxs: dict, sq, device, cache: VerifierCache, part, coins: dict,
                           async_digests: bool = False):
    """One rank's share of a pooled range verification: part ``part`` of the
    sampled prefix of every request, checked for every VN with that VN's
    coins for this part.  -> ({vn: {index: bool}}, {index: slice digest});
    ``async_digests``: the digests as a Future (computed beside the part)."""
    union = sorted({i for idxs in vn_idxs.values() for i in idxs})
    base, parts = _range_parts(reqs, union, sq, device, part)
    digests = {}
    if part[1] > 1:  # only helpers' verdicts need binding to the bytes they checked
        ok_idx = [i for i in union if base[i]]
        if async_digests:
            digests = _slice_digests_async(ok_idx, [parts[i] for i in ok_idx], device)
        else:
            with timers.span("rp.verify.slice_digests"):
                digests = dict(zip(ok_idx, lists_digests([parts[i] for i in ok_idx])))
    P = sq.RosterServers.aggregate()
    mode = int(getattr(sq, "RangeProofMode", 0) or 0)
    by_set: dict = {}
    for vn, idxs in vn_idxs.items():
        by_set.setdefault(tuple(sorted(idxs)), []).append(vn)
    out = {}
    for idxs, group in by_set.items():
        live = [i for i in idxs if base[i] and parts[i]]
        res = [{i: base[i] for i in idxs} for _ in group]
        # work accounting: range items this rank checks, once per VN of the group
        timers.count("pool.range_items", len(group) * sum(len(r) for i in live for r in parts[i]))
        if live:
            sigmat = cache.sigmat(sq, device)
            cl = [coins.get(vn) for vn in group]
            for k, bad in enumerate(_bad_requests(live, parts, sigmat, P, device, mode, cl)):
                for i in live:
                    res[k][i] = i not in bad
        for vn, rv in zip(group, res):
            out[vn] = rv
    return out, digests


_SEG_MAX = 64  # attribution segments per batch (more requests: chunks of requests)


def _u_cap() -> int:
    """Pairing-side U points (verifiers x proofs x servers) per verification
    batch: a batch's working set is ~17 KB of Miller-loop line coefficients
    per U plus the G2 joint tables of its V's, so a million-value range
    (3 x 10M U's per VN) is checked in batches that fit HBM
    (DRYNX_VERIFY_CHUNK_U; the headline inbox, 186k U's, is one batch)."""
    return int(os.environ.get("DRYNX_VERIFY_CHUNK_U", 3 << 20))


def _item_chunks(live: list, parts: dict, n_vn: int) -> list:
    """``live`` / ``parts`` cut into batches of at most ``_u_cap`` U points
    (a list longer than that is split by proof ranges) -> [(live, parts)]."""
    cap = max(1, _u_cap() // max(1, n_vn))
    tot = sum(len(r) * r.S for i in live for r in parts[i])
    if tot <= cap:
        return [(live, parts)]
    out, cur, cur_n = [], {}, 0
    for i in live:
        for r in parts[i]:
            per = max(1, r.S)
            a = 0
            while a < len(r):
                take = min(len(r) - a, max(1, (cap - cur_n) // per))
                cur.setdefault(i, []).append(r if (a, take) == (0, len(r)) else rp.rpl_range(r, a, a + take))
                cur_n += take * per
                a += take
                if cur_n >= cap:
                    out.append(cur)
                    cur, cur_n = {}, 0
    if cur:
        out.append(cur)
    return [(list(c), c) for c in out]


def _bad_requests(live, parts, sigmat, P, device, mode, coins_list) -> list:
    """``_bad_requests_batch`` over batches of at most ``_u_cap`` U points
    (each with fresh weights from every VN's coins); a request is bad for a
    VN when any of its pieces is."""
    chunks = _item_chunks(live, parts, len(coins_list))
    if len(chunks) == 1:
        return _bad_requests_batch(live, parts, sigmat, P, device, mode, coins_list)
    bad = [set() for _ in coins_list]
    for k, (cl, cp) in enumerate(chunks):
        with timers.span(f"rp.verify.chunk[{k}/{len(chunks)}]"):
            for b, more in zip(bad, _bad_requests_batch(cl, cp, sigmat, P, device, mode, coins_list)):
                b |= more
    return bad


def _bad_requests_batch(live, parts, sigmat, P, device, mode, coins_list) -> list:
    """The requests of ``live`` each VN rejects -> [set] per VN.  One batch
    per (u, l, S) group with per-request attribution (rp.verify_range_proof_
    list_multi ``segs``): a passing batch clears everything at once; a
    failing one names its bad segments from a second, segment-grouped pass of
    the failing VN alone.  Only what attribution cannot settle (a segment
    holding several requests when there are more than _SEG_MAX, or a batch
    rejected before the equations) falls back to bisection."""
    n_vn = len(coins_list)
    if len(live) == 1:
        return [set() if ok else set(live) for ok in _check_lists(live, parts, sigmat, P, device, mode, coins_list)]
    units = [[i] for i in live] if len(live) <= _SEG_MAX else \
        [list(c) for c in np.array_split(np.asarray(live), _SEG_MAX) if len(c)]
    groups: dict = {}
    for ui, unit in enumerate(units):
        for i in unit:
            for r in parts[i]:
                if len(r):
                    lists, cnt = groups.setdefault((r.u, r.l, r.S), ([], {}))
                    lists.append(r)
                    cnt[ui] = cnt.get(ui, 0) + len(r)
    bad = [set() for _ in range(n_vn)]
    unsure = [set() for _ in range(n_vn)]
    recheck: set = set()
    try:
        for lists, cnt in groups.values():
            with timers.span("rp.verify.cat"):
                c = rp.rpl_cat(lists)
            uids = list(cnt)
            res = rp.verify_range_proof_list_multi(c, sigmat, P, n_vn, device, mode, coins=coins_list,
                                                   segs=[cnt[u] for u in uids])
            if isinstance(res[0], rp.RangeInvalid):
                # some proofs do not decode: their requests are bad for every VN,
                # the others get a batch without them
                for u, ok in zip(uids, res[0]):
                    if ok:
                        recheck.update(int(i) for i in units[u])
                    elif len(units[u]) == 1:
                        for b in bad:
                            b.add(int(units[u][0]))
                    else:
                        for us in unsure:
                            us.update(int(i) for i in units[u])
                continue
            for k, rk in enumerate(res):
                for u, ok in zip(uids, rk if rk is not None else [None] * len(uids)):
                    if ok is None or (not ok and len(units[u]) > 1):
                        unsure[k].update(int(i) for i in units[u])
                    elif not ok:
                        bad[k].add(int(units[u][0]))
    except Exception as e:
        log.warning(f"batched range verification failed: {e}")
        return [set(int(i) for i in live) for _ in range(n_vn)]
    recheck -= set().union(*bad, *unsure)
    if recheck:  # the decodable requests of a batch that held undecodable ones
        for b, more in zip(bad, _bad_requests_batch(sorted(recheck), parts, sigmat, P, device, mode, coins_list)):
            b |= more
    for k in range(n_vn):
        rest = sorted(unsure[k] - bad[k])
        if rest:
            with timers.span("rp.verify.blame"):
                bad[k] |= _blame(rest, parts, sigmat, P, device, mode, coins_list[k])
    return bad


def _check_lists(live, parts, sigmat, P, device, mode, coins_list) -> list:
    """One batch per (u, l, S) group over the requests ``live``, every VN's
    verdict from its own weights -> [bool] per VN."""
    n_vn = len(coins_list)
    groups: dict = {}
    for i in live:
        for r in parts[i]:
            groups.setdefault((r.u, r.l, r.S), []).append(r)
    oks = [True] * n_vn
    try:
        with timers.span("rp.verify.cat"):
            cats = [rp.rpl_cat(g) for g in groups.values()]
        for c in cats:
            for k, ok in enumerate(rp.verify_range_proof_list_multi(c, sigmat, P, n_vn, device, mode,
                                                                    coins=coins_list)):
                oks[k] = oks[k] and ok
    except Exception as e:
        log.warning(f"batched range verification failed: {e}")
        oks = [False] * n_vn
    return oks


def _blame(live, parts, sigmat, P, device, mode, coins) -> set:
    """The requests of a failed batch that fail on their own, found by
    bisection: a half that passes as one batch is cleared at once, so k bad
    requests among m cost O(k log m) batches instead of m re-checks (each
    batch drawn afresh from the VN's own coins)."""
    bad: set = set()
    stack = [list(live)]
    while stack:
        grp = stack.pop()
        if len(grp) == 1:
            if not _check_lists(grp, parts, sigmat, P, device, mode, [coins])[0]:
                bad.add(grp[0])
            continue
        if _check_lists(grp, parts, sigmat, P, device, mode, [coins])[0]:
            continue
        h = len(grp) // 2
        stack += [grp[h:], grp[:h]]
    return bad


_DECODERS = {"keyswitch": lambda b, d: sigma.KeySwitchProof.from_bytes(b, d),
             "obfuscation": lambda b, d: sigma.ObfuscationProof.from_bytes(b, d),
             "aggregation": lambda b, d: ags.AggregationProof.from_bytes(b, d),
             "shuffle": lambda b, d: shuffle.ShuffleProof.from_bytes(b, d)}


def _decode(req: ProofRequest, device):
    """Unmarshal the SIGNED payload (packed tensor or bytes), never the
    prover's in-memory object; cached per request across the VNs of a rank
    (decoded data, not a verdict)."""
    if req.decoded is None:
        t = None
        if req.kind in PACKED_KINDS:
            if req.tensor is not None and req._data is None:
                t = req.tensor.to(device)
            elif _is_packed(req.kind, req.data):  # a packed payload that travelled as bytes
                t = torch.from_numpy(np.frombuffer(req.data, dtype=np.int32).copy()).to(device)
        if t is not None:
            req.decoded = (ags.AggregationProof.unpack(t) if req.kind == "aggregation"
                           else sigma.unpack_many(req.kind, [t])[0])
        else:
            req.decoded = _DECODERS[req.kind](req.data, device)
    if isinstance(req.decoded, Exception):
        raise req.decoded
    return req.decoded


_PACKED_MAGIC = {"aggregation": ags.AGG_MAGIC, "keyswitch": sigma.KS_MAGIC, "obfuscation": sigma.OBF_MAGIC}


def _is_packed(kind: str, b: bytes) -> bool:
    return len(b) >= 4 and len(b) % 4 == 0 and int.from_bytes(b[:4], "little") == _PACKED_MAGIC[kind]


def export_reference_bytes(kind: str, value: bytes) -> bytes:
    """A stored payload in the reference-style byte layout (GetProofs): packed
    raw-limb payloads are decoded and re-encoded; anything else is served as
    stored.  A packed payload that does not decode raises."""
    if kind == "range":
        from . import range_wire

        if value and range_wire.is_raw_bundle(value):
            return range_wire.encode_bundle(range_bundle_from_bytes(value, "cpu"))
        return value
    if kind in PACKED_KINDS and _is_packed(kind, value):
        t = torch.from_numpy(np.frombuffer(value, dtype=np.int32).copy())
        pr = ags.AggregationProof.unpack(t) if kind == "aggregation" else sigma.unpack_many(kind, [t])[0]
        if isinstance(pr, Exception):
            raise pr
        return pr.to_bytes()
    return value


def _prefetch_packed(reqs: list, idxs: list, device):
    """Decode the packed per-CN proofs of an inbox with one header copy per kind."""
    by_kind: dict = {}
    for i in idxs:
        r = reqs[i]
        if r.decoded is None and r.kind in PACKED_KINDS and r.tensor is not None and r._data is None:
            by_kind.setdefault(r.kind, []).append(i)
    for kind, ii in by_kind.items():
        ts = [reqs[i].tensor.to(device) for i in ii]
        dec = ags.unpack_many(ts) if kind == "aggregation" else sigma.unpack_many(kind, ts)
        for i, d in zip(ii, dec):
            reqs[i].decoded = d


def prefetch_digests(reqs: list):
    """Envelope digests (decoded data: a function of the signed payload) of
    every tensor payload of an inbox in ONE segmented launch per device."""
    todo = [r for r in reqs if not r.data_digest and r.tensor is not None and r._data is None]
    by_dev: dict = {}
    for r in todo:
        by_dev.setdefault(r.tensor.device, []).append(r)
    for rs in by_dev.values():
        for r, d in zip(rs, payload_digest.digest_many([r.tensor for r in rs])):
            r.data_digest = d


def verify_requests(reqs: list, sq, vn_id: str, vn_index: int, n_vns: int, device, cache: VerifierCache,
                    range_pooled=None, defer: bool = False, coins=None):
    """VerifyProof for a VN's whole inbox, with the VN's own verdicts: its
    Schnorr checks of every envelope (one batch), its sampling decisions and
    random weights (``coins``, crypto/coins.py), its Fiat-Shamir checks.
    Only decoded data is shared with co-hosted VNs (envelope digests,
    unpacked proofs, transcript digests).  The per-CN proofs are verified in
    one batched launch sequence per kind (aggregation sums as device booleans
    read back together); range proofs are one batch each.
    ``range_pooled``: {base_key: None (not sampled) | bool} -- this VN's range
    results from the pooled verification (a dict or a Future of one).
    ``defer``: return a callable that waits for the pooled range results and
    returns the codes (everything else is already checked)."""
    codes = [None] * len(reqs)
    todo: dict = {}
    pooled_idx: list = []
    pre = cache.sig_pre.pop((sq.SurveyID, vn_id), None)
    with timers.span("verify.digests"):
        prefetch_digests(reqs)
    keys = [(sq.IDtoPublic.get(r.sender_id), r.digest(), r.signature) for r in reqs]
    if pre is not None and pre[0] == _inbox_tag(reqs):
        sigs_ok = pre[1]  # this VN's checks of exactly these envelopes, from the co-hosted batch
    else:
        with timers.span("verify.signature.batch"):
            sigs_ok = sigma.schnorr_verify_batch(keys, device) if reqs else []
    for i, req in enumerate(reqs):
        if not sigs_ok[i]:
            codes[i] = PROOF_FALSE_SIGN
        elif range_pooled is not None and req.kind == "range" and not req.header_only:
            pooled_idx.append(i)  # resolved below: the pooled batch may still be running
        elif not should_verify(sq, req, vn_index, n_vns, coins):
            codes[i] = PROOF_RECEIVED
        else:
            todo.setdefault(req.kind, []).append(i)
    range_future = None
    if "range" in todo and len(todo) > 1 and torch.device(device).type == "cuda":
        # the range lists (the heavy pairing work) verify on a worker thread with
        # their own HIP stream while this thread checks the short per-CN proofs
        idxs = todo.pop("range")
        range_future = _side_pool(device).submit(_verify_range_side, reqs, idxs, sq, vn_id, device, cache,
                                                 torch.cuda.current_stream(torch.device(device)), coins)
    _prefetch_packed(reqs, [i for k in PACKED_KINDS for i in todo.get(k, [])], device)
    pre = cache.ks_pre.pop((sq.SurveyID, vn_id), None)
    if pre is not None and "keyswitch" in todo and all(i in pre for i in todo["keyswitch"]):
        for i in todo.pop("keyswitch"):
            codes[i] = PROOF_TRUE if pre[i] else PROOF_FALSE
        timers.record(f"{vn_id}_{TIMER['keyswitch']}", pre.get("dt", 0.0))
    dev_flags = []  # (request index, device bool): read back with ONE copy
    for kind, idxs in todo.items():
        with timers.timed(f"{vn_id}_{TIMER[kind]}"):
            if kind == "range":
                for i, ok in verify_range_many(reqs, idxs, sq, device, cache, coins=coins).items():
                    codes[i] = PROOF_TRUE if ok else PROOF_FALSE
            elif kind == "aggregation":
                for i in idxs:
                    try:
                        dev_flags.append((i, ags.aggregation_check(_decode(reqs[i], device),
                                                                   sq.AggregationProofThreshold)))
                    except Exception as e:
                        log.warning(f"{vn_id}: aggregation proof from {reqs[i].sender_id} rejected: {e}")
                        codes[i] = PROOF_FALSE
            elif kind in ("keyswitch", "obfuscation"):
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
                    res = sigma.key_switch_batch_verification(objs, sq.KeySwitchingProofThreshold, coins=coins)
                else:
                    res = sigma.obfuscation_batch_verification(objs, sq.ObfuscationProofThreshold, coins=coins)
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
    # the device verdicts (aggregation sums) are read back when the codes are
    # resolved: co-hosted VNs then queue all their checks before the first
    # read, and pay one device round trip between them instead of one each
    flag_t = torch.stack([f.reshape(()) for _, f in dev_flags]) if dev_flags else None

    def read_flags():
        if flag_t is not None:
            with timers.span("verify.flags"):
                flags = flag_t.cpu().tolist()
            for (i, _), ok in zip(dev_flags, flags):
                codes[i] = PROOF_TRUE if ok else PROOF_FALSE
        if range_future is not None:
            for i, code in range_future.result():
                codes[i] = code

    if not defer:
        read_flags()

    def resolve():
        if defer:
            read_flags()
        if pooled_idx:
            with timers.span("rp.verify.pooled_wait"):
                pooled = range_pooled.result() if hasattr(range_pooled, "result") else range_pooled
                pooled = pooled.get(vn_id, {}) if vn_id in pooled else pooled
            for i in pooled_idx:
                res = pooled.get(reqs[i].base_key(), False)
                codes[i] = PROOF_RECEIVED if res is None else (PROOF_TRUE if res else PROOF_FALSE)
        return codes

    return resolve if defer else resolve()


_pools: dict = {}
_streams: dict = {}


def _side_pool(device):
    """The VN range side worker of ``device`` (pinned to it)."""
    from ..utils import streams

    key = str(torch.device(device))
    if key not in _pools:
        _pools[key] = streams.executor(device, 1, "drynx-vn-range")
    return _pools[key]


def _verify_range_side(reqs, idxs, sq, vn_id, device, cache, main, coins=None) -> list:
    dev = torch.device(device)
    side = _streams.get(str(dev))
    if side is None:
        side = _streams[str(dev)] = torch.cuda.Stream(dev)
    side.wait_stream(main)  # payloads / decoded lists are ready
    out = []
    with torch.cuda.stream(side), timers.timed(f"{vn_id}_{TIMER['range']}"):
        for i, ok in verify_range_many(reqs, idxs, sq, device, cache, coins=coins).items():
            out.append((i, PROOF_TRUE if ok else PROOF_FALSE))
    side.synchronize()
    return out


def verify_proof(req: ProofRequest, sq, vn_id: str, vn_index: int, n_vns: int, device, cache: VerifierCache,
                 coins=None) -> int:
    """<Kind>ProofRequest.VerifyProof -> bitmap code."""
    with timers.timed(f"{vn_id}_{TIMER[req.kind]}"):
        if not verify_signature(req, sq.IDtoPublic.get(req.sender_id)):
            return PROOF_FALSE_SIGN
        if not should_verify(sq, req, vn_index, n_vns, coins):
            return PROOF_RECEIVED
        try:
            ok = verify_content(req, sq, device, cache)
        except Exception as e:  # malformed proof bytes => false, never a crash of the VN
            log.warning(f"{vn_id}: {req.kind} proof from {req.sender_id} rejected: {e}")
            ok = False
        return PROOF_TRUE if ok else PROOF_FALSE
