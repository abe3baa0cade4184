"""ProofCollection: every proof request reaches the verifying nodes, which
verify (sampled), persist, fill their bitmaps and append a ledger block.

Reference: protocols/proof_collection_protocol.go — star tree prover root +
all VNs (:84-305): each VN verifies, stores the proof in bbolt
(``storeProof`` :307-406; bucket surveyID/type, key
surveyID/type/sender/differInfo/VN; shuffle proofs are not stored), updates
the bitmap, decrements the expected count; when done it persists its bitmap
(bucket <VN>, key surveyID/map) and forwards it to the root VN, which builds
the DataBlock and appends the skipchain (services/service_skipchain.go:96-158).

MI355X mapping: the per-proof star broadcasts collapse into one personalised
exchange of all requests to the ranks hosting VNs (xGMI all-to-all); each VN
verifies every request it is assigned as one device batch; bitmaps and the
block travel on the control plane.
"""
from __future__ import annotations

import json
import os
import time

import torch

from ..ledger import skipchain as skc
from ..parallel.comm import bytes_to_obj, obj_to_bytes
from ..proofs import requests as prq
from ..query import query_to_proofs_nbrs
from ..utils import timers
from ..utils.log import get_logger

log = get_logger("proof_collection")


def expected_counts(sq) -> dict:
    """QueryToProofsNbrs reordered to the VN order (service_skipchain.go:57-63)."""
    q = query_to_proofs_nbrs(sq)
    return dict(zip(prq.QUERY_ORDER, q))


def use_pool(ctx) -> bool:
    """Pooled range verification: every rank checks a 1/world slice of every
    range-proof list on behalf of every VN (so three VNs keep eight GPUs busy;
    on one GPU the co-hosted VNs' batches share the decode and run back to
    back); the VN's own rank keeps the signature checks, the sampling
    decision, the bitmap and the ledger.  ``DRYNX_VN_POOL=0`` leaves each VN's
    range checks to the VN's own rank, one VN at a time."""
    return os.environ.get("DRYNX_VN_POOL", "1") != "0"


def fan_out(ctx, sq, local_requests: list, all_ranks: bool = False) -> list:
    """All requests, on every rank that hosts a VN (others get nothing), or on
    every rank (``all_ranks``: pooled verification)."""
    vns = [ctx.cluster.by_id(si.id) for si in sq.Query.RosterVNs.list]
    vn_ranks = list(range(ctx.comm.world)) if all_ranks else sorted({v.rank for v in vns})
    if ctx.comm.world == 1:
        return list(local_requests)
    # sharded verification: ship the payload only to ranks hosting an assigned
    # VN; the others get the signed header (signature + digest) and record 2
    # range-proof payloads (tens of MB per DP) go as raw limb tensors over RCCL;
    # envelopes and small proofs as pickled control messages
    per_rank = {d: [] for d in vn_ranks}
    per_rank_t = {d: [] for d in vn_ranks}
    packed = {}
    for idx, r in enumerate(local_requests):
        assigned = prq.assigned_vns(sq, r, len(vns))
        full_ranks = vn_ranks if (assigned is None or all_ranks) else {vns[i].rank for i in assigned}
        for d in vn_ranks:
            if d not in full_ranks:
                per_rank[d].append(r.header().to_wire())
            elif r.kind == "range" and r.obj is not None and d != ctx.rank:
                if idx not in packed:
                    packed[idx] = (r.tensor if r.tensor is not None else prq.range_bundle_pack(r.obj)).to(ctx.device)
                w = r.header().to_wire()
                w["digest"], w["tensor"] = b"", packed[idx].numel()
                per_rank[d].append(w)
                per_rank_t[d].append(packed[idx])
            else:
                per_rank[d].append(r.to_wire())
    got = ctx.comm.exchange_bytes({d: obj_to_bytes(per_rank[d]) for d in vn_ranks})
    wires = {src: bytes_to_obj(b) for src, b in got.items()}
    tens = {d: torch.cat(per_rank_t[d]) for d in vn_ranks if per_rank_t[d]}
    # the envelopes announced every tensor's size: no size round for the payloads
    sizes = {src: sum(w.get("tensor") or 0 for w in ws) for src, ws in wires.items() if src != ctx.rank}
    got_t = ctx.comm.exchange(tens, recv_sizes={s_: n_ for s_, n_ in sizes.items() if n_})
    out = []
    for src in sorted(got):
        if src == ctx.rank:
            out += list(local_requests)  # keep decoded objects for locally produced proofs
            continue
        off = 0
        for w in wires[src]:
            req = prq.ProofRequest.from_wire(w)
            n = w.get("tensor")
            if n:
                t = got_t[src][off: off + n]
                off += n
                req.set_tensor(t)  # signed bytes: the VN re-hashes and decodes them on its device
            out.append(req)
    return out


def pool_verify_ranges(ctx, sq, reqs: list, vns: list) -> dict:
    """Pooled range verification (see ``use_pool``).  Sampling is decided by
    each VN's own rank (reference ``rand.Float64() <= Threshold``, or the
    sharding extension) and shared; rank k then checks slice k/W of the
    sampled prefix of every list, one batch per VN with that VN's own random
    weights; the slice verdicts are all-gathered and AND-ed.
    -> {vn_id: {base_key: None (not sampled) | bool}} on every rank."""
    W, k = ctx.comm.world, ctx.comm.rank
    rng = [i for i, r in enumerate(reqs) if r.kind == "range" and not r.header_only]
    local = {}
    for vi, vn in enumerate(vns):
        if vn.rank == ctx.rank:
            local[vn.id] = {reqs[i].base_key(): prq.should_verify(sq, reqs[i], vi, len(vns)) for i in rng}
    sampled = {}
    for d in ctx.comm.all_gather_object(local):
        sampled.update(d)
    vn_idxs = {vn.id: [i for i in rng if sampled[vn.id].get(reqs[i].base_key())] for vn in vns}
    t0 = time.perf_counter()
    res = prq.verify_range_many_multi(reqs, vn_idxs, sq, ctx.device, ctx.verifier_cache, part=(k, W))
    dt = time.perf_counter() - t0
    mine = {}
    for vn in vns:
        timers.record(f"{vn.id}_VerifyRange", dt)  # one shared pass for the co-hosted VNs
        mine[vn.id] = {reqs[i].base_key(): bool(ok) for i, ok in res.get(vn.id, {}).items()}
    verdicts = ctx.comm.all_gather_object(mine)
    out = {}
    for vn in vns:
        out[vn.id] = {key: (None if not smp else all(v[vn.id].get(key, False) for v in verdicts))
                      for key, smp in sampled[vn.id].items()}
    return out


def _pool_async(ctx, sq, reqs, vns):
    """pool_verify_ranges on a worker thread with its own HIP stream: the
    range batches (the GPU's long pole) run while this thread checks the
    short per-CN proofs of each VN.  On a multi-rank node the worker also
    owns the pool's collectives (the main thread issues none meanwhile)."""
    import concurrent.futures as cf

    if not hasattr(ctx, "_pool_exec"):
        ctx._pool_exec = cf.ThreadPoolExecutor(max_workers=1, thread_name_prefix="drynx-vn-pool")
    if ctx.device.type != "cuda":
        return ctx._pool_exec.submit(pool_verify_ranges, ctx, sq, reqs, vns)
    if not hasattr(ctx, "_pool_stream"):
        # DRYNX_POOL_RESERVE_CUS=k: the pool's heavy kernels (long-running
        # workgroups) leave k CUs to the short plan / per-CN-proof launches
        from .. import native as nt

        k = int(os.environ.get("DRYNX_POOL_RESERVE_CUS", "0"))
        ctx._pool_stream = nt.cu_masked_stream(ctx.device, k) if k > 0 else torch.cuda.Stream(ctx.device)
    side, main = ctx._pool_stream, torch.cuda.current_stream(ctx.device)
    side.wait_stream(main)

    def run():
        with torch.cuda.stream(side):
            out = pool_verify_ranges(ctx, sq, reqs, vns)
        side.synchronize()
        return out

    return ctx._pool_exec.submit(run)


def verify_and_store(ctx, sq, vn, vn_index: int, n_vns: int, requests: list, range_pooled=None) -> dict:
    return store_verdicts(ctx, sq, vn, requests, check_requests(ctx, sq, vn, vn_index, n_vns, requests, range_pooled))


def check_requests(ctx, sq, vn, vn_index: int, n_vns: int, requests: list, range_pooled=None):
    """VerifyProof over one VN's inbox; with pooled range checks the range
    codes are left pending (``codes`` holds a resolver) so the VN's short
    per-CN checks run while the pooled batch is still on the GPU."""
    return prq.verify_requests(requests, sq, vn.id, vn_index, n_vns, ctx.device, ctx.verifier_cache, range_pooled,
                               defer=True)


def store_verdicts(ctx, sq, vn, requests: list, pending) -> dict:
    """storeProof for every request of the inbox: bitmap entry, ledger write
    (surveyID/type bucket, shuffle proofs not stored), expected-count check
    and the VN's bitmap (proof_collection_protocol.go:307-406)."""
    codes = pending() if callable(pending) else pending
    store = ctx.store(vn.id)
    bitmap = {}
    counts = {k: 0 for k in prq.VN_ORDER}
    stored = [req for req in requests if req.kind != "shuffle"]  # storeProof skips shuffle proofs (:318-331)
    values = dict(zip(map(id, stored), ctx.ledger_values(stored)))
    for req, code in zip(requests, codes):
        key = req.key(vn.id)
        bitmap[key] = code
        counts[req.kind] += 1
        if req.kind != "shuffle":
            store.update_async(f"{sq.SurveyID}/{req.kind}", key, values[id(req)])
    exp = expected_counts(sq)
    for k in prq.VN_ORDER:
        if counts[k] != exp[k]:
            log.warning(f"{vn.id}: received {counts[k]} {k} proofs, expected {exp[k]}")
    store.update_async(vn.id, f"{sq.SurveyID}/map", json.dumps(bitmap, sort_keys=True).encode())
    ctx.local_bitmaps[(sq.SurveyID, vn.id)] = bitmap
    return bitmap


def proof_collection(ctx, sq, local_requests: list):
    """Returns the new SkipBlock (on every rank)."""
    vns = [ctx.cluster.by_id(si.id) for si in sq.Query.RosterVNs.list]
    pool = use_pool(ctx)
    with timers.timed("ProofFanOut"):
        reqs = fan_out(ctx, sq, local_requests, all_ranks=pool)
    bitmaps = {}
    with timers.timed("ProofVerification"):
        pooled = _pool_async(ctx, sq, reqs, vns) if pool else None
        local_vns = [vn.id for vn in vns if vn.rank == ctx.rank]
        if len(local_vns) > 1:  # co-hosted VNs: one grouped key-switch MSM for all of them
            with timers.span("verify.keyswitch.multi"):
                prq.prewarm_keyswitch(reqs, sq, local_vns, ctx.device, ctx.verifier_cache)
        pending = {vn.id: check_requests(ctx, sq, vn, idx, len(vns), reqs, pooled)
                   for idx, vn in enumerate(vns) if vn.rank == ctx.rank}
        for vn in vns:
            if vn.id in pending:
                bitmaps[vn.id] = store_verdicts(ctx, sq, vn, reqs, pending[vn.id])
        if pooled is not None:
            pooled.result()
    # bitmaps -> root VN (SharedBMChannel)
    allbm = {}
    for d in ctx.comm.all_gather_object(bitmaps):
        allbm.update(d)
    root = vns[0]
    block = None
    t = timers.start_timer("BI", sync=False)
    if ctx.rank == root.rank:
        merged = {}
        for vn in vns:
            merged.update(allbm.get(vn.id, {}))
        data = skc.new_data_block(sq.SurveyID, merged, [v.identity() for v in vns])
        if ctx.last_block is None:
            # resume an existing chain from the root VN's ledger (restart of a
            # node over a persisted workdir) instead of starting a new genesis
            ctx.last_block = ctx.get_latest_block(root.id)
        block = skc.make_block(ctx.last_block, data, [v.identity() for v in vns])
    block_bytes = ctx.comm.broadcast_object(block.to_bytes() if block is not None else None, src=root.rank)
    block = skc.SkipBlock.from_bytes(block_bytes)
    # every VN runs its verifiers (verifyFuncBitmap, VerifyBase against its own
    # latest block), then signs the block and the forward link from its latest
    signers = []
    for vn in vns:
        if vn.rank == ctx.rank:
            prev = ctx.vn_latest(vn.id)
            if skc.verify_bitmap(block, ctx.local_bitmaps.get((sq.SurveyID, vn.id), {}), vn.id) \
                    and skc.verify_base(prev, block):
                signers.append((vn.id, vn.keypair.secret, prev))
            else:
                log.warning(f"{vn.id} refused block for survey {sq.SurveyID}")
    sigs, links = skc.cosign_many(block, signers)  # the co-hosted VNs' partials in one batch
    for d, fl in ctx.comm.all_gather_object((sigs, links)):
        block.ForwardSignatures.update(d)
        links.update(fl)
    skc.finalize_cosig(block)  # BLS collective signature of the VN roster
    for vn in vns:
        if vn.rank == ctx.rank:
            # proof blobs keep persisting on the store's writer thread (GetProofs /
            # CloseDB flush); the block only depends on the bitmap
            st = ctx.store(vn.id)
            prev = ctx.vn_latest(vn.id)
            if prev is not None and links:
                skc.add_forward_link(prev, block.Hash, links)   # stored with the previous block
                st.update_async("skipchain", prev.Hash, prev.to_bytes())
            ctx.set_vn_latest(vn.id, block)
            raw = block.to_bytes()
            st.update_async("skipchain", block.Hash, raw)
            st.update_async("skipchain", "latest", raw)
            if block.Index == 0:
                st.update_async("genesis", "genesis", raw)
            st.update_async("mapping", sq.SurveyID, block.Hash.encode())
    ctx.last_block = block
    timers.end_timer(t)
    ctx.end_verification(sq.SurveyID, block)  # EndVerificationChannel <- block (service_skipchain.go:158)
    return block
