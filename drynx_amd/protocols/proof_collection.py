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

from .. import native as nt
from ..ledger import skipchain as skc
from ..parallel.netem import CT_BYTES, POINT_BYTES, SCALAR_BYTES, SIG_BYTES, flow_hops, range_proof_bytes
from .data_collection import all_possible_groups as dcp_groups
from ..parallel.comm import bytes_to_obj, obj_to_bytes
from ..crypto.coins import Coins
from ..proofs import requests as prq
from ..query import query_to_proofs_nbrs
from ..utils import streams, timers
from ..utils.log import get_logger

log = get_logger("proof_collection")


def expected_counts(sq) -> dict:
    """QueryToProofsNbrs reordered to the VN order (service_skipchain.go:57-63)."""
    q = query_to_proofs_nbrs(sq)
    return dict(zip(prq.QUERY_ORDER, q))


def _net_proofs(ctx, sq, reqs: list, vns: list):
    """Every proof envelope from its prover to every VN (one hop, the
    reference wire sizes of SURVEY 2.4)."""
    n_groups = len(dcp_groups(sq.Query.DPDataGen.GroupByValues))
    n_rows = n_groups * sq.Query.Operation.NbrOutput
    S = len(sq.RosterServers.list)
    sizes = {}
    for r in reqs:
        if r.kind == "range":
            rg = sq.Query.Ranges or []
            nb = sum(range_proof_bytes(int(x[0]), int(x[1]), S) for x in rg) * n_groups
        elif r.kind == "aggregation":
            nb = (len((sq.ServerToDP or {}).get(r.sender_id) or []) + 1) * n_rows * CT_BYTES
        elif r.kind == "keyswitch":
            nb = n_rows * (POINT_BYTES + CT_BYTES + 2 * POINT_BYTES + SCALAR_BYTES) + 4 * POINT_BYTES
        elif r.kind == "obfuscation":
            nb = n_rows * (3 * CT_BYTES + SCALAR_BYTES)
        else:
            nb = int(sq.Query.DiffP.NoiseListSize) * 3 * CT_BYTES
        sizes[r.base_key()] = (r.sender_id, nb + SIG_BYTES)
    ctx.net.step("proofs_to_vns", [(src, v.id, nb) for src, nb in sizes.values() for v in vns],
                 hops=flow_hops("proofs_to_vns"))


def verification_mode(ctx) -> str:
    """Who checks a VN's range proofs (``ctx.pool_policy``, else DRYNX_VN_POOL):

    * ``pool`` ("1", default; single-operator deployments): every rank checks
      a slice of every range list on behalf of EVERY VN, with that VN's coins
      (a per-survey seed the VN hands out), so three VNs keep eight GPUs busy;
      the VN's own rank keeps the signature checks, the sampling decisions,
      the bitmap and the ledger, and accepts a helper's slice verdict only if
      the helper's digest of the slice it checked equals the VN's own digest
      of that slice of its signed payload.
    * ``local`` ("vn-local"): the same, but each VN's lists are spread only
      over the ranks assigned to THAT VN (its own rank plus helper ranks no
      other VN uses): no VN's verdict depends on another VN's ranks or
      helpers, and a helper learns only its own VN's seed.
    * ``own`` ("0"; forced by multi-party servers, services/server.py): each
      VN checks its whole inbox on its own rank (the reference: every VN
      verifies what it received, lib/proof/structs_proofs.go:135-182).

    Every mode runs as the range plane beside the CN phases; on one GPU the
    co-hosted VNs' batches share the decode and run back to back."""
    pol = getattr(ctx, "pool_policy", None)
    if pol is None:
        pol = os.environ.get("DRYNX_VN_POOL", "1")
    return {"0": "own", "own": "own", "local": "local", "vn-local": "local"}.get(str(pol), "pool")


def trust_model(ctx) -> str:
    """What a VN's range verdict depends on, as run: ``single-operator-pool``
    (helper ranks that serve every VN) or ``vn-local`` (only ranks assigned
    to that VN; at one rank, or with ``own``, its own rank)."""
    return "single-operator-pool" if verification_mode(ctx) == "pool" and ctx.comm.world > 1 else "vn-local"


def _placement(ctx, sq) -> tuple:
    """(DPs per rank, VNs per rank, VN ranks in roster order) of a survey."""
    W = ctx.comm.world
    dps, vns = [0] * W, [0] * W
    for _, members in (sq.ServerToDP or {}).items():
        for si in members or []:
            dps[ctx.cluster.by_id(si.id).rank] += 1
    vn_ranks = [ctx.cluster.by_id(si.id).rank for si in sq.Query.RosterVNs.list]
    for r in vn_ranks:
        vns[r] += 1
    return dps, vns, vn_ranks


def verification_groups(mode: str, W: int, dps: list, vns: list, vn_ranks: list) -> tuple:
    """-> (groups, parts): ``groups[v]`` the ranks that check VN v's range
    lists (v's own rank first), ``parts[v][rank]`` that rank's slice of each
    list (``prq.sampled_bounds`` part: weighted by ``prq.balanced_parts``
    rules, a rank hosting more DPs or a VN checks a shorter slice).  A
    function of the placement only: identical on every rank.  ``local``:
    every rank hosting no VN serves one VN, the one whose group has the least
    capacity so far (its ranks' weights; a rank hosting k VNs counts 1/k)."""
    n = len(vn_ranks)
    if W <= 1 or mode == "own":
        return [[r] for r in vn_ranks], [{r: (0, 1)} for r in vn_ranks]
    if mode == "pool":
        bp = prq.balanced_parts(W, dps, vns)
        return [list(range(W)) for _ in range(n)], [{k: bp[k] for k in range(W)} for _ in range(n)]
    w = prq.rank_weights(dps, vns)
    groups = [[r] for r in vn_ranks]
    cap = [w[r] / max(1, vns[r]) for r in vn_ranks]
    for h in (k for k in range(W) if vns[k] == 0):
        v = min(range(n), key=lambda i: (cap[i], i))
        groups[v].append(h)
        cap[v] += w[h]
    parts = []
    for g in groups:
        iw = [max(1, int(round(1000 * w[k]))) for k in g]
        cum = [0]
        for x in iw:
            cum.append(cum[-1] + x)
        parts.append({k: (i, len(g), *cum) if len(g) > 1 else (0, 1) for i, k in enumerate(g)})
    return groups, parts


def groups_of(ctx, sq) -> tuple:
    """``verification_groups`` of this node's mode for a survey -> (groups, parts)
    as dicts keyed by VN id."""
    dps, vns, vn_ranks = _placement(ctx, sq)
    groups, parts = verification_groups(verification_mode(ctx), ctx.comm.world, dps, vns, vn_ranks)
    ids = [si.id for si in sq.Query.RosterVNs.list]
    return dict(zip(ids, groups)), dict(zip(ids, parts))


def fan_out(ctx, sq, local_requests: list, pool: bool = False, stage: int = 0) -> list:
    """Every request to the ranks that host a VN; with ``pool`` (the range
    plane: ``verification_groups``), a helper rank gets only ITS slice of
    every range bundle its VN(s) may check (~1/group of the payload) plus the
    envelope header, and each local VN's per-survey seed goes to exactly the
    ranks of that VN's group.  Payload tensors (range bundles, packed per-CN
    proofs) travel as raw limbs in one all-to-all with sizes announced by the
    control message (no size round); envelopes and byte payloads ride on the
    control message."""
    vns = [ctx.cluster.by_id(si.id) for si in sq.Query.RosterVNs.list]
    W = ctx.comm.world
    vn_ranks = sorted({v.rank for v in vns})
    mode = verification_mode(ctx)
    groups, gparts = groups_of(ctx, sq) if pool else ({}, {})
    helpers: dict = {}  # helper rank (hosting no VN) -> (its slice part, indices of the VNs it serves)
    for vi, v in enumerate(vns):
        for k in groups.get(v.id, ()):
            if k not in vn_ranks:
                helpers.setdefault(k, (gparts[v.id][k], []))[1].append(vi)
    dests = sorted(set(vn_ranks) | set(helpers))
    seeds = {}
    if pool:
        # each local VN's per-survey seed for its group's helpers rides on this
        # exchange (no control round of its own): helper k derives that VN's
        # coins for its slice from it
        seeds = {vn.id: ctx.vn_coins(vn.id).seed() for vn in vns if vn.rank == ctx.rank}
        ctx.__dict__.setdefault("_pool_seeds", {})[(sq.SurveyID, stage)] = dict(seeds)
        if len(ctx._pool_seeds) > 64:
            ctx._pool_seeds.pop(next(iter(ctx._pool_seeds)))
    if W == 1:
        return list(local_requests)
    per_rank = {d: [] for d in dests}
    per_rank_t = {d: [] for d in dests}
    packed = {}
    for idx, r in enumerate(local_requests):
        assigned = prq.assigned_vns(sq, r, len(vns))
        # in the pool every VN rank checks a slice for every VN: all get the payload
        full_ranks = set(vn_ranks) if (assigned is None or (pool and mode == "pool")) \
            else {vns[i].rank for i in assigned}
        for d in dests:
            if d == ctx.rank:
                continue
            if d not in full_ranks:
                serves = helpers.get(d)
                if (serves is not None and r.kind == "range" and r.obj is not None
                        and (assigned is None or any(vi in assigned for vi in serves[1]))):
                    # a helper: its slice of the bundle (its part of its group)
                    sl = _helper_slice(r.obj, sq, serves[0])
                    w = r.header().to_wire()
                    if sl:
                        t = prq.range_bundle_pack(sl).to(ctx.device)
                        w["tensor"], w["slice"] = t.numel(), list(serves[0])
                        per_rank_t[d].append(t)
                    per_rank[d].append(w)
                else:
                    per_rank[d].append(r.header().to_wire())
            elif r.tensor is not None and r._data is None:
                if idx not in packed:
                    packed[idx] = r.tensor.to(ctx.device)
                w = r.header().to_wire()
                w["digest"], w["tensor"] = b"", packed[idx].numel()
                per_rank[d].append(w)
                per_rank_t[d].append(packed[idx])
            else:
                per_rank[d].append(r.to_wire())
    # a VN's seed only to the ranks of its group (a vn-local helper never
    # learns another VN's coins)
    got = ctx.comm.exchange_bytes({d: obj_to_bytes({"w": per_rank[d],
                                                    "seeds": {v: s for v, s in seeds.items() if d in groups[v]}})
                                   for d in dests if d != ctx.rank})
    msgs = {src: bytes_to_obj(b) for src, b in got.items()}
    wires = {src: m["w"] for src, m in msgs.items()}
    if pool:
        for m in msgs.values():
            ctx._pool_seeds[(sq.SurveyID, stage)].update(m["seeds"])
    tens = {d: t for d, t in zip([d for d in dests if per_rank_t[d]],
                                  nt.cat_rows([per_rank_t[d] for d in dests if per_rank_t[d]]))}
    # the envelopes announced every tensor's size: no size round for the payloads
    sizes = {src: sum(w.get("tensor") or 0 for w in ws) for src, ws in wires.items()}
    got_t = ctx.comm.exchange(tens, recv_sizes={s_: n_ for s_, n_ in sizes.items() if n_})
    out = []
    for src in sorted(set(wires) | {ctx.rank}):
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
                if w.get("slice"):
                    # helper copy: the payload is this slice; the digest stays the signed one
                    req._data, req.tensor, req.slice_of = None, t, tuple(w["slice"])
                else:
                    req.set_tensor(t)  # signed bytes: the VN re-hashes and decodes them on its device
            out.append(req)
    return out


def _helper_slice(lists, sq, part) -> list:
    """What the prover sends pool helper ``part[0]`` (tests substitute an
    equivocating prover here)."""
    return prq.slice_lists(lists, sq, part)


def _pkey(part) -> str:
    return ",".join(str(int(x)) for x in part)


def pool_verify_ranges(ctx, sq, reqs: list, vns: list, comm=None, arrived: float | None = None, stage: int = 0,
                       record: bool = True, second=None) -> dict:
    """Range verification through the verification groups (see
    ``verification_mode``).  Each VN's rank decides that VN's sampling
    (reference ``rand.Float64() <= Threshold``, from the VN's own coins, or
    the sharding extension) and draws a per-survey seed; every rank of VN v's
    group checks its slice of the sampled prefix of every list with coins
    derived from v's seed and reports its verdicts with the digest of each
    slice it checked.  v's rank then accepts a helper's slice verdict only
    when the digest matches its own digest of that slice of the signed
    payload, and re-checks any other slice itself.  Groups of one (``own``)
    need no gather.  ``<vn>_VerifyRange`` (structs_proofs.go:137) runs from
    ``arrived`` (the VN's inbox: the range fan-out's end on its rank) to that
    VN's own verdict (after its digest checks and any slice it re-checked).
    ``second``: a Future of the staged plane's second batch's local part
    (``_pool_local`` on another worker): both batches' results travel in ONE
    gather and the verdicts cover both.
    -> {vn_id: {base_key: None (not sampled) | bool}} for the VNs of this rank."""
    comm = comm or ctx.comm
    t0 = arrived if arrived is not None else time.perf_counter()
    states = [_pool_local(ctx, sq, reqs, vns, comm.rank, comm.world, stage)]
    if second is not None:
        with timers.span("rp.verify.pool_second"):
            states.append(second.result(timeout=float(os.environ.get("DRYNX_STAGE_WAIT_S", "120"))))
    return _pool_finish(ctx, sq, states, comm, t0, record)


def _pool_local(ctx, sq, reqs: list, vns: list, k: int, W: int, stage: int) -> dict:
    """This rank's share of one batch of a pooled verification: its slices
    checked for the VNs whose group holds it, their digests, and (a VN's
    rank) its sampling and the digests of its helpers' slices (queued)."""
    rng = [i for i, r in enumerate(reqs) if r.kind == "range" and not r.header_only]
    groups, gparts = groups_of(ctx, sq)
    # every VN's seed arrived with the fan-out; the helpers check every list a
    # VN may sample (the sharding extension's assignment is public; a random
    # Threshold sample stays the VN's own decision, applied to the verdicts
    # below) -- no control round before the checks
    seeds = getattr(ctx, "_pool_seeds", {}).pop((sq.SurveyID, stage), {})
    serve = [vn for vn in vns if k in groups[vn.id]]  # the VNs this rank checks a slice for
    missing = [vn.id for vn in serve if vn.id not in seeds]
    if missing:
        raise RuntimeError(f"pool: no fan-out seed for {missing} (survey {sq.SurveyID})")

    def may_check(i, vi):
        a_ = prq.assigned_vns(sq, reqs[i], len(vns))
        return a_ is None or vi in a_
    vn_idxs = {vn.id: [i for i in rng if may_check(i, vi)] for vi, vn in enumerate(vns)}
    sampled = {vn.id: {reqs[i].base_key(): prq.should_verify(sq, reqs[i], vi, len(vns), ctx.vn_coins(vn.id))
                       for i in rng} for vi, vn in enumerate(vns) if vn.rank == ctx.rank}
    local_vns = [vn for vn in vns if vn.rank == ctx.rank]
    helped = [vn for vn in local_vns if len(groups[vn.id]) > 1]
    # a VN rank's digests of its helpers' slices of its own payloads run beside
    # this rank's part (their own thread and stream: the part's latency-bound
    # kernels leave the GPU room), not after the gather
    exp_f = _expected_async(ctx, sq, reqs, vn_idxs, helped, groups, gparts) if helped else None
    # this rank's parts: the VNs it serves grouped by the slice it checks for them
    by_part: dict = {}
    for vn in serve:
        by_part.setdefault(tuple(gparts[vn.id][k]), []).append(vn)
    mine, mydig, futs = {}, {}, []
    for part, pvns in by_part.items():
        coins = {vn.id: Coins(seeds[vn.id]).derive(("slice", k, W)) for vn in pvns}
        res, digests = prq.verify_range_pool_part(reqs, {vn.id: vn_idxs[vn.id] for vn in pvns}, sq, ctx.device,
                                                  ctx.verifier_cache, part, coins, async_digests=True)
        for vn in pvns:
            mine[vn.id] = {reqs[i].base_key(): bool(ok) for i, ok in res.get(vn.id, {}).items()}
        futs.append((part, digests))
    for part, digests in futs:
        if hasattr(digests, "result"):
            digests = digests.result()
        mydig[_pkey(part)] = {reqs[i].base_key(): d for i, d in digests.items()}
    return {"reqs": reqs, "vn_idxs": vn_idxs, "sampled": sampled, "helped": helped, "exp_f": exp_f,
            "mine": mine, "mydig": mydig, "groups": groups, "gparts": gparts, "local_vns": local_vns}


def _pool_finish(ctx, sq, states: list, comm, t0: float, record: bool) -> dict:
    """One gather of every batch's (verdicts, slice digests), then each local
    VN's verdicts: helper verdicts bound to its own digests of their slices,
    mismatching slices re-checked, unsampled lists left None."""
    k = comm.rank
    groups = states[0]["groups"]
    payload = [(s["mine"], s["mydig"]) for s in states]
    if any(len(g) > 1 for g in groups.values()):
        gathered = comm.all_gather_object(payload)
    else:  # every VN checks alone on its own rank: nothing to gather
        gathered = {k: payload}
    out: dict = {}
    for si, st in enumerate(states):
        reqs, vn_idxs, sampled, gparts = st["reqs"], st["vn_idxs"], st["sampled"], st["gparts"]
        got = {j: gathered[j][si] for j in (gathered if isinstance(gathered, dict) else range(len(gathered)))}
        trusted = {}
        if st["helped"]:
            trusted = _check_helper_digests(ctx, sq, reqs, vn_idxs, st["helped"], got, groups, gparts,
                                            st["exp_f"].result())
        for vn in st["local_vns"]:
            g = groups[vn.id]
            tr = trusted[vn.id] if len(g) > 1 else {}
            verdict = {}
            for key, smp in sampled[vn.id].items():
                if not smp:
                    verdict[key] = None
                    continue
                verdict[key] = all(got[j][0][vn.id].get(key, False) for j in g if j == k or (key, j) in tr)
            # slices whose helper digest did not match: this VN checks them itself
            # (only lists this VN sampled: an unsampled one keeps None = code 2,
            # whatever a helper reported for it)
            redo = {j: [i for i in idxs if sampled[vn.id].get(reqs[i].base_key())]
                    for j, idxs in tr.get("redo", {}).items()}
            redo = {j: idxs for j, idxs in redo.items() if idxs}
            if redo:
                with timers.span("rp.verify.pool_redo"):
                    c = ctx.vn_coins(vn.id)
                    for j, idxs in redo.items():
                        r2, _ = prq.verify_range_pool_part(reqs, {vn.id: idxs}, sq, ctx.device, ctx.verifier_cache,
                                                           gparts[vn.id][j], {vn.id: c})
                        for i, ok in r2[vn.id].items():
                            key = reqs[i].base_key()
                            verdict[key] = bool(verdict.get(key)) and bool(ok)
            out.setdefault(vn.id, {}).update(verdict)
    if record:
        for vn in states[0]["local_vns"]:
            timers.record(f"{vn.id}_VerifyRange", time.perf_counter() - t0)
    return out


def _expected_async(ctx, sq, reqs, vn_idxs: dict, local_vns: list, groups: dict, gparts: dict):
    """``_expected_digests`` as an idle task of this rank's pool part (run
    while its verifier waits for the device, on a HIP stream of its own
    ordered after the caller's, where the payloads were received): no second
    thread contending for the GIL with the part's host work."""
    from ..proofs import range_proof as rp

    def work():
        return _expected_digests(ctx, sq, reqs, vn_idxs, local_vns, groups, gparts)
    if ctx.device.type != "cuda":
        return rp.add_idle_task(rp.Deferred(work))
    # one digest stream per pool thread (a staged range plane runs two)
    dstreams = ctx.__dict__.setdefault("_dig_streams", {})
    tid = __import__("threading").get_ident()
    if tid not in dstreams:
        dstreams[tid] = torch.cuda.Stream(ctx.device)
    st, cur = dstreams[tid], torch.cuda.current_stream(ctx.device)
    st.wait_stream(cur)

    def run():
        with torch.cuda.stream(st):
            return work()
    return rp.add_idle_task(rp.Deferred(run))


def _expected_digests(ctx, sq, reqs, vn_idxs: dict, local_vns: list, groups: dict, gparts: dict):
    """Digests of the local VNs' helpers' slices of their signed payloads ->
    ({(request, rank): digest}, {(request, rank) with an empty slice})."""
    me = ctx.rank
    want: dict = {}  # (request, rank) -> part
    for vn in local_vns:
        for i in vn_idxs[vn.id]:
            for j in groups[vn.id]:
                if j != me:
                    want.setdefault((i, j), gparts[vn.id][j])
    expected: dict = {}
    empty: set = set()  # (request, rank) whose slice is empty: nothing to check there
    with timers.span("rp.verify.expected_digests"):
        entries, keys = [], []
        for (i, j), part in sorted(want.items()):
            try:
                lists = prq._range_lists(reqs[i], ctx.device)
            except Exception:  # noqa: BLE001 -- undecodable: every slice is redone (and fails)
                continue
            sl = prq.slice_lists(lists, sq, part)
            if not sl:
                empty.add((i, j))
                continue
            entries.append(sl)
            keys.append((i, j))
        for key, d in zip(keys, prq.lists_digests(entries)):
            expected[key] = d
    return expected, empty


def _check_helper_digests(ctx, sq, reqs, vn_idxs: dict, local_vns: list, gathered, groups: dict, gparts: dict,
                          pre) -> dict:
    """For each local VN: the (base_key, rank) pairs whose helper-reported
    slice digest equals the digest of that slice of the VN's own signed
    payload, and the mismatches to redo ({rank: [request index]}).  A helper
    whose slice of a list is empty (a list shorter than the group) has no
    verdict on it and is in neither.  ``pre``: the (expected, empty) of
    ``_expected_digests``."""
    me = ctx.rank
    expected, empty = pre
    out = {}
    for vn in local_vns:
        ok_pairs, redo = set(), {}
        for i in vn_idxs[vn.id]:
            bk = reqs[i].base_key()
            for j in groups[vn.id]:
                if j == me:
                    continue
                got = gathered[j][1].get(_pkey(gparts[vn.id][j]), {}).get(bk)
                if (i, j) in empty:
                    continue
                if expected.get((i, j)) is not None and got == expected[(i, j)]:
                    ok_pairs.add((bk, j))
                else:
                    redo.setdefault(j, []).append(i)
        ok_pairs_d = {p_: True for p_ in ok_pairs}
        ok_pairs_d["redo"] = redo
        out[vn.id] = ok_pairs_d
    return out


def _pool_async(ctx, sq, reqs, vns, comm=None, second=None):
    """pool_verify_ranges on a worker thread with its own HIP stream: the
    range batches (the GPU's long pole) run while this thread checks the
    short per-CN proofs of each VN.  On a multi-rank node the worker also
    owns the pool's collectives (the main thread issues none meanwhile).
    ``second``: see ``pool_verify_ranges`` (a staged range plane)."""
    if not hasattr(ctx, "_pool_exec"):
        ctx._pool_exec = streams.executor(ctx.device, 1, "drynx-vn-pool")
    arrived = time.perf_counter()  # the fan-out just delivered the VNs' inboxes
    if ctx.device.type != "cuda":
        return ctx._pool_exec.submit(pool_verify_ranges, ctx, sq, reqs, vns, comm, arrived, 0, True, second)
    if not hasattr(ctx, "_pool_stream"):
        ctx._pool_stream = torch.cuda.Stream(ctx.device, priority=streams.priority(POOL_PRIORITY))
    side, main = ctx._pool_stream, torch.cuda.current_stream(ctx.device)
    side.wait_stream(main)

    def run():
        with torch.cuda.stream(side):
            out = pool_verify_ranges(ctx, sq, reqs, vns, comm, arrived, 0, True, second)
        side.synchronize()
        return out

    return ctx._pool_exec.submit(run)


def _pool_local_async(ctx, sq, reqs, vns, stage: int):
    """``_pool_local`` of a staged plane's later batch on a second worker and
    HIP stream (no collectives: its results go out in the first batch's
    gather) -> Future of its state."""
    if not hasattr(ctx, "_pool_exec2"):
        ctx._pool_exec2 = streams.executor(ctx.device, 1, "drynx-vn-pool2")
    k, W = ctx.comm.rank, ctx.comm.world
    if ctx.device.type != "cuda":
        return ctx._pool_exec2.submit(_pool_local, ctx, sq, reqs, vns, k, W, stage)
    if not hasattr(ctx, "_pool_stream2"):
        ctx._pool_stream2 = torch.cuda.Stream(ctx.device, priority=streams.priority(POOL_PRIORITY))
    side, main = ctx._pool_stream2, torch.cuda.current_stream(ctx.device)
    side.wait_stream(main)

    def run():
        with torch.cuda.stream(side):
            st = _pool_local(ctx, sq, reqs, vns, k, W, stage)
            if st["exp_f"] is not None:  # the helper digests are queued on this thread: compute them here
                st["exp_f"].result()
        side.synchronize()
        return st

    return ctx._pool_exec2.submit(run)


def verify_and_store(ctx, sq, vn, vn_index: int, n_vns: int, requests: list, range_pooled=None) -> dict:
    return store_verdicts(ctx, sq, vn, requests, check_requests(ctx, sq, vn, vn_index, n_vns, requests, range_pooled))


def check_requests(ctx, sq, vn, vn_index: int, n_vns: int, requests: list, range_pooled=None):
    """VerifyProof over one VN's inbox; with pooled range checks the range
    codes are left pending (``codes`` holds a resolver) so the VN's short
    per-CN checks run while the pooled batch is still on the GPU."""
    return prq.verify_requests(requests, sq, vn.id, vn_index, n_vns, ctx.device, ctx.verifier_cache, range_pooled,
                               defer=True, coins=ctx.vn_coins(vn.id))


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


def start_range_plane(ctx, sq, range_requests: list, staged: bool = False) -> dict:
    """The range-proof plane, started as soon as this rank's range proofs are
    signed (the reference streams them to the VNs while the CNs aggregate,
    data_collection_protocol.go:278-348): their fan-out on the data plane
    (main thread: every RCCL collective stays on one thread), then the pooled
    verification on a worker with its own HIP stream and its own control
    group (``Comm.plane("pool")``), overlapping the CN phases.  ``staged``:
    a second batch follows (``extend_range_plane``); the first batch's worker
    waits for that batch's local part and gathers both at once."""
    import concurrent.futures as cf

    vns = [ctx.cluster.by_id(si.id) for si in sq.Query.RosterVNs.list]
    with timers.timed("RangeFanOut"):
        reqs = fan_out(ctx, sq, range_requests, pool=True)
    second = cf.Future() if staged else None
    out = {"reqs": reqs, "pooled": _pool_async(ctx, sq, reqs, vns, ctx.comm.plane("pool"), second),
           "second_state": second}
    _prefetch_range(ctx, sq, reqs, vns)
    return out


def _prefetch_range(ctx, sq, reqs, vns):
    if any(vn.rank == ctx.rank for vn in vns) and hasattr(ctx, "ledger_values"):
        # the stored payloads' device-to-host copy starts now, under the pooled
        # verification, instead of at the verdicts (store_verdicts finds them
        # in the rank's blob segment); payloads whose digest is not known yet
        # (received ones: a digest here would wait for the exchange) go then
        with timers.span("ledger.prefetch"):
            ctx.ledger_values([r for r in reqs if r.kind == "range" and r.data_digest], range_shape(sq))


def range_stages(ctx, sq) -> int:
    """How many DPs of each rank prove in the range plane's FIRST batch, or 0
    for one batch.  With DPs spread unevenly over the ranks (10 DPs on 8
    GPUs: two ranks prove two), a single fan-out waits for the slowest
    prover and every pool part starts late; staged, the first exchange
    carries every rank's first min(DPs per rank) DPs, the pool parts start on
    it, and the rest follows in a second exchange whose batch verifies
    concurrently (the reference streams each DP's proofs as they are made,
    data_collection_protocol.go:278-348).  A function of the placement:
    identical on every rank.  Opt-in (DRYNX_RANGE_STAGES=1): measured at
    W = 8 on one GPU the second batch beside the first lengthens every part
    from ~30 to ~39-40 ms (its kernels and host work contend with the
    first's), which outweighs starting ~5 ms earlier (projection 51.7 vs
    50.0 ms, profiles/r6/staged/)."""
    W = ctx.comm.world
    if W <= 1 or os.environ.get("DRYNX_RANGE_STAGES", "0") != "1":
        return 0
    dps, _, _ = _placement(ctx, sq)
    lo, hi = min(dps), max(dps)
    return lo if 0 < lo < hi else 0


def extend_range_plane(ctx, sq, early: dict, range_requests: list) -> dict:
    """The second batch of a staged range plane (``range_stages``): its
    fan-out (collective: every rank calls it, with or without requests of
    its own), then its local part on a second worker and stream, concurrent
    with the first batch's; ``early`` then holds both batches' requests."""
    vns = [ctx.cluster.by_id(si.id) for si in sq.Query.RosterVNs.list]
    with timers.timed("RangeFanOut2"):
        reqs = fan_out(ctx, sq, range_requests, pool=True, stage=1)
    fut = _pool_local_async(ctx, sq, reqs, vns, 1)
    ph = early["second_state"]

    def relay(f):
        e = f.exception()
        if e is not None:
            ph.set_exception(e)
        else:
            ph.set_result(f.result())
    fut.add_done_callback(relay)
    _prefetch_range(ctx, sq, reqs, vns)
    return {**early, "reqs": early["reqs"] + reqs, "second_state": None}


def range_shape(sq):
    """(S, l) of the query's range proofs -- servers signing the digits, digits
    per proof -- when every output has the same (u, l), else None: the ledger's
    compact form locates the GT block of a payload from it before decoding."""
    q = sq.Query
    rs = {tuple(r[:2]) for r in (q.Ranges or [])}
    sigs = q.IVSigs.InputValidationSigs if q.IVSigs is not None else None
    if len(rs) != 1 or not sigs:
        return None
    u, l = next(iter(rs))
    return (len(sigs), int(l)) if u and l else None


def early_plane_ok(ctx, sq) -> bool:
    """The range plane starts before the CN phases (whatever the
    verification mode) when the survey has VNs and proofs, and there are range
    proofs to verify: with ranges (0, 0) the DPs ship commitments only, and
    starting the plane early would just put their signing and fan-out on the
    CN phases' thread instead of beside them."""
    q = sq.Query
    return bool(q.Proofs) and q.RosterVNs is not None and len(q.RosterVNs.list) > 0 \
        and any(r[0] and r[1] for r in (q.Ranges or [])) \
        and os.environ.get("DRYNX_RANGE_PLANE", "1") != "0"


LEDGER_PREFETCH = True  # A/B constants (tools/ab_patch.py --no-ledger-prefetch / --pool-priority)
POOL_PRIORITY = -1  # the U chain ahead of validation and ledger kernels (profiles/r6/pool_prio/)


def proof_collection(ctx, sq, local_requests: list, early: dict | None = None, late=None):
    """Returns the new SkipBlock (on every rank).  ``early``: the range plane
    started by ``start_range_plane`` (its requests and pooled verdicts);
    ``local_requests`` then holds the remaining (per-CN) proofs.  ``late``: a
    callable returning the proofs still being finished (the key-switch proofs
    of the last CN phase): the VNs check everything else first, then fan out
    and check these -- as the reference's VNs verify each proof as it arrives
    (proof_collection_protocol.go:183-305) -- and store one bitmap."""
    vns = [ctx.cluster.by_id(si.id) for si in sq.Query.RosterVNs.list]
    with timers.timed("ProofFanOut"):
        # (range lists not already out on the range plane go through the verification groups now)
        reqs = fan_out(ctx, sq, local_requests, pool=early is None)
    if early is not None:
        reqs = early["reqs"] + reqs
    bitmaps = {}
    with timers.timed("ProofVerification"):
        pooled = early["pooled"] if early is not None else _pool_async(ctx, sq, reqs, vns)
        local_vns = [vn.id for vn in vns if vn.rank == ctx.rank]

        def checks(rs, range_pooled):
            if len(local_vns) > 1:  # co-hosted VNs: their signature checks in one host batch
                prq.prewarm_signatures(rs, sq, local_vns, ctx.verifier_cache)
                with timers.span("verify.keyswitch.multi"):  # one grouped key-switch MSM for all of them
                    prq.prewarm_keyswitch(rs, sq, local_vns, ctx.device, ctx.verifier_cache,
                                          {v: ctx.vn_coins(v) for v in local_vns})
            return {vn.id: check_requests(ctx, sq, vn, idx, len(vns), rs, range_pooled)
                    for idx, vn in enumerate(vns) if vn.rank == ctx.rank}

        def prefetch(rs):
            # the stored payloads' host copy and blob write run under their
            # verification instead of after the verdicts (store_verdicts finds
            # them in the rank's blob segment); payloads whose digest is known.
            # On a worker of its own: the main thread goes on to the checks
            # (the late key-switch proofs' prefetch sat on the serial path)
            if not (LEDGER_PREFETCH and local_vns and hasattr(ctx, "ledger_values")):
                return None
            sel = [r for r in rs if r.kind != "shuffle" and r.data_digest and r.tensor is not None]
            if not sel:
                return None
            ex = getattr(ctx, "_prefetch_exec", None)
            if ex is None:
                ex = ctx._prefetch_exec = streams.executor(ctx.device, 1, "drynx-ledger-prefetch")

            def run():
                with timers.span("ledger.prefetch"):
                    ctx.ledger_values(sel, range_shape(sq))
            return ex.submit(run)

        pfs = [prefetch(reqs)]
        pending = checks(reqs, pooled)
        reqs2, pending2 = [], {}
        if late is not None:
            with timers.timed("ProofFanOut"):
                reqs2 = fan_out(ctx, sq, late(), pool=False)
            pfs.append(prefetch(reqs2))
            pending2 = checks(reqs2, None)
        for f in pfs:  # store_verdicts reads the blob segment the prefetch fills
            if f is not None:
                f.result()
        for vn in vns:
            if vn.id in pending:
                codes = pending[vn.id]()
                if vn.id in pending2:
                    codes = list(codes) + list(pending2[vn.id]())
                bitmaps[vn.id] = store_verdicts(ctx, sq, vn, reqs + reqs2, codes)
        if pooled is not None:
            pooled.result()
    reqs = reqs + reqs2
    if getattr(ctx, "net", None) is not None:
        _net_proofs(ctx, sq, reqs, vns)
    # bitmaps -> root VN (SharedBMChannel): every rank gets every VN's bitmap
    # plus the root VN's block parameters (its timestamp; its chain head when
    # it resumed from its ledger) and builds the same block itself -- no
    # broadcast round for the block
    root = vns[0]
    # every rank's chain head rides along: all ranks see whether they would
    # build on the root VN's head before anyone signs a block
    mine = {"bm": bitmaps, "head": ctx.last_block.Hash if ctx.last_block is not None else None}
    if ctx.rank == root.rank:
        resumed = None
        if ctx.last_block is None:
            # resume an existing chain from the root VN's ledger (restart of a
            # node over a persisted workdir) instead of starting a new genesis
            ctx.last_block = ctx.get_latest_block(root.id)
            resumed = ctx.last_block.to_bytes() if ctx.last_block is not None else None
        mine["root"] = {"time": time.time(), "prev": resumed,
                        "head": ctx.last_block.Hash if ctx.last_block is not None else None}
    allbm, rootp = {}, None
    gathered = ctx.comm.all_gather_object(mine)
    for d in gathered:
        allbm.update(d["bm"])
        rootp = d.get("root", rootp)
    if rootp["prev"] is None:
        # no resumed head to adopt: every rank must already hold the root's
        # head (a rank left behind by a survey that failed on it would build a
        # block with another hash); decided from the gathered heads, so every
        # rank raises together instead of hanging in the co-signing round
        lag = [r for r, d in enumerate(gathered) if d["head"] != rootp["head"]]
        if lag:
            raise RuntimeError(f"survey {sq.SurveyID}: rank(s) {lag} hold another chain head than the root VN "
                               f"({rootp['head']}); refusing to build diverging blocks")
    if hasattr(ctx, "take_proof_starts"):
        # the VNs' verdicts are back on every DP's rank: the reference's
        # <dp>_AllProofs ends here (its proof collection's feedback channel,
        # data_collection_protocol.go:343-345)
        now = time.perf_counter()
        for dp_id, t_start in ctx.take_proof_starts(sq.SurveyID).items():
            timers.record(f"{dp_id}_AllProofs", now - t_start)
    t = timers.start_timer("BI", sync=False)
    merged = {}
    for vn in vns:
        merged.update(allbm.get(vn.id, {}))
    data = skc.new_data_block(sq.SurveyID, merged, [v.identity() for v in vns], t=rootp["time"])
    prev = ctx.last_block
    if rootp["prev"] is not None and ctx.rank != root.rank:
        prev = skc.SkipBlock.from_bytes(rootp["prev"])
    block = skc.make_block(prev, data, [v.identity() for v in vns])
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
    if getattr(ctx, "net", None) is not None:
        ids = [v.id for v in vns]
        bsz = len(block.to_bytes())
        ctx.net.step("bitmaps", [(i, ids[0], 64 * len(allbm.get(i, {})) + 64) for i in ids[1:]],
                     hops=flow_hops("bitmaps"))
        ctx.net.step("skipchain", [(ids[0], i, bsz) for i in ids[1:]] + [(i, ids[0], SIG_BYTES) for i in ids[1:]],
                     hops=flow_hops("skipchain", n_vns=len(ids), genesis=block.Index == 0))
        ctx.net.step("end_verification", [(ids[0], "client", bsz)], hops=flow_hops("end_verification"))
    ctx.end_verification(sq.SurveyID, block)  # EndVerificationChannel <- block (service_skipchain.go:158)
    return block
