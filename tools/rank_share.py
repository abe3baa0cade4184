"""One rank's share of the W-rank headline schedule, measured on ONE GPU.

bench.py at --gpus 8 places CNs on ranks 0-2, VNs on ranks 3-5 and the 10 DPs
round robin from rank 6 (ranks 6 and 7 host two DPs each); every VN's range
checks are pooled, rank k checking slice k/W of every list for every VN
(protocols/proof_collection.py).  This tool runs one real d = 44 query on one
GPU (the bench's configuration), captures its DPs' encoded results and the
signed range-proof inbox, and then times, alone and synchronised (median of
``--reps``):

* prove(k): range proofs + signed envelopes of exactly rank k's DPs;
* pool(k): rank k's pooled share for all three VNs -- on a helper rank from
  the slice payloads it would receive (unpack included), on a VN rank from
  the full signed payloads (decode of the whole inbox included);
* digests(k): a VN rank's recomputation of the other ranks' slice digests
  (run inside its pool part while the verifier waits for the device, on a
  stream of their own, as the framework does; also timed alone for reference);
* serial: the query's non-range critical path (CN phases, querier, per-CN
  proofs, block), taken from a ``--u 0 --l 0`` bench JSON (``--serial-json``).

* ctrl: the query's control-plane rounds on the host TCP plane (one query
  broadcast and three all-gathers per query per rank: verdicts, bitmaps with
  the block seed, co-signatures), from a ``tools/ctrl_round.py`` JSON of W
  processes (``--ctrl-json``), added in full to every rank (not overlapped).

Every rank's pool part starts when the range fan-out (ONE exchange after
every rank has signed its proofs) completes, so the projected step is
max(serial on rank 0, fan-out end + max_k pool(k)) + ctrl
(``projection_step_ms``), the fan-out ending when the last link has
delivered: max over senders of prove(k) + its largest per-peer payload
(full bundles to VN ranks, slices to helpers) at ``--xgmi-link-gbs`` (one
direction of one link; the ``xgmi`` term).  ``projection_ms`` keeps each
rank's own prove + pool (+ ctrl), the bound without that synchronisation.
Usage: python tools/rank_share.py [--world 8] [--reps 5] [--serial-json f] [--ctrl-json f]
"""
from __future__ import annotations

import argparse
import contextlib
import copy
import json
import os
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from drynx_amd.crypto.coins import Coins  # noqa: E402
from drynx_amd.protocols import proof_collection as pcp  # noqa: E402
from drynx_amd.proofs import range_proof as rp  # noqa: E402
from drynx_amd.proofs import requests as prq  # noqa: E402
from drynx_amd.query import LogisticRegressionParameters, new_survey_id  # noqa: E402
from drynx_amd.services.api import DrynxClient  # noqa: E402
from drynx_amd.services.local import local_cluster, make_survey  # noqa: E402
from drynx_amd.services.service import DrynxNode  # noqa: E402


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


_PSTREAM: dict = {}


def pool_part(*a):
    """prq.verify_range_pool_part as pool_verify_ranges runs it (slice digests
    beside the part, on a stream of proof_collection.POOL_PRIORITY), digests
    resolved."""
    dev = a[3]
    if not isinstance(dev, torch.device) or dev.type != "cuda":
        res, dig = prq.verify_range_pool_part(*a, async_digests=True)
        return res, (dig.result() if hasattr(dig, "result") else dig)
    from drynx_amd.protocols import proof_collection as pc
    from drynx_amd.utils import streams

    import threading

    key = (str(dev), pc.POOL_PRIORITY, threading.get_ident())  # one stream per pool thread (a staged plane: two)
    if key not in _PSTREAM:
        _PSTREAM[key] = torch.cuda.Stream(dev, priority=streams.priority(pc.POOL_PRIORITY))
    st = _PSTREAM[key]
    st.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(st):
        res, dig = prq.verify_range_pool_part(*a, async_digests=True)
        out = res, (dig.result() if hasattr(dig, "result") else dig)
    torch.cuda.current_stream(dev).wait_stream(st)
    return out


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        _sync()
        t = time.perf_counter()
        fn()
        _sync()
        ts.append(1e3 * (time.perf_counter() - t))
    return round(statistics.median(ts), 2)


def _torch_glue(path, *fns):
    """GPU time of the torch ops launched by ``fns`` (run on this thread),
    grouped by (op, innermost framework frame), plus every kernel's total."""
    from collections import defaultdict

    from torch.profiler import ProfilerActivity, profile

    from drynx_amd.utils import timers

    for fn in fns:
        fn()
    _sync()
    timers.PROFILE_SPANS = True  # every framework span is a profiler range (GPU time of what it launched)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as p:
        for fn in fns:
            fn()
        _sync()
    timers.PROFILE_SPANS = False
    agg, cnt = defaultdict(float), defaultdict(int)
    for e in p.events():
        if not e.name.startswith("aten::") or e.cpu_parent is not None and e.cpu_parent.name.startswith("aten::"):
            continue
        t = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
        if t <= 0:
            continue
        frames = [fr for fr in (e.stack or []) if "drynx_amd" in fr or "tools/" in fr]
        key = (e.name, frames[0] if frames else "?")
        agg[key] += t
        cnt[key] += 1
    with open(path, "w") as f:
        f.write(p.key_averages().table(sort_by="device_time_total", row_limit=50, max_name_column_width=60))
        f.write("\n\n# framework spans and torch ops (device time incl. children)\n")
        f.write(p.key_averages().table(sort_by="device_time_total", row_limit=80, max_name_column_width=50))
        f.write("\n\n# GPU time of torch ops by (op, innermost framework frame)\n")
        for (name, fr), t in sorted(agg.items(), key=lambda kv: -kv[1])[:80]:
            f.write(f"{t / 1e3:9.2f} ms {cnt[(name, fr)]:5d}  {name:28s} {fr}\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--features", type=int, default=44)
    ap.add_argument("--records", type=int, default=1_000_000)
    ap.add_argument("--serial-json", default=None, help="bench.py --u 0 --l 0 JSON (the non-range critical path)")
    ap.add_argument("--torch-prof-query", default=None,
                    help="torch.profiler of one whole 1-GPU query (every thread): GPU time per framework span / op")
    ap.add_argument("--ctrl-json", default=None, help="tools/ctrl_round.py JSON (W-process control round latency)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--xgmi-link-gbs", type=float, default=76.5,
                    help="one direction of one xGMI link (GB/s): the fan-out term of the projection")
    ap.add_argument("--passes", type=int, default=2, help="1, or 2: a second pass in the reverse order (min of both)")
    ap.add_argument("--order", default=None, help="comma list: the order the ranks are measured in (default 0..W-1)")
    ap.add_argument("--staged", action="store_true", default=os.environ.get("DRYNX_RANGE_STAGES") == "1",
                    help="project the staged range plane (DRYNX_RANGE_STAGES=1, proof_collection.range_stages) "
                         "instead of ONE fan-out after every rank's proving (the default)")
    ap.add_argument("--vn-mode", default="pool", choices=["pool", "local", "own"],
                    help="proof_collection.verification_mode of the projected run: pool (every rank for every VN, "
                         "single operator), local (each VN's own rank + helpers serving only it), own")
    ap.add_argument("--torch-prof", default=None,
                    help="also profile the 1-GPU pooled check of the whole inbox and the proving of every DP "
                         "(torch.profiler on this thread): the GPU time of torch ops per framework frame")
    a = ap.parse_args()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    W, n_cns, n_vns, n_dps, d = a.world, 3, 3, 10, a.features
    cl, node = local_cluster(n_cns, n_dps, n_vns, device=dev, workdir=tempfile.mkdtemp(prefix="drynx_share_"))
    rec = max(1, a.records // n_dps)
    g = torch.Generator(device=dev).manual_seed(1234)
    node.dp_data = {}
    for dp in cl.dps:
        X = torch.randint(0, 4, (rec, d), generator=g, device=dev).to(torch.float64)
        X += torch.rand((rec, d), generator=g, device=dev, dtype=torch.float64)
        node.dp_data[dp.id] = (X, torch.randint(0, 2, (rec,), generator=g, device=dev))
    lp = LogisticRegressionParameters(NbrRecords=rec * n_dps, NbrFeatures=d, Means=[2.0] * d,
                                      StandardDeviations=[1.15] * d, Lambda=1.0, Step=0.012, MaxIterations=450,
                                      InitialWeights=[0.1] * (d + 1), K=2, PrecisionApproxCoefficients=100.0)
    client = DrynxClient(node, device=dev)
    sq0 = make_survey(client, cl, "logistic regression", proofs=1, ranges=[16, 16, 1 << 62], lr_params=lp,
                      thresholds=[1.0, 1.0, 1.0, 0.0, 1.0], sig_device=dev)
    cap = {}
    orig_async, orig_plane = DrynxNode._range_proofs_async, pcp.start_range_plane

    def cap_async(self, sq, dp_results):
        cap["dp_results"], cap["sq"] = dp_results, sq
        return orig_async(self, sq, dp_results)

    def cap_plane(ctx, sq, reqs, **kw):
        cap["reqs"] = list(reqs)
        return orig_plane(ctx, sq, reqs, **kw)

    DrynxNode._range_proofs_async, pcp.start_range_plane = cap_async, cap_plane
    for _ in range(2):  # the first query builds the prover tables
        sq = copy.copy(sq0)
        sq.SurveyID = new_survey_id()
        client.send_survey_query(sq)
    DrynxNode._range_proofs_async, pcp.start_range_plane = orig_async, orig_plane
    if a.torch_prof_query:
        def one_query():
            q = copy.copy(sq0)
            q.SurveyID = new_survey_id()
            client.send_survey_query(q)
        _torch_glue(a.torch_prof_query, one_query)
    sq, reqs, dp_results = cap["sq"], cap["reqs"], cap["dp_results"]
    rng = [i for i, r in enumerate(reqs) if r.kind == "range"]
    vn_idxs = {vn.id: rng for vn in cl.vns}
    cache = node.verifier_cache
    # the bench's placement at world W
    place = {}
    for i, c in enumerate(cl.cns):
        place.setdefault(i % W, []).append(c.id)
    for i, v in enumerate(cl.vns):
        place.setdefault((n_cns + i) % W, []).append(v.id)
    dps_of = {k: [dp.id for i, dp in enumerate(cl.dps) if (n_cns + n_vns + i) % W == k] for k in range(W)}
    vn_rank_list = [(n_cns + i) % W for i in range(n_vns)]
    vn_ranks = set(vn_rank_list)
    vn_ids = [vn.id for vn in cl.vns]
    # the framework's verification groups and weighted parts for this placement
    # (proof_collection.verification_groups: the pool, vn-local or own)
    groups, gparts = pcp.verification_groups(a.vn_mode, W, [len(dps_of[k]) for k in range(W)],
                                             [vn_rank_list.count(k) for k in range(W)], vn_rank_list)
    groups, gparts = dict(zip(vn_ids, groups)), dict(zip(vn_ids, gparts))

    def parts_of(k):
        """{part: [VN ids]} rank k checks (the VNs whose group holds k)."""
        out = {}
        for v in vn_ids:
            if k in groups[v]:
                out.setdefault(tuple(gparts[v][k]), []).append(v)
        return out

    def helper_part(k):
        """The slice part a rank hosting no VN receives (it serves one part)."""
        ps = list(parts_of(k))
        return ps[0] if ps else None

    def digest_slices(full, k):
        """The slices a VN rank k digests: its local VNs' helpers' parts."""
        want = {}
        for v, r in zip(vn_ids, vn_rank_list):
            if r != k:
                continue
            for j in groups[v]:
                if j != k:
                    want.setdefault(j, gparts[v][j])
        return [prq.slice_lists(ls, sq, p_) for ls in full for p_ in want.values()]

    def helper_reqs(part):
        out = []
        for i in rng:
            r = reqs[i]
            sl = prq.slice_lists(prq._range_lists(r, dev), sq, part)
            c = copy.copy(r)
            c._data, c.decoded, c.slice_of = None, None, tuple(part)
            c.tensor = prq.range_bundle_pack(sl).to(dev)
            out.append(c)
        return out

    def full_reqs():
        out = []
        for i in rng:
            c = copy.copy(reqs[i])
            c.decoded = None  # a VN rank decodes its signed payloads itself
            out.append(c)
        return out

    if a.torch_prof:
        _torch_glue(a.torch_prof, lambda: prq.verify_range_pool_part(
            full_reqs(), {v: list(range(len(rng))) for v in vn_idxs}, sq, dev, cache, (0, 1),
            {vn.id: Coins() for vn in cl.vns}), lambda: node._sign_range(sq, node._prove_range(sq, dp_results)))
    if os.environ.get("DRYNX_TRACE"):
        # a span trace of rank 3's (a VN rank) and rank 6's (a helper) pool share alone
        from drynx_amd.utils import timers

        timers._events.clear()
        reps = int(os.environ.get("RANK_SHARE_TRACE_REPS", "1"))  # > 1: the last one is the steady state
        for k in [int(x) for x in os.environ.get("RANK_SHARE_PARTS", "3,6").split(",") if x]:
            for _ in range(reps):
                reqs_k = full_reqs() if k in vn_ranks else helper_reqs(helper_part(k))
                _sync()
                time.sleep(1.0)  # an idle gap: a kernel trace shows this part as its own burst (tools/kernel_bursts.py)
                with timers.span(f"pool_part[{k}]"):
                    for part, pv in parts_of(k).items():
                        pool_part(reqs_k, {v: list(range(len(rng))) for v in pv}, sq, dev, cache, part,
                                  {v: Coins() for v in pv})
                _sync()
        for k in [int(x) for x in os.environ.get("RANK_SHARE_PROVE", "").split(",") if x]:
            # rank k's proving (its DPs' range proofs + signed envelopes), after the pool parts
            mine = {dp: dp_results[dp] for dp in dps_of[k]}
            for _ in range(reps):
                _sync()
                time.sleep(1.0)
                with timers.span(f"prove[{k}]"):
                    node._sign_range(sq, node._prove_range(sq, mine))
                _sync()
        timers.dump_trace(os.environ["DRYNX_TRACE"])
        if os.environ.get("RANK_SHARE_TRACE_ONLY") == "1":
            node.close(remove=True)
            return
    res = {"world": W, "features": d, "vn_mode": a.vn_mode,
           "trust_model": "single-operator-pool" if a.vn_mode == "pool" and W > 1 else "vn-local",
           "groups": groups,
           "placement": {k: {"parties": place.get(k, []), "dps": dps_of[k]} for k in range(W)},
           "ranks": {}}
    order = [int(x) for x in a.order.split(",")] if a.order else list(range(W))
    # --passes 2 (default): a second pass in the reverse order, each rank's
    # times the min of its two: the rank measured last read ~2 ms slow in
    # either order (profiles/r5/order), a drift of the process, not of the rank
    seq = order + (order[::-1] if a.passes > 1 else [])
    # the staged range plane (proof_collection.range_stages): every rank's first
    # m DPs fan out first, the rest (the ranks proving more DPs) in a second
    # exchange whose pool batch runs beside the first
    counts = [len(dps_of[k]) for k in range(W)]
    m = min(counts) if (a.staged and 0 < min(counts) < max(counts)) else 0
    first = {dp for k in range(W) for dp in (dps_of[k][:m] if m else dps_of[k])}
    sel_a = [j for j, i in enumerate(rng) if reqs[i].sender_id in first]
    sel_b = [j for j, i in enumerate(rng) if reqs[i].sender_id not in first]
    res["stages"] = {"first_dps_per_rank": m or None, "first_lists": len(sel_a), "second_lists": len(sel_b)}

    def sub(rs, sel):
        return [rs[j] for j in sel]

    # 1. proving: every rank's whole proving and (staged) its first batch
    prove = {}
    for k in seq:
        mine = {dp: dp_results[dp] for dp in dps_of[k]}
        t_all = timed(lambda: node._sign_range(sq, node._prove_range(sq, mine)), a.reps) if mine else 0.0
        mine_a = {dp: dp_results[dp] for dp in (dps_of[k][:m] if m else dps_of[k])}
        t_a = t_all if len(mine_a) == len(mine) else \
            timed(lambda: node._sign_range(sq, node._prove_range(sq, mine_a)), a.reps)
        prev = prove.get(k)
        prove[k] = (t_a, t_all) if prev is None else (min(prev[0], t_a), min(prev[1], t_all))
    # 2. the exchanges over xGMI: every rank's payloads to each peer over that
    # peer's link (full bundles to VN ranks, the helper's slice to the others);
    # each batch's parts start when its last link has delivered
    dp_rank = {dp: k for k, ids in dps_of.items() for dp in ids}
    link = [{}, {}]
    for j, i in enumerate(rng):
        r = reqs[i]
        src = dp_rank.get(r.sender_id)
        if src is None:
            continue
        full = r.tensor.numel() * r.tensor.element_size() if r.tensor is not None else len(r.data)
        lists = prq._range_lists(r, dev)
        st = 0 if r.sender_id in first else 1
        for dst in range(W):
            if dst == src:
                continue
            hp = helper_part(dst) if dst not in vn_ranks else None
            if dst in vn_ranks:
                nb = full
            elif hp is not None:
                nb = prq.range_bundle_pack(prq.slice_lists(lists, sq, hp)).numel() * 4
            else:
                continue
            link[st][(src, dst)] = link[st].get((src, dst), 0) + nb
    bw = a.xgmi_link_gbs * 1e6  # bytes per ms

    def exch_end(st, t):
        return max(t[s_] + max((b_ for (s2, _), b_ in link[st].items() if s2 == s_), default=0) / bw
                   for s_ in range(W))
    end_a = exch_end(0, {k: prove[k][0] for k in range(W)})
    end_b = exch_end(1, {k: prove[k][1] for k in range(W)}) if sel_b else end_a
    delay = max(0.0, end_b - end_a)  # the second batch's parts start this much after the first's
    # 3. every rank's pool share: the first batch's part, and (staged) the
    # second batch's on a second thread and stream, started ``delay`` later
    res["passes"] = {}
    import concurrent.futures as cf

    ex2 = cf.ThreadPoolExecutor(max_workers=1)
    for pi, k in enumerate(seq):
        mp_ = parts_of(k)
        coins = {vn.id: Coins() for vn in cl.vns}
        is_vn = k in vn_ranks

        def run_parts(reqs_k, sel):
            idx = list(range(len(sel)))
            for part, pv in mp_.items():
                pool_part(reqs_k, {v: idx for v in pv}, sq, dev, cache, part, {v: coins[v] for v in pv})
        full = [prq._range_lists(reqs[i], dev) for i in rng] if is_vn else None
        dig = digest_slices(full, k) if is_vn else []

        def batch(sel):
            if not sel or not mp_:
                return
            if is_vn:
                dst = torch.cuda.Stream(dev) if dev.type == "cuda" else None
                dg = digest_slices(sub(full, sel), k)

                def digests_side():
                    ctx = torch.cuda.stream(dst) if dst is not None else contextlib.nullcontext()
                    with ctx:
                        if dg:
                            prq.lists_digests(dg)
                    if dst is not None:
                        dst.synchronize()
                # as proof_collection: the VN's digests of its helpers' slices run on
                # their own stream as an idle task of the part
                if dst is not None:
                    dst.wait_stream(torch.cuda.current_stream(dev))
                fut = rp.add_idle_task(rp.Deferred(digests_side))
                run_parts(sub(full_reqs(), sel), sel)
                fut.result()
            else:
                run_parts(sub(helper_reqs(helper_part(k)), sel), sel)
            _sync()

        def both():
            if sel_b and mp_:
                def late():
                    time.sleep(delay / 1e3)
                    batch(sel_b)
                f = ex2.submit(late)
                batch(sel_a)
                f.result()
            else:
                batch(sel_a)
        t_pool = timed(both, a.reps) if mp_ else 0.0
        t_dig = timed(lambda: prq.lists_digests(dig), a.reps) if (is_vn and dig) else 0.0
        rec = {"prove_ms": prove[k][1], "prove_first_ms": prove[k][0], "pool_ms": t_pool, "vn_digest_ms": t_dig,
               "vn_rank": is_vn, "dps": len(dps_of[k])}
        res["passes"].setdefault(k, []).append(rec)
        prev = res["ranks"].get(k)
        res["ranks"][k] = rec if prev is None else {**rec, **{f: min(prev[f], rec[f]) for f in
                                                              ("pool_ms", "vn_digest_ms")}}
        print(json.dumps({"rank": k, "pass": 1 + (pi >= len(order)), **rec}), flush=True)
    ex2.shutdown()
    if a.serial_json:
        s = json.load(open(a.serial_json))
        res["serial_ms"] = s["ms_per_step"]
        res["serial_source"] = a.serial_json
    serial = res.get("serial_ms", 0.0)
    ctrl = 0.0
    if a.ctrl_json:
        c = json.load(open(a.ctrl_json))
        ctrl = c["bcast_ms_median"] + 3 * c["gather_ms_median"]
        res["ctrl_ms"] = round(ctrl, 3)
        res["ctrl_source"] = a.ctrl_json
    proj = {}
    for k, v in res["ranks"].items():
        # each rank's range path: its first batch's parts start at that exchange's end
        # (a VN rank's pool_ms includes its overlapped digests)
        proj[k] = round(max(serial if k == 0 else 0.0, end_a + v["pool_ms"]) + ctrl, 2)
    res["projection_ms"] = proj
    prove_max = max(v[1] for v in prove.values())
    pool_max = max(v["pool_ms"] for v in res["ranks"].values())
    xgmi = round(end_a - max(v[0] for v in prove.values()), 3)
    res["xgmi_link_bytes_max"] = max([b_ for lk in link for b_ in lk.values()], default=0)
    res["projection_step_ms"] = round(max(serial, end_a + pool_max) + ctrl, 2)
    res["projection_terms_ms"] = {"prove_max": prove_max, "first_exchange_end": round(end_a, 3),
                                  "second_exchange_delay": round(delay, 3), "xgmi": xgmi, "pool_max": pool_max,
                                  "serial": serial, "ctrl": round(ctrl, 3)}
    print(json.dumps({"vn_mode": a.vn_mode, "projection_ms": proj, "step_ms": res["projection_step_ms"],
                      "terms": res["projection_terms_ms"]}), flush=True)
    if a.json_out:
        json.dump(res, open(a.json_out, "w"), indent=1)
    node.close(remove=True)


if __name__ == "__main__":
    main()
