"""The Drynx node runtime (one instance per rank = per GPU).

Reference: services/service.go (CN orchestration, ``HandleSurveyQuery`` :263,
phases :711-868), services/service_data_provider.go (DP), and
services/service_skipchain.go (VN + skipchain + bbolt getters).  The reference
runs each party as its own onet server and wires phases with goroutines and
channels (with known ordering fragility); here every rank runs
the same explicit phase sequence (SPMD) with collective barriers between
phases, hosting any number of logical CN/DP/VN parties:

  broadcast query -> DRO noise shuffle -> DataCollection (+ range proofs)
  -> CollectiveAggregation (+ aggregation proofs) -> [Obfuscation (+ proofs)]
  -> KeySwitching (+ proofs) -> result to the querier
  -> ProofCollection at the VNs -> skipchain block

Timer names follow the reference.
"""
from __future__ import annotations

import copy
import os
import time
from dataclasses import dataclass, field

import torch

from .. import native as nt
from ..crypto.elgamal import CipherVector
from ..ledger.skipchain import SkipBlock
from ..ledger.skipchain import update_chain as skc_update_chain
from ..ops.encoding import cat_proof_batches as dcp_batch_cat
from ..ledger.store import Store
from ..parallel.comm import Comm, LocalComm
from ..parallel.ec_collectives import KeyIndex
from ..parallel.netem import CT_BYTES, POINT_BYTES, flow_hops, tree_edges
from ..parallel.topology import Cluster
from ..proofs import range_proof as rp
from ..proofs import requests as prq
from ..protocols import computing_nodes as cnp
from ..protocols import data_collection as dcp
from ..protocols import proof_collection as pcp
from ..query import PublishSignatureBytes, SurveyQuery, add_diff_p, check_parameters, ivsigs_digest
from ..utils import streams, timers

from ..utils.faults import FaultPlan
from ..utils.log import get_logger

log = get_logger("service")


@dataclass
class SurveyResult:
    survey_id: str
    result: CipherVector | None            # key-switched ciphertexts, groups x NbrOutput (root rank)
    n_groups: int
    n_out: int
    block: SkipBlock | None = None
    clear_dp: dict = field(default_factory=dict)
    client_out: object = None

    def groups(self):
        return [self.result[g * self.n_out:(g + 1) * self.n_out] for g in range(self.n_groups)]


LEDGER_GT_T2 = True  # range payloads stored in their compact form (A/B constant: tools/ab_patch.py)
# smaller payloads stay raw: a one-record DP's 27 KB bundle saves little and
# its own launches and header reads cost more (6000 one-record DPs: 1.7 -> 9.4 s
# per query when every bundle was compacted, profiles/r5/allops)
LEDGER_COMPACT_MIN_BYTES = 1 << 20


class DrynxNode:
    """Per-rank runtime hosting the logical parties placed on this rank."""

    def __init__(self, cluster: Cluster, comm: Comm | None = None, workdir: str = "./drynx_db", device=None,
                 dp_data: dict | None = None):
        self.comm = comm or LocalComm(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.rank = self.comm.rank
        self.device = torch.device(device) if device is not None else self.comm.device
        if self.device.type == "cuda":
            if self.device.index is None:
                self.device = torch.device("cuda", torch.cuda.current_device())
            timers.set_device(self.device)
        self.cluster = cluster
        self.key_index = KeyIndex([p.id for p in cluster.parties])
        self.workdir = workdir
        self.dp_data = dp_data or {}
        self._stores: dict = {}
        self.verifier_cache = prq.VerifierCache()
        self.local_bitmaps: dict = {}
        self.last_block: SkipBlock | None = None
        self.surveys: dict = {}
        self.fault_plan = FaultPlan.from_env()  # misbehaving parties (tests / simulations)
        from ..parallel.netem import NetEmulator

        self.net = NetEmulator.from_env()  # emulated party-to-party links (simulation Bandwidth / Delay)
        # VN side of the API (service_skipchain.go:31-166): surveys announced to
        # the VNs (SurveyQueryToVN) and the EndVerificationChannel per survey
        self.vn_surveys: dict = {}
        self._end_cv = __import__("threading").Condition()
        self._end_blocks: dict = {}

    # ------------------------------------------------------------------ VN API
    def vn_coins(self, vn_id: str):
        """The VN's private coins (crypto/coins.py): its sampling decisions and
        the random weights of all of its batched checks, never shared with
        another VN hosted on this rank."""
        if not hasattr(self, "_vn_coins"):
            self._vn_coins = {}
        c = self._vn_coins.get(vn_id)
        if c is None:
            from ..crypto.coins import Coins

            c = self._vn_coins[vn_id] = Coins()
        return c

    def register_vn_survey(self, sq: SurveyQuery):
        """HandleSurveyQueryToVN: the VNs learn the survey (expected proof
        counts, DB, chain) before any proof arrives.  A survey that reaches the
        VNs without this call is registered implicitly when it runs."""
        from ..protocols.proof_collection import expected_counts

        with self._end_cv:
            self.vn_surveys[sq.SurveyID] = {"sq": sq, "expected": expected_counts(sq)}
            if len(self.vn_surveys) > 256:
                self.vn_surveys.pop(next(iter(self.vn_surveys)))

    def end_verification(self, survey_id: str, block: SkipBlock):
        """The root VN appended the survey's block: release the waiters."""
        with self._end_cv:
            self._end_blocks[survey_id] = block
            if len(self._end_blocks) > 256:
                self._end_blocks.pop(next(iter(self._end_blocks)))
            self._end_cv.notify_all()

    def wait_end_verification(self, survey_id: str, timeout: float | None = None) -> SkipBlock | None:
        """SendEndVerification (api_skipchain.go:30, service_skipchain.go:166):
        block until every VN finished the survey's proofs and the block is
        appended; None on timeout."""
        with self._end_cv:
            self._end_cv.wait_for(lambda: survey_id in self._end_blocks, timeout)
            return self._end_blocks.get(survey_id)

    # ------------------------------------------------------------------ VN storage
    def ledger_value(self, req):
        return self.ledger_values([req])[0]

    def ledger_values(self, reqs: list, shape: tuple | None = None) -> list:
        """What a VN stores for each proof request (storeProof,
        proof_collection_protocol.go:318-331): the signed payload.  Range
        bundles' raw-limb tensors go to the rank's shared blob segment once
        (however many co-hosted VNs store them): every new one of the call is
        gathered into one device buffer and moved by ONE pinned, asynchronous
        device-to-host copy on the ledger's own stream (thousands of one-proof
        DPs would otherwise cost one copy + event each); ``get_proofs`` serves
        them in the reference RangeProofListBytes layout (proofs/range_wire.py)."""
        out: list = [None] * len(reqs)
        fresh: dict = {}
        for i, req in enumerate(reqs):
            if req.header_only or req.tensor is None or req._data is not None:
                out[i] = req.payload()
            else:
                fresh.setdefault(req.digest().hex(), []).append(i)
        if not fresh:
            return out
        if not hasattr(self, "_blobs"):
            self._blobs = self._blob_store()
        refs = {k: self._blobs.get(k) for k in fresh}
        new = [k for k, v in refs.items() if v is None]
        if new:
            tensors = {k: reqs[fresh[k][0]].tensor.contiguous().reshape(-1).view(torch.uint8) for k in new}
            claims = self._blobs.claim(new) if hasattr(self._blobs, "claim") else [True] * len(new)
            mine = [k for k, c in zip(new, claims) if c]
            theirs = [k for k, c in zip(new, claims) if not c]
            timers.count("ledger.written", len(mine))
            timers.count("ledger.referenced", len(theirs))
            if mine:
                items = [self._ledger_item(reqs[fresh[k][0]], tensors[k], shape) for k in mine]
                for k, ref in zip(mine, self._blobs.put_many(mine, self._host_bytes(items))):
                    refs[k] = ref
            if theirs:  # another VN rank of this node claimed them: references only, no device-to-host copy
                for k, ref in zip(theirs, self._blobs.put_refs(theirs)):
                    refs[k] = ref
        for k, idxs in fresh.items():
            for i in idxs:
                out[i] = refs[k]
        return out

    def _blob_store(self):
        """This rank's store of large ledger values.  On a single node with VNs
        on several ranks (LOCAL_WORLD_SIZE == WORLD_SIZE), the VN ranks share
        one content-addressed node directory and each payload is copied and
        written once, by the first VN rank of the node holding it that claims
        it (``ledger.store.NodeBlobs``: three VN ranks would otherwise write
        ~1.7 GB per query to one disk); DRYNX_LEDGER_NODE_SHARE=0 keeps one
        private store per rank."""
        from ..ledger.store import BlobSegment, NodeBlobs

        W = self.comm.world
        vn_ranks = sorted({vn.rank for vn in self.cluster.vns})
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", "0") or 0)
        # one directory per job: torchrun's run id (often "none" when standalone)
        # plus the rendezvous port, so consecutive or concurrent jobs never share it
        run = "_".join(x for x in (os.environ.get("TORCHELASTIC_RUN_ID"), os.environ.get("MASTER_PORT")) if x)
        if (W > 1 and lws == W and run and len(vn_ranks) > 1 and self.rank in vn_ranks
                and os.environ.get("DRYNX_LEDGER_NODE_SHARE", "1") == "1"):
            root = os.path.join(os.path.dirname(os.path.abspath(self.workdir)), f"drynx_node_ledger_{run}")
            return NodeBlobs(root, device=self.device)
        return BlobSegment(os.path.join(self.workdir, f"ledger_r{self.rank}.blobs"), self.device)

    def _ledger_item(self, req, tensor, shape=None):
        """What ``_host_bytes`` copies for one stored payload: a range bundle
        on the GPU in its compact ledger form (``proofs.ledger_codec``: GT
        elements as torus images, rebuilt bit for bit when read), anything
        else as is."""
        if LEDGER_GT_T2 and req.kind == "range" and tensor.is_cuda and tensor.numel() >= LEDGER_COMPACT_MIN_BYTES:
            from ..proofs import ledger_codec

            pend = ledger_codec.prepare(req, shape)
            if pend is not None:
                return pend
        return tensor

    def _host_bytes(self, tensors: list):
        """A producer of the host bytes of ``tensors`` (run by the ledger
        thread): on a GPU one concatenation on the compute stream, then one
        pinned copy on the ledger stream, so the producer only waits for it.
        An item may be a ``ledger_codec.Pending``: the producer builds its
        compact image on the ledger stream and copies that instead."""
        from ..ledger.store import Compact
        from ..proofs.ledger_codec import Pending

        items = list(tensors)
        if not any(isinstance(t, Pending) for t in items) and not items[0].is_cuda:
            return lambda: [memoryview(t.numpy()) for t in items]
        if not hasattr(self, "_ledger_stream"):
            self._ledger_stream = torch.cuda.Stream(self.device)
        st = self._ledger_stream
        st.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(st):
            for t in items:
                (t.tensor if isinstance(t, Pending) else t).record_stream(st)
            # compact images whose GT blocks are known now are built here, on
            # the ledger stream, and copied with the raw payloads; the others
            # (layout from the header) are built by the producer
            raw = [t.launch() if isinstance(t, Pending) and t.regions is not None else t for t in items]
            raw = [t for t in raw if not isinstance(t, Pending)]
            # each payload straight into its slice of one pinned buffer (no
            # device-side concatenation of the ~600 MB of range payloads), by a
            # small persistent copy grid (nt.copy_to_host) instead of the
            # runtime's blit kernel, whose thousands of PCIe-stalled waves sat
            # beside the verification (~5 ms per query, tools/ab_ledger_copy.py)
            sizes = [t.numel() for t in raw]
            host = torch.empty((max(1, sum(sizes)),), dtype=torch.uint8, pin_memory=True)
            pairs, slow, o = [], [], 0
            for t, n in zip(raw, sizes):
                (pairs if n % 4 == 0 and t.data_ptr() % 4 == 0 else slow).append((t, host[o: o + n]))
                o += n
            if pairs:
                nt.copy_to_host(pairs, host)
            for t, h in slow:
                h.copy_(t, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)

        def produce():
            ev.synchronize()
            mv = memoryview(host.numpy())
            out, o, k = [], 0, 0
            for it in items:
                if isinstance(it, Pending) and it.image is None:
                    v = it.produce(st)
                else:
                    v = mv[o: o + sizes[k]]
                    v = it.finish(v) if isinstance(it, Pending) else v
                    o += sizes[k]
                    k += 1
                # compact images are tagged as such for the store (never sniffed when read)
                out.append(Compact(v) if isinstance(it, Pending) and it.compact else v)
            return out
        return produce

    def store(self, vn_id: str) -> Store:
        s = self._stores.get(vn_id)
        if s is None or s.closed:
            s = self._stores[vn_id] = Store(os.path.join(self.workdir, f"db_{vn_id}.sqlite"))
        return s

    # ------------------------------------------------------------------ main entry
    def run_survey(self, sq: SurveyQuery | None, on_result=None) -> SurveyResult:
        """Collective: every rank calls it; rank 0 passes the SurveyQuery.

        ``on_result(SurveyResult)`` (querier side) is handed the key-switched
        result as soon as the CNs produce it and runs on a worker thread with
        its own device stream, overlapping the VNs' proof collection -- as in
        the reference, where the querier decodes while the VNs verify
        (service.go:805-868 vs proof_collection_protocol.go); its return value
        lands in ``SurveyResult.client_out``.

        On a GPU the survey's own (latency-bound: CN phases, short proof
        checks) launches run on a HIGH-priority stream, so the dispatcher hands
        them the next free CU slots instead of queueing them behind the
        long-running workgroups of the range prover / verifier, which keep
        normal-priority streams."""
        if self.device.type != "cuda":
            return self._run_survey(sq, on_result)
        if not hasattr(self, "_hp_stream"):
            self._hp_stream = torch.cuda.Stream(self.device, priority=streams.priority(-1))
        hp, outer = self._hp_stream, torch.cuda.current_stream(self.device)
        hp.wait_stream(outer)
        with torch.cuda.stream(hp):
            out = self._run_survey(sq, on_result)
        outer.wait_stream(hp)
        return out

    def _run_survey(self, sq: SurveyQuery | None, on_result=None) -> SurveyResult:
        sq = self._broadcast_query(sq)
        self.surveys[sq.SurveyID] = sq
        if sq.Query.Proofs and sq.Query.RosterVNs is not None and sq.SurveyID not in self.vn_surveys:
            self.register_vn_survey(sq)
        if self.rank == 0 and not check_parameters(sq, add_diff_p(sq.Query.DiffP)):
            log.warning("query parameters failed CheckParameters; continuing as the reference does")
        proofs: list = []
        q = sq.Query
        n_groups = len(dcp.all_possible_groups(q.DPDataGen.GroupByValues))
        n_out = q.Operation.NbrOutput
        t_exec = timers.start_timer("JustExecution")
        if self.net is not None:
            self._net_dissemination(sq)
        cn_sums, cn_inputs, dp_results = dcp.data_collection(self, sq)
        # range proofs start right after encoding (the reference fires them
        # asynchronously, data_collection_protocol.go:278-348): proving is queued
        # on the GPU now, envelope marshalling + signing runs on a worker thread
        # while the CN phases below proceed
        range_future = range_future2 = None
        if q.Proofs:
            # staged range plane (pcp.range_stages): the first min(DPs per
            # rank) DPs of every rank fan out first, the rest in a second batch
            m = pcp.range_stages(self, sq) if pcp.early_plane_ok(self, sq) else 0
            if m:
                items = list(dp_results.items())
                range_future = self._range_proofs_async(sq, dict(items[:m]), staged=True)
                range_future2 = self._range_proofs_async(sq, dict(items[m:]), staged=True) if items[m:] else None
                if range_future2 is None:  # no second-stage DP here: the rank still joins that exchange
                    import concurrent.futures as cf

                    range_future2 = cf.Future()
                    range_future2.set_result([])
            else:
                range_future = self._range_proofs_async(sq, dp_results)
        # DRO noise shuffle: after the DPs' encoding and with their range
        # proofs already queued, so its shuffles and shuffle proofs run beside
        # the proving instead of before it (the reference runs the DRO phase in
        # its own goroutine beside data collection and waits for it only before
        # key switching, services/service.go:341-352, 733-736)
        noise = cnp.dro_phase(self, sq, proofs)
        if self.net is not None and noise is not None:
            cns = [si.id for si in sq.RosterServers.list]
            nb = int(sq.Query.DiffP.NoiseListSize) * 3 * CT_BYTES
            self.net.step("dro", [(a, b, nb) for a, b in zip(cns, cns[1:] + cns[:1])], hops=flow_hops("dro", len(cns)))
        want = dcp.expected_n_out(sq)
        if dp_results:  # (a width that does not fit ``want`` aborted the route on every rank)
            n_out = len(next(iter(dp_results.values()))["cv"]) // n_groups
        if want is None:  # ranks without DPs learn the width from the others
            n_out = max(self.comm.all_gather_object(n_out if dp_results else 0)) or n_out
        else:
            n_out = want
        early = None
        if range_future is not None and pcp.early_plane_ok(self, sq):
            # the range-proof plane starts now, beside the CN phases
            with timers.span("range.plane.start"):
                rreqs = range_future.result()
                # the signed payloads are complete (a staged batch's signing
                # waited for its own proving only: the prove stream may still
                # run the second batch, which the exchange must not wait for)
                src = "_sign_stream" if range_future2 is not None else "_prove_stream"
                if hasattr(self, src):
                    torch.cuda.current_stream(self.device).wait_stream(getattr(self, src))
                if self.fault_plan:
                    self.fault_plan.apply(rreqs, lambda pid: self.cluster.by_id(pid).keypair.secret)
                early = pcp.start_range_plane(self, sq, rreqs, staged=range_future2 is not None)
                if range_future2 is not None:
                    early["second"] = range_future2
            range_future = None
        # range proofs on the GPU during this query's CN phases and querier (``_side_stream``)
        self._range_active = bool(early is not None or range_future is not None) and \
            any(u and ll for u, ll in (tuple(r[:2]) for r in (q.Ranges or [])))
        n_rows = n_groups * n_out
        net = self.net
        cn_ids = [si.id for si in sq.RosterServers.list]
        nc = len(cn_ids)
        if net is not None:
            with_dps = sum(1 for dps in (sq.ServerToDP or {}).values() if dps)
            net.step("data_collection", [(si.id, cn, n_rows * CT_BYTES) for cn, dps in (sq.ServerToDP or {}).items()
                                         for si in (dps or [])],
                     hops=flow_hops("data_collection", nc, cns_with_dps=with_dps))
        agg = cnp.collective_aggregation(self, sq, cn_sums, cn_inputs, n_rows, proofs)
        if net is not None:
            net.step("aggregation", [(c, p, n_rows * CT_BYTES) for c, p in tree_edges(cn_ids)],
                     hops=flow_hops("aggregation", nc))
        if q.Obfuscation:
            agg = cnp.obfuscation(self, sq, agg, n_rows, proofs)
            if net is not None:
                e = tree_edges(cn_ids)
                net.step("obfuscation", [(p, c, n_rows * CT_BYTES) for c, p in e] +
                         [(c, p, n_rows * CT_BYTES) for c, p in e], hops=flow_hops("obfuscation", nc))
        result = cnp.key_switching(self, sq, agg, n_groups, n_out, noise, proofs)
        if net is not None:
            e = tree_edges(cn_ids)
            net.step("key_switching", [(p, c, n_rows * POINT_BYTES) for c, p in e] +
                     [(c, p, n_rows * CT_BYTES) for c, p in e], hops=flow_hops("key_switching", nc))
            net.step("result", [(cn_ids[0], "client", n_rows * CT_BYTES)], hops=flow_hops("result"))
        if q.CuttingFactor and result is not None:
            # CN truncates the replicated response (service.go:760-761)
            per = n_out // q.CuttingFactor
            result = CipherVector.cat([result[g * n_out: g * n_out + per] for g in range(n_groups)])
            n_out = per
        timers.end_timer(t_exec)
        client = {"f": None}
        # the last CN phase's proofs (key switching) are still being finished:
        # the VNs check every other proof first (pcp.proof_collection ``late``)
        late_f = proofs.pop() if proofs and hasattr(proofs[-1], "result") else None
        with timers.span("cn.proofs.wait"):
            proofs = self._resolve_proofs(proofs)

        def start_client():
            if on_result is not None and result is not None and client["f"] is None:
                client["f"] = self._submit_client(on_result, SurveyResult(sq.SurveyID, result, n_groups, n_out))
        # the querier decodes beside the VNs' checks.  Without range proofs the
        # key-switch proof chain is the step's critical path: the decode then
        # starts once those proofs are signed (its decryption kernels held the
        # CUs the chain's short launches wait for: --u 0 --l 0 27.2 -> 26.0 ms);
        # with range proofs it starts at once (later: +3.8 ms, profiles/r5/ab19)
        if late_f is None or self._range_active:
            start_client()
        if range_future is not None:
            proofs.extend(range_future.result())
            if hasattr(self, "_prove_stream"):
                torch.cuda.current_stream(self.device).wait_stream(self._prove_stream)
        secret_of = lambda pid: self.cluster.by_id(pid).keypair.secret  # noqa: E731
        if self.fault_plan:
            self.fault_plan.apply(proofs, secret_of)

        def late():
            with timers.span("cn.proofs.wait_late"):
                out = self._resolve_proofs([late_f]) if late_f is not None else []
            start_client()
            if self.fault_plan:
                self.fault_plan.apply(out, secret_of)
            return out

        block = None
        if early is not None and "second" in early:
            # the staged range plane's second batch (every rank: a collective)
            with timers.span("range.plane.extend"):
                rreqs2 = early.pop("second").result()
                if hasattr(self, "_sign_stream"):
                    torch.cuda.current_stream(self.device).wait_stream(self._sign_stream)
                if self.fault_plan:
                    self.fault_plan.apply(rreqs2, secret_of)
                early = pcp.extend_range_plane(self, sq, early, rreqs2)
        if q.Proofs and q.RosterVNs is not None and len(q.RosterVNs.list):
            block = pcp.proof_collection(self, sq, proofs, early, late)
        elif late_f is not None:
            late()
        start_client()  # (no proofs to wait for)
        clear = {k: v["clear"] for k, v in dp_results.items()}
        out = SurveyResult(sq.SurveyID, result, n_groups, n_out, block, clear)
        if client["f"] is not None:
            out.client_out = client["f"].result()
        return out

    def _net_dissemination(self, sq):
        """Client -> root CN, then root CN -> other CNs and its DPs with the
        DPs' acknowledgements (service.go:263-378), carrying the query and its
        input-validation keys (hops: ``netem.flow_hops``)."""
        sigs = sq.Query.IVSigs.InputValidationSigs or []
        size = 1024 + sum(len(x.Public) + len(x.Signature) for row in sigs for x in row)
        cns = [si.id for si in sq.RosterServers.list]
        self.net.step("query_client", [("client", cns[0], size)], hops=flow_hops("query_client"))
        self.net.step("query_dissemination", [(cns[0], c, size) for c in cns[1:]] +
                      [(cn, si.id, size) for cn, dps in (sq.ServerToDP or {}).items() for si in (dps or [])],
                      hops=flow_hops("query_dissemination", len(cns)))

    def _side_stream(self, attr: str, env: str, bulk: int, alone: int):
        """The worker stream of the querier or of the CN-proof finishing, at the
        priority that pays for the query at hand.  With range proofs on the GPU
        (``self._range_active``: the range plane's long-running prover and
        verifier workgroups) the querier's short decrypt/BSGS chain is the
        step's tail and gets the high priority (75 ms vs 10 ms behind the VNs'
        MSM passes) while the CN proofs stay normal; without them the CN
        proofs' signing gates the VNs' checks and the querier only runs beside
        them, so the priorities swap (same-box A/B, profiles/r4/prio_ab.txt:
        headline 186.2 vs 192.8 ms, --u 0 --l 0 30.8-33.0 vs 28.8 ms).
        ``env`` (DRYNX_CLIENT_PRIORITY / DRYNX_CNP_PRIORITY) pins one."""
        pin = os.environ.get(env)
        p = int(pin) if pin is not None else (bulk if getattr(self, "_range_active", False) else alone)
        cache = self.__dict__.setdefault(attr, {})
        if p not in cache:
            cache[p] = torch.cuda.Stream(self.device, priority=streams.priority(p))
        return cache[p]

    def defer_proofs(self, fn, *args, lane: str = ""):
        """Run ``fn(*args) -> [ProofRequest]`` (proof finishing: transcript
        digests, responses, packing, envelope signatures -- each needs one
        device-to-host copy) on the node's CN-proof worker with its own HIP
        stream, ordered after the work queued so far; the query's critical
        path does not wait for it.  ``lane`` = "late": the last CN phase's
        (key-switching) proofs get a worker and stream of their own, so their
        transcript starts when the phase ends instead of queueing behind the
        earlier phases' signing.  -> Future (resolved before proof collection)."""
        import concurrent.futures as cf

        if self.device.type != "cuda":
            fut = cf.Future()
            fut.set_result(fn(*args))
            return fut
        attr = f"_cnp_pool{lane}"
        if not hasattr(self, attr):
            setattr(self, attr, streams.executor(self.device, 1, f"drynx-cn-proofs{lane}"))
        side = self._side_stream(f"_cnp_streams{lane}", "DRYNX_CNP_PRIORITY", bulk=0, alone=-1)
        # the job's inputs are the work queued so far: an event recorded now and
        # waited for when the job STARTS on the worker -- a wait_stream issued
        # here would land on ``side`` while the previous job is still queueing
        # its kernels, putting them behind this caller's later launches (the
        # aggregation proofs' signing waited ~4 ms behind the key-switch proof
        # kernels that way)
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))

        def run():
            side.wait_event(ready)
            with torch.cuda.stream(side):
                out = fn(*args)
            done = torch.cuda.Event()
            done.record(side)
            done.synchronize()  # this job's packed payloads are complete before anyone reads them
            return out

        return getattr(self, attr).submit(run)

    @staticmethod
    def _resolve_proofs(proofs: list) -> list:
        out = []
        for p in proofs:
            if hasattr(p, "result"):
                out.extend(p.result())
            elif isinstance(p, list):
                out.extend(p)
            else:
                out.append(p)
        return out

    def _submit_client(self, fn, partial: SurveyResult):
        if not hasattr(self, "_client_pool"):
            self._client_pool = streams.executor(self.device, 1, "drynx-querier")
        if self.device.type != "cuda":
            return self._client_pool.submit(fn, partial)
        side = self._side_stream("_client_streams", "DRYNX_CLIENT_PRIORITY", bulk=-1, alone=0)
        side.wait_stream(torch.cuda.current_stream(self.device))  # result tensors are ready on `side`

        def run():
            with torch.cuda.stream(side):
                r = fn(partial)
            side.synchronize()
            return r

        return self._client_pool.submit(run)

    def _broadcast_query(self, sq: SurveyQuery | None) -> SurveyQuery:
        """Query to every rank (the reference broadcasts it down the CN tree,
        service.go:263-330) in ONE control collective.  The CN input-validation
        signatures (MBs for wide queries) ride along, as raw bytes, only the
        first time their set is sent: every rank keeps the same bounded cache
        of sets keyed by digest (rank 0 mirrors it), so rank 0 knows which
        sets the others hold without asking."""
        if self.comm.world == 1:
            return sq
        if not hasattr(self, "_ivsigs"):
            self._ivsigs = {}
        msg = None
        if sq is not None:
            sigs = sq.Query.IVSigs.InputValidationSigs
            dg = ivsigs_digest(sigs)
            lite = copy.copy(sq)
            lite.Query = copy.copy(sq.Query)
            lite.Query.IVSigs = copy.copy(sq.Query.IVSigs)
            lite.Query.IVSigs.InputValidationSigs = None
            raw = None
            if dg and dg not in self._ivsigs:
                raw = [[(x.Public, x.Signature) for x in row] for row in sigs]
                self._cache_ivsigs(dg, sigs)
            msg = (lite.to_dict(), dg, raw)
        d, dg, raw = self.comm.broadcast_object(msg, src=0)
        if self.rank != 0 and raw is not None:
            self._cache_ivsigs(dg, [[PublishSignatureBytes(p, g) for p, g in row] for row in raw])
        out = SurveyQuery.from_dict(d)
        if dg:
            out.Query.IVSigs.InputValidationSigs = self._ivsigs[dg]
        return out

    def _cache_ivsigs(self, dg, sigs):
        """The same insertion / eviction on every rank (see ``_broadcast_query``)."""
        if len(self._ivsigs) >= 8:
            self._ivsigs.pop(next(iter(self._ivsigs)))
        self._ivsigs[dg] = sigs

    def _range_proofs(self, sq, dp_results: dict, proofs: list):
        """Synchronous variant (kept for callers/tests that patch it)."""
        t0 = time.perf_counter()
        reqs = self._sign_range(sq, self._prove_range(sq, dp_results))
        self._record_all_proofs(sq, reqs, t0)
        proofs.extend(reqs)

    def _record_all_proofs(self, sq, reqs: list, t0: float):
        """``RangeProving``: this rank's proving batch, from the start of
        proving until the signed envelopes exist (device work included:
        measured after the prover stream has drained).  Each DP's proving start
        is kept for its ``<dp>_AllProofs``, which -- as in the reference
        (data_collection_protocol.go:280-345: the timer ends when the proof
        collection protocol's feedback channel fires) -- runs until the VNs'
        verdicts on that DP's proofs are back on the DP's rank
        (``take_proof_starts``, proof_collection.py)."""
        timers.record("RangeProving", time.perf_counter() - t0)
        if not hasattr(self, "_proof_t0"):
            self._proof_t0 = {}
        if len(self._proof_t0) > 64:
            self._proof_t0.clear()
        starts = self._proof_t0.setdefault(sq.SurveyID, {})
        for r in reqs:
            starts.setdefault(r.sender_id, t0)

    def take_proof_starts(self, survey_id) -> dict:
        """{dp_id: proving start} of the DPs of this rank for a survey (once)."""
        return getattr(self, "_proof_t0", {}).pop(survey_id, {})

    def _prove_range(self, sq, dp_results: dict) -> list:
        """Range proofs of every DP hosted here as ONE prover batch per (u, l)
        (ten DPs with one output each would otherwise be ten latency-bound
        launch sequences), split back per DP afterwards."""
        P = sq.RosterServers.aggregate()
        out = {dp_id: [] for dp_id in dp_results}
        owners, batches = [], []
        for dp_id, res in dp_results.items():
            bs = [b for b in res["proofs"] if b is not None and len(b)]
            if bs:
                for b in bs:
                    owners.append((dp_id, b))
                    batches.append(b)
            elif not any(b is not None for b in res["proofs"]):
                # no range proofs (ranges 0): ship the commitments only (dcp.go:283-288)
                out[dp_id].append(rp.RangeProofList(0, 0, 0, [0] * len(res["cv"]), list(range(len(res["cv"]))),
                                                    res["cv"]))
        if batches:
            sigmat = self.verifier_cache.sigmat(sq, self.device)
            if not hasattr(sigmat, "_shard"):
                # every rank hosts DPs: the prover tables are built 1/W per rank and shared
                sigmat.attach_shard(self.comm, all(self.cluster.local(r, "dp") for r in range(self.comm.world)))
            big = dcp_batch_cat(batches)
            lists = rp.create_range_proofs(big, sigmat, P, self.device, sq.RangeProofMode)  # one list per (u, l)
            # every DP's items of a given (u, l) are contiguous inside that list
            cursor = {}
            for dp_id, b in owners:
                for key in dict.fromkeys(zip(b.u, b.l)):
                    cnt = sum(1 for uu, ll in zip(b.u, b.l) if (uu, ll) == key)
                    gi = next(g for g, r in enumerate(lists) if (r.u, r.l) == key)
                    a = cursor.get(gi, 0)
                    out[dp_id].append(rp.rpl_range(lists[gi], a, a + cnt))
                    cursor[gi] = a + cnt
        return list(out.items())

    def _sign_range(self, sq, proved: list) -> list:
        """Every hosted DP's range request: one packing, digest and signing
        pass for all of them (``prq.new_range_requests``)."""
        items = list(proved)
        secrets = [self.cluster.by_id(dp_id).keypair.secret for dp_id, _ in items]
        return prq.new_range_requests(items, sq.SurveyID, secrets, self.device)

    def _range_proofs_async(self, sq, dp_results: dict, staged: bool = False):
        """Prove the range proofs of ``dp_results`` on the prove stream and sign
        them on the proof worker -> Future of the signed requests.
        ``staged``: one of several batches queued back to back on the prove
        stream; its signing then waits for ITS proving only (an event) and
        runs on a stream of its own, so the first batch's envelopes do not
        wait for the second batch's kernels."""
        import concurrent.futures as cf

        if not hasattr(self, "_pool"):
            self._pool = streams.executor(self.device, 1, "drynx-proofs")
        if type(self)._range_proofs is not DrynxNode._range_proofs or "_range_proofs" in self.__dict__:
            # a patched (e.g. fault-injecting) prover: run it synchronously
            lst: list = []
            self._range_proofs(sq, dp_results, lst)
            fut = cf.Future()
            fut.set_result(lst)
            return fut
        t0 = time.perf_counter()
        if self.device.type != "cuda":
            proved = self._prove_range(sq, dp_results)

            def sign_host():
                reqs = self._sign_range(sq, proved)
                self._record_all_proofs(sq, reqs, t0)
                return reqs
            return self._pool.submit(sign_host)
        # proving runs on its own HIP stream so the CN phases (aggregation, key
        # switching: short latency-bound launches) overlap it on the GPU instead
        # of queueing behind ~20 ms of range-proof kernels
        if not hasattr(self, "_prove_stream"):
            self._prove_stream = torch.cuda.Stream(self.device)
        side, main = self._prove_stream, torch.cuda.current_stream(self.device)
        side.wait_stream(main)  # the DP ciphertexts / randomness are ready
        with torch.cuda.stream(side):
            proved = self._prove_range(sq, dp_results)
        if staged:
            done = torch.cuda.Event()
            done.record(side)
            if not hasattr(self, "_sign_stream"):
                self._sign_stream = torch.cuda.Stream(self.device)
            sst = self._sign_stream

            def sign_staged():
                sst.wait_event(done)
                with torch.cuda.stream(sst):
                    reqs = self._sign_range(sq, proved)
                sst.synchronize()
                self._record_all_proofs(sq, reqs, t0)
                return reqs

            return self._pool.submit(sign_staged)

        def sign():
            with torch.cuda.stream(side):
                reqs = self._sign_range(sq, proved)  # packing + digest kernels follow the proofs on `side`
            side.synchronize()
            self._record_all_proofs(sq, reqs, t0)
            return reqs

        return self._pool.submit(sign)

    # ------------------------------------------------------------------ VN getters (api_skipchain.go)
    def get_genesis(self, vn_id: str):
        raw = self.store(vn_id).get("genesis", "genesis")
        return SkipBlock.from_bytes(raw) if raw else None

    def vn_latest(self, vn_id: str):
        """The VN's own latest block (its chain head), cached in memory."""
        if not hasattr(self, "_vn_latest"):
            self._vn_latest = {}
        if vn_id not in self._vn_latest:
            raw = self.store(vn_id).get("skipchain", "latest")
            self._vn_latest[vn_id] = SkipBlock.from_bytes(raw) if raw else None
        return self._vn_latest[vn_id]

    def set_vn_latest(self, vn_id: str, block: SkipBlock):
        if not hasattr(self, "_vn_latest"):
            self._vn_latest = {}
        self._vn_latest[vn_id] = block

    def get_latest_block(self, vn_id: str, from_block: SkipBlock | None = None):
        """GetLatestBlock (service_skipchain.go:195-205): without ``from_block``
        the VN's head; with it, the last block of the update chain walked and
        verified from ``from_block`` through the forward links (GetUpdateChain)."""
        if from_block is not None:
            return self.get_update_chain(vn_id, from_block)[-1]
        raw = self.store(vn_id).get("skipchain", "latest")
        return SkipBlock.from_bytes(raw) if raw else None

    def get_update_chain(self, vn_id: str, from_block: SkipBlock) -> list:
        """GetUpdateChain from ``from_block`` (re-read from this VN's ledger, so
        its forward links are the current ones) to the head."""
        st = self.store(vn_id)

        def get(h):
            raw = st.get("skipchain", h)
            return SkipBlock.from_bytes(raw) if raw else None

        start = get(from_block.Hash) or from_block
        publics = {p.id: p.public for p in self.cluster.vns}
        return skc_update_chain(get, start, publics)

    def get_block(self, vn_id: str, survey_id: str):
        st = self.store(vn_id)
        h = st.get("mapping", survey_id)
        if h is None:
            return None
        raw = st.get("skipchain", h.decode())
        return SkipBlock.from_bytes(raw) if raw else None

    def get_proofs(self, vn_id: str, survey_id: str) -> dict:
        """HandleGetProofs (service_skipchain.go:240-320): the VN's stored proofs;
        range bundles in the reference layout network.Marshal(&RangeProofListBytes),
        the per-CN proofs in their kyber-encoding export."""
        st = self.store(vn_id)
        st.flush()
        out = {}
        for kind in prq.VN_ORDER:
            for k, v in st.bucket(f"{survey_id}/{kind}").items():
                # raw-limb payloads are served in the reference layout; one
                # that does not decode is an error, not silently raw bytes
                out[k] = prq.export_reference_bytes(kind, v)
        return out

    def get_bitmap(self, vn_id: str, survey_id: str) -> dict:
        import json

        raw = self.store(vn_id).get(vn_id, f"{survey_id}/map")
        return json.loads(raw) if raw else {}

    def flush_stores(self):
        """Wait until every queued ledger write is durable (blob writes are
        fdatasync'ed by the ledger worker, SQLite commits sync the WAL)."""
        for s in self._stores.values():
            s.flush()
        if hasattr(self, "_blobs"):
            self._blobs.flush()

    def close_db(self, vn_id: str, remove: bool = False):
        s = self._stores.pop(vn_id, None)
        if s is not None:
            s.close(remove)

    def close(self, remove: bool = False):
        for k in list(self._stores):
            self.close_db(k, remove)
        if hasattr(self, "_blobs"):
            self._blobs.close(remove)
            del self._blobs
