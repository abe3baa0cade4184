#!/usr/bin/env python3
"""Headline benchmark: full verifiable logistic-regression query on the
reference's own LR-SPECTF configuration.

BASELINE.json metric: "end-to-end query latency + range-proof verifications/sec,
logreg on 1e6 records".  Configuration = the reference's LR SPECTF run
(AllResults.xlsx LogRegr row 7, simul/runfiles/drynx.toml:13): 3 CNs, 3 VNs,
10 DPs, logistic regression k=2 over 44 features (2070 encrypted outputs per
DP), range proofs u = l = 16 on every output, every VN verifying every proof
(threshold 1.0, no sharding), Boneh-Boyen input-validation keys drawn at random
per CN and per column (InitRangeProofSignature, simul/drynx_simul.go:292-296).
1e6 synthetic SPECTF-shaped records in total (1e5 per DP).

One step = one complete survey through the framework:
  10 DPs: fp64-MFMA encoding -> 20,700 ElGamal ciphertexts -> 20,700 range
  proofs (signed offset 2^62) -> collective aggregation (+ proofs) -> key
  switching (+ proofs) -> querier decryption (BSGS) + gradient descent ->
  proof collection: 3 VNs x 20,700 range proofs (993,600 pairing equations
  each) + aggregation / key-switch proofs -> DataBlock -> BLS-cosigned
  skipchain block.

value  = range-proof verifications per second of end-to-end query time
         (20,700 proofs x 3 VNs per query), whole job.
ms_per_step = end-to-end latency of one verifiable query (max over ranks).
scaling = strong: the query is fixed; N GPUs share it (DPs round robin over the
         ranks, CNs and VNs on distinct ranks, every VN's range checks pooled
         over all ranks by default).  The JSON's ``config.trust_model`` says
         what a VN's verdict depended on in the run: ``single-operator-pool``
         (helper ranks serve every VN, their slice verdicts bound to the VN's
         own digests of the bytes they checked) or ``vn-local`` (only ranks
         assigned to that VN: ``--vn-mode local``, or the VN's own rank:
         ``--vn-mode own``; one GPU: every VN on its own coins).
vs_baseline = value / 315.6, the reference's verifications per second of
         end-to-end time in that run (20,700 x 3 / 196.77 s).

Run: python bench.py [--gpus N --steps K --warmup W].  N > 1 runs one rank
per GPU (RCCL over xGMI): under torch.distributed.run, or, when started
directly, bench.py launches torch.distributed.run with N ranks itself.

Other BASELINE.json configs (``--query``; same harness, one JSON line each;
value = end-to-end latency in seconds of one verifiable query, lower is
better, vs_baseline = value / the reference's AllOps total for that operation):
  --query mean | variance   config 2: 1e5 synthetic records (10 DPs x 1e4,
                            values in [0, 3]), range proofs (16, 5) (the
                            simulation's Ranges code 18), 3 CNs, 3 VNs;
                            reference AllOps rows 6-7: 2.57 s / 2.74 s
  --query lin_reg           config 3: Pima-shaped linear regression, d = 8,
                            8 DPs x 960 records, feature values in [0, 200),
                            range proofs (16, 8); reference AllOps row 16
                            (lin_reg, d = 9): 15.97 s
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from drynx_amd.parallel.comm import init_distributed, make_comm  # noqa: E402
from drynx_amd.query import LogisticRegressionParameters, QueryDiffP, new_survey_id  # noqa: E402
from drynx_amd.services.api import DrynxClient  # noqa: E402
from drynx_amd.services.local import local_cluster, make_survey  # noqa: E402
from drynx_amd.utils import timers  # noqa: E402

REFERENCE_LR_SPECTF_S = 196.77  # AllResults.xlsx LogRegr row 7
REFERENCE_DIFFPRI_10K_S = 82.0  # AllResults.xlsx DiifPri row 6: query with a 10k-entry noise list
# the reference's DiffPri sheet by noise-list size (simul/test_data/graphs/TIFS/diffPri.py:9-12): totals
REFERENCE_DIFFPRI_S = {0: 2.3, 10_000: 81.9, 100_000: 657.0, 1_000_000: 5872.0}
DRO_LAP_SCALE, DRO_LIMIT = 2.0, 50.0  # noise list parameters of the config-4 line
REFERENCE_VERIFICATIONS_PER_S = 10 * 2070 * 3 / REFERENCE_LR_SPECTF_S  # 10 DPs x 2070 proofs x 3 VNs
# AllOps totals (AllResults.xlsx rows 6, 7, 16) and this bench's shape for them
QUERY_CONFIGS = {
    "mean": dict(ref_s=2.57, dps=10, records=100_000, d=1, lo=0, hi=3, ranges=(16, 5)),
    "variance": dict(ref_s=2.74, dps=10, records=100_000, d=1, lo=0, hi=3, ranges=(16, 5)),
    "lin_reg": dict(ref_s=15.97, dps=8, records=7_680, d=8, lo=0, hi=199, ranges=(16, 8)),
    # the reference's MaxOptimized sheet (simul/test_data/graphs/TIFS/maxOpti.py:9-12): max with the
    # unary encoding over a range of --range values (one ciphertext + one (2, 1) range proof per value
    # and DP: the simulation's Ranges code 1), 3 CNs, 3 VNs, 10 DPs; totals 5.5 / 28.5 / 246 / 2226 s
    "max": dict(ref_s=None, dps=10, records=1_000, d=1, lo=0, hi=None, ranges=(2, 1)),
}
REFERENCE_MAX_UNARY_S = {1_000: 5.5, 10_000: 28.5, 100_000: 246.0, 1_000_000: 2226.0}  # maxOpti.py:9-12


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--records", type=int, default=1_000_000, help="records in total, split over the DPs")
    ap.add_argument("--features", type=int, default=44, help="SPECTF-shaped: 44 features -> 2070 outputs")
    ap.add_argument("--cns", type=int, default=3)
    ap.add_argument("--dps", type=int, default=10)
    ap.add_argument("--vns", type=int, default=3)
    ap.add_argument("--deterministic-sigs", action="store_true",
                    help="InitRangeProofSignatureDeterministic keys (the reference uses them only with CuttingFactor)")
    ap.add_argument("--u", "--base", dest="u", type=int, default=16)
    ap.add_argument("--l", "--digits", dest="l", type=int, default=16)
    ap.add_argument("--precision", type=float, default=100.0)
    ap.add_argument("--max-iter", type=int, default=450)
    ap.add_argument("--device", default=None)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--range", dest="value_range", type=int, default=1_000,
                    help="--query max: values in [0, RANGE) -> RANGE unary outputs per DP (maxOpti rows: "
                         "1000 / 10000 / 100000 / 1000000)")
    ap.add_argument("--range-mode", type=int, default=0,
                    help="SurveyQuery.RangeProofMode: 0 reference semantics, 1 recomputed challenge + V in G2")
    ap.add_argument("--query", default="lr", choices=["lr", "lr_dro", *QUERY_CONFIGS],
                    help="lr = the headline; lr_dro = BASELINE.json config 4; mean/variance/lin_reg = configs 2 and 3")
    ap.add_argument("--fault-dp", type=int, default=None,
                    help="fault-injected run: DP k's range-proof payload is corrupted after proving and re-signed "
                         "(one false proof among all); the bench then checks that every VN blames exactly that DP")
    ap.add_argument("--vn-mode", default=None, choices=["pool", "local", "own"],
                    help="who checks each VN's range proofs at W > 1 (proof_collection.verification_mode): pool = "
                         "every rank for every VN (single operator, the default), local = ranks assigned to that "
                         "VN only (vn-local trust), own = the VN's own rank (default: DRYNX_VN_POOL, else pool)")
    ap.add_argument("--verification-sharding", type=int, default=0,
                    help="SurveyQuery.VerificationSharding: each proof verified by exactly k VNs (0: every VN)")
    ap.add_argument("--check-ledger", action="store_true",
                    help="after the timed steps, read every local VN's stored proofs of the last survey back "
                         "(GetProofs) and report ledger_readback in the rank records")
    ap.add_argument("--table-digest", action="store_true",
                    help="report a SHA-256 of each rank's prover tables (small configs: compares sharded builds)")
    ap.add_argument("--dro", type=int, default=None,
                    help="differential-privacy noise list size (DRO shuffle by every CN, with shuffle proofs); "
                         "--query lr_dro sets 10000 (the reference's DiffPri 10k row)")
    return ap.parse_args()


def _forward_args(argv: list) -> list:
    """The script's arguments for the launcher's command line: its own parser
    takes abbreviations of ITS options out of them ("--l" would read as
    --log-dir...), so the short aliases travel as their long forms."""
    alias = {"--u": "--base", "--l": "--digits"}
    out = []
    for a in argv:
        if a.startswith("--"):
            name, eq, val = a.partition("=")
            a = alias.get(name, name) + eq + val
        out.append(a)
    return out


def _launch_ranks(args) -> int | None:
    """``--gpus N`` (N > 1) run directly, not under a launcher: start N ranks
    through torch.distributed.run as a CHILD process (this process has made
    no GPU call yet -- nothing here may touch HIP) and hand back its exit
    code; rank 0's JSON line reaches our stdout unchanged.  The reference
    likewise runs every party as its own process (simul/drynx_simul.go:83-98).
    Under a launcher (WORLD_SIZE set) returns None and the ranks run here."""
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return None
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__),
           *_forward_args(sys.argv[1:])]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    return subprocess.call(cmd, env=env)


def _check_world(args, comm):
    if comm.world != args.gpus:
        sys.exit(f"bench: --gpus {args.gpus} but the job has {comm.world} rank(s)")


def _rank_record(comm, cl, step_ms, elapsed, setup_s, b0, extra: dict | None = None) -> dict:
    """This rank's share of the job: its parties, step times, data-plane
    traffic over the timed steps, the range items it checked for the VN
    pool and the range payloads it wrote / referenced in the node's ledger
    (gathered to rank 0 into the JSON's ``ranks``)."""
    roles = {r: [p.id for p in cl.local(comm.rank, r)] for r in ("cn", "vn", "dp")}
    c = timers.counters()
    return {"rank": comm.rank, "roles": roles, "step_ms": step_ms, "elapsed_ms": round(1000 * elapsed, 1),
            "setup_s": round(setup_s, 3), "bytes_sent": comm.bytes_sent - b0[0], "bytes_recv": comm.bytes_recv - b0[1],
            "pool_range_items": c.get("pool.range_items", 0),
            "ctrl_collectives": c.get("comm.ctrl_collectives", 0),
            "data_exchanges": c.get("comm.data_exchanges", 0),
            "ledger_written": c.get("ledger.written", 0), "ledger_referenced": c.get("ledger.referenced", 0),
            "ledger_blob_bytes": c.get("ledger.blob_bytes", 0),
            **(extra or {})}


def _ledger_readback(node, cl, rank: int, survey_id: str) -> dict:
    """GetProofs of every VN hosted here for ``survey_id`` (each stored value
    read back and exported in the reference layout) -> {vn: n proofs}."""
    node.flush_stores()
    return {vn.id: len(node.get_proofs(vn.id, survey_id)) for vn in cl.local(rank, "vn")}


def _table_digest(node) -> str:
    """SHA-256 over this rank's prover tables (every signature set, every layout)."""
    import hashlib

    h = hashlib.sha256()
    for sm in node.verifier_cache._sig.values():
        for key in sorted(sm._ptab, key=str):
            v = sm._ptab[key]
            ts = v[:2] if isinstance(v, tuple) else ((v.get("g2"), v.get("gt")) if isinstance(v, dict) else ())
            for t in ts:
                if isinstance(t, torch.Tensor):
                    h.update(t.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def main():
    args = parse()
    rc = _launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    from drynx_amd.utils.streams import node_process_setup

    node_process_setup()
    if args.query == "lr_dro" and args.dro is None:
        args.dro = 10_000
    if args.query not in ("lr", "lr_dro"):
        return main_query(args)
    init_distributed()
    comm = make_comm(args.device)
    _check_world(args, comm)
    world, rank = comm.world, comm.rank
    device = comm.device
    if device.type == "cuda":
        torch.cuda.set_device(device)
    workdir = tempfile.mkdtemp(prefix=f"drynx_bench_r{rank}_")
    n_dps, n_vns = args.dps, args.vns
    # CNs on ranks 0.., VNs right after them, DPs round robin over every rank
    # starting after the CN / VN ranks (the ranks that draw an extra DP are the
    # ones without a CN or VN role: N=4 -> ranks 2, 3; N=8 -> ranks 6, 7)
    offsets = {"cn": 0, "vn": args.cns % world, "dp": (args.cns + args.vns) % world}
    cl, node = local_cluster(args.cns, n_dps, n_vns, comm=comm, device=device, workdir=workdir, offsets=offsets)
    if args.vn_mode:
        node.pool_policy = args.vn_mode
    from drynx_amd.protocols import proof_collection as pcp

    trust = pcp.trust_model(node)
    mode = pcp.verification_mode(node)
    pool_note = {"pool": f"pooled over {world} ranks for every VN (single operator; helper verdicts bound to "
                         f"slice digests)",
                 "local": "each VN's lists spread over its own rank + helper ranks serving only that VN "
                          "(helper verdicts bound to slice digests)",
                 "own": "each VN verifies its whole inbox on its own rank"}[mode] if world > 1 \
        else "every VN verifies its whole inbox with its own coins (co-hosted on one GPU)"
    if args.fault_dp is not None:
        from drynx_amd.utils.faults import FaultPlan

        node.fault_plan = FaultPlan({(cl.dps[args.fault_dp].id, "range"): "corrupt_proof"})
    rec_per_dp = max(1, args.records // n_dps)
    d = args.features
    # the DP's database: generated once on its device (synthetic, random-init)
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    dp_data = {}
    for dp in cl.local(rank, "dp"):
        X = torch.randint(0, 4, (rec_per_dp, d), generator=g, device=device).to(torch.float64)
        X += torch.rand((rec_per_dp, d), generator=g, device=device, dtype=torch.float64)
        y = torch.randint(0, 2, (rec_per_dp,), generator=g, device=device)
        dp_data[dp.id] = (X, y)
    node.dp_data = dp_data
    # global standardisation parameters (as the reference passes Means/SDs in the query)
    means = [2.0] * d
    sds = [1.15] * d
    lp = LogisticRegressionParameters(NbrRecords=rec_per_dp * n_dps, NbrFeatures=d, Means=means,
                                      StandardDeviations=sds, Lambda=1.0, Step=0.012, MaxIterations=args.max_iter,
                                      InitialWeights=[0.1] * (d + 1), K=2,
                                      PrecisionApproxCoefficients=args.precision)
    # signed coefficients: prove m + offset in [0, u^l) (offset fits the int64 wire field)
    offset = min((args.u ** args.l) // 2, 1 << 62)
    client = DrynxClient(node, device=device) if rank == 0 else None
    template = None
    t_setup = time.perf_counter()
    diffp = None
    if args.dro:
        # config 4: the DP noise list (discretised Laplace, unlynx GenerateNoiseValuesScale) is
        # encrypted by the root CN, shuffled + re-randomised by every CN in turn with a proof of
        # shuffle (DRO, service.go:619-665), and added to the aggregate before key switching
        diffp = QueryDiffP(LapMean=0.0, LapScale=DRO_LAP_SCALE, NoiseListSize=args.dro, Quanta=1.0, Scale=1.0,
                           Limit=DRO_LIMIT)
    if rank == 0:  # CN input-validation keys are set up once, before the queries (as in the reference simulation)
        template = make_survey(client, cl, "logistic regression", proofs=1, ranges=[args.u, args.l, offset],
                               lr_params=lp, thresholds=[1.0, 1.0, 1.0, 0.0, 1.0],
                               verification_sharding=args.verification_sharding, diffp=diffp,
                               sig_device=device, deterministic_sigs=args.deterministic_sigs,
                               range_proof_mode=args.range_mode)

    def one_step():
        if rank == 0:
            sq = copy.copy(template)
            sq.SurveyID = new_survey_id()
            _, vals, res = client.send_survey_query(sq)
            weights = (vals[0], list(client.last_plaintexts[0]))
        else:
            res = node.run_survey(None)
            weights = None
        return res, weights

    # setup: the CN keys / signatures above, then the first query, which also
    # builds the prover tables of the signature set in HBM (cached afterwards)
    t_first = time.perf_counter()
    for w in range(args.warmup):
        one_step()
        if w == 0:
            first_s = time.perf_counter() - t_first
    if args.warmup == 0:
        first_s = 0.0
    my_setup_s = time.perf_counter() - t_setup if args.warmup else 0.0
    setup_s = max(comm.all_gather_object(my_setup_s))
    table_bytes = sum(comm.all_gather_object(sum(sm.table_bytes() for sm in node.verifier_cache._sig.values())))
    timers.reset()
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    b0 = (comm.bytes_sent, comm.bytes_recv)
    t0 = time.perf_counter()
    blocks, checks, step_ms = [], [], []
    prof = _torch_profiler(rank)
    for _ in range(args.steps):
        ts = time.perf_counter()
        with timers.span("bench.step"):  # a roctx range under DRYNX_ROCTX=1 (tools/span_kernels.py)
            res, weights = one_step()
        step_ms.append(round(1000 * (time.perf_counter() - ts), 1))
        blocks.append(res.block)
        checks.append((weights, res.clear_dp))
    node.flush_stores()  # proof persistence overlaps the next step; the tail is timed too
    _torch_profiler_dump(prof, rank)
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    my_elapsed = time.perf_counter() - t0
    elapsed = max(comm.all_gather_object(my_elapsed))
    extra = {}
    if args.check_ledger:
        extra["ledger_readback"] = _ledger_readback(node, cl, rank, blocks[-1].data_block().SurveyID
                                                    if blocks and blocks[-1] is not None else "")
    if args.table_digest:
        extra["table_digest"] = _table_digest(node)
    ranks = comm.all_gather_object(_rank_record(comm, cl, step_ms, my_elapsed, my_setup_s, b0, extra))
    n_out = (d + 1) + (d + 1) ** 2
    proofs_per_step = n_dps * n_out
    # threshold 1.0: every VN checks every proof (VerificationSharding k: exactly k VNs per proof)
    verifs_per_step = proofs_per_step * (min(args.verification_sharding, n_vns) if args.verification_sharding
                                         else n_vns)
    ms = 1000.0 * elapsed / args.steps
    value = verifs_per_step * args.steps / elapsed
    if args.fault_dp is not None:
        # exactly the forged DP's range proof is false (code 0) at every VN; everything else true
        bad = f"/range/{cl.dps[args.fault_dp].id}/"
        ok = all(b is not None and all((v == 0) if bad in k else (v == 1) for k, v in b.data_block().Proofs.items())
                 for b in blocks)
    elif args.verification_sharding:  # the VNs not assigned a proof record "received, not checked" (2)
        ok = all(b is not None and set(b.data_block().Proofs.values()) <= {1, 2}
                 and 1 in b.data_block().Proofs.values() for b in blocks)
    else:
        ok = all(b is not None and all(v == 1 for v in b.data_block().Proofs.values()) for b in blocks)
    result_ok = _check_lr_results(comm, checks, lp, diffp)
    allt = comm.all_gather_object(timers.summary())
    if rank == 0:
        phase = {}
        for t in allt:
            for k, v in t.items():
                phase[k] = max(phase.get(k, 0.0), v["sum"] / args.steps)
        if args.dro:
            config4 = {
                "metric": "end-to-end verifiable LR query latency with DP noise (DRO shuffle) + key switching",
                "value": round(ms / 1000.0, 5), "unit": "s per query (whole job)", "higher_is_better": False,
                "vs_baseline": round((ms / 1000.0) / REFERENCE_LR_SPECTF_S, 6),
                "speedup_vs_reference_lr_spectf": round(REFERENCE_LR_SPECTF_S / (ms / 1000.0), 1),
                "speedup_vs_reference_diffpri_10k": round(REFERENCE_DIFFPRI_10K_S / (ms / 1000.0), 1),
                "obfuscation": "DRO: encrypted Laplace noise list shuffled + re-randomised by every CN with a "
                               "proof of shuffle, added to the aggregate before key switching (the reference's "
                               "Obfuscation protocol is only legal for bit operations, structs.go:450-462)",
                "noise_list": {"size": args.dro, "lap_scale": DRO_LAP_SCALE, "limit": DRO_LIMIT},
                "reference_row": ({"sheet": "DiffPri", "source": "simul/test_data/graphs/TIFS/diffPri.py:9-12",
                                   "noise_list": args.dro, "total_s": REFERENCE_DIFFPRI_S[args.dro],
                                   "speedup": round(REFERENCE_DIFFPRI_S[args.dro] / (ms / 1000.0), 1)}
                                  if args.dro in REFERENCE_DIFFPRI_S else None),
            }
        line = {
            "metric": "end-to-end query latency + range-proof verifications/sec, logreg on 1e6 records",
            "value": round(value, 3),
            "unit": "range-proof verifications/s (whole job) over full verifiable LR queries",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / REFERENCE_VERIFICATIONS_PER_S, 3),
            "dtype": "bn254-exact/fp64",
            "data": "synthetic (random SPECTF-shaped records, random keys and input-validation signatures)",
            "config": {
                "model": f"logistic regression k=2, d={d} ({n_out} encrypted outputs per DP), full verifiable query",
                "global_batch": rec_per_dp * n_dps,
                "seq_len": None,
                "parallelism": f"{world} ranks: {n_dps} DPs, {args.cns} CNs, {n_vns} VNs, VN range checks: {pool_note}",
                "dps": n_dps, "cns": args.cns, "vns": n_vns,
                "records_per_dp": rec_per_dp,
                "sigs": "deterministic" if args.deterministic_sigs else "random (per CN, per column)",
                "verification": (f"each proof verified by {args.verification_sharding} VNs (VerificationSharding)"
                                 if args.verification_sharding else "every VN verifies every proof (threshold 1.0)"),
                "range_proof": {"u": args.u, "l": args.l, "servers": args.cns, "proofs_per_query": proofs_per_step,
                                "verifications_per_query": verifs_per_step},
                "vn_independent": trust == "vn-local",
                "trust_model": trust,
                "verification_mode": mode,
                "vn_pool": pool_note,
            },
            "e2e_latency_s": round(ms / 1000.0, 4),
            "latency_vs_reference_lr_spectf": round(REFERENCE_LR_SPECTF_S / (ms / 1000.0), 2),
            "all_proofs_valid": ok,
            **({"fault_injected": f"{cl.dps[args.fault_dp].id} range proof corrupted and re-signed",
                "blame_ok": ok} if args.fault_dp is not None else {}),
            "result_ok": result_ok,
            "setup_s": round(setup_s, 3),
            "first_query_s": round(first_s, 3),
            "prover_table_bytes": int(table_bytes),
            "step_ms_rank0": step_ms,
            "rccl_world": world if dist.is_initialized() and dist.get_backend() == "nccl" else 0,
            "ranks": ranks,
            "phase_s": {k: round(v, 4) for k, v in sorted(phase.items()) if not k.startswith("dp") or "AllProofs" in k},
        }
        if args.dro:  # config 4: latency is the metric (one JSON line, same harness)
            line.update(config4)
            line["config"]["model"] = f"logistic regression k=2, d={d} + DRO noise + key switching, verifiable"
        print(json.dumps(line), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(line, f, indent=1)
    timers.dump_trace(os.environ.get("DRYNX_TRACE") and f"{os.environ['DRYNX_TRACE']}.r{rank}.json")
    node.close(remove=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    if not (ok and result_ok):
        sys.exit("bench: a proof was rejected or the decrypted result is wrong (see all_proofs_valid / result_ok)")


def _check_lr_results(comm, checks: list, lp, diffp=None) -> bool:
    """Outside the timed region: for every timed query, the querier's
    decrypted aggregate must equal the clear sum of every DP's coefficient
    vector (all ranks' DPs) -- plus, with DP noise, one distinct entry of the
    (shuffled) noise list per output -- and its weights the gradient descent
    run on what was decrypted."""
    from collections import Counter

    from drynx_amd.models.logistic_regression import decode_logistic_regression_values
    from drynx_amd.proofs.aggregation_shuffle import generate_noise_values_scale

    sums = []
    for _, clear in checks:
        tot = None
        for v in clear.values():
            g0 = [int(x) for x in v[0]]
            tot = g0 if tot is None else [a + b for a, b in zip(tot, g0)]
        sums.append(tot)
    every = comm.all_gather_object(sums)
    if comm.rank != 0:
        return True
    good = True
    for q, (weights, _) in enumerate(checks):
        clear_sum = None
        for per_rank in every:
            s_ = per_rank[q]
            if s_ is not None:
                clear_sum = s_ if clear_sum is None else [a + b for a, b in zip(clear_sum, s_)]
        (w, plain) = weights
        if diffp is not None:
            noise = Counter(generate_noise_values_scale(diffp.NoiseListSize, diffp.LapMean, diffp.LapScale,
                                                        diffp.Quanta, diffp.Scale or 1.0, diffp.Limit))
            k = min(len(plain), diffp.NoiseListSize)
            used = Counter(p_ - c_ for p_, c_ in zip(plain[:k], clear_sum[:k]))
            if any(noise[v] < c for v, c in used.items()) or plain[k:] != clear_sum[k:]:
                good = False
                continue
        elif plain != clear_sum:
            good = False
            continue
        w_clear = decode_logistic_regression_values(plain, lp)
        good = good and all(abs(a - b) <= 1e-9 * max(1.0, abs(b)) for a, b in zip(w, w_clear))
    return good


def _torch_profiler(rank):
    """DRYNX_TORCH_PROF=<file>: torch.profiler over the timed steps (which
    torch ops launch the framework kernels' helper copies/fills); off by default."""
    path = os.environ.get("DRYNX_TORCH_PROF")
    if not path or rank != 0:
        return None
    from torch.profiler import ProfilerActivity, profile

    p = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True)
    p.__enter__()
    return p


def _torch_profiler_dump(p, rank):
    if p is None:
        return
    torch.cuda.synchronize()
    p.__exit__(None, None, None)
    path = os.environ["DRYNX_TORCH_PROF"]
    with open(path, "w") as f:
        f.write(p.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=60,
                                                                max_name_column_width=40, max_shapes_column_width=60))
        f.write("\n\n# GPU time of torch ops by (op, innermost framework frame)\n")
        from collections import defaultdict

        agg, cnt = defaultdict(float), defaultdict(int)
        for e in p.events():
            if not e.name.startswith("aten::") or e.cpu_parent is not None and e.cpu_parent.name.startswith("aten::"):
                continue
            t = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
            if t <= 0:
                continue
            frames = [fr for fr in (e.stack or []) if "drynx_amd" in fr or "bench.py" in fr]
            key = (e.name, frames[0] if frames else "?")
            agg[key] += t
            cnt[key] += 1
        for (name, fr), t in sorted(agg.items(), key=lambda kv: -kv[1])[:60]:
            f.write(f"{t / 1e3:9.2f} ms {cnt[(name, fr)]:5d}  {name:28s} {fr}\n")


def main_query(args):
    """BASELINE.json configs 2 and 3, and the MaxOptimized rows (``--query max
    --range N``): one verifiable integer query per step."""
    cfg = dict(QUERY_CONFIGS[args.query])
    if args.query == "max":
        cfg["hi"] = args.value_range - 1
        cfg["ref_s"] = REFERENCE_MAX_UNARY_S.get(args.value_range)
    init_distributed()
    comm = make_comm(args.device)
    _check_world(args, comm)
    world, rank = comm.world, comm.rank
    device = comm.device
    if device.type == "cuda":
        torch.cuda.set_device(device)
    n_dps = cfg["dps"]
    offsets = {"cn": 0, "vn": args.cns % world, "dp": (args.cns + args.vns) % world}
    cl, node = local_cluster(args.cns, n_dps, args.vns, comm=comm, device=device,
                             workdir=tempfile.mkdtemp(prefix=f"drynx_bench_r{rank}_"), offsets=offsets)
    if args.vn_mode:
        node.pool_policy = args.vn_mode
    rows = cfg["records"] // n_dps
    d = cfg["d"]
    n_in = d + 1 if args.query == "lin_reg" else 1
    g = torch.Generator(device=device).manual_seed(99 + rank)
    node.dp_data = {dp.id: list(torch.randint(cfg["lo"], cfg["hi"] + 1, (n_in, rows), generator=g, device=device))
                    for dp in cl.local(rank, "dp")}
    u, l = cfg["ranges"]
    client = DrynxClient(node, device=device) if rank == 0 else None
    template = None
    t_setup = time.perf_counter()
    if rank == 0:
        template = make_survey(client, cl, args.query, query_min=cfg["lo"], query_max=cfg["hi"], d=d, rows=rows,
                               proofs=1, ranges=[u, l], thresholds=[1.0, 1.0, 1.0, 0.0, 1.0], sig_device=device,
                               deterministic_sigs=args.deterministic_sigs)
    sig_s = time.perf_counter() - t_setup
    decoded = []

    def one_step():
        if rank == 0:
            sq = copy.copy(template)
            sq.SurveyID = new_survey_id()
            _, vals, res = client.send_survey_query(sq)
            decoded.append(vals[0])
            return res
        return node.run_survey(None)

    t_first = time.perf_counter()
    for _ in range(args.warmup):
        one_step()
    first_s = (time.perf_counter() - t_first) / max(1, args.warmup) if args.warmup else 0.0
    timers.reset()
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    blocks = [one_step().block for _ in range(args.steps)]
    node.flush_stores()
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    elapsed = max(comm.all_gather_object(time.perf_counter() - t0))
    ok = all(b is not None and all(v == 1 for v in b.data_block().Proofs.values()) for b in blocks)
    sec = elapsed / args.steps
    n_out = len(template.Query.Ranges) if rank == 0 else None
    result_ok = None
    if args.query == "max":  # the decoded max equals the max over every DP's records
        mx = comm.all_gather_object(max((int(c.max()) for cols in node.dp_data.values() for c in cols), default=None))
        want = max(v for v in mx if v is not None)
        result_ok = rank != 0 or all(int(round(v[0])) == want for v in decoded)
    allt = comm.all_gather_object(timers.summary())
    if rank == 0:
        phase = {}
        for t in allt:
            for k, v in t.items():
                phase[k] = max(phase.get(k, 0.0), v["sum"] / args.steps)
        line = {
            "metric": f"end-to-end verifiable {args.query} query latency",
            "value": round(sec, 5),
            "unit": "s per query (whole job)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * sec, 2),
            "higher_is_better": False, "scaling": "strong",
            "vs_baseline": round(sec / cfg["ref_s"], 5) if cfg["ref_s"] else None,
            "speedup_vs_reference": round(cfg["ref_s"] / sec, 1) if cfg["ref_s"] else None,
            "dtype": "bn254-exact/int64",
            "data": "synthetic (uniform integer records, random keys and input-validation signatures)",
            "config": {"model": f"{args.query}" + (f" d={d}" if args.query == "lin_reg" else "")
                       + (f" unary encoding over [0, {args.value_range})" if args.query == "max" else ""),
                       "global_batch": rows * n_dps, "seq_len": None,
                       "parallelism": f"{world} ranks: {n_dps} DPs, {args.cns} CNs, {args.vns} VNs",
                       "dps": n_dps, "records_per_dp": rows, "outputs_per_dp": n_out,
                       "range_proof": {"u": u, "l": l, "proofs_per_query": n_dps * n_out,
                                       "verifications_per_query": n_dps * n_out * args.vns},
                       "sigs": ("deterministic (InitRangeProofSignatureDeterministic)" if args.deterministic_sigs
                                else "random (per CN, per column)"),
                       "verification": "every VN verifies every proof"},
            "reference_row": ({"sheet": "MaxOptimized", "source": "simul/test_data/graphs/TIFS/maxOpti.py:9-12",
                               "range": args.value_range, "total_s": cfg["ref_s"]} if args.query == "max" else None),
            "all_proofs_valid": ok,
            "result_ok": result_ok,
            "signature_setup_s": round(sig_s, 3),
            "first_query_s": round(first_s, 3),
            "phase_s": {k: round(v, 4) for k, v in sorted(phase.items())
                        if not k[:2] in ("dp", "vn", "cn") or k[2:3] == "0"},
        }
        print(json.dumps(line), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(line, f, indent=1)
    node.close(remove=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
