#!/usr/bin/env python3
"""Headline benchmark: full verifiable logistic-regression query.

BASELINE.json metric: "end-to-end query latency + range-proof verifications/sec,
logreg on 1e6 records" — config 5: full verifiable query (logistic regression
over 1e6 records, skipchain proof collection, batched range-proof
verification).

One step = one complete survey through the framework:
  DP (one per rank/GPU): 1e6 synthetic SPECTF-shaped records (44 features,
  random-init data, generated once on the device = the DP's database) ->
  approximation-coefficient encoding (fp64 MFMA) -> 2070 ElGamal ciphertexts
  -> 2070 range proofs (u=16, l=16 as in the reference's service tests, signed offset 2^62) with S = 3 CNs ->
  collective aggregation -> key switching (+ aggregation / key-switch proofs)
  -> querier decryption (BSGS) + gradient descent -> proof collection at the
  VNs (one per rank, every proof verified by exactly one VN: batched
  pairing verification) -> DataBlock -> signed skipchain block.

value  = range proofs verified per second of end-to-end query time, summed
         over the whole job (weak scaling: per-GPU work is fixed).
ms_per_step = end-to-end latency of one verifiable query (max over ranks).
vs_baseline = value / 114.6, the reference's range-proof throughput derived
         from its LR-SPECTF run (10 DPs x 2070 proofs, 180.59 s of proof
         overhead; AllResults.xlsx LogRegr row 7).

Run: python bench.py [--gpus N --steps K --warmup W]; for N>1 under
torch.distributed.run (one rank per GPU, RCCL over xGMI).
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import sys
import tempfile
import time

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from drynx_amd.parallel.comm import init_distributed, make_comm  # noqa: E402
from drynx_amd.query import LogisticRegressionParameters, new_survey_id  # noqa: E402
from drynx_amd.services.api import DrynxClient  # noqa: E402
from drynx_amd.services.local import local_cluster, make_survey  # noqa: E402
from drynx_amd.utils import timers  # noqa: E402

REFERENCE_RANGE_PROOFS_PER_S = 10 * 2070 / 180.59  # LR SPECTF, BASELINE.md
REFERENCE_LR_SPECTF_S = 196.77


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--records", type=int, default=1_000_000, help="records per DP (one DP per GPU)")
    ap.add_argument("--features", type=int, default=44, help="SPECTF-shaped: 44 features -> 2070 outputs")
    ap.add_argument("--cns", type=int, default=3)
    ap.add_argument("--u", "--base", dest="u", type=int, default=16)
    ap.add_argument("--l", "--digits", dest="l", type=int, default=16)
    ap.add_argument("--precision", type=float, default=100.0)
    ap.add_argument("--max-iter", type=int, default=450)
    ap.add_argument("--device", default=None)
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def main():
    args = parse()
    init_distributed()
    comm = make_comm(args.device)
    world, rank = comm.world, comm.rank
    device = comm.device
    if device.type == "cuda":
        torch.cuda.set_device(device)
    workdir = tempfile.mkdtemp(prefix=f"drynx_bench_r{rank}_")
    n_dps, n_vns = world, world
    cl, node = local_cluster(args.cns, n_dps, n_vns, comm=comm, device=device, workdir=workdir)
    d = args.features
    # the DP's database: generated once on its device (synthetic, random-init)
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    dp_data = {}
    for dp in cl.local(rank, "dp"):
        X = torch.randint(0, 4, (args.records, d), generator=g, device=device).to(torch.float64)
        X += torch.rand((args.records, d), generator=g, device=device, dtype=torch.float64)
        y = torch.randint(0, 2, (args.records,), generator=g, device=device)
        dp_data[dp.id] = (X, y)
    node.dp_data = dp_data
    # global standardisation parameters (as the reference passes Means/SDs in the query)
    means = [2.0] * d
    sds = [1.15] * d
    lp = LogisticRegressionParameters(NbrRecords=args.records * n_dps, NbrFeatures=d, Means=means,
                                      StandardDeviations=sds, Lambda=1.0, Step=0.012, MaxIterations=args.max_iter,
                                      InitialWeights=[0.1] * (d + 1), K=2,
                                      PrecisionApproxCoefficients=args.precision)
    # signed coefficients: prove m + offset in [0, u^l) (offset fits the int64 wire field)
    offset = min((args.u ** args.l) // 2, 1 << 62)
    client = DrynxClient(node, device=device) if rank == 0 else None
    template = None
    if rank == 0:  # CN input-validation keys are set up once, before the queries (as in the reference simulation)
        template = make_survey(client, cl, "logistic regression", proofs=1, ranges=[args.u, args.l, offset],
                               lr_params=lp, thresholds=[1.0, 1.0, 1.0, 0.0, 1.0], verification_sharding=1,
                               sig_device=device, deterministic_sigs=True)

    def one_step():
        if rank == 0:
            sq = copy.copy(template)
            sq.SurveyID = new_survey_id()
            _, vals, res = client.send_survey_query(sq)
            weights = vals[0]
        else:
            res = node.run_survey(None)
            weights = None
        return res, weights

    for _ in range(args.warmup):
        one_step()
    timers.reset()
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    blocks = []
    for _ in range(args.steps):
        res, weights = one_step()
        blocks.append(res.block)
    node.flush_stores()  # proof persistence overlaps the next step; the tail is timed too
    comm.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = max(comm.all_gather_object(elapsed))
    n_out = (d + 1) + (d + 1) ** 2
    proofs_per_step = n_dps * n_out
    ms = 1000.0 * elapsed / args.steps
    value = proofs_per_step * args.steps / elapsed
    ok = all(b is not None and all(v in (1, 2) for v in b.data_block().Proofs.values()) for b in blocks)
    allt = comm.all_gather_object(timers.summary())
    if rank == 0:
        phase = {}
        for t in allt:
            for k, v in t.items():
                phase[k] = max(phase.get(k, 0.0), v["sum"] / args.steps)
        line = {
            "metric": "end-to-end query latency + range-proof verifications/sec, logreg on 1e6 records",
            "value": round(value, 3),
            "unit": "range-proof verifications/s (whole job) over full verifiable LR queries",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / REFERENCE_RANGE_PROOFS_PER_S, 3),
            "dtype": "bn254-exact/fp64",
            "data": "synthetic (random SPECTF-shaped records, random keys)",
            "config": {
                "model": f"logistic regression k=2, d={d} ({n_out} encrypted outputs per DP), full verifiable query",
                "global_batch": args.records * n_dps,
                "seq_len": None,
                "parallelism": f"{world} ranks: {n_dps} DPs, {args.cns} CNs, {n_vns} VNs (sharded verification)",
                "records_per_dp": args.records,
                "range_proof": {"u": args.u, "l": args.l, "servers": args.cns, "proofs_per_query": proofs_per_step},
            },
            "e2e_latency_s": round(ms / 1000.0, 4),
            "latency_vs_reference_lr_spectf": round(REFERENCE_LR_SPECTF_S / (ms / 1000.0), 2),
            "all_proofs_valid": ok,
            "phase_s": {k: round(v, 4) for k, v in sorted(phase.items()) if not k.startswith("dp") or "AllProofs" in k},
        }
        print(json.dumps(line), flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                json.dump(line, f, indent=1)
    timers.dump_trace(os.environ.get("DRYNX_TRACE") and f"{os.environ['DRYNX_TRACE']}.r{rank}.json")
    node.close(remove=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
