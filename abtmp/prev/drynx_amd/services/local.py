"""Cluster bootstrap helpers shared by tests, the simulation, bench.py and the CLI.

Mirrors the reference's test/simulation wiring: ``generateNodes`` /
``repartitionDPs`` (services/service_test.go:29-66), signature creation per CN
and output (simul/drynx_simul.go:283-305), thresholds ordering
``[general, aggregation, range, obfuscation, keyswitch]``.
"""
from __future__ import annotations

import tempfile

import torch

from ..crypto import oracle as O
from ..parallel.comm import Comm, LocalComm
from ..parallel.topology import build_cluster
from ..proofs import range_proof as rp
from ..query import QueryDiffP, QueryDPDataGen, choose_operation, lr_nbr_outputs
from .api import DrynxClient
from .service import DrynxNode

RANGE_PRESETS = {  # simul/drynx_simul.go:133-281 `Ranges` codes -> (u, l)
    -1: None, 0: (0, 0), 1: (2, 1), 16: (16, 16), 17: (8, 3), 18: (16, 5), 19: (4, 16),
}


def local_cluster(n_cns=3, n_dps=5, n_vns=3, comm: Comm | None = None, device=None, workdir=None,
                  deterministic_keys=False, dp_data=None, offsets=None):
    comm = comm or LocalComm(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    cl = build_cluster(n_cns, n_dps, n_vns, comm.world, comm.rank, comm, deterministic_keys, offsets)
    node = DrynxNode(cl, comm, workdir or tempfile.mkdtemp(prefix="drynx_db_"), device or comm.device, dp_data)
    return cl, node


def make_signatures(cluster, ranges, device="cpu", deterministic=False):
    """InputValidationSigs[cn][col]: one BB key + u signatures per (CN, output)."""
    if not deterministic:  # the reference default: fresh random keys per CN and per column
        flat = rp.init_range_proof_signatures([int(r[0]) for _ in cluster.cns for r in ranges], device)
        n = len(ranges)
        return [flat[i * n:(i + 1) * n] for i in range(len(cluster.cns))]
    out = []
    det: dict = {}
    for _ in cluster.cns:
        row = []
        for r in ranges:
            u = int(r[0])
            # InitRangeProofSignatureDeterministic: identical keys (x = 12), computed once per u
            if u not in det:
                det[u] = rp.init_range_proof_signature_deterministic(u, device)
            row.append(det[u])
        out.append(row)
    return out


def make_survey(client: DrynxClient, cluster, op_name: str, *, query_min=0, query_max=10, d=1, rows=10,
                group_by=(1,), proofs=0, ranges=None, obfuscation=False, thresholds=None, diffp=None,
                cutting_factor=0, lr_params=None, survey_id=None, sig_device="cpu", deterministic_sigs=False,
                verification_sharding=0, with_vns=None, range_proof_mode=0):
    op = choose_operation(op_name, query_min, query_max, d, cutting_factor)
    if op_name == "logistic regression":
        op.LRParameters = lr_params
        op.NbrOutput = lr_nbr_outputs(lr_params.NbrFeatures, lr_params.K)
    n_out = op.NbrOutput
    if ranges is not None and (len(ranges) == 0 or not isinstance(ranges[0], (list, tuple))):
        ranges = [list(ranges) for _ in range(n_out)]  # one (u, l[, offset]) for every output
    ps = None
    if proofs and ranges is not None and not all(r[0] == 0 and r[1] == 0 for r in ranges):
        ps = make_signatures(cluster, ranges, sig_device, deterministic_sigs)
    if thresholds is None:
        thresholds = [1.0, 1.0, 1.0, 1.0 if obfuscation else 0.0, 1.0] if proofs else [0.0] * 5
    with_vns = bool(proofs) if with_vns is None else with_vns
    id_to_public = {p.id: p.public for p in cluster.parties}
    gen = QueryDPDataGen(GroupByValues=list(group_by), GenerateRows=rows, GenerateDataMin=query_min,
                         GenerateDataMax=query_max)
    return client.generate_survey_query(
        cluster.roster_cns(), cluster.roster_vns() if with_vns else None, cluster.server_to_dp(), id_to_public,
        survey_id, op, ranges, ps, proofs, obfuscation, thresholds, diffp or QueryDiffP(), gen, cutting_factor,
        verification_sharding, range_proof_mode)


def clear_expected(op_name, clear_dp: dict):
    """Sum of the DPs' clear responses (first group) for checking decoded results."""
    tot = None
    for v in clear_dp.values():
        g0 = v[0]
        tot = list(g0) if tot is None else [a + b for a, b in zip(tot, g0)]
    return tot


__all__ = ["local_cluster", "make_survey", "make_signatures", "RANGE_PRESETS", "clear_expected", "O"]
