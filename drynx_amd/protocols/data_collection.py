"""DataCollection: DPs encode + encrypt, responses are gathered at their CN.

Reference: protocols/data_collection_protocol.go — star tree CN root + its
DPs (:73-172); each DP generates or loads its data (:178-373,
createFakeDataForOperation :376), encodes per group-by group, fires its range
proofs asynchronously, sends ``ResponseDPBytes`` to the CN which sums per
group (:144-168).

Here: every rank encodes the DPs it hosts (one batched encryption kernel per
response), the (DP -> CN) star gather is one ``route`` all-to-all over
xGMI, and each CN sums its DPs with the K5 reduction kernel.
"""
from __future__ import annotations

import itertools
import zlib

import torch

from ..crypto import elgamal as eg
from ..ops import encoding as enc
from ..parallel import ec_collectives as ec
from ..utils import timers


def all_possible_groups(group_by_values) -> list:
    """unlynx AllPossibleGroups: every combination of category indices."""
    vals = [int(v) for v in (group_by_values or [1])]
    return [list(g) for g in itertools.product(*[range(v) for v in vals])]


def _seed(survey_id: str, dp_id: str) -> int:
    return zlib.crc32(f"{survey_id}/{dp_id}".encode()) & 0x7FFFFFFF


def generate_fake_data(op, nbr_rows: int, lo: int, hi: int, device, gen: torch.Generator):
    """createFakeDataForOperation: NbrInput columns of uniform ints in [lo, hi]."""
    n_in = max(1, op.NbrInput)
    t = torch.randint(lo, hi + 1, (n_in, max(1, nbr_rows)), generator=gen, dtype=torch.int64)
    if torch.device(device).type == "cuda":
        # one pinned, asynchronous upload: a pageable copy per column waits for
        # the previous DP's kernels, which serialised thousands of small DPs
        t = t.pin_memory().to(device, non_blocking=True)
    return list(t.unbind(0))


def generate_lr_data(params, device, gen: torch.Generator):
    """Synthetic LR records (data_collection_protocol.go:226-241 dummy rows):
    features uniform in [0, 4) as float64, labels uniform {0,1}; generated on
    the DP's device so 1e6-record DPs never touch the host."""
    n, m = int(params.NbrRecords), int(params.NbrFeatures)
    g = torch.Generator(device=device) if torch.device(device).type == "cuda" else gen
    if torch.device(device).type == "cuda":
        g.manual_seed(int(gen.initial_seed()))
    X = torch.randint(0, 4, (n, m), generator=g, device=device).to(torch.float64)
    y = torch.randint(0, 2, (n,), generator=g, device=device)
    return X, y


def dp_encode(ctx, sq, dp, sync_timer: bool = True) -> dict:
    """Encode one DP's response for every group. Returns a dict with the
    stacked CipherVector (groups x NbrOutput), per-group proof batches, clear values."""
    q = sq.Query
    op = q.Operation
    device = ctx.device
    pk = eg.pk_table(sq.RosterServers.aggregate(), device)
    gen = torch.Generator().manual_seed(_seed(sq.SurveyID, dp.id))
    data = lr = None
    if op.NameOp == "logistic regression":
        if ctx.dp_data and dp.id in ctx.dp_data:
            lr = ctx.dp_data[dp.id]
        else:
            lr = generate_lr_data(op.LRParameters, device, gen)
    else:
        if ctx.dp_data and dp.id in ctx.dp_data:
            data = ctx.dp_data[dp.id]
        else:
            g = q.DPDataGen
            data = generate_fake_data(op, g.GenerateRows, g.GenerateDataMin, g.GenerateDataMax, device, gen)
    groups = all_possible_groups(q.DPDataGen.GroupByValues)
    with_proofs = q.Proofs != 0 and q.Ranges is not None and q.IVSigs.InputValidationSigs is not None \
        and not all(r[0] == 0 and r[1] == 0 for r in q.Ranges)
    cf = q.CuttingFactor
    op_eff = op
    if cf:
        import copy

        op_eff = copy.copy(op)
        op_eff.NbrOutput = op.NbrOutput // cf
    cvs, proofs, clears = [], [], []
    with timers.timed(f"{dp.id}_DPencoding", sync=sync_timer):
        for _ in groups:
            r = enc.encode(data, pk, op_eff, ranges=q.Ranges, with_proofs=with_proofs, lr_data=lr)
            cv = r.cv
            if cf:
                cv = eg.CipherVector.cat([cv] * cf)
            cvs.append(cv)
            proofs.append(r.proofs)
            clears.append(r.clear)
    return {"cv": eg.CipherVector.cat(cvs), "proofs": proofs, "clear": clears, "n_groups": len(groups)}


def data_collection(ctx, sq) -> tuple:
    """Run every local DP, route responses to their CN's rank, sum per CN.

    Returns (cn_sums: {cn_id: CipherVector}, cn_inputs: {cn_id: {dp_id: CipherVector}},
    dp_results: {dp_id: dict}) for the parties hosted on this rank."""
    cl = ctx.cluster
    dp_to_cn = {}
    for cn_id, dps in sq.ServerToDP.items():
        for si in dps or []:
            dp_to_cn[si.id] = cn_id
    dp_results, items = {}, []
    local_dps = [dp for dp in cl.local(ctx.rank, "dp") if dp.id in dp_to_cn]
    # the per-DP timer syncs the device only for a handful of DPs per rank: with
    # thousands (ScaleDPs, one record each) the syncs serialise the encoders
    sync_timer = len(local_dps) <= 16
    for dp in local_dps:
        res = dp_encode(ctx, sq, dp, sync_timer)
        dp_results[dp.id] = res
        cn = cl.by_id(dp_to_cn[dp.id])
        items.append((cn.rank, dp.id, res["cv"]))
    with timers.timed("DataCollectionRoute"):
        got = ec.route(ctx.comm, items, ctx.key_index)
    cn_inputs, cn_sums = {}, {}
    for cn in cl.local(ctx.rank, "cn"):
        inputs = {si.id: got[si.id] for si in (sq.ServerToDP.get(cn.id) or []) if si.id in got}
        cn_inputs[cn.id] = inputs
        with timers.timed(f"{cn.id}_DataCollectionProtocol"):
            if inputs:
                cn_sums[cn.id] = eg.CipherVector.sum(list(inputs.values()))
    return cn_sums, cn_inputs, dp_results
