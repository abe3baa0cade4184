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
import time
import zlib

import torch

from ..crypto import elgamal as eg
from ..ops import encoding as enc
from ..parallel import ec_collectives as ec
from ..query import lr_nbr_outputs
from ..utils import timers


def all_possible_groups(group_by_values) -> list:
    """unlynx AllPossibleGroups: every combination of category indices."""
    vals = [int(v) for v in (group_by_values or [1])]
    return [list(g) for g in itertools.product(*[range(v) for v in vals])]


def expected_n_out(sq) -> int | None:
    """Ciphertexts per group every DP of the survey encodes, from the query
    alone (None when it does not say): ranks hosting no DP size the CN phases
    with it instead of asking the others (one control round fewer)."""
    q = sq.Query
    op = q.Operation
    cf = max(1, q.CuttingFactor or 1)
    if op.NameOp == "logistic regression":
        p = op.LRParameters
        return None if p is None else lr_nbr_outputs(p.NbrFeatures, p.K) * cf
    return (op.NbrOutput // cf) * cf if op.NbrOutput > 0 else None


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


def _with_proofs(q) -> bool:
    return q.Proofs != 0 and q.Ranges is not None and q.IVSigs.InputValidationSigs is not None \
        and not all(r[0] == 0 and r[1] == 0 for r in q.Ranges)


def dp_encode_batch(ctx, sq, dps: list) -> dict:
    """Encode every DP of ``dps`` as ONE batch: their records are stacked into
    one matrix (one pinned upload), the outputs of all DPs come from one K14
    launch (or one bincount / scatter for histograms and bit encodings), all
    ciphertexts of all groups from one encryption launch, and the values reach
    the host in one copy (the clear results and the provers' inputs).

    Same per-DP data (seeds), outputs, group replication and CuttingFactor
    replication as :func:`dp_encode`; returns ``{dp_id: result}`` in its format.
    The reference encodes DP by DP (data_collection_protocol.go:178-373); with
    thousands of one-record DPs (ScaleDPs) per-DP launch sequences and syncs
    were the whole cost."""
    q = sq.Query
    op = q.Operation
    device = torch.device(ctx.device)
    pk = eg.pk_table(sq.RosterServers.aggregate(), device)
    g = q.DPDataGen
    groups = all_possible_groups(g.GroupByValues)
    if op.NameOp == "logistic regression":
        return _encode_batch_tail(ctx, sq, dps, _lr_values(ctx, sq, dps, device), groups, pk)
    n_in = max(1, op.NbrInput)
    mats, rows = [], []
    for dp in dps:
        if ctx.dp_data and dp.id in ctx.dp_data:
            cols = [enc._t(c, device).reshape(-1).to(torch.int64) for c in ctx.dp_data[dp.id]]
            mats.append(torch.stack(cols, dim=1))
        else:  # generate_fake_data's draw, kept on the host until the one upload below
            gen = torch.Generator().manual_seed(_seed(sq.SurveyID, dp.id))
            t = torch.randint(g.GenerateDataMin, g.GenerateDataMax + 1, (n_in, max(1, g.GenerateRows)), generator=gen,
                              dtype=torch.int64)
            mats.append(t.t())
        rows.append(mats[-1].shape[0])
    if all(m.device.type == "cpu" for m in mats):
        Z = torch.cat(mats).contiguous()
        if device.type == "cuda":
            Z = Z.pin_memory().to(device, non_blocking=True)
    else:
        Z = torch.cat([m.to(device) for m in mats]).contiguous()
    vals = enc.batch_values(op.NameOp, Z, rows, op.QueryMin, op.QueryMax)  # [n_dp, n_out]
    return _encode_batch_tail(ctx, sq, dps, vals, groups, pk)


def _lr_values(ctx, sq, dps: list, device) -> torch.Tensor:
    """[n_dp, n_out] int64 coefficient vectors of every DP's logistic-regression
    data (the fused fp64-MFMA encoder per DP, no host round trip in between)."""
    from ..models.logistic_regression import encode_coefficients_int, encode_coefficients_int_many, n_coeffs

    op = sq.Query.Operation
    params = op.LRParameters
    data = []
    for dp in dps:
        if ctx.dp_data and dp.id in ctx.dp_data:
            X, y = ctx.dp_data[dp.id]
        else:
            X, y = generate_lr_data(params, device, torch.Generator().manual_seed(_seed(sq.SurveyID, dp.id)))
        data.append((X, y))
    if device.type == "cuda":
        # every DP of the rank through the fused encoder at once: one reduction and
        # one rounding pass instead of ~20 launches per DP on the critical path
        Xs = [torch.as_tensor(X, device=device) if X is not None else None for X, _ in data]
        ys = [torch.as_tensor(y, device=device) if y is not None else None for _, y in data]
        many = encode_coefficients_int_many(Xs, ys, params)
        if many is not None:
            return many
    out = []
    for X, y in data:
        if X is None or len(X) == 0:
            out.append(torch.zeros(n_coeffs(params.NbrFeatures, params.K), dtype=torch.int64, device=device))
        else:
            out.append(encode_coefficients_int(torch.as_tensor(X, device=device), torch.as_tensor(y, device=device),
                                               params).to(device))
    return torch.stack(out)


def _encode_batch_tail(ctx, sq, dps: list, vals: torch.Tensor, groups, pk) -> dict:
    """Shared tail of ``dp_encode_batch``: one encryption launch for every
    (DP, group, output), CuttingFactor replication, one host copy, the proof
    batches per DP."""
    q = sq.Query
    op = q.Operation
    device = torch.device(ctx.device)
    ng, cf = len(groups), q.CuttingFactor
    n_dp, n_out = vals.shape
    with_proofs = _with_proofs(q)
    bits = op.NameOp in enc.BIT_OPS and not with_proofs
    # one fresh encryption per (DP, group, output); CuttingFactor replicates a
    # group's ciphertexts cf times (same randomness), as dp_encode does
    cv, r = enc.encrypt_batch(pk, vals[:, None, :].expand(n_dp, ng, n_out), bits)
    rep = max(1, cf or 1)
    idx = (torch.arange(ng, device=device)[:, None, None] * n_out
           + torch.arange(n_out, device=device)[None, None, :]).expand(ng, rep, n_out).reshape(-1)
    per_dp = ng * n_out
    K = cv.K.reshape(n_dp, per_dp, -1)[:, idx]
    C = cv.C.reshape(n_dp, per_dp, -1)[:, idx]
    host = vals.cpu().tolist()
    us = ls = offs = None
    if with_proofs:
        us, ls, offs = enc._ranges_uvl(q.Ranges, n_out)
    out = {}
    for i, dp in enumerate(dps):
        v = host[i]
        proofs = []
        if with_proofs:
            base = i * per_dp
            for j in range(ng):
                lo = base + j * n_out
                proofs.append(enc.CreateProofBatch(list(v), r[lo: lo + n_out], cv[lo: lo + n_out], us, ls,
                                                   list(range(n_out)), offs, vals[i]))
        else:
            proofs = [None] * ng
        out[dp.id] = {"cv": eg.CipherVector(K[i], C[i]), "proofs": proofs, "clear": [list(v) for _ in groups],
                      "n_groups": ng}
    return out


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
    batchable = sq.Query.Operation.NameOp in enc.BATCH_OPS + ("logistic regression",)
    abort = None
    try:
        if local_dps and batchable:
            # every DP of this rank in one batch; each DP's encoding latency is the batch's
            with timers.timed("DPencodingBatch", sync=sync_timer) as t:
                batch = dp_encode_batch(ctx, sq, local_dps)
            dt = time.perf_counter() - t.t0
            for dp in local_dps:
                timers.record(f"{dp.id}_DPencoding", dt)
        else:
            batch = {dp.id: dp_encode(ctx, sq, dp, sync_timer) for dp in local_dps}
    except Exception as e:  # noqa: BLE001 -- a DP that cannot answer aborts the survey on every rank
        abort = f"survey {sq.SurveyID}: a DP of rank {ctx.rank} failed to encode: {type(e).__name__}: {e}"
        batch, local_dps = {}, []
    want = expected_n_out(sq)
    n_groups = len(all_possible_groups(sq.Query.DPDataGen.GroupByValues))
    for dp in local_dps:
        res = batch[dp.id]
        dp_results[dp.id] = res
        cn = cl.by_id(dp_to_cn[dp.id])
        items.append((cn.rank, dp.id, res["cv"]))
        if want is not None and len(res["cv"]) != want * n_groups and abort is None:
            # (raised on EVERY rank by the route's size round, not only here:
            # ranks without DPs would otherwise wait in the CN collectives)
            abort = (f"survey {sq.SurveyID}: DP {dp.id} encoded {len(res['cv']) // max(1, n_groups)} outputs, "
                     f"the query announces {want}")
    with timers.timed("DataCollectionRoute"):
        got = ec.route(ctx.comm, items, ctx.key_index, abort=abort)
    cn_inputs, cn_sums = {}, {}
    for cn in cl.local(ctx.rank, "cn"):
        inputs = {si.id: got[si.id] for si in (sq.ServerToDP.get(cn.id) or []) if si.id in got}
        cn_inputs[cn.id] = inputs
        with timers.timed(f"{cn.id}_DataCollectionProtocol"):
            if inputs:
                cn_sums[cn.id] = eg.CipherVector.sum(list(inputs.values()))
    return cn_sums, cn_inputs, dp_results
