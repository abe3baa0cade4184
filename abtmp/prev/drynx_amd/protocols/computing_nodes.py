"""Computing-node protocols: collective aggregation, obfuscation, DRO noise
shuffle and collective key switching.

Reference:
  * CollectiveAggregation (unlynx, binary CN tree; services/service.go:515-560,
    :775-790)
  * Obfuscation (protocols/obfuscation_protocol.go:113-314): every CN
    multiplies each ciphertext by a fresh secret and the tree sums -> root
    holds (sum_i s_i) C
  * DRO (unlynx ShufflingProtocol as DROProtocolName; services/service.go
    :619-665, :810-830): encrypted Laplace noise list shuffled + re-randomised
    by every CN in sequence
  * KeySwitching (unlynx; services/service.go:566-616, :854-868): root adds the
    noise (:600-604), every CN adds its share (v B, v Q - x K), shares summed
MI355X mapping: the tree sweeps become ``sum_to_root`` / ``broadcast_cv`` EC
collectives (exchange over xGMI + K5 HIP reduction), the shuffle chain a
send/recv ring.
"""
from __future__ import annotations

import torch

from .. import native as nt
from ..crypto import bn254 as bn
from ..crypto import elgamal as eg
from ..parallel import ec_collectives as ec
from ..proofs import aggregation_shuffle as ags
from ..proofs import shuffle
from ..proofs import requests as prq
from ..proofs import sigma
from ..query import add_diff_p
from ..utils import timers


def _root_rank(ctx, sq) -> int:
    return ctx.cluster.by_id(sq.RosterServers.list[0].id).rank


def collective_aggregation(ctx, sq, cn_sums: dict, cn_inputs: dict, n_rows: int, proofs: list):
    """Sum every CN's DP aggregate onto the root CN; each CN publishes an
    aggregation proof (its inputs + its claimed sum).  The proofs (packed
    device tensors, digest, signature) are finished on the node's proof worker
    while the aggregation proceeds (the reference's ProofFunc runs in its own
    goroutine, service.go:533-560)."""
    root = _root_rank(ctx, sq)
    local, items = [], []
    roster = {s.id for s in sq.RosterServers.list}
    for cn in ctx.cluster.local(ctx.rank, "cn"):
        if cn.id not in roster:
            continue
        with timers.timed(f"{cn.id}_AggregationPhase"):
            s = cn_sums.get(cn.id) or eg.CipherVector.zeros(n_rows, ctx.device)
            local.append(s)
            if sq.Query.Proofs:
                pr = ags.aggregation_list_proof_creation(list(cn_inputs.get(cn.id, {}).values()), s)
                items.append(("aggregation", pr, cn.id, "", cn.keypair.secret))
    if items:
        proofs.append(ctx.defer_proofs(prq.new_proof_requests, items, sq.SurveyID))
    with timers.timed("CollectiveAggregation"):
        return ec.sum_to_root(ctx.comm, local, n_rows, root)


def obfuscation(ctx, sq, agg, n_rows: int, proofs: list):
    root = _root_rank(ctx, sq)
    agg = ec.broadcast_cv(ctx.comm, agg, n_rows, root)
    local, pend = [], []
    for cn in ctx.cluster.local(ctx.rank, "cn"):
        with timers.timed(f"{cn.id}_ObfuscationPhase"):
            s = bn.random_scalars(n_rows, ctx.device)
            co = agg.mul_scalars(s)
            local.append(co)
            if sq.Query.Proofs:
                pend.append((cn, co, s))
    if pend:
        def finish(agg=agg, pend=pend):
            items = [("obfuscation", sigma.obfuscation_list_proof_creation(agg, co, s), cn.id, "", cn.keypair.secret)
                     for cn, co, s in pend]
            return prq.new_proof_requests(items, sq.SurveyID)
        proofs.append(ctx.defer_proofs(finish))
    return ec.sum_to_root(ctx.comm, local, n_rows, root)


def dro_phase(ctx, sq, proofs: list):
    """Differential-privacy noise: root creates the trivially-encrypted noise
    list, every CN (in roster order) shuffles + re-randomises it under the
    collective key (with a shuffle proof); returns the final list on the root."""
    if not add_diff_p(sq.Query.DiffP):
        return None
    d = sq.Query.DiffP
    P = sq.RosterServers.aggregate()
    cns = [ctx.cluster.by_id(si.id) for si in sq.RosterServers.list]
    n = int(d.NoiseListSize)
    cur = None
    if ctx.rank == cns[0].rank:
        noise = ags.generate_noise_values_scale(n, d.LapMean, d.LapScale, d.Quanta, d.Scale or 1.0, d.Limit)
        m = torch.tensor(noise, dtype=torch.int64, device=ctx.device)
        C = nt.g1_fb_mul_i64(bn.base_table(ctx.device), m)  # IntArrayToCipherVector: (0, v B)
        cur = eg.CipherVector(bn.g1_infinity_jac(n, ctx.device), C)
    holder = cns[0].rank
    with timers.timed("DROPhase"):
        for idx, cn in enumerate(cns):
            if cn.rank != holder:  # hand the list to the next CN's rank (ring send/recv)
                if ctx.rank == holder:
                    ctx.comm.send(ec.cv_to_rows(cur).reshape(-1), cn.rank)
                elif ctx.rank == cn.rank:
                    cur = ec.rows_to_cv(ctx.comm.recv(n * ec.ROW, holder))
                holder = cn.rank
            if ctx.rank == cn.rank:
                Y, perm, rho = ags.shuffle_sequence(cur, P)
                if sq.Query.Proofs:
                    pr = shuffle.prove(cur, Y, perm, rho, P)
                    proofs.append(prq.new_proof_request("shuffle", pr, sq.SurveyID, cn.id, "", cn.keypair.secret))
                cur = Y
        root = cns[0].rank
        if holder != root:
            if ctx.rank == holder:
                ctx.comm.send(ec.cv_to_rows(cur).reshape(-1), root)
            elif ctx.rank == root:
                cur = ec.rows_to_cv(ctx.comm.recv(n * ec.ROW, holder))
    return cur if ctx.rank == cns[0].rank else None


def key_switching(ctx, sq, agg, n_groups: int, n_out: int, noise, proofs: list):
    """Switch the root's aggregate from the collective key to the querier key."""
    root = _root_rank(ctx, sq)
    n_rows = n_groups * n_out
    if ctx.rank == root and noise is not None and len(noise) > 0:
        # survey.QueryResponseState.Data[i].Add(v.Data, Noises[:len(v.Data)]) for every group
        k = min(n_out, len(noise))
        idx = torch.arange(n_rows, device=ctx.device) % n_out
        take = idx < k
        noise_rows = eg.CipherVector.zeros(n_rows, ctx.device)
        sel = torch.nonzero(take).reshape(-1)
        noise_rows.K[sel] = noise.K[idx[sel]]
        noise_rows.C[sel] = noise.C[idx[sel]]
        agg = agg.add(noise_rows)
    agg = ec.broadcast_cv(ctx.comm, agg, n_rows, root)
    Q = sq.ClientPubKey
    local_K = []
    cns = [cn for cn in ctx.cluster.local(ctx.rank, "cn") if cn.id in {s.id for s in sq.RosterServers.list}]
    if cns:
        # all co-located CNs in one batch of launches (short vectors are latency-bound);
        # the proofs' challenges / responses / envelopes finish on the proof worker
        with timers.timed("KeySwitchingPhase"):
            local_K, pend = sigma.key_switch_shares_batch([c.keypair.secret for c in cns], [c.public for c in cns],
                                                          agg.K, Q, bool(sq.Query.Proofs))
        if pend is not None:
            def finish(pend=pend, cns=cns):
                prs = sigma.finish_keyswitch_proofs(pend)
                return prq.new_proof_requests([("keyswitch", pr, cn.id, "", cn.keypair.secret)
                                               for cn, pr in zip(cns, prs)], sq.SurveyID)
            proofs.append(ctx.defer_proofs(finish, lane="_late"))
    total = ec.sum_to_root(ctx.comm, local_K, n_rows, root)
    if ctx.rank != root:
        return None
    # (K', C') = (sum v B, C + sum (v Q - x K))
    return eg.CipherVector(total.K, nt.g1_add(agg.C, total.C))
