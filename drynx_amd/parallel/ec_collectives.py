"""Elliptic-curve-aware collectives (no RCCL reduction op can add BN254 points).

Ciphertext vectors travel between ranks as raw Jacobian limb tensors
([n, 48] int32 = K||C) — intra-cluster traffic never pays the affine
normalisation / big-endian conversion that the external wire format needs.

* ``route``: personalised all-to-all of keyed CipherVectors (star gather
  DP -> CN of DataCollection, C6; CN -> root of CollectiveAggregation, C8;
  obfuscation / key-switch shares, C9/C11).
* ``sum_to_root``: every rank contributes CipherVectors; the root rank reduces
  them with the K5 kernel.  For long vectors (>= ``shard_threshold`` rows)
  it does a reduce-scatter by ownership (each rank sums 1/W of the rows) and
  gathers the shards to the root — on a full xGMI mesh that is 2 one-hop
  steps instead of a (W-1)-hop ring.
* ``all_reduce_cv``: every rank ends with the sum: the same reduce-scatter
  by ownership, then an all-gather of the reduced shards (C8/C9/C11 when
  every CN needs the aggregate, e.g. to re-randomise it locally).
* ``broadcast_cv``: root -> all ranks.
"""
from __future__ import annotations

import torch

from .. import native as nt
from ..crypto.elgamal import CipherVector
from .comm import Comm

ROW = 48  # K||C Jacobian limbs per ciphertext


def cv_to_rows(cv: CipherVector) -> torch.Tensor:
    return torch.cat([cv.K, cv.C], dim=1)


def rows_to_cv(rows: torch.Tensor) -> CipherVector:
    rows = rows.reshape(-1, ROW)
    return CipherVector(rows[:, :24].contiguous(), rows[:, 24:].contiguous())


def route(comm: Comm, items: list, key_index, abort: str | None = None) -> dict:
    """items: list of (dst_rank, key, CipherVector).  Returns {key: CipherVector}
    of the items addressed to this rank.  ``key_index``: key -> int and back
    (a ``KeyIndex``) shared by all ranks.  Per destination the buffer is
    [count, key_0, n_0, key_1, n_1, ..., rows_0, rows_1, ...]: the receiver
    copies only the 1 + 2 count header words to the host.  ``abort``: this
    rank cannot send (every rank raises, ``Comm.exchange``)."""
    if abort is not None:
        comm.exchange({}, abort=abort)
    per_dst: dict = {}
    for dst, key, cv in items:
        per_dst.setdefault(dst, []).append((key_index.encode(key), len(cv), cv_to_rows(cv).to(comm.device).reshape(-1)))
    outgoing = {}
    for dst, parts in per_dst.items():
        hdr = [len(parts)] + [v for k, n, _ in parts for v in (k, n)]
        outgoing[dst] = torch.cat([torch.tensor(hdr, dtype=torch.int32).to(comm.device)] + [r for _, _, r in parts])
    got = comm.exchange(outgoing)
    out = {}
    srcs = sorted(got)
    if not srcs:
        return out
    # every source's header words in ONE device-to-host copy (up to _HDR_ITEMS
    # items per source; a longer header is fetched on its own)
    H = 1 + 2 * _HDR_ITEMS
    heads = torch.nn.utils.rnn.pad_sequence([got[s][:H] for s in srcs], batch_first=True).cpu().tolist()
    for src, head in zip(srcs, heads):
        buf = got[src]
        n_items = int(head[0])
        if n_items < 0 or 1 + 2 * n_items > buf.numel():
            raise ValueError(f"route: malformed header from rank {src}")
        hdr = head[1: 1 + 2 * n_items] if n_items <= _HDR_ITEMS else buf[1: 1 + 2 * n_items].cpu().tolist()
        off = 1 + 2 * n_items
        for q in range(n_items):
            k, n = hdr[2 * q], hdr[2 * q + 1]
            if n < 0 or off + n * ROW > buf.numel():
                raise ValueError(f"route: item {q} from rank {src} overruns its buffer")
            out[key_index.decode(k)] = rows_to_cv(buf[off: off + n * ROW])
            off += n * ROW
    return out


_HDR_ITEMS = 64


class KeyIndex:
    """Bijective key <-> int map known to every rank (e.g. party ids)."""

    def __init__(self, keys):
        self.keys = list(keys)
        self.idx = {k: i for i, k in enumerate(self.keys)}

    def encode(self, k) -> int:
        return self.idx[k]

    def decode(self, i: int):
        return self.keys[i]


def sum_local(cvs: list) -> CipherVector:
    return CipherVector.sum(cvs)


def sum_to_root(comm: Comm, local_cvs: list, n_rows: int, root: int = 0,
                shard_threshold: int = 1 << 16) -> CipherVector | None:
    """Homomorphically sum CipherVectors held by all ranks onto ``root``.
    Every rank contributes exactly ``n_rows`` rows (zeros if it hosts no
    contributor), so every receive size is known: no size round."""
    local = CipherVector.sum(local_cvs) if local_cvs else CipherVector.zeros(n_rows, comm.device)
    if comm.world == 1:
        return local
    W = comm.world
    if n_rows < shard_threshold:
        known = {s: n_rows * ROW for s in range(W)} if comm.rank == root else {}
        got = comm.exchange({root: cv_to_rows(local)}, recv_sizes=known)
        if comm.rank != root:
            return None
        parts = [rows_to_cv(got[s]) for s in sorted(got)]
        return CipherVector.sum(parts)
    # reduce-scatter by ownership then gather shards at root
    bounds = [(n_rows * i) // W for i in range(W + 1)]
    rows = cv_to_rows(local)
    mine_n = bounds[comm.rank + 1] - bounds[comm.rank]
    got = comm.exchange({d: rows[bounds[d]: bounds[d + 1]] for d in range(W)},
                        recv_sizes={s: mine_n * ROW for s in range(W)})
    mine = CipherVector.sum([rows_to_cv(got[s]) for s in sorted(got)]) if mine_n else None
    known = {s: (bounds[s + 1] - bounds[s]) * ROW for s in range(W)} if comm.rank == root else {}
    got2 = comm.exchange({root: cv_to_rows(mine)} if mine is not None else {}, recv_sizes=known)
    if comm.rank != root:
        return None
    return CipherVector.cat([rows_to_cv(got2[s]) for s in range(W) if s in got2])


def all_reduce_cv(comm: Comm, local_cvs: list, n_rows: int) -> CipherVector:
    """Homomorphic all-reduce: reduce-scatter by row ownership (rank d sums
    rows [b_d, b_{d+1}) of every rank's vector with the K5 kernel), then an
    all-gather of the W reduced shards.  Each rank sends and receives about
    2 (W-1)/W of the vector over one hop of the xGMI mesh: no ring, and no
    size round (every size follows from ``n_rows``)."""
    local = CipherVector.sum(local_cvs) if local_cvs else CipherVector.zeros(n_rows, comm.device)
    if comm.world == 1:
        return local
    W = comm.world
    bounds = [(n_rows * i) // W for i in range(W + 1)]
    rows = cv_to_rows(local)
    mine_n = bounds[comm.rank + 1] - bounds[comm.rank]
    got = comm.exchange({d: rows[bounds[d]: bounds[d + 1]] for d in range(W) if bounds[d + 1] > bounds[d]},
                        recv_sizes={s: mine_n * ROW for s in range(W)})
    known = {s: (bounds[s + 1] - bounds[s]) * ROW for s in range(W)}
    if mine_n:
        mine = cv_to_rows(CipherVector.sum([rows_to_cv(got[s]) for s in sorted(got)]))
        got2 = comm.exchange({d: mine for d in range(W)}, recv_sizes=known)
    else:
        got2 = comm.exchange({}, recv_sizes=known)
    return CipherVector.cat([rows_to_cv(got2[s]) for s in range(W) if s in got2])


def broadcast_cv(comm: Comm, cv: CipherVector | None, n_rows: int, root: int = 0) -> CipherVector:
    if comm.world == 1:
        return cv
    known = {root: n_rows * ROW}
    if comm.rank == root:
        rows = cv_to_rows(cv)
        got = comm.exchange({d: rows for d in range(comm.world)}, recv_sizes=known)
    else:
        got = comm.exchange({}, recv_sizes=known)
    return rows_to_cv(got[root])


def g1_sum_rows(x: torch.Tensor) -> torch.Tensor:
    return nt.g1_sum(x)
