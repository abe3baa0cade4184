"""Emulated party-to-party network (the simulation's Bandwidth / Delay).

Reference: the onet simulation runs every party on its own host and shapes
the links (``Bandwidth = 100`` Mbps, ``Delay = 20`` ms in
simul/runfiles/drynx.toml:6-7; the published "Bandwith" sheet sweeps them).
Here parties share GPUs and talk over xGMI or in memory, so the emulated
network is applied per protocol step, at the point of the flow where the
reference sends its messages:

* every step is a set of messages (sender party, receiver party, bytes in the
  reference's wire format: CipherText 128 B, range proof ~256 + 32 l +
  544 S l B per value, ... SURVEY 2.4) plus the number of sequential hops it
  needs (a star announcement + reply is 2, a binary CN tree up and down 2 x
  depth);
* each party has one full-duplex interface of ``bandwidth_mbps``: a step
  lasts ``hops * delay + max over parties (bytes out, bytes in) / bandwidth``;
* ``mode="sleep"`` waits that long where the step happens (every rank
  computes the same global step, so ranks stay in step); ``"account"`` only
  records it.  Each step is recorded under the timer ``net_<step>`` and the
  total under ``NetworkEmulated``.

Flows that the reference overlaps with computation (range proofs streamed to
the VNs while the CNs aggregate) are charged where this framework sends them
(proof collection after the CN phases): a conservative model.
"""
from __future__ import annotations

import os
import time
from collections import defaultdict

from ..utils import timers

# reference wire sizes (range_proof.go:89-155, structs.go:403)
CT_BYTES = 128
POINT_BYTES = 64
SCALAR_BYTES = 32
SIG_BYTES = 96


def range_proof_bytes(u: int, l: int, S: int) -> int:
    """One value's range proof on the wire (Commit, c, Zr, D, Zphi, Zv, V, A)."""
    if u == 0 and l == 0:
        return CT_BYTES
    return 256 + 32 * l + 544 * S * l


class NetEmulator:
    def __init__(self, bandwidth_mbps: float, delay_ms: float, mode: str = "sleep"):
        if mode not in ("sleep", "account"):
            raise ValueError(f"unknown network emulation mode {mode}")
        self.bw = float(bandwidth_mbps) * 1e6 / 8.0  # bytes / s
        self.delay = float(delay_ms) / 1e3
        self.mode = mode
        self.total = 0.0

    @staticmethod
    def from_env():
        """DRYNX_NETEM="<Mbps>,<delay ms>[,sleep|account]" (simulation runs)."""
        spec = os.environ.get("DRYNX_NETEM", "").strip()
        if not spec:
            return None
        parts = [p.strip() for p in spec.split(",")]
        return NetEmulator(float(parts[0]), float(parts[1]), parts[2] if len(parts) > 2 else "sleep")

    def step_time(self, msgs, hops: int = 1) -> float:
        out_b, in_b = defaultdict(int), defaultdict(int)
        for src, dst, n in msgs:
            if src == dst:
                continue
            out_b[src] += int(n)
            in_b[dst] += int(n)
        worst = max([0] + list(out_b.values()) + list(in_b.values()))
        return hops * self.delay + (worst / self.bw if self.bw > 0 else 0.0)

    def step(self, name: str, msgs, hops: int = 1) -> float:
        t = self.step_time(list(msgs), hops)
        self.total += t
        timers.record(f"net_{name}", t)
        timers.record("NetworkEmulated", t)
        if self.mode == "sleep" and t > 0:
            time.sleep(t)
        return t


# ---------------------------------------------------------------- reference flows
# Sequential one-way messages ("hops") on the critical path of each step of a
# reference query, read off the reference sources; every step's messages are
# charged with these counts (the simulation's Delay per hop).  Transport
# overhead that the reference sources do not show (onet's websocket setup per
# client call, tree propagation to nodes that do not know a protocol's tree)
# is NOT in these counts: ``DRYNX_NETEM_SETUP_HOPS`` adds that many hops per
# client call and per new protocol tree when set (default 0).
def setup_hops() -> int:
    return int(os.environ.get("DRYNX_NETEM_SETUP_HOPS", "0"))


def flow_hops(step: str, n_cns: int = 3, n_vns: int = 3, cns_with_dps: int = 1, genesis: bool = False) -> int:
    """Hops of one reference step (the table below cites the reference flow
    of each); ``n_*`` size the CN / VN trees."""
    d_cn, d_vn = tree_depth(n_cns), tree_depth(n_vns)
    st = setup_hops()
    table = {
        # simul client -> every VN, one request/reply after the other
        # (api_skipchain.go SendSurveyQueryToVNs loop; drynx_simul.go:382-393)
        "query_vns": n_vns * (2 + st),
        # client -> root CN request (api.go SendSurveyQuery; the reply is "result")
        "query_client": 1 + st,
        # root CN -> CNs and DPs (service.go:319-339), DPs' DPqueryReceived
        # back (service_data_provider.go), CNs' SyncDCP (service.go:367-378,
        # sent by the other CNs on arrival, so it is there with the DP acks)
        "query_dissemination": 2,
        # DataCollection star announce + reply (data_collection_protocol.go),
        # then DPdataFinished among the CNs (service.go:391-408): one more hop
        # when several CNs collect from DPs and finish together
        "data_collection": 2 + st + (1 if cns_with_dps > 1 else 0),
        # unlynx collective aggregation / obfuscation / key switching: the
        # binary CN tree down (announcement) and up (reply)
        # (service.go:667-700 GenerateNaryTreeWithRoot(2, root))
        "aggregation": 2 * d_cn + st,
        "obfuscation": 2 * d_cn + st,
        "key_switching": 2 * d_cn + st,
        "dro": n_cns,
        # root CN -> client reply
        "result": 1,
        # the last proofs (key switch) leave their CN when the key switching
        # ends: prover -> VN (proof_collection_protocol.go:154-165)
        "proofs_to_vns": 1 + st,
        # non-root VN -> root VN BitmapCollectionMessage (:360-372)
        "bitmaps": 1,
        # cothority skipchain store: BFT-CoSi prepare + commit over the VN tree
        # (down + up each) for the new block, the same for the previous block's
        # forward link, then the block's propagation to the roster (announce +
        # ack); the genesis has no forward link (service_skipchain.go:120-150)
        "skipchain": 4 * max(1, d_vn) * (1 if genesis else 2) + 2,
        # root VN -> client: the pending SendEndVerification reply (:158, :164-169)
        "end_verification": 1,
        # simul client -> every VN CloseDB, one after the other (api_skipchain.go SendCloseDB)
        "close_db": n_vns * (2 + st),
        # simul client -> a VN GetLatestBlock request/reply, and that VN's
        # skipchain GetUpdateChain request/reply (service_skipchain.go:185-200)
        "latest_block": 4 + 2 * st,
    }
    return table[step]


def tree_depth(n: int) -> int:
    """Depth of onet's binary tree over n nodes (GenerateNaryTreeWithRoot(2, root))."""
    d, cap = 0, 1
    while cap < n:
        d += 1
        cap += 2 ** d
    return d


def tree_edges(ids: list) -> list:
    """(child, parent) edges of the binary tree over ``ids`` rooted at ids[0]."""
    return [(ids[i], ids[(i - 1) // 2]) for i in range(1, len(ids))]
