"""One rank's share of the W-rank setup, measured on ONE GPU.

The setup a W-rank bench pays before its first timed query (bench.py
``setup_s``) is dominated by the prover's comb tables of the signature set
(GLS-8 layout, ~114 GB for the bench's 3-CN SPECTF-shaped set): at W > 1
every rank builds points [k n / W, (k+1) n / W) and the slices are then
broadcast into every rank's full table (``SigMaterial.attach_shard`` /
``_prover_tables4``, RCCL over xGMI).  This tool times, on one GPU:

* ``sigs_s``: the CN input-validation keys and signatures (``make_survey``);
* ``build_full_s``: the whole table build (what the 1-GPU bench pays);
* ``build_share_s``: rank k's 1/W of it, through the same sharded code path
  with an emulated communicator whose ``broadcast_into`` lands the other
  ranks' slices by HBM copies (``landing_hbm_s``: the write side of the
  broadcast at the device's copy rate, a lower bound for the real receive);
* ``recv_bytes``: what rank k receives, and ``xgmi_s`` at the assumed
  per-rank receive rate ``--xgmi-gbs`` (stated, not measured: no multi-GPU
  box is available to this tool).

``projected_setup_s`` = bench setup_s (``--bench-json``) - build_full_s +
build_share_s + max(landing_hbm_s, xgmi_s).

Usage: python tools/setup_share.py [--world 8] [--rank 0] [--bench-json f] [--json-out f]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from drynx_amd.query import LogisticRegressionParameters  # noqa: E402
from drynx_amd.services.api import DrynxClient  # noqa: E402
from drynx_amd.services.local import local_cluster, make_survey  # noqa: E402
from drynx_amd.utils import timers  # noqa: E402


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


class EmuShard:
    """Rank ``rank`` of a ``world``-rank communicator on one GPU: the table
    layout agreement is trivial and a broadcast from another rank lands as an
    HBM copy of this rank's own (equally sized) slice into the target view."""

    def __init__(self, world, rank, dev):
        self.world, self.rank, self.dev = world, rank, dev
        self.landing_s, self.recv_bytes = 0.0, 0
        self.first_landing = None  # perf_counter() when the first slice lands (the build loop has drained)

    def all_gather_object(self, obj):
        return [obj] * self.world

    def broadcast_into(self, t, src):
        if src == self.rank:
            return t
        base = t._base if t._base is not None else t
        m = t.shape[0]
        # a same-sized source region of the same table that does not overlap the target
        off = (t.storage_offset() - base.storage_offset()) // t.shape[1]
        own = base[:m] if off >= m else base[base.shape[0] - m:]
        _sync()
        t0 = time.perf_counter()
        if self.first_landing is None:
            self.first_landing = t0
        t.copy_(own)
        _sync()
        self.landing_s += time.perf_counter() - t0
        self.recv_bytes += t.numel() * t.element_size()
        return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--features", type=int, default=44)
    ap.add_argument("--xgmi-gbs", type=float, default=150.0,
                    help="assumed per-rank receive rate of the table broadcasts (GB/s): one xGMI link's worth")
    ap.add_argument("--bench-json", default=None, help="1-GPU bench.py JSON (its setup_s)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--mode", choices=("share", "full"), default="share")
    ap.add_argument("--full-json", default=None, help="JSON of a --mode full run (its build_full_s)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    n_cns, n_dps, n_vns, d = 3, 10, 3, a.features
    cl, node = local_cluster(n_cns, n_dps, n_vns, device=dev, workdir=tempfile.mkdtemp(prefix="drynx_setup_"))
    lp = LogisticRegressionParameters(NbrRecords=1_000_000, NbrFeatures=d, Means=[2.0] * d,
                                      StandardDeviations=[1.15] * d, Lambda=1.0, Step=0.012, MaxIterations=450,
                                      InitialWeights=[0.1] * (d + 1), K=2, PrecisionApproxCoefficients=100.0)
    client = DrynxClient(node, device=dev)
    _sync()
    t = time.perf_counter()
    sq = make_survey(client, cl, "logistic regression", proofs=1, ranges=[16, 16, 1 << 62], lr_params=lp,
                     thresholds=[1.0, 1.0, 1.0, 0.0, 1.0], sig_device=dev)
    _sync()
    sigs_s = time.perf_counter() - t
    sm = node.verifier_cache.sigmat(sq, dev)
    mode = sm.table_mode(dev) or 4
    res = {"world": a.world, "rank": a.rank, "features": d, "table_mode": mode, "distinct_points": sm.n_distinct,
           "sigs_s": round(sigs_s, 3)}

    def build(label):
        with timers.span(f"setup.build[{label}]"):
            return _build()

    def _build():
        old = sm._ptab.pop((mode, str(dev)), None)
        del old  # the previous build's tables are freed before the next one allocates its own
        if dev.type == "cuda":
            torch.cuda.empty_cache()
            res.setdefault("hbm_in_use_before_build_gb", []).append(round(torch.cuda.memory_allocated() / 1e9, 2))
        _sync()
        t0 = time.perf_counter()
        sm._prover_tables4(dev, mode)
        _sync()
        return t0, time.perf_counter() - t0

    sm.attach_shard(None, False)
    # ONE build per process, as a real rank allocates its tables once: a
    # second ~110 GB allocation after a free stalled 3-6 s before its build
    # started on some boxes, whichever build it was (profiles/r5/final/,
    # profiles/r5/final2/setup_host_trace.txt).  --mode full: the whole
    # 1-rank build (module / kernel first-use costs included, as in bench.py's
    # setup_s); --mode share (default): this rank's share, with build_full_s
    # taken from a --full-json of the other mode
    if a.mode == "full":
        res["build_full_s"] = round(build("full")[1], 3)
        res["table_bytes"] = sm.table_bytes()
        print(json.dumps(res), flush=True)
        if a.json_out:
            json.dump(res, open(a.json_out, "w"), indent=1)
        timers.dump_trace()
        node.close(remove=True)
        return
    if a.full_json:
        res["build_full_s"] = json.load(open(a.full_json))["build_full_s"]
    emu = EmuShard(a.world, a.rank, dev)
    sm._shard = emu  # as attach_shard does for a W-rank communicator
    t0, total = build("share")
    res["table_bytes"] = sm.table_bytes()
    res["landing_hbm_s"] = round(emu.landing_s, 3)
    res["build_share_s"] = round((emu.first_landing or (t0 + total)) - t0, 3)
    res["share_total_s"] = round(total, 3)
    res["recv_bytes"] = emu.recv_bytes
    res["xgmi_gbs_assumed"] = a.xgmi_gbs
    res["xgmi_s"] = round(emu.recv_bytes / (a.xgmi_gbs * 1e9), 3)
    if a.bench_json and "build_full_s" in res:
        b = json.load(open(a.bench_json))
        res["bench_setup_s"] = b["setup_s"]
        res["projected_setup_s"] = round(b["setup_s"] - res["build_full_s"] + res["build_share_s"]
                                         + max(res["landing_hbm_s"], res["xgmi_s"]), 3)
    print(json.dumps(res), flush=True)
    if a.json_out:
        json.dump(res, open(a.json_out, "w"), indent=1)
    timers.dump_trace()  # DRYNX_TRACE=<path>: the builds' host spans
    node.close(remove=True)


if __name__ == "__main__":
    main()
