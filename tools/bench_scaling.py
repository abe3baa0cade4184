"""Scaling sweeps of the reference's TIFS sheets on one MI355X.

Reference (simul/test_data/graphs/TIFS/AllResults.xlsx, BASELINE.md / SURVEY.md §6;
CPU cluster, 100 Mbps / 20 ms links; plots scalingServers.py, scalingVNs.py,
threshold.py):
  * ScaleServers rows 5-12: 6 -> 48 CNs, 10 DPs in total: 1.87 -> 5.25 s
  * ScaleVNs rows 5-26: 7 -> 42 VNs, threshold 1.0: 9.45 -> 25.04 s;
    threshold 0.3: 6.07 -> 15.8 s
  * ScaleDPs rows 5-8 / 10-13: 600 -> 600k records with #DPs = #records:
    9.7 / 62.9 / 489 / 3287 s; with 10 DPs: 2.2 / 3.4 / 3.8 / 4.4 s
  * Threshold rows 5-13, 26: (T, T_sub) = (1, 1) 8.75 s ... (0.2, 0.2) 4.35 s;
    (0, 0) 2.15 s
Only the end points of each sweep are quoted in the survey, so
``reference_s`` is null for the points between them.

Every point is one complete verifiable ``sum`` survey (range proofs (16, 16),
every CN signs its input-validation set, skipchain block) with all parties on
one GPU in one process.  It is the median of ``reps`` runs after one warm-up
(signature and decryption tables).  Output: one JSON line per point.

    python tools/bench_scaling.py [reps] [sweep,...]   # sweeps: servers, vns, threshold
"""
import json
import statistics
import sys
import tempfile
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from drynx_amd.services.api import DrynxClient  # noqa: E402
from drynx_amd.services.local import local_cluster, make_survey  # noqa: E402

RANGES = [16, 16]


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def _point(dev, n_cns, n_dps, n_vns, thresholds, reps, rows=10):
    cl, node = local_cluster(n_cns, n_dps, n_vns, device=dev, workdir=tempfile.mkdtemp(prefix="drynx_scale_"))
    client = DrynxClient(node, device=dev)
    times, codes = [], set()
    for i in range(reps + 1):
        sq = make_survey(client, cl, "sum", query_min=0, query_max=100, rows=rows, proofs=1, ranges=RANGES,
                         thresholds=thresholds, sig_device=dev, deterministic_sigs=True)
        _sync(dev)
        t0 = time.perf_counter()
        _, vals, res = client.send_survey_query(sq)
        _sync(dev)
        dt = time.perf_counter() - t0
        expect = sum(v[0][0] for v in res.clear_dp.values())
        assert int(vals[0][0]) == expect, (vals, expect)
        codes |= set(res.block.data_block().Proofs.values()) if res.block is not None else set()
        if i:
            times.append(dt)
    node.close(remove=True)
    return statistics.median(times), sorted(codes)


def main():
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    sweeps = set(sys.argv[2].split(",")) if len(sys.argv) > 2 else {"servers", "vns", "threshold", "dps"}
    full = [1.0, 1.0, 1.0, 0.0, 1.0]  # [general, aggregation, range, obfuscation, keyswitch] (api.go:79-83)
    points = []
    if "servers" in sweeps:
        for n, ref in ((6, 1.87), (12, None), (24, None), (48, 5.25)):
            points.append(("ScaleServers", dict(cns=n, dps=10, vns=3), full, ref))
    if "vns" in sweeps:
        for thr, refs in ((1.0, {7: 9.45, 42: 25.04}), (0.3, {7: 6.07, 42: 15.8})):
            for n in (7, 14, 28, 42):
                t = [thr, 1.0, 1.0, 0.0, 1.0]
                points.append((f"ScaleVNs threshold {thr}", dict(cns=3, dps=10, vns=n), t, refs.get(n)))
    if "threshold" in sweeps:
        for (T, Ts), ref in (((1.0, 1.0), 8.75), ((0.6, 0.6), None), ((0.2, 0.2), 4.35), ((0.0, 0.0), 2.15)):
            points.append((f"Threshold (T, T_sub) = ({T}, {Ts})", dict(cns=3, dps=10, vns=3), [T, Ts, Ts, 0.0, Ts],
                           ref))
    if "dps" in sweeps:
        # ScaleDPs: 600 ... 600k records held by #DPs = #records (rows 5-8) or by 10 DPs (rows 10-13)
        for total, ref in ((600, 2.2), (6000, 3.4), (60000, 3.8), (600000, 4.4)):
            points.append((f"ScaleDPs 10 DPs, {total} records", dict(cns=3, dps=10, vns=3, rows=total // 10), full,
                           ref))
        for total, ref in ((600, 9.7), (6000, 62.9)):
            points.append(("ScaleDPs #DPs = #records", dict(cns=3, dps=total, vns=3, rows=1), full, ref))
    for label, topo, thr, ref in points:
        sec, codes = _point(dev, topo["cns"], topo["dps"], topo["vns"], thr, reps, topo.get("rows", 10))
        print(json.dumps({"sweep": label, **topo, "seconds": round(sec, 4), "reference_s": ref,
                          "speedup": round(ref / sec, 1) if ref else None, "proof_codes": codes}), flush=True)


if __name__ == "__main__":
    main()
