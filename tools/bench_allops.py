"""Every operation of the reference's AllOps benchmark on one MI355X.

Reference: simul/test_data/graphs/TIFS/AllResults.xlsx sheet AllOps (rows
5-18): 3 CNs, 3 VNs, 10 DPs, proofs on, total time per query
(execution + proof overhead) on a CPU cluster with 100 Mbps / 20 ms links.
Here all parties run on one GPU (one process); the time is one complete
verifiable survey (DP encoding + range proofs, CN aggregation [+ obfuscation],
key switching, querier decoding, VN verification of every proof, skipchain
block).  Output: one JSON line per operation with our seconds and the
reference's.

Ranges follow the reference's service tests: (u, l) = (16, 16) for numeric
outputs, (2, 1) for the bit vectors of bool/min/max/set operations.
"""
import json
import statistics
import sys
import tempfile
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from drynx_amd.query import LogisticRegressionParameters  # noqa: E402
from drynx_amd.services.api import DrynxClient  # noqa: E402
from drynx_amd.services.local import local_cluster, make_survey  # noqa: E402

# (label, op, kwargs, reference seconds)
CASES = [
    ("sum", "sum", dict(query_min=0, query_max=100), 1.98),
    ("mean", "mean", dict(query_min=0, query_max=100), 2.57),
    ("variance", "variance", dict(query_min=0, query_max=100), 2.74),
    ("bool_OR (obfuscation)", "bool_OR", dict(query_min=0, query_max=1, obfuscation=True), 2.11),
    ("bool_AND", "bool_AND", dict(query_min=0, query_max=1), 1.88),
    ("max, 100 values (obfuscation)", "max", dict(query_min=0, query_max=99, obfuscation=True), 8.04),
    ("max, 100 values", "max", dict(query_min=0, query_max=99), 2.19),
    ("frequencyCount, 100 buckets", "frequencyCount", dict(query_min=0, query_max=99), 2.63),
    ("intersection (obfuscation)", "inter", dict(query_min=0, query_max=99, obfuscation=True), 2.35),
    ("intersection", "inter", dict(query_min=0, query_max=99), 1.94),
    ("cosim", "cosim", dict(query_min=0, query_max=100, d=2), 3.84),
    ("lin_reg, d=9 (65 outputs)", "lin_reg", dict(query_min=0, query_max=10, d=9), 15.97),
    ("MLeval", "MLeval", dict(query_min=0, query_max=100), 3.25),
    ("logistic regression, d=6 (56 outputs)", "logistic regression", dict(), 12.42),
]
def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


BIT_OPS = {"bool_OR", "bool_AND", "max", "min", "union", "inter"}


def main():
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    cl, node = local_cluster(3, 10, 3, device=dev, workdir=tempfile.mkdtemp(prefix="drynx_allops_"))
    client = DrynxClient(node, device=dev)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    only = set(sys.argv[2].split(",")) if len(sys.argv) > 2 else None
    for label, op, kw, ref in CASES:
        if only and op not in only:
            continue
        kw = dict(kw)
        obf = kw.pop("obfuscation", False)
        ranges = [2, 1] if op in BIT_OPS else [16, 16]
        if op in BIT_OPS and not obf:
            ranges = [0, 0]  # reference: bit ops without obfuscation carry no range proof (u = l = 0)
        lp = None
        if op == "logistic regression":
            d = 6
            lp = LogisticRegressionParameters(NbrRecords=100, NbrFeatures=d, Means=[0.0] * d,
                                              StandardDeviations=[1.0] * d, Lambda=1.0, Step=0.1, MaxIterations=25,
                                              InitialWeights=[0.1] * (d + 1), K=2, PrecisionApproxCoefficients=1e2)
            ranges = [16, 16, 1 << 62]
        times, codes = [], set()
        for i in range(reps + 1):
            sq = make_survey(client, cl, op, rows=10, proofs=1, ranges=ranges, obfuscation=obf, lr_params=lp,
                             sig_device=dev, deterministic_sigs=True, **kw)
            _sync(dev)
            t0 = time.perf_counter()
            _, vals, res = client.send_survey_query(sq)
            _sync(dev)
            dt = time.perf_counter() - t0
            codes |= set(res.block.data_block().Proofs.values()) if res.block is not None else set()
            if i:  # first run is the warm-up (signature tables, decryption tables)
                times.append(dt)
        med = statistics.median(times)
        print(json.dumps({"op": label, "seconds": round(med, 4), "reference_s": ref, "speedup": round(ref / med, 1),
                          "proof_codes": sorted(codes)}), flush=True)
    node.close(remove=True)


if __name__ == "__main__":
    main()
