#!/usr/bin/env python3
"""Which framework lines launch torch "glue" ops (copies, cats, fills) in a
verifiable query, and how many bytes they move: a TorchFunctionMode records
every torch call made from drynx_amd code with the innermost framework frame
and the bytes of its output.  Run on CPU with a small LR query (the call
sites are the same as on the GPU; the bytes scale with the query shape).

usage: python tools/op_audit.py [features] [dps] [device]
(views are not counted: only ops whose output has its own storage)
"""
import collections
import os
import sys
import tempfile
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

class Audit:
    """Wraps torch entry points process-wide (worker threads included: the
    prover and the pooled verifier run on their own threads)."""

    TARGETS = [(torch, "cat"), (torch, "stack"), (torch, "zeros"), (torch, "full"), (torch, "zeros_like"),
               (torch.Tensor, "contiguous"), (torch.Tensor, "clone"), (torch.Tensor, "to"),
               (torch.Tensor, "repeat"), (torch.Tensor, "index_select"), (torch.Tensor, "repeat_interleave"),
               (torch.Tensor, "__getitem__"), (torch.Tensor, "flip"), (torch.Tensor, "cpu"),
               (torch.nn.utils.rnn, "pad_sequence")]

    def __init__(self):
        self.stats = collections.defaultdict(lambda: [0, 0])
        self._orig = []

    def _wrap(self, owner, name):
        orig = getattr(owner, name)
        stats = self.stats

        def wrapped(*args, **kwargs):
            out = orig(*args, **kwargs)
            if isinstance(out, torch.Tensor) and out.numel():
                ins = set()
                for a in list(args) + list(kwargs.values()):
                    for t in (a if isinstance(a, (list, tuple)) else [a]):
                        if isinstance(t, torch.Tensor):
                            ins.add(t.untyped_storage().data_ptr())
                if out.untyped_storage().data_ptr() not in ins:  # views move no memory
                    frame = "?"
                    for fs in reversed(traceback.extract_stack(limit=14)[:-1]):
                        if "drynx_amd" in fs.filename:
                            frame = f"{fs.filename.split('drynx_amd/')[-1]}:{fs.lineno} {fs.name}"
                            break
                    st = stats[(name, frame)]
                    st[0] += 1
                    st[1] += out.numel() * out.element_size()
            return out
        self._orig.append((owner, name, orig))
        setattr(owner, name, wrapped)

    def __enter__(self):
        for owner, name in self.TARGETS:
            self._wrap(owner, name)
        return self

    def __exit__(self, *a):
        for owner, name, orig in reversed(self._orig):
            setattr(owner, name, orig)
        return False


def main():
    d = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    n_dps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = sys.argv[3] if len(sys.argv) > 3 else "cpu"
    from drynx_amd.query import LogisticRegressionParameters, new_survey_id
    from drynx_amd.services.api import DrynxClient
    from drynx_amd.services.local import local_cluster, make_survey

    cl, node = local_cluster(3, n_dps, 3, device=dev, workdir=tempfile.mkdtemp())
    lp = LogisticRegressionParameters(NbrRecords=200 * n_dps, NbrFeatures=d, Means=[2.0] * d,
                                      StandardDeviations=[1.15] * d, Lambda=1.0, Step=0.012, MaxIterations=5,
                                      InitialWeights=[0.1] * (d + 1), K=2, PrecisionApproxCoefficients=100.0)
    client = DrynxClient(node, device=dev)
    sq = make_survey(client, cl, "logistic regression", proofs=1, ranges=[16, 16, 1 << 62], lr_params=lp,
                     thresholds=[1.0, 1.0, 1.0, 0.0, 1.0], sig_device=dev)
    client.send_survey_query(sq)  # warm caches (tables), not audited
    sq.SurveyID = new_survey_id()
    a = Audit()
    with a:
        client.send_survey_query(sq)
    rows = sorted(a.stats.items(), key=lambda kv: -kv[1][1])
    tot = sum(v[1] for _, v in rows)
    print(f"glue bytes {tot / 2**20:.1f} MiB over {sum(v[0] for _, v in rows)} calls (d={d}, {n_dps} DPs)")
    for (name, frame), (n, b) in rows[:40]:
        print(f"{b / 2**20:10.2f} MiB {n:6d}  {name:18s} {frame}")
    node.close(remove=True)


if __name__ == "__main__":
    main()
