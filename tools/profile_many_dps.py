"""cProfile of one verifiable ``sum`` survey with many DPs (ScaleDPs shape,
#DPs = #records) -- finds the per-DP host costs that dominate when each DP
contributes one value.  Usage: python tools/profile_many_dps.py [n_dps] [out.txt]"""
import cProfile
import io
import pstats
import sys
import tempfile
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from drynx_amd.services.api import DrynxClient  # noqa: E402
from drynx_amd.services.local import local_cluster, make_survey  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 600
    out = sys.argv[2] if len(sys.argv) > 2 else None
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    cl, node = local_cluster(3, n, 3, device=dev, workdir=tempfile.mkdtemp(prefix="drynx_prof_"))
    client = DrynxClient(node, device=dev)

    def run():
        sq = make_survey(client, cl, "sum", query_min=0, query_max=100, rows=1, proofs=1, ranges=[16, 16],
                         thresholds=[1.0, 1.0, 1.0, 0.0, 1.0], sig_device=dev, deterministic_sigs=True)
        t0 = time.perf_counter()
        client.send_survey_query(sq)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        return time.perf_counter() - t0

    print("warm-up", round(run(), 3), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    t = run()
    pr.disable()
    s = io.StringIO()
    s.write(f"{n} DPs: {t:.3f} s\n")
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(40)
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(100)
    txt = s.getvalue()
    if out:
        with open(out, "w") as f:
            f.write(txt)
    print(txt[:200])
    from drynx_amd.utils import timers

    timers.dump_trace()
    node.close(remove=True)


if __name__ == "__main__":
    main()
