set -o pipefail
mkdir -p gpurun_out
DRYNX_TRACE=gpurun_out/trsum timeout -k 10 300 python - > gpurun_out/trsum.log 2>&1 <<'PY'
import sys, tempfile, time, torch
sys.path.insert(0, ".")
from drynx_amd.services.api import DrynxClient
from drynx_amd.services.local import local_cluster, make_survey
from drynx_amd.utils import timers
dev = torch.device("cuda", 0)
cl, node = local_cluster(3, 10, 3, device=dev, workdir=tempfile.mkdtemp())
client = DrynxClient(node, device=dev)
for i in range(4):
    with timers.span("MAKE_SURVEY"):
        sq = make_survey(client, cl, "sum", rows=10, proofs=1, ranges=[16, 16], sig_device=dev, deterministic_sigs=True, query_min=0, query_max=100)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    with timers.span("QUERY"):
        client.send_survey_query(sq)
    torch.cuda.synchronize(); print("query", time.perf_counter() - t0, flush=True)
timers.dump_trace("gpurun_out/trsum.json")
PY
python tools/host_trace.py gpurun_out/trsum.json 3 > gpurun_out/trsum.txt; tail -3 gpurun_out/trsum.log
