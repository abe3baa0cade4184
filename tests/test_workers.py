"""Every worker thread of a node is pinned to the rank's device
(``utils.streams.executor``): no executor is made anywhere else in the
package, a CPU survey creates its workers through the factory, and on a GPU
every worker's current device is the node's (one process per GPU: a worker
of rank k must never default to device 0)."""
import os
import re

import pytest
import torch

from drynx_amd.utils import streams

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "drynx_amd")


def test_no_executor_outside_the_factory():
    allowed = {os.path.join("utils", "streams.py"), os.path.join("native", "build.py")}
    bad = []
    for d, _, files in os.walk(PKG):
        for f in files:
            if not f.endswith(".py"):
                continue
            rel = os.path.relpath(os.path.join(d, f), PKG)
            if rel in allowed:
                continue
            src = open(os.path.join(d, f)).read()
            if re.search(r"ThreadPoolExecutor\(|ProcessPoolExecutor\(", src):
                bad.append(rel)
    assert not bad, f"executors made outside utils.streams.executor: {bad}"


def _survey(device, tmp_path):
    from drynx_amd.services.api import DrynxClient
    from drynx_amd.services.local import local_cluster, make_survey

    cl, node = local_cluster(2, 3, 2, device=device, workdir=str(tmp_path))
    client = DrynxClient(node, device=device)
    sq = make_survey(client, cl, "sum", query_min=0, query_max=8, rows=6, proofs=1, ranges=[4, 2],
                     sig_device=device)
    client.send_survey_query(sq)
    return node


def test_survey_workers_come_from_the_factory(tmp_path):
    before = len(streams._made)
    node = _survey("cpu", tmp_path)
    made = streams._made[before:]
    assert "drynx-vn-pool" in made or "drynx-ledger" in made, made
    node.close(remove=True)


@pytest.mark.gpu
def test_workers_pinned_to_node_device(tmp_path, gpu_device):
    node = _survey(gpu_device, tmp_path)
    pools = [getattr(node, a) for a in ("_pool", "_client_pool", "_cnp_pool", "_cnp_poollate", "_pool_exec")
             if hasattr(node, a)]
    assert pools
    for ex in pools:
        assert ex.submit(streams.pinned_device).result() == gpu_device.index
        assert ex.submit(torch.cuda.current_device).result() == gpu_device.index
    node.close(remove=True)
