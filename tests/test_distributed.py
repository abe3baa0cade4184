"""Multi-process (gloo, world_size 2) surveys: parties spread over ranks, EC
collectives over torch.distributed, proof fan-out, shared skipchain block."""
import os
import socket
import subprocess
import sys
import tempfile

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _diffp():
    from drynx_amd.query import QueryDiffP

    return QueryDiffP(LapMean=0.0, LapScale=1.0, NoiseListSize=40, Quanta=1.0, Scale=1.0, Limit=5.0)


def _worker(rank, world, port, outdir):
    import json

    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from drynx_amd.parallel.comm import DistComm
    from drynx_amd.services.api import DrynxClient
    from drynx_amd.services.local import local_cluster, make_survey

    comm = DistComm("cpu")
    cl, node = local_cluster(3, 4, 2, comm=comm, device="cpu", workdir=os.path.join(outdir, f"r{rank}"))
    out = {}
    for op, kw in [("sum", {}), ("variance", {}), ("frequencyCount", {}), ("sum", {"proofs": 1, "ranges": [16, 3]}),
                   ("max", {"proofs": 1, "ranges": [2, 1], "obfuscation": True}),
                   # DRO noise list shuffled by CNs on both ranks, beside the range proving
                   ("sum", {"proofs": 1, "ranges": [16, 3], "diffp": _diffp()})]:
        if rank == 0:
            client = DrynxClient(node)
            sq = make_survey(client, cl, op, query_min=0, query_max=4, rows=6, **kw)
            _, vals, res = client.send_survey_query(sq)
            out[f"{op}{len(out)}"] = {"vals": vals[0], "block": res.block.Hash if res.block else None,
                                      "codes": sorted(set(res.block.data_block().Proofs.values())) if res.block else []}
        else:
            res = node.run_survey(None)
            out[f"{op}{len(out)}"] = {"block": res.block.Hash if res.block else None,
                                      "clear": res.clear_dp}
    with open(os.path.join(outdir, f"out{rank}.json"), "w") as f:
        json.dump(out, f, default=str)
    node.close()
    dist.destroy_process_group()


def test_two_rank_gloo_surveys():
    import json

    outdir = tempfile.mkdtemp()
    mp.spawn(_worker, args=(2, _free_port(), outdir), nprocs=2, join=True)
    o0 = json.load(open(os.path.join(outdir, "out0.json")))
    o1 = json.load(open(os.path.join(outdir, "out1.json")))
    for k in o0:
        assert o0[k]["block"] == o1[k]["block"]
    assert o0["sum3"]["codes"] == [1] and o0["max4"]["codes"] == [1] and o0["sum5"]["codes"] == [1]
    assert o0["max4"]["vals"][0] <= 4.0


@pytest.mark.slow
def test_bench_two_ranks_torchrun():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "1", "--warmup", "0", "--records", "2000", "--features", "2", "--max-iter", "5", "--device", "cpu"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line) if (json := __import__("json")) else None
    assert d["n_gpus"] == 2 and d["all_proofs_valid"] and d["value"] > 0


def _bench_line(r):
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


_SMALL = ["--steps", "1", "--warmup", "0", "--records", "2000", "--features", "2", "--max-iter", "5", "--device", "cpu"]


@pytest.mark.slow
def test_bench_self_launches_eight_ranks():
    """``python bench.py --gpus 8`` with no launcher (the driver's BENCH form)
    starts 8 ranks itself and runs the targeted placement: CNs on ranks 0-2,
    VNs on 3-5, DPs round robin from rank 6 (ranks 6 and 7 host 2 DPs each),
    every VN's range checks pooled in 1/8 slices over all ranks."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", *_SMALL],
                       capture_output=True, text=True, timeout=900, env=env)
    d = _bench_line(r)
    assert d["n_gpus"] == 8 and d["all_proofs_valid"] and d["result_ok"]
    ranks = {x["rank"]: x for x in d["ranks"]}
    assert sorted(ranks) == list(range(8))
    assert [ranks[k]["roles"]["cn"] for k in range(3)] == [["cn0"], ["cn1"], ["cn2"]]
    assert [ranks[k]["roles"]["vn"] for k in range(3, 6)] == [["vn0"], ["vn1"], ["vn2"]]
    assert sorted(ranks[6]["roles"]["dp"]) == ["dp0", "dp8"] and sorted(ranks[7]["roles"]["dp"]) == ["dp1", "dp9"]
    assert all(len(ranks[k]["roles"]["dp"]) == 1 for k in range(6))
    # pooled range checks: every (proof, VN) verification is done once, split in
    # 8 slices weighted by each rank's other work (prq.balanced_parts: ranks 6
    # and 7 prove two DPs, ranks 3-5 host a VN -> shorter slices)
    from drynx_amd.proofs import requests as prq

    n_out = d["config"]["range_proof"]["proofs_per_query"] // d["config"]["dps"]
    items = [ranks[k]["pool_range_items"] for k in range(8)]
    assert sum(items) == d["config"]["range_proof"]["verifications_per_query"]
    parts = prq.balanced_parts(8, [1, 1, 1, 1, 1, 1, 2, 2], [0, 0, 0, 1, 1, 1, 0, 0])

    class _Sq:
        RangeProofThreshold = 1.0
    for k in range(8):
        lo, hi = prq.sampled_bounds(_Sq, n_out, parts[k])
        assert items[k] == (hi - lo) * d["config"]["dps"] * d["config"]["vns"], k
    # control plane: at most 4 host collectives per query per rank (query
    # broadcast, pooled verdicts, bitmaps, co-signatures); + 1 for the bench's
    # own elapsed-time gather after the timed steps
    assert all(ranks[k]["ctrl_collectives"] <= 4 * d["steps"] + 1 for k in range(8)), \
        [ranks[k]["ctrl_collectives"] for k in range(8)]
    # per-party timers: every DP's <dp>_AllProofs is measured on its own rank
    # (proving start -> the VNs' verdicts back on that rank); DPs on different
    # ranks get their own values, none longer than the query
    ap = {k: v for k, v in d["phase_s"].items() if k.endswith("_AllProofs")}
    assert sorted(ap) == sorted(f"dp{i}_AllProofs" for i in range(10))
    by_rank = {k: [ap[f"{dp}_AllProofs"] for dp in ranks[k]["roles"]["dp"]] for k in range(8)}
    assert len({round(v[0], 6) for v in by_rank.values()}) > 1
    assert max(ap.values()) <= max(ranks[0]["step_ms"]) / 1000.0 + 1e-3
    # traffic: every rank took part in the data plane; the VN ranks receive the most
    assert all(ranks[k]["bytes_sent"] > 0 and ranks[k]["bytes_recv"] > 0 for k in range(8))
    assert min(ranks[k]["bytes_recv"] for k in (3, 4, 5)) > max(ranks[k]["bytes_recv"] for k in (0, 1, 2, 6, 7))


@pytest.mark.slow
def test_bench_self_launches_two_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *_SMALL],
                       capture_output=True, text=True, timeout=600, env=env)
    d = _bench_line(r)
    assert d["n_gpus"] == 2 and d["all_proofs_valid"] and d["result_ok"] and len(d["ranks"]) == 2


def test_bench_rejects_world_mismatch():
    """Under a launcher whose world differs from --gpus the bench refuses to
    print a number labelled with the wrong GPU count."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *_SMALL],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0 and "rank(s)" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_forwarded_args_avoid_launcher_abbreviations():
    """bench.py's self-launch hands its arguments to torch.distributed.run,
    whose parser would read "--l" as an abbreviation of its own --log-dir:
    the short aliases travel in their long forms, values untouched."""
    sys.path.insert(0, ROOT)
    import bench

    fwd = bench._forward_args(["--gpus", "8", "--u", "4", "--l=2", "--steps", "3", "--features", "12"])
    assert fwd == ["--gpus", "8", "--base", "4", "--digits=2", "--steps", "3", "--features", "12"]
    argv = sys.argv
    try:
        sys.argv = ["bench.py", *fwd]
        a = bench.parse()
    finally:
        sys.argv = argv
    assert (a.gpus, a.u, a.l, a.steps, a.features) == (8, 4, 2, 3, 12)


def _run_bench(gpus: int, extra: list, env_extra: dict | None = None, timeout: int = 900):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), *extra],
                       capture_output=True, text=True, timeout=timeout, env=env)
    return _bench_line(r)


@pytest.mark.slow
def test_two_ranks_sharded_tables_and_node_ledger():
    """Two ranks on one node, VerificationSharding 2 (each proof checked by 2
    of the 3 VNs, per-CN payloads fanned out to the assigned VNs only):
    the prover tables are built 1/2 per rank and broadcast (GLS-8 layout
    forced) and equal a one-rank build bit for bit; the VN ranks share
    content-addressed ledger payloads (each written once on the node, the
    other rank referencing it) and every VN's stored proofs read back."""
    small = ["--steps", "1", "--warmup", "1", "--records", "2000", "--features", "2", "--max-iter", "5",
             "--device", "cpu", "--deterministic-sigs", "--table-digest"]
    env = {"DRYNX_PROVER_TABLE_BITS": "7"}
    d2 = _run_bench(2, small + ["--verification-sharding", "2", "--check-ledger"], env)
    d1 = _run_bench(1, small, env)
    assert d2["n_gpus"] == 2 and d2["all_proofs_valid"] and d2["result_ok"]
    ranks = d2["ranks"]
    assert all(r["bytes_recv"] > 0 for r in ranks)
    assert {r["table_digest"] for r in ranks} == {d1["ranks"][0]["table_digest"]}
    # node-shared payloads: written once on the node, the other VN rank references them
    assert sum(r["ledger_written"] for r in ranks) > 0 and sum(r["ledger_referenced"] for r in ranks) > 0
    stored = {vn: n for r in ranks for vn, n in r["ledger_readback"].items()}
    assert sorted(stored) == ["vn0", "vn1", "vn2"] and all(n > 0 for n in stored.values())
