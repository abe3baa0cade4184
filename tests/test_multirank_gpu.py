"""Multi-rank device paths on the GPU box: ``bench.py --gpus 2`` as a fresh
child job whose two ranks share cuda:0 over a gloo data plane (RCCL refuses
two ranks on one device), so every W > 1 path runs the HIP kernels: helper
slices of the pooled range checks bound to their digests, the prover tables
built 1/2 per rank and broadcast into each rank's copy (``attach_shard`` /
``broadcast_into``), node-shared ledger payloads, and fault attribution
across ranks.  The reference runs every party as its own process
(simul/drynx_simul.go:83-98, 284-305)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = ["--steps", "2", "--warmup", "1", "--records", "20000", "--features", "6", "--max-iter", "20",
         "--device", "cuda:0", "--deterministic-sigs", "--table-digest"]


def _bench(gpus: int, extra: list, timeout: int = 300) -> dict:
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(DRYNX_DIST_BACKEND="gloo", DRYNX_PROVER_TABLE_BITS="7", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), *SMALL, *extra],
                       capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.gpu
def test_two_ranks_on_device(gpu_device):
    d1 = _bench(1, [])
    d2 = _bench(2, ["--check-ledger"])
    assert d2["n_gpus"] == 2 and d2["all_proofs_valid"] and d2["result_ok"]
    ranks = d2["ranks"]
    assert len(ranks) == 2 and all(r["bytes_recv"] > 0 and r["bytes_sent"] > 0 for r in ranks)
    # pooled range checks: both ranks checked a slice for every VN
    assert all(r["pool_range_items"] > 0 for r in ranks)
    assert sum(r["pool_range_items"] for r in ranks) == \
        d2["config"]["range_proof"]["verifications_per_query"] * d2["steps"]
    # sharded GLS-8 prover tables: bit-identical to the one-rank build
    assert {r["table_digest"] for r in ranks} == {d1["ranks"][0]["table_digest"]}
    # node-shared ledger payloads and every VN's proofs readable
    assert sum(r["ledger_written"] for r in ranks) > 0 and sum(r["ledger_referenced"] for r in ranks) > 0
    stored = {vn: n for r in ranks for vn, n in r["ledger_readback"].items()}
    assert sorted(stored) == ["vn0", "vn1", "vn2"] and all(n > 0 for n in stored.values())


@pytest.mark.gpu
def test_two_ranks_fault_blame(gpu_device):
    """One DP's range proof forged on a rank that is not the VNs' only rank:
    every VN blames exactly that DP (the bench asserts the bitmap)."""
    d = _bench(2, ["--fault-dp", "1"])
    assert d["n_gpus"] == 2 and d["blame_ok"] and d["result_ok"]
