"""Ledger blob segments (ledger/store.py BlobSegment): values rotate into
generation files and every file is kept by default (as bbolt keeps every
proof); under the opt-in disk budget (DRYNX_LEDGER_RETAIN=budget) the oldest
generations are deleted when a write would leave less than the reserve free,
their references fail loudly and everything newer still reads back."""
import os

import numpy as np
import pytest

from drynx_amd.ledger.store import BlobSegment, Store


def _put(seg, store, i, size=4096):
    data = np.full(size, i % 251, dtype=np.uint8)
    ref = seg.put_many([f"b{i}"], lambda d=data: [memoryview(d)])[0]
    store.update("proofs", f"k{i}", ref)
    return data.tobytes()


@pytest.mark.parametrize("retain", ["budget", "all"])
def test_blob_generations_and_pruning(tmp_path, monkeypatch, retain):
    monkeypatch.setenv("DRYNX_LEDGER_SEGMENT_GB", str(10000 / (1 << 30)))   # ~10 KB generations
    if retain == "budget":
        monkeypatch.setenv("DRYNX_LEDGER_RETAIN", "budget")
    seg = BlobSegment(str(tmp_path / "ledger_r0.blobs"))
    store = Store(str(tmp_path / "db_vn0.sqlite"))
    want = {i: _put(seg, store, i) for i in range(3)}
    seg.flush()
    assert all(store.get("proofs", f"k{i}") == want[i] for i in range(3))
    gens_before = list(seg._gens)
    assert len(gens_before) >= 2                       # 4 KB values, ~10 KB generations
    # no disk left above the reserve: every older generation goes, the newest stays
    monkeypatch.setenv("DRYNX_LEDGER_RESERVE_GB", str(1 << 40))
    want[3] = _put(seg, store, 3)
    seg.flush()
    assert store.get("proofs", "k3") == want[3]
    if retain == "all":
        assert all(os.path.exists(p) for p in gens_before)
        assert store.get("proofs", "k0") == want[0]
    else:
        assert not os.path.exists(gens_before[0]) and len(seg._gens) < len(gens_before) + 1
        from drynx_amd.ledger.store import PrunedError

        with pytest.raises(PrunedError, match="pruned"):
            store.get("proofs", "k0")
    store.close()
    seg.close(remove=True)
    assert not any(p.name.startswith("ledger_r0.blobs") for p in tmp_path.iterdir())


def test_node_shared_payloads(tmp_path):
    """The VN ranks of one node share content-addressed payload files: the
    first rank to claim a digest copies and writes it, another rank holding
    the same payload stores a reference only and its reads wait until the
    claimant's file is complete."""
    from drynx_amd.ledger.store import NodeBlobs

    root = str(tmp_path / "node")
    writer = NodeBlobs(root)
    reader = NodeBlobs(root)
    assert writer.claim(["d1"]) == [True]
    assert reader.claim(["d1"]) == [False]           # already claimed on the node
    rstore = Store(str(tmp_path / "db_vn1.sqlite"))
    data = np.arange(100000, dtype=np.uint32).view(np.uint8)
    ref = reader.put_refs(["d1"])[0]
    rstore.update("proofs", "k", ref)               # a reference before the claimant has written anything
    import threading
    import time

    def late_write():
        time.sleep(0.2)
        writer.put_many(["d1"], lambda: [memoryview(data)])
        writer.flush()

    th = threading.Thread(target=late_write)
    th.start()
    assert rstore.get("proofs", "k") == data.tobytes()   # waited for the claimant
    th.join()
    assert os.path.exists(os.path.join(root, "d1.blob")) and not os.path.exists(os.path.join(root, "d1.blob.tmp"))
    rstore.close()
    reader.close(remove=True)
    writer.close(remove=True)
    assert not os.path.exists(root)


def test_node_blobs_claim_by_holder_only(tmp_path):
    """Sharded fan-out: the lowest VN rank of the node may receive a
    header-only envelope.  Whichever rank holds the payload claims and writes
    it, so every VN's stored reference reads back (the old fixed-writer
    scheme left the other VN waiting for a file nobody wrote)."""
    from drynx_amd.ledger.store import NodeBlobs

    root = str(tmp_path / "node")
    low, high = NodeBlobs(root), NodeBlobs(root)      # VN ranks 3 and 4 of a node
    data = np.full(70000, 7, dtype=np.uint8)
    # rank 3 got only the header: it claims nothing; rank 4 holds the payload
    assert high.claim(["p"]) == [True]
    ref = high.put_many(["p"], lambda: [memoryview(data)])[0]
    st = Store(str(tmp_path / "db_vn1.sqlite"))
    st.update("proofs", "k", ref)
    assert st.get("proofs", "k") == data.tobytes()
    st.close()
    low.close(remove=True)
    high.close(remove=True)


def test_first_survey_reads_back_after_many(tmp_path):
    """Keep-everything default: after 100 surveys of large payloads the first
    survey's values read back bit-identically (bbolt keeps every proof,
    services/service_skipchain.go:240-320), and each write was synced."""
    seg = BlobSegment(str(tmp_path / "ledger_r0.blobs"))
    store = Store(str(tmp_path / "db_vn0.sqlite"))
    pruned0 = BlobSegment.pruned
    first = {}
    for s_ in range(100):
        rows = []
        for j in range(2):
            data = np.random.default_rng(s_ * 7 + j).integers(0, 256, 70000, dtype=np.uint8)
            ref = seg.put_many([f"s{s_}p{j}"], lambda d=data: [memoryview(d)])[0]
            rows.append((f"survey{s_}/range", f"dp{j}", ref))
            if s_ == 0:
                first[f"dp{j}"] = data.tobytes()
        for b, k, r in rows:
            store.update_async(b, k, r)
    seg.flush()
    store.flush()
    assert store.bucket("survey0/range") == first
    assert BlobSegment.pruned == pruned0
    store.close()
    seg.close(remove=True)
