"""Ledger blob segments under a disk budget (ledger/store.py BlobSegment):
values rotate into generation files; when a write would leave less than the
reserve free, the oldest generations are deleted, their references fail
loudly and everything newer still reads back; DRYNX_LEDGER_RETAIN=all keeps
every file."""
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
    if retain == "all":
        monkeypatch.setenv("DRYNX_LEDGER_RETAIN", "all")
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
        with pytest.raises(FileNotFoundError, match="pruned"):
            store.get("proofs", "k0")
    store.close()
    seg.close(remove=True)
    assert not any(p.name.startswith("ledger_r0.blobs") for p in tmp_path.iterdir())


def test_node_shared_payloads(tmp_path):
    """The VN ranks of one node share content-addressed payload files: the
    writer copies and writes, a reader rank stores references only and its
    reads wait until the writer's file is complete."""
    from drynx_amd.ledger.store import NodeBlobs

    root = str(tmp_path / "node")
    reader = NodeBlobs(root, writer=False)
    rstore = Store(str(tmp_path / "db_vn1.sqlite"))
    data = np.arange(100000, dtype=np.uint32).view(np.uint8)
    ref = reader.put_many(["d1"], None, [data.nbytes])[0]
    rstore.update("proofs", "k", ref)               # a reference before the writer has written anything
    writer = NodeBlobs(root, writer=True)
    import threading
    import time

    def late_write():
        time.sleep(0.2)
        writer.put_many(["d1"], lambda: [memoryview(data)])
        writer.flush()

    th = threading.Thread(target=late_write)
    th.start()
    assert rstore.get("proofs", "k") == data.tobytes()   # waited for the writer
    th.join()
    assert os.path.exists(os.path.join(root, "d1.blob")) and not os.path.exists(os.path.join(root, "d1.blob.tmp"))
    rstore.close()
    reader.close(remove=True)
    writer.close(remove=True)
    assert not os.path.exists(root)
