"""Embedded bucketed key-value store (bbolt equivalent) for verifying nodes.

Reference: each VN opens bbolt at ``"db:"+ServerIdentity.ID``
(services/service_skipchain.go:77-86) and writes with ``libdrynx.UpdateDB``
(lib/structs.go:571-588: batch put, create bucket if missing).  Buckets:
  surveyID/<type>  key surveyID/type/sender/differInfo/VN -> proof bytes
  <VN address>     key surveyID/map                        -> bitmap
  genesis          key genesis                             -> genesis block
  mapping          key surveyID                            -> block hash
Here: SQLite (WAL) with one (bucket, key) -> value table; values above
``BLOB_MIN`` bytes (range-proof bundles: tens of MB per DP) go to an
append-only segment file next to the database and the table keeps a
(offset, length) reference, so a wide query's proofs land with one sequential
write instead of B-tree page churn.  Writes can be queued to a background
writer thread so proof persistence never sits on the verification critical
path (``flush`` joins them); a queued value may be a device tensor, copied to
the host by the writer.

Durability: as a bbolt batch is committed before ``UpdateDB`` returns
(lib/structs.go:571-588), every blob write is fdatasync'ed by the ledger
worker before its job completes and SQLite runs with ``synchronous=FULL`` (each
commit syncs the WAL), so ``flush`` returning means the values are on disk.
Retention: every proof is kept (bbolt never drops one and ``GetProofs`` serves
all of them, services/service_skipchain.go:240-320); a full disk fails the
write loudly.  ``DRYNX_LEDGER_RETAIN=budget`` opts into deleting the oldest
blob generations below a disk reserve; a read of a pruned value then raises
``PrunedError``.
"""
from __future__ import annotations

import os
import queue
import sqlite3
import struct
import threading

from ..utils import streams, timers


BLOB_MIN = 1 << 16
_REF = b"\x00DXBLOB1"
_REF2 = b"\x00DXBLOB2"  # + offset, length (u64) + path of a shared BlobSegment (raw bytes)
_REF3 = b"\x00DXBLOB3"  # the same, holding a compact range payload (proofs/ledger_codec.py)
_REF4 = b"\x00DXBLOB4"  # + path of a node-shared payload file (its own tag word says raw / compact)
_NODE_RAW, _NODE_COMPACT = b"DXNODER1", b"DXNODEC1"  # first bytes of a node-shared payload file


class Compact:
    """A produced ledger value in the compact range-payload form: the writer
    tags it explicitly (``_REF3`` / the node file's tag), and only tagged
    values are decompressed when read -- nothing is recognised by sniffing."""

    def __init__(self, buf):
        self.buf = buf


def _unwrap(d) -> tuple:
    """(bytes view, compact flag) of a produced value."""
    if isinstance(d, Compact):
        return memoryview(d.buf).cast("B"), True
    return memoryview(d).cast("B"), False


def _addr(mv: memoryview) -> int:
    import numpy as np

    return np.frombuffer(mv, dtype=np.uint8).__array_interface__["data"][0] if mv.nbytes else 0


def _coalesce(bufs: list) -> list:
    """Runs of buffers that sit back to back in one exporter (the slices of
    one pinned device-to-host buffer: thousands of small payloads of a
    many-DP query) merged into single views, so they are written by one
    positioned write instead of one pool task each; written bytes unchanged."""
    if len(bufs) < 64:
        return bufs
    out, run = [], None  # run: (exporter, base view, base address, start, end)
    for b in bufs:
        b = memoryview(b).cast("B") if b.format != "B" or b.ndim != 1 else b
        obj = b.obj
        a = _addr(b)
        if run is not None and obj is run[0] and a == run[2] + run[4]:
            run = (run[0], run[1], run[2], run[3], run[4] + b.nbytes)
            continue
        if run is not None:
            out.append(run[1][run[3]: run[4]])
        try:
            base = memoryview(obj).cast("B")
            base_a = _addr(base)
            if not base_a <= a <= base_a + base.nbytes - b.nbytes:
                raise ValueError
            run = (obj, base, base_a, a - base_a, a - base_a + b.nbytes)
        except (TypeError, ValueError):
            out.append(b)
            run = None
    if run is not None:
        out.append(run[1][run[3]: run[4]])
    return out


class BlobRef:
    """A value living in a rank-level BlobSegment (written once, referenced by
    the stores of every VN hosted on the rank)."""

    def __init__(self, segment: "BlobSegment", future):
        self.segment, self.future = segment, future

    def result(self):
        return self.future.result()


class _Item:
    """Future of the i-th value of a ``put_many`` job."""

    def __init__(self, job, i):
        self.job, self.i = job, i

    def result(self):
        return self.job.result()[self.i]


def _copies() -> int:
    """DRYNX_LEDGER_COPIES=k (diagnostics): every blob is also written to k-1
    extra files, reproducing on one rank the ledger write volume of k VN ranks
    (on an 8-GPU node each of the 3 VN ranks persists its own copy of every
    proof, proof_collection_protocol.go:307-406)."""
    return max(1, int(os.environ.get("DRYNX_LEDGER_COPIES", "1")))


def _mark_pruned(path: str):
    """Record a deleted value file next to it (readers then fail at once
    instead of waiting for a node-shared file that will never appear)."""
    with open(os.path.join(os.path.dirname(os.path.abspath(path)), "_pruned"), "a") as f:
        f.write(os.path.basename(path) + "\n")


def _was_pruned(path: str) -> bool:
    try:
        with open(os.path.join(os.path.dirname(os.path.abspath(path)), "_pruned")) as f:
            return os.path.basename(path) in {ln.strip() for ln in f}
    except FileNotFoundError:
        return False


def _gb_env(name: str, default: float) -> float:
    return float(os.environ.get(name, default)) * (1 << 30)


def _budget() -> bool:
    """Pruning below a disk reserve is opt-in (DRYNX_LEDGER_RETAIN=budget)."""
    return os.environ.get("DRYNX_LEDGER_RETAIN", "all") == "budget"


class PrunedError(FileNotFoundError):
    """A ledger value deleted under DRYNX_LEDGER_RETAIN=budget."""


def _fsync_dir(path: str):
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
    finally:
        os.close(fd)


class BlobSegment:
    """Append-only files of large ledger values shared by the VNs of one rank:
    the same proof payload is written once, however many co-hosted VNs store
    it.  Values are produced by a callable on the segment's own worker thread
    (and, on a GPU, its own HIP stream: device-to-host copies never queue on
    the compute streams).

    Values go to generation files of at most DRYNX_LEDGER_SEGMENT_GB (default
    4), each write fdatasync'ed before its job completes.  Everything is kept
    (a full disk fails the write, as the reference's bbolt store would).
    Opt-in disk budget (DRYNX_LEDGER_RETAIN=budget): before a write that would
    leave less than DRYNX_LEDGER_RESERVE_GB (default 8) free, the oldest
    generations of this rank are deleted (their proofs are no longer served
    by ``get_proofs``, which raises ``PrunedError``; bitmaps, blocks and small
    proofs stay in the database)."""

    def __init__(self, path: str, device=None):
        self.base = self.path = path
        self._gens: list = [path]  # generation files, oldest first
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self._f = open(path, "ab")
        self._ex = streams.executor(device, 1, "drynx-ledger")
        self._done: dict = {}
        self._lock = threading.Lock()
        self._device = device
        self._stream = None

    def put(self, blob_id: str, produce) -> BlobRef:
        with self._lock:
            fut = self._done.get(blob_id)
            if fut is None:
                fut = self._done[blob_id] = self._ex.submit(self._write, produce)
                while len(self._done) > 1 << 16:
                    self._done.pop(next(iter(self._done)))
        return BlobRef(self, fut)

    def get(self, blob_id: str):
        """The BlobRef of a value already put (None if unknown)."""
        with self._lock:
            fut = self._done.get(blob_id)
        return None if fut is None else BlobRef(self, fut)

    def put_many(self, blob_ids: list, produce_all) -> list:
        """Put several values produced together: ``produce_all()`` returns one
        buffer per id (e.g. slices of one device-to-host copy); they are written
        back to back by one job."""
        job = self._ex.submit(self._write, produce_all, True)
        refs = []
        with self._lock:
            for i, bid in enumerate(blob_ids):
                fut = self._done.get(bid)
                if fut is None:
                    fut = self._done[bid] = _Item(job, i)
                refs.append(BlobRef(self, fut))
            while len(self._done) > 1 << 16:
                self._done.pop(next(iter(self._done)))
        return refs

    def _write(self, produce, many: bool = False):
        import torch

        dev = torch.device(self._device) if self._device is not None else None
        if dev is not None and dev.type == "cuda":
            if self._stream is None:
                self._stream = torch.cuda.Stream(dev)
            with torch.cuda.stream(self._stream), timers.span("ledger.encode"):
                data = produce()
        else:
            with timers.span("ledger.encode"):
                data = produce()
        with timers.span("ledger.write"):
            pairs = [_unwrap(d) for d in (data if many else [data])]
            bufs, flags = [b for b, _ in pairs], [f for _, f in pairs]
            timers.count("ledger.blob_bytes", sum(b.nbytes for b in bufs))
            self._make_room(sum(b.nbytes for b in bufs) * _copies())
            self._f.flush()
            off = self._f.seek(0, os.SEEK_END)
            out, pos = [], off
            for b, fl in zip(bufs, flags):
                out.append((pos, b.nbytes, self.path, fl))  # the generation file it lands in
                pos += b.nbytes
            self._pwrite_all(bufs, off)
            self._f.seek(0, os.SEEK_END)
            for j in range(1, _copies()):
                # diagnostics: the write volume of several VN ranks, each
                # persisting its own copy (DRYNX_LEDGER_COPIES, see _copies)
                self._pwrite_all(bufs, off, f"{self.path}.copy{j}")
        with timers.span("ledger.sync"):
            for p in self._files_of(self.path):
                os.fdatasync(self._pfds[p])
        return out if many else out[0]

    _PIECE = 32 << 20  # bytes per parallel write
    pruned = 0  # generation files deleted for disk space (this process)

    def _files_of(self, path: str) -> list:
        return [path] + [f"{path}.copy{j}" for j in range(1, _copies())]

    def _rotate(self):
        """Start a new generation file (the old one stays readable)."""
        self._f.close()
        fds = self.__dict__.get("_pfds", {})
        for p in self._files_of(self.path):
            fd = fds.pop(p, None)
            if fd is not None:
                os.close(fd)
        self.path = f"{self.base}.{len(self._gens)}"
        self._gens.append(self.path)
        self._f = open(self.path, "ab")
        _fsync_dir(os.path.dirname(os.path.abspath(self.path)))

    def _make_room(self, need: int):
        import shutil

        if self._f.seek(0, os.SEEK_END) + need > _gb_env("DRYNX_LEDGER_SEGMENT_GB", 4) and \
                self._f.tell() > 0:
            self._rotate()
        if not _budget():
            return
        reserve = _gb_env("DRYNX_LEDGER_RESERVE_GB", 8)
        d = os.path.dirname(os.path.abspath(self.path))
        while shutil.disk_usage(d).free - need < reserve and len(self._gens) > 1 and self._gens[0] != self.path:
            old = self._gens.pop(0)
            _mark_pruned(old)
            for p in self._files_of(old):
                try:
                    os.remove(p)
                except FileNotFoundError:
                    pass
            BlobSegment.pruned += 1
            if BlobSegment.pruned == 1:
                import logging

                logging.getLogger("drynx_amd").warning(
                    f"ledger: disk below the {reserve / (1 << 30):.0f} GB reserve, deleting the oldest proof "
                    f"segments of {self.base} (DRYNX_LEDGER_RETAIN=budget)")

    def _pwrite_all(self, bufs: list, off: int, path: str | None = None):
        """The buffers back to back from ``off``, in pieces written by several
        threads with positioned writes (they release the GIL; one sequential
        write of a query's ~540 MB of range proofs took ~50 ms)."""
        pieces, pos = [], off
        for b in _coalesce(bufs):
            for a in range(0, b.nbytes, self._PIECE):
                pieces.append((b[a: a + self._PIECE], pos + a))
            pos += b.nbytes
        fds = self.__dict__.setdefault("_pfds", {})
        path = path or self.path
        if path not in fds:
            # positioned writes need a descriptor WITHOUT O_APPEND (Linux
            # appends every pwrite on an O_APPEND descriptor, ignoring the offset)
            fds[path] = os.open(path, os.O_WRONLY | os.O_CREAT, 0o644)
        fd = fds[path]

        def put(item):
            view, at = item
            while view.nbytes:
                k = os.pwrite(fd, view, at)
                view, at = view[k:], at + k

        if len(pieces) <= 1:
            for it in pieces:
                put(it)
            return
        if not hasattr(self, "_wpool"):
            self._wpool = streams.executor(self._device, 4, "drynx-ledger-w")
        list(self._wpool.map(put, pieces))

    def flush(self):
        with self._lock:
            futs = list(self._done.values())
        for f in futs:
            f.result()

    def close(self, remove: bool = False):
        self._ex.shutdown(wait=True)
        self._f.close()
        for path, fd in self.__dict__.pop("_pfds", {}).items():
            os.close(fd)
        if remove:
            for g in self._gens:
                for p in self._files_of(g):
                    try:
                        os.remove(p)
                    except FileNotFoundError:
                        pass


class _Done:
    """An already-known result (a reference that needs no write)."""

    def __init__(self, v):
        self.v = v

    def result(self):
        return self.v


class NodeBlobs(BlobSegment):
    """Range payloads shared by the VN ranks of ONE node, content-addressed
    (one file per payload digest under a node directory).  On an 8-GPU node
    several VN ranks receive the same signed payloads: the first rank to
    CLAIM a digest (an ``O_CREAT | O_EXCL`` marker file, atomic across the
    node's processes) copies it to the host and writes it; every other rank
    holding the same payload stores a reference to that file and skips the
    device-to-host copy -- as the VNs co-hosted on a rank already share one
    BlobSegment.  Only a rank that actually holds the payload claims it, so a
    VN rank that got a header-only envelope (``VerificationSharding``, or
    per-CN proofs fanned out to the assigned VNs only) never leaves a
    reference nobody writes.  A payload file appears under its final name
    only once fully written and fdatasync'ed (write to .tmp, sync, rename,
    directory sync); a reader that finds it missing waits for it."""

    def __init__(self, root: str, device=None):
        os.makedirs(root, exist_ok=True)
        super().__init__(os.path.join(root, f"_rank_{os.getpid()}_{id(self):x}.unused"), device)
        self.root = root
        self._files: list = []  # this rank's payload files, oldest first
        # this user's open marker: the directory goes only with its last user
        self._open_mark = os.path.join(root, f"_open_{os.getpid()}_{id(self):x}")
        open(self._open_mark, "w").close()

    def file_of(self, blob_id: str) -> str:
        return os.path.join(self.root, f"{blob_id}.blob")

    def claim(self, blob_ids: list) -> list:
        """[bool]: True where THIS rank writes the payload (first claimant on
        the node), False where another rank of the node already claimed it."""
        out = []
        for bid in blob_ids:
            try:
                os.close(os.open(self.file_of(bid) + ".claim", os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o644))
                out.append(True)
            except FileExistsError:
                out.append(False)
        return out

    def put_refs(self, blob_ids: list, sizes: list | None = None) -> list:
        """References to payloads another rank of the node claimed and writes
        (the whole file: its length and form are the writer's, which may store
        the smaller compact image; ``sizes`` is not needed)."""
        refs = []
        with self._lock:
            for bid in blob_ids:
                fut = self._done.setdefault(bid, _Done((0, 0, self.file_of(bid), None)))
                refs.append(BlobRef(self, fut))
        return refs

    def put_many(self, blob_ids: list, produce_all) -> list:
        """Write payloads this rank claimed (``claim``)."""
        job = self._ex.submit(self._write_files, list(blob_ids), produce_all)
        refs = []
        with self._lock:
            for i, bid in enumerate(blob_ids):
                fut = self._done.get(bid)
                if fut is None:
                    fut = self._done[bid] = _Item(job, i)
                refs.append(BlobRef(self, fut))
        return refs

    def _write_files(self, blob_ids: list, produce_all):
        import shutil

        import torch

        dev = torch.device(self._device) if self._device is not None else None
        if dev is not None and dev.type == "cuda":
            if self._stream is None:
                self._stream = torch.cuda.Stream(dev)
            with torch.cuda.stream(self._stream), timers.span("ledger.encode"):
                data = produce_all()
        else:
            with timers.span("ledger.encode"):
                data = produce_all()
        out = []
        with timers.span("ledger.write"):
            reserve = _gb_env("DRYNX_LEDGER_RESERVE_GB", 8)
            for bid, d in zip(blob_ids, data):
                b, compact = _unwrap(d)
                timers.count("ledger.blob_bytes", b.nbytes)
                if _budget():
                    while shutil.disk_usage(self.root).free - b.nbytes < reserve and self._files:
                        old = self._files.pop(0)
                        _mark_pruned(old)
                        try:
                            os.remove(old)
                        except FileNotFoundError:
                            pass
                        BlobSegment.pruned += 1
                final = self.file_of(bid)
                tmp = final + ".tmp"
                self._pwrite_all([memoryview(_NODE_COMPACT if compact else _NODE_RAW), b], 0, tmp)
                fd = self._pfds.pop(tmp)
                with timers.span("ledger.sync"):
                    os.fdatasync(fd)
                os.close(fd)
                os.replace(tmp, final)
                self._files.append(final)
                out.append((0, 0, final, compact))
            if blob_ids:
                _fsync_dir(self.root)
        return out

    def close(self, remove: bool = False):
        """``remove``: this rank's files go; the node directory goes only with
        its last open user (other VN ranks may still write or read there)."""
        super().close(remove)
        try:
            os.remove(self._open_mark)
        except FileNotFoundError:
            pass
        if remove:
            for p in self._files:
                for q in (p, p + ".claim"):
                    try:
                        os.remove(q)
                    except FileNotFoundError:
                        pass
            try:
                users = [n for n in os.listdir(self.root) if n.startswith("_open_")]
            except FileNotFoundError:
                return
            if not users:
                __import__("shutil").rmtree(self.root, ignore_errors=True)


class Store:
    def __init__(self, path: str):
        self.path = path
        self.blob_path = path + ".blobs"
        self._blob_f = None
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        self._lock = threading.RLock()
        self._db = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        self._db.execute("PRAGMA journal_mode=WAL")
        self._db.execute("PRAGMA synchronous=FULL")  # every commit syncs the WAL (a committed bbolt batch)
        self._db.execute("CREATE TABLE IF NOT EXISTS kv (bucket TEXT, key TEXT, value BLOB, PRIMARY KEY(bucket, key))")
        self._q: queue.Queue = queue.Queue()
        self._writer = None
        self.closed = False

    # ------------------------------------------------------------- values / blob segment
    def _encode(self, value) -> bytes:
        """Caller holds the lock.  Large values are written straight from the
        host buffer (no bytes() copy under the GIL)."""
        if isinstance(value, BlobRef):
            res = value.result()
            if isinstance(value.segment, NodeBlobs):
                return _REF4 + res[2].encode()
            off, n, path = res[:3]
            compact = len(res) > 3 and bool(res[3])
            return (_REF3 if compact else _REF2) + struct.pack("<QQ", off, n) + path.encode()
        if hasattr(value, "cpu") and hasattr(value, "numpy"):
            buf = memoryview(value.detach().cpu().contiguous().numpy()).cast("B")
        else:
            buf = memoryview(value).cast("B") if not isinstance(value, bytes) else memoryview(value)
        if buf.nbytes < BLOB_MIN:
            return buf.tobytes()
        if self._blob_f is None:
            self._blob_f = open(self.blob_path, "ab")
        off = self._blob_f.seek(0, os.SEEK_END)
        self._blob_f.write(buf)
        return _REF + struct.pack("<QQ", off, buf.nbytes)

    def _decode(self, v) -> bytes:
        """The stored value; a payload the writer TAGGED compact (``_REF3``,
        or a node file's compact tag) is rebuilt into the signed bytes."""
        v = bytes(v)
        compact = False
        if v.startswith(_REF4):
            raw = self._read_shared(v[len(_REF4):].decode(), 0, 0)
            tag, v = raw[:8], raw[8:]
            if tag not in (_NODE_RAW, _NODE_COMPACT):
                raise ValueError("ledger: node-shared payload file without its tag")
            compact = tag == _NODE_COMPACT
        elif v.startswith(_REF3) or v.startswith(_REF2):
            off, n = struct.unpack("<QQ", v[len(_REF2): len(_REF2) + 16])
            compact = v.startswith(_REF3)
            v = self._read_shared(v[len(_REF2) + 16:].decode(), off, n)
        else:
            v = self._decode_raw(v)
        if compact:
            from ..proofs import ledger_codec

            return ledger_codec.decompress_bytes(v)
        return v

    @staticmethod
    def _read_shared(path: str, off: int, n: int) -> bytes:
        """``n`` bytes at ``off`` of a file another thread or rank writes
        (n = 0: all of it), waiting for a node-shared file not written yet."""
        import time as _t

        deadline = _t.monotonic() + float(os.environ.get("DRYNX_LEDGER_WAIT_S", "60"))
        while True:
            try:
                with open(path, "rb") as f:
                    f.seek(off)
                    return f.read(n) if n else f.read()
            except FileNotFoundError:
                # a node-shared payload not yet written by the node's writer
                # rank: wait for it, unless the writer pruned it
                if _was_pruned(path):
                    raise PrunedError(f"ledger value pruned for disk space ({path}; "
                                      f"DRYNX_LEDGER_RETAIN=budget)") from None
                if _t.monotonic() < deadline:
                    _t.sleep(0.01)
                    continue
                raise FileNotFoundError(f"ledger value {path} was never written") from None

    def _decode_raw(self, v) -> bytes:
        v = bytes(v)
        if len(v) == len(_REF) + 16 and v.startswith(_REF):
            off, n = struct.unpack("<QQ", v[len(_REF):])
            if self._blob_f is not None:
                self._blob_f.flush()
            with open(self.blob_path, "rb") as f:
                f.seek(off)
                return f.read(n)
        return v

    # ------------------------------------------------------------- sync API
    def update(self, bucket: str, key: str, value: bytes):
        """UpdateDB(db, bucket, key, value)."""
        with self._lock:
            v = self._encode(value)
            if self._blob_f is not None:
                self._blob_f.flush()
                os.fdatasync(self._blob_f.fileno())
            self._db.execute("INSERT OR REPLACE INTO kv(bucket, key, value) VALUES (?,?,?)", (bucket, key, v))

    def update_many(self, rows):
        with self._lock:
            enc = [(b, k, self._encode(v)) for b, k, v in rows]
            if self._blob_f is not None:
                self._blob_f.flush()
                os.fdatasync(self._blob_f.fileno())
            self._db.execute("BEGIN")
            self._db.executemany("INSERT OR REPLACE INTO kv(bucket, key, value) VALUES (?,?,?)", enc)
            self._db.execute("COMMIT")

    def get(self, bucket: str, key: str):
        self.flush()  # read-your-writes over queued updates
        with self._lock:
            r = self._db.execute("SELECT value FROM kv WHERE bucket=? AND key=?", (bucket, key)).fetchone()
            return None if r is None else self._decode(r[0])

    def bucket(self, bucket: str) -> dict:
        self.flush()  # read-your-writes over queued updates
        with self._lock:
            rows = self._db.execute("SELECT key, value FROM kv WHERE bucket=? ORDER BY key", (bucket,)).fetchall()
            return {k: self._decode(v) for k, v in rows}

    def buckets(self) -> list:
        self.flush()  # read-your-writes over queued updates
        with self._lock:
            return [r[0] for r in self._db.execute("SELECT DISTINCT bucket FROM kv ORDER BY bucket").fetchall()]

    def cursor_prefix(self, bucket_prefix: str) -> dict:
        self.flush()  # read-your-writes over queued updates
        with self._lock:
            rows = self._db.execute("SELECT bucket, key, value FROM kv WHERE bucket LIKE ? ORDER BY bucket, key",
                                    (bucket_prefix + "%",)).fetchall()
            return {(b, k): self._decode(v) for b, k, v in rows}

    # ------------------------------------------------------------- async writer
    def update_async(self, bucket: str, key: str, value: bytes):
        if self._writer is None:
            self._writer = threading.Thread(target=self._drain, daemon=True)
            self._writer.start()
        self._q.put((bucket, key, value))

    def _drain(self):
        while True:
            item = self._q.get()
            if item is None:
                self._q.task_done()
                return
            batch = [item]
            while True:
                try:
                    nxt = self._q.get_nowait()
                except queue.Empty:
                    break
                if nxt is None:
                    self._q.put(None)
                    self._q.task_done()
                    break
                batch.append(nxt)
            with timers.span("store.write"):
                self.update_many(batch)
            for _ in batch:
                self._q.task_done()

    def flush(self):
        if self._writer is not None:
            self._q.join()

    def close(self, remove: bool = False):
        """HandleCloseDB: close and optionally delete the file (service_skipchain.go:323-342)."""
        self.flush()
        if self._writer is not None:
            self._q.put(None)
            self._writer.join(timeout=5)
            self._writer = None
        with self._lock:
            self._db.close()
            if self._blob_f is not None:
                self._blob_f.close()
                self._blob_f = None
        self.closed = True
        if remove:
            for suf in ("", "-wal", "-shm", ".blobs"):
                try:
                    os.remove(self.path + suf)
                except FileNotFoundError:
                    pass
