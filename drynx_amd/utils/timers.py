"""Named wall-clock timers (reference: unlynx ``StartTimer/EndTimer`` over onet
``simul/monitor``, 25 call sites; names kept identical for comparability:
``<node>_DataCollectionProtocol``, ``JustExecution``, ``<node>_AggregationPhase``,
``<node>_KeySwitchingPhase``, ``<name>_DPencoding``, ``<name>_AllProofs``,
``<VN>_VerifyRange``, ``BI``, ``Decode``, ``Decryption``, ``GradientDescent``,
``Simulation``...).  A timer is wall time from the host's start of the phase
to the completion of the device work the phase queued (see ``Timer``), and
each timer also emits a roctx range when profiling under rocprofv3."""
from __future__ import annotations

import contextlib
import csv
import json
import os
import threading
import time
from collections import defaultdict

import torch

_lock = threading.Lock()
_records: dict = defaultdict(list)
# host-side span trace (DRYNX_TRACE=<path>): chrome://tracing JSON of every timer
# and span, per thread, without extra device syncs -- lines up with a rocprofv3
# kernel trace to show where the host sits between kernels
_TRACE = os.environ.get("DRYNX_TRACE")
_events: list = []


def _emit(name: str, t0_ns: int, t1_ns: int):
    th = threading.current_thread()
    with _lock:
        _events.append({"name": name, "ph": "X", "pid": os.getpid(), "tid": th.name, "ts": t0_ns / 1e3,
                        "dur": (t1_ns - t0_ns) / 1e3})


# DRYNX_SPAN_SYNC=1 (diagnostics, with DRYNX_TRACE): every span synchronises
# the device on entry and exit, so its duration is its own host + GPU cost
# with nothing overlapping (a serialized cost breakdown of a code path)
_SPAN_SYNC = os.environ.get("DRYNX_SPAN_SYNC") == "1"


def _dev_sync():
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


PROFILE_SPANS = False  # tools set this under torch.profiler: spans become record_function ranges
# DRYNX_ROCTX=1: every span is also a roctx range, so a rocprofv3
# --runtime-trace run attributes each kernel to the innermost span that
# launched it (tools/span_kernels.py)
_ROCTX = os.environ.get("DRYNX_ROCTX") == "1"


@contextlib.contextmanager
def span(name: str):
    """A no-sync traced region (free when DRYNX_TRACE is unset)."""
    if PROFILE_SPANS:
        with torch.profiler.record_function(name):
            yield
        return
    if not _TRACE and not _ROCTX:
        yield
        return
    if _SPAN_SYNC:
        _dev_sync()
    if _ROCTX:
        torch.cuda.nvtx.range_push(name)
    t0 = time.perf_counter_ns()
    try:
        yield
    finally:
        if _SPAN_SYNC:
            _dev_sync()
        if _ROCTX:
            torch.cuda.nvtx.range_pop()
        if _TRACE:
            _emit(name, t0, time.perf_counter_ns())


def dump_trace(path: str | None = None):
    path = path or _TRACE
    if not path:
        return
    with _lock:
        ev = list(_events)
    with open(path, "w") as f:
        json.dump({"traceEvents": ev, "displayTimeUnit": "ms"}, f)


def _device_timed() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_initialized()


_DEVICE = None  # the rank's GPU (``set_device``); None: the calling thread's current device


def set_device(device):
    """The node's device: phase-end events are recorded on ITS current stream
    (a phase may end on a worker thread)."""
    global _DEVICE
    d = torch.device(device)
    _DEVICE = d if d.type == "cuda" else None


# Phase timers measure WALL time from the host's start of the phase to the
# completion of the last operation the phase queued on its stream (the
# reference's StartTimer/EndTimer bracket goroutines that block until their
# work is done).  ``end`` records a HIP event instead of synchronising the
# query's thread; a watcher thread stamps the host time at which the event
# completes (polling, 0.2 ms) and records ``completion - start``.  A phase that
# starts behind a stream backlog therefore counts the wait, and work the phase
# joined from other streams (wait_stream before ``end``) is covered.
_watch: list = []          # (name, host start, end event) not yet complete
_watch_cv = threading.Condition(_lock)
_watcher = None


def _watch_loop():
    while True:
        with _watch_cv:
            while not _watch:
                _watch_cv.wait()
            items = list(_watch)
        done = []
        for it in items:
            if it[2].query():
                done.append((it, time.perf_counter()))
        with _watch_cv:
            for it, t1 in done:
                _watch.remove(it)
                _records[it[0]].append(t1 - it[1])
            if done:
                _watch_cv.notify_all()
        time.sleep(0.0002)


def _resolve():
    """Wait until every watched phase has completed and been recorded."""
    with _watch_cv:
        while _watch:
            _watch_cv.wait(0.05)


class Timer:
    def __init__(self, name: str, sync: bool = True):
        self.name = name
        self.sync = sync
        self.t0 = None

    def start(self):
        self.t0 = time.perf_counter()
        return self

    def end(self) -> float:
        global _watcher
        t1 = time.perf_counter()
        if _TRACE:
            _emit(self.name, int(self.t0 * 1e9), int(t1 * 1e9))
        if self.sync and _device_timed():
            e1 = torch.cuda.Event()
            # on the rank's device explicitly (``set_device``), whatever thread ends the phase
            e1.record(torch.cuda.current_stream(_DEVICE))
            if not e1.query():  # the phase's device work is still running: the watcher stamps its end
                with _watch_cv:
                    _watch.append((self.name, self.t0, e1))
                    if _watcher is None:
                        _watcher = threading.Thread(target=_watch_loop, daemon=True, name="drynx-timers")
                        _watcher.start()
                    _watch_cv.notify_all()
                return t1 - self.t0
            t1 = time.perf_counter()
        dt = t1 - self.t0
        with _lock:
            _records[self.name].append(dt)
        return dt


def start_timer(name: str, sync: bool = True) -> Timer:
    return Timer(name, sync).start()


def end_timer(t: Timer) -> float:
    return t.end()


@contextlib.contextmanager
def timed(name: str, sync: bool = True):
    rng = None
    try:
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            rng = torch.cuda.nvtx.range_push(name)
    except Exception:  # roctx not present
        rng = None
    t = Timer(name, sync).start()
    try:
        yield t
    finally:
        t.end()
        if rng is not None:
            try:
                torch.cuda.nvtx.range_pop()
            except Exception:
                pass


def record(name: str, seconds: float):
    """Add an externally measured interval under ``name``."""
    with _lock:
        _records[name].append(seconds)


def records() -> dict:
    _resolve()
    with _lock:
        return {k: list(v) for k, v in _records.items()}


_counts: dict = defaultdict(int)


def count(name: str, n: int = 1):
    """Add ``n`` to a named work counter (e.g. range items this rank checked
    for the VN pool); reported next to the timers, cleared by ``reset``."""
    with _lock:
        _counts[name] += int(n)


def counters() -> dict:
    with _lock:
        return dict(_counts)


def reset():
    _resolve()
    with _lock:
        _records.clear()
        _counts.clear()


def summary() -> dict:
    _resolve()
    with _lock:
        return {k: {"n": len(v), "sum": sum(v), "mean": sum(v) / len(v), "max": max(v)} for k, v in _records.items()}


def write_csv(path: str):
    """onet-simul-like CSV: one row per timer with n/sum/mean/max (parsed by simul.parse_time_data)."""
    s = summary()
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "n", "sum", "mean", "max"])
        for k in sorted(s):
            w.writerow([k, s[k]["n"], f"{s[k]['sum']:.6f}", f"{s[k]['mean']:.6f}", f"{s[k]['max']:.6f}"])
