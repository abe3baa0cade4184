"""Named wall-clock timers (reference: unlynx ``StartTimer/EndTimer`` over onet
``simul/monitor``, 25 call sites; names kept identical for comparability:
``<node>_DataCollectionProtocol``, ``JustExecution``, ``<node>_AggregationPhase``,
``<node>_KeySwitchingPhase``, ``<name>_DPencoding``, ``<name>_AllProofs``,
``<VN>_VerifyRange``, ``BI``, ``Decode``, ``Decryption``, ``GradientDescent``,
``Simulation``...).  GPU work inside a timer is synchronised at the end so the
interval is real device time, and each timer also emits a roctx range when
profiling under rocprofv3."""
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


def _sync():
    # the calling thread's stream only: phases running on other threads/streams
    # (querier decode, proof signing) keep overlapping
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.current_stream().synchronize()


def _use_events() -> bool:
    """Device-timed phases measure with HIP events on the phase's stream
    (resolved when the timers are read) instead of synchronising the host at
    both ends: a phase timer then costs the query no host-device round trip.
    DRYNX_TIMER_SYNC=1 restores the synchronising timers."""
    return (os.environ.get("DRYNX_TIMER_SYNC") != "1" and torch.cuda.is_available()
            and torch.cuda.is_initialized())


_pending: list = []  # (name, start event, end event) of event-timed phases


def _resolve():
    """Turn finished event pairs into recorded intervals (device time from
    the phase's first to its last queued operation on its stream)."""
    with _lock:
        todo = list(_pending)
        _pending.clear()
    done = []
    for name, e0, e1 in todo:
        e1.synchronize()
        done.append((name, e0.elapsed_time(e1) / 1e3))
    with _lock:
        for name, dt in done:
            _records[name].append(dt)


class Timer:
    def __init__(self, name: str, sync: bool = True):
        self.name = name
        self.sync = sync
        self.t0 = None
        self.ev = None

    def start(self):
        if self.sync and _use_events():
            self.ev = torch.cuda.Event(enable_timing=True)
            self.ev.record()
        elif self.sync:
            _sync()
        self.t0 = time.perf_counter()
        return self

    def end(self) -> float:
        if self.ev is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            t1 = time.perf_counter()
            with _lock:
                _pending.append((self.name, self.ev, e1))
                if len(_pending) > 4096:
                    todo = _pending[:2048]
                    del _pending[:2048]
                    for name, a, b in todo:
                        b.synchronize()
                        _records[name].append(a.elapsed_time(b) / 1e3)
            if _TRACE:
                _emit(self.name, int(self.t0 * 1e9), int(t1 * 1e9))
            return t1 - self.t0
        if self.sync:
            _sync()
        t1 = time.perf_counter()
        dt = t1 - self.t0
        with _lock:
            _records[self.name].append(dt)
        if _TRACE:
            _emit(self.name, int(self.t0 * 1e9), int(t1 * 1e9))
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
    with _lock:
        _pending.clear()
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
