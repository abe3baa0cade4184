"""Stream priorities of the framework's HIP streams, and the node's worker
threads pinned to the rank's device.

``priority(p)`` is the priority a stream asks for; DRYNX_STREAM_PRIO=0 turns
every request into the normal priority.  ROCm gives each priority level its
own hardware queue, so only then does a measurement run with
GPU_MAX_HW_QUEUES=1 and AMD_SERIALIZE_KERNEL=3 put every stream on ONE queue
and run every kernel alone on the chip (tools/gpu/r4_spans.sh: per-kernel
costs with no overlap inflation)."""
from __future__ import annotations

import os
import threading


def priority(p: int) -> int:
    return 0 if os.environ.get("DRYNX_STREAM_PRIO", "1") == "0" else int(p)


NODE_SWITCH_INTERVAL = 0.0005


def node_process_setup():
    """Process-wide settings for a process whose job is to run a node (bench,
    ``server run``; a library user's process is left alone): a 0.5 ms GIL
    switch interval, so the node's worker threads (ledger writers, CN-proof
    finishing, the pool, the querier) hand the interpreter back to the
    query's thread sooner than Python's 5 ms (--u 0 --l 0 25.8-28.2 ->
    23.4-23.9 ms on one box, the headline unchanged: profiles/r4/serial/v_*.json)."""
    import sys

    sys.setswitchinterval(NODE_SWITCH_INTERVAL)


_made: list = []  # thread-name prefixes of every executor made here (tests audit the node's workers)
_tls = threading.local()


def executor(device=None, max_workers: int = 1, name: str = "drynx"):
    """Every worker thread of a node comes from here: a ThreadPoolExecutor
    whose threads start by making the rank's GPU their current device
    (``torch.cuda.set_device``), so a worker of rank k never launches or
    allocates on device 0 by default (one process per GPU: on an 8-GPU node
    a device-k worker touching device 0 would only show in the 8-GPU run).
    ``device`` None / CPU: plain threads."""
    import concurrent.futures as cf

    import torch

    dev = torch.device(device) if device is not None else None
    init = None
    if dev is not None and dev.type == "cuda" and os.environ.get("DRYNX_PIN_WORKERS", "1") != "0":
        idx = dev.index if dev.index is not None else torch.cuda.current_device()

        def init():
            torch.cuda.set_device(idx)
            _tls.device = idx
    _made.append(name)
    return cf.ThreadPoolExecutor(max_workers=max_workers, thread_name_prefix=name, initializer=init)


def pinned_device():
    """The device index this worker thread was pinned to (None: not a pinned worker)."""
    return getattr(_tls, "device", None)
