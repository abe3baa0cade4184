"""Stream priorities of the framework's HIP streams.

``priority(p)`` is the priority a stream asks for; DRYNX_STREAM_PRIO=0 turns
every request into the normal priority.  ROCm gives each priority level its
own hardware queue, so only then does a measurement run with
GPU_MAX_HW_QUEUES=1 and AMD_SERIALIZE_KERNEL=3 put every stream on ONE queue
and run every kernel alone on the chip (tools/gpu/r4_spans.sh: per-kernel
costs with no overlap inflation)."""
from __future__ import annotations

import os


def priority(p: int) -> int:
    return 0 if os.environ.get("DRYNX_STREAM_PRIO", "1") == "0" else int(p)
