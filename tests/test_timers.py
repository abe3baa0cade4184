"""Reference-named phase timers are wall time (unlynx StartTimer/EndTimer
around blocking goroutines): from the host's start of the phase to the
completion of the device work it queued (utils/timers.py)."""
import threading
import time

import pytest
import torch

from drynx_amd.utils import timers


def test_host_only_phase_is_wall_time():
    timers.reset()
    with timers.timed("HostPhase"):
        time.sleep(0.03)
    with timers.timed("HostPhaseNoSync", sync=False):
        time.sleep(0.01)
    s = timers.summary()
    assert 0.03 <= s["HostPhase"]["sum"] < 0.5
    assert 0.01 <= s["HostPhaseNoSync"]["sum"] < 0.5


def test_timers_from_threads():
    timers.reset()

    def work(k):
        with timers.timed(f"T{k}"):
            time.sleep(0.005 * (k + 1))

    ths = [threading.Thread(target=work, args=(k,)) for k in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    s = timers.summary()
    assert all(s[f"T{k}"]["sum"] >= 0.005 * (k + 1) for k in range(4))


@pytest.mark.gpu
def test_phase_behind_stream_backlog_counts_the_wait(gpu_device):
    """A phase started while its stream still runs earlier work ends when its
    own (queued-after) work completes: the timer covers the backlog, and the
    phase's device work that outlives ``end`` is counted too."""
    a = torch.randn(8192, 8192, device=gpu_device)
    for _ in range(2):
        a = a @ a / 8192                        # library warm-up (kernel selection) outside the reference time
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(6):
        a = a @ a / 8192
    torch.cuda.synchronize()
    backlog = time.perf_counter() - t
    timers.reset()
    for _ in range(6):
        a = a @ a / 8192                    # the backlog, queued before the phase
    with timers.timed("Behind"):
        b = a + 1                           # a tiny phase behind the backlog
    host_end = time.perf_counter()
    torch.cuda.synchronize()
    s = timers.summary()
    assert s["Behind"]["sum"] >= 0.5 * backlog, (s["Behind"], backlog)
    assert s["Behind"]["sum"] > 0.5 * (time.perf_counter() - host_end)
    del b
    # a phase whose own device work outlives end(): counted until it completes
    timers.reset()
    with timers.timed("LongDevice"):
        for _ in range(6):
            a = a @ a / 8192
    torch.cuda.synchronize()
    assert timers.summary()["LongDevice"]["sum"] >= 0.5 * backlog
