"""Lifetime of cached device-resident bucket plans (native._device_layout).

Round 5 captured the pool verifier's passes in HIP graphs and saw replays
fault (profiles/r6/graph_fault.md): the plan cache evicts layouts (32 shapes)
while a captured graph -- or, eagerly, another stream's queued kernels --
still read them, and the caching allocator handed the freed blocks to new
allocations.  Now every stream that reads a layout is recorded on its tensors
(eviction waits for them) and a capture keeps every layout it reads."""
import pytest
import torch

from drynx_amd import native as nt


def _shape(i):
    return ((64 + i, 64),)


def test_capture_keep_collects_layouts():
    with nt.capture_keep() as ck:
        a = nt._device_layout(_shape(0), 8, 8, 32, "cpu")
        b = nt._device_layout(_shape(1), 8, 8, 32, "cpu")
    assert ck.items[0] is a and ck.items[1] is b
    nt._device_layout(_shape(2), 8, 8, 32, "cpu")
    assert len(ck.items) == 2  # collection ends with the block


def test_eviction_keeps_captured_layouts_alive(monkeypatch):
    monkeypatch.setattr(nt, "_PLAN_LIMIT", 2)
    with nt.capture_keep() as ck:
        held = nt._device_layout(_shape(10), 8, 8, 32, "cpu")
    for i in range(11, 20):  # evicts shape 10 from the cache
        nt._device_layout(_shape(i), 8, 8, 32, "cpu")
    key = (_shape(10), 8, 8, 32, "cpu")
    assert key not in nt._DPLANS and ck.items[0] is held
    assert held["lane_bucket"].numel() == held["n_lanes"]  # still a live tensor the graph can read


@pytest.mark.gpu
def test_layout_records_every_user_stream(gpu_device):
    s1, s2 = torch.cuda.Stream(gpu_device), torch.cuda.Stream(gpu_device)
    with torch.cuda.stream(s1):
        lay = nt._device_layout(_shape(40), 8, 8, 32, gpu_device)
    with torch.cuda.stream(s2):
        again = nt._device_layout(_shape(40), 8, 8, 32, gpu_device)
    assert again is lay and {s1.stream_id, s2.stream_id} <= lay["_streams"]


@pytest.mark.gpu
def test_lazy_constant_published_across_streams(gpu_device):
    """A device constant built lazily on a busy stream (the GLV beta of the
    variable-base multiplication: its pinned upload queues behind that
    stream's kernels) is complete before another stream can read it
    (``bn.publish``).  Round 6 found the verifier's pool stream creating it
    while the key-switching stream used it at once: garbage shares, and the
    querier's decryption of an LR aggregate failed (tests/test_multirank_gpu.py)."""
    from drynx_amd.crypto import bn254 as bn

    n = 1 << 16
    pts = nt.g1_fb_mul(bn.base_table(gpu_device), bn.random_scalars(n, gpu_device))
    k = bn.random_scalars(n, gpu_device)
    want = nt.g1_to_affine(nt.g1_mul(pts.cpu(), k.cpu()))
    busy, other = torch.cuda.Stream(gpu_device), torch.cuda.Stream(gpu_device)
    busy.wait_stream(torch.cuda.current_stream(gpu_device))
    other.wait_stream(torch.cuda.current_stream(gpu_device))
    nt._glv_consts.clear()
    tab = bn.base_table(gpu_device)
    with torch.cuda.stream(busy):
        for _ in range(8):  # a backlog on the creating stream (kernels that do not read the constant)
            nt.g1_fb_mul(tab, k)
        nt._glv_const("beta", gpu_device)
    with torch.cuda.stream(other):
        got = nt.g1_to_affine(nt.g1_mul(pts, k))
    torch.cuda.synchronize()
    assert torch.equal(got.cpu(), want)
