"""Batched data movement (csrc/kernels/dx_copy.hip): one-launch copies of
many regions (nt.batched_copy / nt.cat_rows, used by rp.rpl_cat and the
verifier's stacked GT image) and the per-row AND of validity flags
(nt.rows_all, used by rp.validate_list), each against plain torch."""
import pytest
import torch

from drynx_amd import native as nt

DEVICES = ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)]


def _dev(name):
    if name == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device(name)


@pytest.mark.parametrize("device", DEVICES)
def test_cat_rows_matches_torch_cat(device):
    dev = _dev(device)
    g = torch.Generator().manual_seed(7)
    groups = []
    for width, rows in [(96, [5000, 1, 37, 4097]), (8, [3, 100000]), (24, [1]), (32, [0, 9, 70000])]:
        groups.append([torch.randint(-2**31, 2**31 - 1, (r, width), generator=g, dtype=torch.int32).to(dev)
                       for r in rows])
    # a non-contiguous member and a float64 group
    groups.append([torch.arange(64, dtype=torch.int32).view(8, 8).t().to(dev), torch.ones((3, 8), dtype=torch.int32,
                                                                                           device=dev)])
    groups.append([torch.rand((11, 3), generator=g, dtype=torch.float64).to(dev) for _ in range(3)])
    outs = nt.cat_rows(groups)
    for grp, out in zip(groups, outs):
        assert torch.equal(out, torch.cat(grp))


@pytest.mark.parametrize("device", DEVICES)
def test_batched_copy_into_views(device):
    dev = _dev(device)
    src = torch.arange(3 * 50000, dtype=torch.int32, device=dev).view(3, 50000)
    dst = torch.zeros((2, 3 * 50000), dtype=torch.int32, device=dev)
    nt.batched_copy([(src[i].contiguous(), dst[1, i * 50000:(i + 1) * 50000]) for i in range(3)])
    assert torch.equal(dst[1], src.reshape(-1)) and int(dst[0].abs().sum()) == 0


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("n", [1, 5, 777])
def test_rows_all_matches_torch(device, n):
    dev = _dev(device)
    g = torch.Generator().manual_seed(n)
    flags = []
    for k in [1, 3, 48, 200, 576] + [2] * 14:                     # 19 arrays: two launches of <= 16
        f = (torch.rand((n * k,), generator=g) > 0.002 / k).to(torch.uint8)
        flags.append(f.to(dev))
    flags.append(torch.ones((n * 4,), dtype=torch.bool, device=dev))
    want = torch.stack([f.bool().view(n, -1).all(dim=1) for f in flags]).all(dim=0)
    got = nt.rows_all(flags, n)
    assert got.dtype == torch.uint8 and torch.equal(got.bool(), want)
    # a single failing entry fails exactly its row
    flags[3] = torch.ones_like(flags[3])
    flags = [torch.ones_like(f) for f in flags]
    flags[4][(n // 2) * 576 + 575] = 0
    got = nt.rows_all(flags, n).bool()
    assert not bool(got[n // 2]) and int(got.sum()) == n - 1
