"""Three-lanes-per-item GT product kernels (csrc/bn254/gt_coop.h) against the
host path of the same ops, bit for bit: the verifier's segmented bucket
products (dx_gt_slice_prod) and the GLS-8 table prover passes
(dx_rp_prove_a_gls8: gT^t from the 16-bit table, then E_phi^e * gT^t).
Sizes are not multiples of the 21 items per wave, slices include empty and
one-factor ones, and scalars include 0 and r - 1 (every window digit sign)."""
import random

import pytest
import torch

from drynx_amd import native as nt
from drynx_amd.crypto import bn254 as bn
from drynx_amd.crypto import oracle as O

pytestmark = pytest.mark.gpu
RNG = random.Random(2026)


def _gt_rows(n: int, device) -> torch.Tensor:
    g = O.pairing(O.G1_GEN, O.G2_GEN)
    base = bn.gt_tensor([g ** RNG.randrange(1, O.R) for _ in range(4)], device)
    k = bn.scalars_tensor([RNG.randrange(O.R) for _ in range(n)], device)
    return nt.gt_pow(base.repeat(-(-n // 4), 1)[:n].contiguous(), k)


def test_gt_slice_prod_coop_matches_host(gpu_device):
    src = _gt_rows(50, gpu_device)
    lens = [0, 1, 2, 7, 8, 3, 0, 5] * 6 + [9]                              # 49 slices
    start = torch.tensor([sum(lens[:i]) % 40 for i in range(len(lens))], dtype=torch.int64)
    length = torch.tensor(lens, dtype=torch.int32)
    idx = torch.tensor([RNG.randrange(50) for _ in range(int(start.max()) + max(lens))], dtype=torch.int64)
    for ix in (None, idx):
        got = nt.gt_slice_prod(src, None if ix is None else ix.to(gpu_device), start.to(gpu_device),
                               length.to(gpu_device))
        ref = nt.gt_slice_prod(src.cpu(), ix, start, length)
        assert torch.equal(got.cpu(), ref)


def test_gls8_prover_coop_matches_host(gpu_device):
    S, L, n_p = 3, 5, 3                                                     # 45 items, 15 (p, j) pairs
    bases = _gt_rows(4, gpu_device)
    tabs = nt.gt_gls8_table(bases)
    n = n_p * S * L
    tidx = torch.tensor([RNG.randrange(4) for _ in range(n)], dtype=torch.int32)
    es = [RNG.randrange(O.R) for _ in range(n - 2)] + [0, O.R - 1]
    ts = [RNG.randrange(O.R) for _ in range(n_p * L - 2)] + [O.R - 1, 0]
    e_sc, t_sc = bn.scalars_tensor(es, "cpu"), bn.scalars_tensor(ts, "cpu")
    from drynx_amd.proofs.range_proof import gt_generator_table

    _, comb = gt_generator_table("cpu")
    got = nt.rp_prove_a_tab(tabs, tidx.to(gpu_device), e_sc.to(gpu_device), t_sc.to(gpu_device), None, S, L, 7)
    ref = nt.rp_prove_a_tab(tabs.cpu(), tidx, e_sc, t_sc, comb, S, L, 7)
    assert torch.equal(got.cpu(), ref)
