"""GLV decomposition of full scalars (csrc/bn254/glv_split.h): k = k1 + k2
lambda mod r with 0 <= k1 < 2^128, |k2| < 2^128 for every k < 2^256, checked
against Python integers on the host build; the GPU test checks the GLV
variable-base kernel (``native.g1_mul``) against the host build and the
oracle."""
import random

import pytest
import torch

from drynx_amd import native as nt
from drynx_amd.crypto import bn254 as bn
from drynx_amd.crypto import oracle as O


def _words_to_int(ws):
    return sum((int(w) & 0xFFFFFFFF) << (32 * i) for i, w in enumerate(ws))


def _scalars(vals, device="cpu"):
    t = torch.zeros((len(vals), 8), dtype=torch.int32)
    for i, v in enumerate(vals):
        for w in range(8):
            x = (v >> (32 * w)) & 0xFFFFFFFF
            t[i, w] = x - (1 << 32) if x >= 1 << 31 else x
    return t.to(device)


def test_glv_split_bounds_and_identity():
    rng = random.Random(7)
    vals = [0, 1, 2, O.R - 1, O.R, O.R + 1, (1 << 256) - 1, 1 << 255, nt.GLV_LAMBDA, O.R - nt.GLV_LAMBDA]
    vals += [rng.randrange(1 << 256) for _ in range(3000)] + [rng.randrange(1 << 64) for _ in range(200)]
    out = nt.glv_split(_scalars(vals))
    for v, row in zip(vals, out.tolist()):
        k1 = _words_to_int(row[:4])
        k2 = _words_to_int(row[4:8]) * (-1 if row[8] else 1)
        assert (k1 + k2 * nt.GLV_LAMBDA - v) % O.R == 0, v
        assert 0 <= k1 < 1 << 128 and abs(k2) < 1 << 128


@pytest.mark.gpu
def test_g1_mul_glv_matches_host_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    dev = "cuda"
    rng = random.Random(11)
    n = 777
    pts = [O.g1_mul(rng.randrange(1, O.R), O.G1_GEN) for _ in range(n)]
    pts[3] = None  # infinity
    ks = [rng.randrange(1 << 256) for _ in range(n)]
    ks[:6] = [0, 1, O.R, O.R - 1, (1 << 256) - 1, 3]
    P = bn.g1_jac_tensor(pts, dev)
    K = _scalars(ks, dev)
    ref = nt.g1_mul(P.cpu(), K.cpu())  # host build of the generic double-and-add
    keep = nt.G1_MUL_PAIR_ROWS
    try:
        for rows in (0, n):  # one lane per row, two lanes per row
            nt.G1_MUL_PAIR_ROWS = rows
            got = nt.g1_mul(P, K)
            assert bool(nt.g1_eq(got.cpu(), ref).all()), rows
    finally:
        nt.G1_MUL_PAIR_ROWS = keep
    for i in (0, 1, 2, 3, 4, 5, 100, 776):
        want = O.g1_mul(ks[i], pts[i]) if pts[i] is not None else None
        assert bn.g1_points_from_jac(got[i:i + 1].cpu())[0] == want
    # broadcast forms (one point / one scalar for all rows)
    one = nt.g1_mul(P[7:8].contiguous(), K)
    assert bool(nt.g1_eq(one, nt.g1_mul(P[7:8].expand(n, 24).contiguous(), K)).all())
    ones = nt.g1_mul(P, K[9:10].contiguous())
    assert bool(nt.g1_eq(ones, nt.g1_mul(P, K[9:10].expand(n, 8).contiguous())).all())
