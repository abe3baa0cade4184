"""Field inversion (csrc/bn254/field.h ``finv``: Bernstein-Yang safegcd,
10 x 59 half-delta divsteps) against Python's modular exponentiation, on
the host build of the same source; the GPU suite compares the device build
against the host one (tests/test_gpu.py Fr inverse, G1 to_affine)."""
import random

import torch

from drynx_amd import native as nt
from drynx_amd.crypto import bn254 as bn
from drynx_amd.crypto import oracle as O

R_ORDER = O.R


def _limbs(x: int) -> list:
    return [(x >> (32 * i)) & 0xFFFFFFFF for i in range(8)]


def _int(row) -> int:
    return sum((v & 0xFFFFFFFF) << (32 * i) for i, v in enumerate(row))


def test_fr_inverse_matches_pow():
    rng = random.Random(7)
    r = R_ORDER
    vals = [0, 1, 2, 3, r - 1, r - 2, (r + 1) // 2, 1 << 200, (1 << 253) % r]
    vals += [rng.randrange(r) for _ in range(3000)]
    vals += [rng.randrange(1 << 64) for _ in range(200)]   # short inputs (many divsteps on a small g)
    t = torch.tensor([_limbs(v) for v in vals], dtype=torch.int64).to(torch.int32)
    out = nt.fr_arith(nt.FR_INV, t.contiguous(), t.contiguous()).tolist()
    for v, row in zip(vals, out):
        assert _int(row) == (pow(v, r - 2, r) if v else 0), v


def test_fp_inverse_through_affine_conversion():
    """Jacobian -> affine divides by Z^2, Z^3 with one Fp inversion per point:
    points with random Z (scalar multiples) against the oracle's affine ones."""
    rng = random.Random(11)
    ks = [1, 2, 3] + [rng.randrange(1, R_ORDER) for _ in range(400)]
    jac = nt.g1_mul(bn.g1_jac_tensor([O.G1_GEN] * len(ks)), bn.scalars_tensor(ks))
    got = bn.g1_points_from_aff(nt.g1_to_affine(jac))
    for k, pt in zip(ks, got):
        assert pt == O.g1_mul(k, O.G1_GEN), k
