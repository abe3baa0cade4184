"""Chunked payload digest (host hashlib vs native kernel) and the ChaCha20
scalar CSPRNG.  GPU variants compare the device kernels with the host path."""
import hashlib
import os

import numpy as np
import pytest
import torch

from drynx_amd import native as nt
from drynx_amd.crypto import bn254 as bn
from drynx_amd.crypto import digest as D
from drynx_amd.crypto import oracle as O


def _t(b: bytes, device="cpu"):
    return torch.from_numpy(np.frombuffer(b, dtype="<i4").copy()).to(device)


@pytest.mark.parametrize("n", [0, 4, 60, 64, 124, 4092, 4096, 4100, 3 * 4096 + 44, 65536])
def test_digest_tensor_matches_bytes(n):
    b = os.urandom(n)
    assert D.digest_bytes(b) == D.digest_tensor(_t(b))


def test_slice_digest_is_plain_sha256():
    b = os.urandom(2 * D.CHUNK + 100)
    w = nt.sha256_chunks(_t(b), D.CHUNK).numpy().view(np.uint32).astype(">u4")
    for i in range(3):
        assert w[i].tobytes() == hashlib.sha256(b[i * D.CHUNK:(i + 1) * D.CHUNK]).digest()


def test_digest_sensitive_to_every_byte():
    b = bytearray(os.urandom(3 * D.CHUNK))
    d0 = D.digest_bytes(bytes(b))
    for pos in (0, D.CHUNK - 1, D.CHUNK, len(b) - 1):
        c = bytearray(b)
        c[pos] ^= 1
        assert D.digest_tensor(_t(bytes(c))) != d0


def test_random_scalars_range_and_freshness():
    a = bn.scalars_from_tensor(bn.random_scalars(20000))
    b = bn.scalars_from_tensor(bn.random_scalars(20000))
    assert all(0 < x < O.R for x in a)
    assert len(set(a) | set(b)) == 40000  # fresh key per call
    # top-bit frequency of a uniform value in [0, r): P(x >= 2^253) = 1 - 2^253/r
    p = 1 - (1 << 253) / O.R
    f = sum(x >> 253 for x in a) / len(a)
    assert abs(f - p) < 0.02


@pytest.mark.gpu
def test_gpu_digest_and_rng(gpu_device):
    b = os.urandom(5 * D.CHUNK + 12)
    assert D.digest_tensor(_t(b, gpu_device)) == D.digest_bytes(b)
    s = bn.scalars_from_tensor(bn.random_scalars(50000, gpu_device))
    assert all(0 < x < O.R for x in s) and len(set(s)) == 50000


def test_digest_many_matches_single():
    import torch

    from drynx_amd.crypto import digest as dg

    ts = [torch.arange(n, dtype=torch.int32) * 7 + n for n in (0, 1, 1023, 1024, 1025, 5000, 3)]
    ts.append(torch.arange(300, dtype=torch.uint8))
    got = dg.digest_many(ts)
    for t, d in zip(ts, got):
        assert d == dg.digest_bytes(t.numpy().tobytes())


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_prg_glv_matches_generator_then_glv(device):
    """The fused GLV-weight draw equals the generator's scalars turned into
    GLV weights (32-bit halves a, b of each scalar; rho = a + b lambda)."""
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    key = bytes(range(32))
    ab, rho = nt.prg_glv(key, 1000, device)
    ab2, rho2 = nt.glv_weights(1000, device, raw=nt.prg_scalars(key, 1000, device))
    assert torch.equal(ab.cpu(), ab2.cpu()) and torch.equal(rho.cpu(), rho2.cpu())
    a, b = int(ab[7, 0]) & 0xFFFFFFFF, int(ab[7, 1]) & 0xFFFFFFFF
    assert bn.scalars_from_tensor(rho[7:8].cpu())[0] == (a + b * nt.GLV_LAMBDA) % O.R


@pytest.mark.gpu
def test_gpu_slice_hashes_match_hashlib(gpu_device):
    """The LDS-staged slice hashing (csrc/kernels/dx_hash.hip sha_slices_kernel)
    against hashlib: payloads of every tail shape (empty, < 1 block, exact
    blocks, several 4 KiB slices with a partial last one), 4-byte-offset views,
    many segments in one launch (more lanes than slices in the last wave) and
    equal-length rows."""
    rng = np.random.default_rng(5)
    sizes = [0, 4, 60, 64, 120, 4096, 4100, 3 * 4096 + 64, 70000, 1 << 20]
    host = [rng.integers(0, 2**31, size=(n + 3) // 4, dtype=np.int64).astype(np.int32)[: n // 4] for n in sizes]
    ts = [torch.from_numpy(h).to(gpu_device) for h in host]
    base = torch.from_numpy(rng.integers(0, 2**31, size=50001, dtype=np.int64).astype(np.int32)).to(gpu_device)
    ts.append(base[1:])                                   # a view starting 4 bytes into its storage
    host.append(base[1:].cpu().numpy())
    for t, h in zip(ts, host):
        assert D.digest_tensor(t) == D.digest_bytes(h.tobytes()), len(h)
    assert D.digest_many(ts) == [D.digest_bytes(h.tobytes()) for h in host]
    rows = torch.from_numpy(rng.integers(0, 2**31, size=(7, 3000), dtype=np.int64).astype(np.int32)).to(gpu_device)
    assert D.digest_rows(rows) == [D.digest_bytes(r.tobytes()) for r in rows.cpu().numpy()]


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("bits", [32, 40, 64, 254])
def test_prg_bits_matches_generator_then_mask(device, bits):
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    from drynx_amd.crypto.coins import mask_bits

    key = bytes(range(1, 33))
    got = nt.prg_bits(key, 777, bits, device).cpu()
    want = mask_bits(nt.prg_scalars(key, 777, device).cpu(), bits)
    assert torch.equal(got, want)
