"""Tensor-level BN254 API on top of the native library.

Converts between Python integers / oracle points and limb tensors, owns the
per-device fixed-base tables of the generators B (G1) and B2 (G2), provides
the CSPRNG for scalars (kernel ``getrandom`` via ``os.urandom``, never a
non-cryptographic PRNG — reference: every ``Scalar().Pick(RandomStream())``),
and the kyber wire codecs (G1 64 B, G2 128 B, GT 384 B, scalar 32 B,
big-endian; reference lib/range/range_proof.go:72-246, lib/structs.go:403).
"""
from __future__ import annotations

import os
import threading

import numpy as np
import torch

from .. import native as nt
from . import oracle as O

P, R = O.P, O.R
RM = 1 << 256
RINV_P = pow(RM, -1, P)

# ----------------------------------------------------------------------------- limb conversion


def ints_to_limbs(vals, n_limbs: int = 8) -> np.ndarray:
    vals = list(vals)
    nbytes = 4 * n_limbs
    buf = b"".join(int(v).to_bytes(nbytes, "little") for v in vals)
    return np.frombuffer(buf, dtype="<u4").reshape(len(vals), n_limbs).copy()


def limbs_to_ints(arr) -> list[int]:
    a = np.ascontiguousarray(np.asarray(arr, dtype=np.uint32).reshape(-1, 8))
    raw = a.astype("<u4").tobytes()
    return [int.from_bytes(raw[32 * i: 32 * i + 32], "little") for i in range(a.shape[0])]


def to_tensor(a: np.ndarray, device) -> torch.Tensor:
    return h2d(torch.from_numpy(np.ascontiguousarray(a).view(np.int32)), device)


def h2d(t: torch.Tensor, device) -> torch.Tensor:
    """Host tensor -> ``device``.  To a GPU through pinned memory and an
    asynchronous copy: a pageable copy blocks the host until every kernel
    already queued on the stream has finished, which stalls the launch
    sequences of the prover and verifier threads."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return t
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("h2d: host upload inside a HIP graph capture")
    return t.pin_memory().to(dev, non_blocking=True)


def to_numpy(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().contiguous().numpy().view(np.uint32)


def mont(x: int) -> int:
    return (x % P) * RM % P


def unmont(x: int) -> int:
    return x * RINV_P % P


# ----------------------------------------------------------------------------- scalars
def scalars_tensor(vals, device="cpu") -> torch.Tensor:
    return to_tensor(ints_to_limbs([int(v) % R for v in vals]), device)


def scalars_from_tensor(t: torch.Tensor) -> list[int]:
    return limbs_to_ints(to_numpy(t))


_R_LIMBS = ints_to_limbs([R])[0]


def random_scalars(n: int, device="cpu") -> torch.Tensor:
    """n uniform scalars in [1, r): ChaCha20 keyed from the OS CSPRNG, expanded
    where the scalars are consumed (one GPU launch for a whole proof batch)."""
    return nt.random_scalars(n, device)


def random_scalars_host_rejection(n: int) -> np.ndarray:
    """Reference sampler (os.urandom + rejection) kept for distribution tests."""
    out = np.empty((0, 8), dtype=np.uint32)
    need = n
    while need > 0:
        m = int(need * 1.4) + 8
        raw = np.frombuffer(os.urandom(32 * m), dtype="<u4").reshape(m, 8).copy()
        raw[:, 7] &= 0x3FFFFFFF  # < 2^254
        v = raw.astype(np.uint64)
        rl = _R_LIMBS.astype(np.uint64)
        less = np.zeros(m, dtype=bool)
        eq = np.ones(m, dtype=bool)
        for k in range(7, -1, -1):
            less |= eq & (v[:, k] < rl[k])
            eq &= v[:, k] == rl[k]
        nz = raw.any(axis=1)
        out = np.concatenate([out, raw[less & nz][:need]])
        need = n - out.shape[0]
    return out


# ----------------------------------------------------------------------------- points <-> tensors
def fp_limbs_mont(vals) -> np.ndarray:
    return ints_to_limbs([mont(v) for v in vals])


def g1_aff_tensor(points, device="cpu") -> torch.Tensor:
    coords = []
    for p in points:
        coords += [0, 0] if p is None else [mont(p[0]), mont(p[1])]
    return to_tensor(ints_to_limbs(coords).reshape(-1, 16), device)


def g1_jac_tensor(points, device="cpu") -> torch.Tensor:
    return nt.g1_from_affine(g1_aff_tensor(points, device))


def g1_infinity_jac(n: int, device="cpu") -> torch.Tensor:
    one = mont(1)
    row = ints_to_limbs([one, one, 0]).reshape(1, 24)
    return to_tensor(np.repeat(row, n, axis=0), device)


def g1_points_from_aff(t: torch.Tensor):
    ints = limbs_to_ints(to_numpy(t).reshape(-1, 8))
    out = []
    for i in range(0, len(ints), 2):
        x, y = ints[i], ints[i + 1]
        out.append(None if (x == 0 and y == 0) else (unmont(x), unmont(y)))
    return out


def g1_points_from_jac(t: torch.Tensor):
    return g1_points_from_aff(nt.g1_to_affine(t.contiguous()))


def _fp2_mont(a: O.Fp2):
    return [mont(a.c0), mont(a.c1)]


def g2_aff_tensor(points, device="cpu") -> torch.Tensor:
    coords = []
    for p in points:
        coords += [0, 0, 0, 0] if p is None else _fp2_mont(p[0]) + _fp2_mont(p[1])
    return to_tensor(ints_to_limbs(coords).reshape(-1, 32), device)


def g2_points_from_aff(t: torch.Tensor):
    ints = limbs_to_ints(to_numpy(t).reshape(-1, 8))
    out = []
    for i in range(0, len(ints), 4):
        c = ints[i: i + 4]
        if not any(c):
            out.append(None)
        else:
            out.append((O.Fp2(unmont(c[0]), unmont(c[1])), O.Fp2(unmont(c[2]), unmont(c[3]))))
    return out


def gt_tensor(vals, device="cpu") -> torch.Tensor:
    coeffs = []
    for f in vals:
        coeffs += [mont(c) for c in f.coeffs()]
    return to_tensor(ints_to_limbs(coeffs).reshape(-1, 96), device)


def gt_from_tensor(t: torch.Tensor):
    ints = limbs_to_ints(to_numpy(t).reshape(-1, 8))
    return [O.Fp12.from_coeffs([unmont(c) for c in ints[i: i + 12]]) for i in range(0, len(ints), 12)]


# ----------------------------------------------------------------------------- wire codecs (kyber)
def _mont_rows_to_be(t: torch.Tensor, n_fp: int) -> np.ndarray:
    """Montgomery limbs [n, n_fp*8] -> canonical big-endian bytes [n, n_fp*32]."""
    flat = t.contiguous().view(-1, 8)
    can = to_numpy(nt.fp_from_mont(flat.cpu() if not flat.is_cuda else flat)).reshape(-1, 8)
    be = can[:, ::-1].astype(">u4")
    return np.ascontiguousarray(be).view(np.uint8).reshape(-1, n_fp * 32)


def _be_to_mont_rows(b: np.ndarray, n_fp: int, device) -> torch.Tensor:
    arr = np.ascontiguousarray(b, dtype=np.uint8).reshape(-1, 32)
    limbs = arr.view(">u4").astype("<u4")[:, ::-1].copy()
    return nt.fp_to_mont(to_tensor(limbs, device)).view(-1, n_fp * 8)


def g1_aff_to_bytes(aff: torch.Tensor) -> np.ndarray:
    """[n,16] Montgomery affine -> [n,64] uint8 kyber G1 (x||y BE, inf = zeros)."""
    return _mont_rows_to_be(aff, 2)


def g1_aff_from_bytes(b, device="cpu", check=True) -> torch.Tensor:
    arr = np.frombuffer(bytes(b), dtype=np.uint8) if isinstance(b, (bytes, bytearray)) else np.asarray(b, np.uint8)
    t = _be_to_mont_rows(arr, 2, device)
    if check:
        ok = nt.g1_on_curve(t)
        if not bool(ok.all()):
            raise ValueError("G1 point not on curve")
    return t


def fp2_perm(arr: np.ndarray) -> np.ndarray:
    """kyber gfP2 marshals (imag, real); our limbs store (real, imag)."""
    a = arr.reshape(-1, 2, 32)
    return a[:, ::-1, :].reshape(arr.shape)


def g2_aff_to_bytes(aff: torch.Tensor) -> np.ndarray:
    be = _mont_rows_to_be(aff, 4)  # (x.c0, x.c1, y.c0, y.c1)
    return np.ascontiguousarray(fp2_perm(be.reshape(-1, 64)).reshape(-1, 128))


def g2_aff_from_bytes(b, device="cpu", check=True) -> torch.Tensor:
    arr = np.frombuffer(bytes(b), dtype=np.uint8) if isinstance(b, (bytes, bytearray)) else np.asarray(b, np.uint8)
    arr = fp2_perm(arr.reshape(-1, 64)).reshape(-1)
    t = _be_to_mont_rows(arr, 4, device)
    if check and not bool(nt.g2_on_curve(t).all()):
        raise ValueError("G2 point not on curve")
    return t


def gt_to_bytes(t: torch.Tensor) -> np.ndarray:
    """kyber gfP12 marshal: c1 then c0, each Fp6 (c2, c1, c0), each Fp2 (imag, real)
    == our 12 Fp coefficients in exactly reversed order."""
    be = _mont_rows_to_be(t, 12).reshape(-1, 12, 32)
    return np.ascontiguousarray(be[:, ::-1, :]).reshape(-1, 384)


def gt_from_bytes(b, device="cpu") -> torch.Tensor:
    arr = np.frombuffer(bytes(b), dtype=np.uint8) if isinstance(b, (bytes, bytearray)) else np.asarray(b, np.uint8)
    a = arr.reshape(-1, 12, 32)[:, ::-1, :]
    return _be_to_mont_rows(np.ascontiguousarray(a).reshape(-1), 12, device)


def scalars_to_bytes(t: torch.Tensor) -> np.ndarray:
    a = to_numpy(t).reshape(-1, 8)
    return np.ascontiguousarray(a[:, ::-1].astype(">u4")).view(np.uint8).reshape(-1, 32)


def scalars_from_bytes(b, device="cpu") -> torch.Tensor:
    arr = np.frombuffer(bytes(b), dtype=np.uint8) if isinstance(b, (bytes, bytearray)) else np.asarray(b, np.uint8)
    limbs = arr.reshape(-1, 32).view(">u4").astype("<u4")[:, ::-1].copy()
    t = to_tensor(limbs, device)
    return nt.fr_arith(nt.FR_REDUCE, t)


# ----------------------------------------------------------------------------- shared device caches
def publish(*objs):
    """Before a lazily built device object goes into a cache other threads
    read: wait until its build has landed.  The build (kernels, asynchronous
    pinned uploads) was queued on the building thread's current stream; a
    reader on another stream would otherwise launch on the half-built table
    (no stream orders the two).  One synchronisation per cache entry."""
    seen = set()
    for o in objs:
        ts = [o] if isinstance(o, torch.Tensor) else [v for v in (vars(o).values() if hasattr(o, "__dict__") else o)
                                                      if isinstance(v, torch.Tensor)]
        for t in ts:
            if t.is_cuda and t.device not in seen:
                seen.add(t.device)
                torch.cuda.current_stream(t.device).synchronize()
    return objs[0] if len(objs) == 1 else objs


# ----------------------------------------------------------------------------- generator tables
_tables: dict = {}
_tlock = threading.Lock()


def _dev_key(device) -> str:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return str(d)


def g1_generator_aff(device="cpu") -> torch.Tensor:
    return g1_aff_tensor([O.G1_GEN], device)


def g2_generator_aff(device="cpu") -> torch.Tensor:
    return g2_aff_tensor([O.G2_GEN], device)


def base_table(device="cpu") -> torch.Tensor:
    """Comb table of the G1 base point B (kyber Point().Base()), cached per device."""
    k = ("B", _dev_key(device))
    with _tlock:
        if k not in _tables:
            _tables[k] = publish(nt.g1_fb_table(g1_generator_aff(device)))
        return _tables[k]


def base2_table(device="cpu") -> torch.Tensor:
    k = ("B2", _dev_key(device))
    with _tlock:
        if k not in _tables:
            _tables[k] = publish(nt.g2_fb_table(g2_generator_aff(device)))
        return _tables[k]


def g1_mul_point(k: int, P=None):
    """k * P for one point on the native host path (P = None -> the base B,
    fixed-base comb).  ~50 us instead of ~10 ms for the Python oracle; used
    by Schnorr envelopes, proof transcripts and key generation."""
    ks = scalars_tensor([k], "cpu")
    if P is None or P == O.G1_GEN:
        return g1_points_from_jac(nt.g1_fb_mul(base_table("cpu"), ks))[0]
    return g1_points_from_jac(nt.g1_mul(g1_jac_tensor([P], "cpu"), ks))[0]


def g1_add_points(P, Q):
    """P + Q for oracle-style affine points via the native host path."""
    if P is None:
        return Q
    if Q is None:
        return P
    return g1_points_from_jac(nt.g1_add(g1_jac_tensor([P]), g1_jac_tensor([Q])))[0]


def point_table(point_jac: torch.Tensor) -> torch.Tensor:
    """Comb table for an arbitrary G1 point (collective key P, querier key Q)."""
    return nt.g1_fb_table(nt.g1_to_affine(point_jac.reshape(1, 24).contiguous()))
