"""ctypes binding of the in-tree native library (csrc/ -> libdrynx_native.so).

Every op takes torch tensors.  If the tensors live on a GPU the gfx950 kernel
is launched on torch's current HIP stream; otherwise the same functor runs on
the host thread pool inside the library.  There is no pure-Python fallback for
any op: if the library is missing the import fails loudly (and on a GPU box the
driver can see exactly which .so was loaded).

Tensor conventions (all int32 tensors carrying raw u32 limbs, little endian):
  Fp / scalar : [..., 8]
  G1 affine   : [..., 16]   (x, y) Montgomery, infinity = zeros
  G1 Jacobian : [..., 24]
  G2 affine   : [..., 32]
  Fp12 (GT)   : [..., 96]
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# DRYNX_NATIVE_LIB selects another build of the library (e.g. the host-sanitizer
# build, build/libdrynx_native_asan.so); default: the in-tree gfx950 build
LIB_PATH = os.environ.get("DRYNX_NATIVE_LIB") or os.path.join(_HERE, "libdrynx_native.so")

_lib = None


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        if os.environ.get("DRYNX_AUTOBUILD", "1") == "1":
            from . import build as _b

            _b.build()
        else:
            raise ImportError(f"{LIB_PATH} missing: run `python -m drynx_amd.native.build`")
    _lib = ctypes.CDLL(LIB_PATH)
    _declare(_lib)
    return _lib


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_U64 = ctypes.c_uint64

_SIGS = {
    "dx_fp_to_mont": [_I, _P, _P, _P, _L],
    "dx_fp_from_mont": [_I, _P, _P, _P, _L],
    "dx_fr_arith": [_I, _P, _I, _P, _P, _P, _L, _L],
    "dx_fr_dot_chunks": [_I, _P, _P, _P, _I, _P, _L, _L, _L],
    "dx_fr_seg_sum": [_I, _P, _P, _P, _P, _L],
    "dx_rp_challenges": [_I, _P, _P, _P, _P, _P, _P, _L],
    "dx_g1_fb_table": [_I, _P, _P, _P, _P, _L],
    "dx_g1_fb_mul": [_I, _P, _P, _P, _P, _L],
    "dx_g1_fb_mul_i64": [_I, _P, _P, _P, _P, _L],
    "dx_g1_fb_mul_idx": [_I, _P, _P, _P, _P, _P, _L],
    "dx_g1_mul": [_I, _P, _P, _P, _P, _L, _I, _I],
    "dx_g1_add": [_I, _P, _P, _P, _P, _L, _I, _I],
    "dx_g1_to_affine": [_I, _P, _P, _P, _L],
    "dx_g1_from_affine": [_I, _P, _P, _P, _L],
    "dx_g1_eq": [_I, _P, _P, _P, _P, _L],
    "dx_g1_on_curve": [_I, _P, _P, _P, _L],
    "dx_g1_sum_chunks": [_I, _P, _P, _P, _L, _L, _L],
    "dx_elgamal_encrypt": [_I, _P, _P, _P, _P, _P, _P, _P, _L],
    "dx_bsgs_build": [_I, _P, _P, _L, _P, _P, _L],
    "dx_bsgs_solve": [_I, _P, _P, _P, _P, _P, _L, _L, _L, _L, _P, _P, _L],
    "dx_g2_fb_table": [_I, _P, _P, _P, _P, _L],
    "dx_g2_fb_mul": [_I, _P, _P, _P, _P, _P, _L],
    "dx_g2_mul": [_I, _P, _P, _P, _P, _L, _I],
    "dx_g2_on_curve": [_I, _P, _P, _P, _L],
    "dx_miller_loop": [_I, _P, _P, _P, _P, _L],
    "dx_final_exp": [_I, _P, _P, _P, _L],
    "dx_pairing": [_I, _P, _P, _P, _P, _L],
    "dx_gt_mul": [_I, _P, _P, _P, _P, _L],
    "dx_gt_inv": [_I, _P, _P, _P, _L],
    "dx_prg_glv": [_I, _P, _P, ctypes.c_uint32, _P, _P, _P, _L],
    "dx_prg_bits": [_I, _P, _P, ctypes.c_uint32, _I, _P, _L],
    "dx_batched_copy": [_I, _P, _P, _P, _I, _L],
    "dx_copy_out": [_I, _P, _P, _P, _I, _L, _I],
    "dx_host_device_ptr": [_P, _P],
    "dx_rows_all": [_I, _P, _P, _P, _I, _L, _P],
    "dx_gt_pow": [_I, _P, _P, _P, _P, _L, _I],
    "dx_gt_eq": [_I, _P, _P, _P, _P, _L],
    "dx_gt_fb_table": [_I, _P, _P, _P, _P, _L],
    "dx_gt_fb_pow": [_I, _P, _P, _P, _P, _P, _L],
    "dx_gt_prod_chunks": [_I, _P, _P, _P, _L, _L, _L],
    "dx_version": [],
    "dx_lr_moments": [_P, _P, _P, _L, _I, _P, _I],
    "dx_lr_gd_k2": [_P, _P, _P, _I, ctypes.c_double, ctypes.c_double, ctypes.c_double, _I, ctypes.c_double,
                    ctypes.c_double, ctypes.c_double, _P],
    "dx_random_scalars": [_I, _P, _P, ctypes.c_uint32, _P, _L],
    "dx_sha256_chunks": [_I, _P, _P, _L, _L, _P],
    "dx_hash_to_g1": [_I, _P, _P, _P, _L, _P, _L],
    "dx_lr_encode": [_P, _P, _L, _L, _I, _P, _P, _P, ctypes.c_double, ctypes.c_double, _P, _I],
    "dx_lr_reduce": [_P, _P, _L, _L, _L, _P],
    "dx_g1_mul_glv256": [_P, _P, _P, _P, _P, _L, _I, _I, _I],
    "dx_glv_split": [_I, _P, _P, _P, _L],
    "dx_gt_t2_compress": [_I, _P, _P, _P, _P, _L],
    "dx_g2_x_compress": [_I, _P, _P, _P, _P, _P, _L],
    "dx_g2_x_decompress": [_I, _P, _P, _P, _P, _P, _L],
    "dx_gt_t2_decompress": [_I, _P, _P, _P, _L],
    "dx_rp_verify_fold": [_P, _P, _P, _P, _P, _P, _L, _I, _I],
    "dx_gt_slice_prod": [_I, _P, _P, _P, _P, _P, _P, _L],
    "dx_gt_chunk_weight": [_I, _P, _P, _P, _P, _P, _P, _P, _L],
    "dx_g1_mul_glv": [_P, _P, _P, _P, _P, _L, _I],
    "dx_rp_u_joint_split": [_I, _P, _P, _P, _P, _L, _I, _I, _L, _I, _P, _P],
    "dx_bucket_bounds": [_I, _P, _P, _L, _L, _P, _P],
    "dx_slice_desc": [_I, _P, _P, _P, _P, _I, _L, _L, _P, _P],
    "dx_lane_slices": [_I, _P, _P, _P, _P, _P, _P, _L, _P, _P],
    "dx_g1_slice_sum": [_I, _P, _P, _P, _P, _P, _P, _L],
    "dx_rp_prove_a": [_I, _P, _P, _P, _P, _P, _P, _L, _I, _I],
    "dx_rp_prove_a_tab": [_I, _P, _P, _P, _P, _P, _P, _P, _L, _I, _I, _I],
    "dx_g2_fb4_table": [_I, _P, _P, _P, _P, _L],
    "dx_g2_fb4_mul": [_I, _P, _P, _P, _P, _P, _L],
    "dx_gt_fb4_table": [_I, _P, _P, _P, _P, _L],
    "dx_gt_fb4_pow": [_I, _P, _P, _P, _P, _P, _L],
    "dx_gt_cyclotomic": [_I, _P, _P, _P, _L],
    "dx_gt_membership": [_I, _P, _P, _P, _L],
    "dx_g1_horner_host": [_P, _P, _L, _I, _I],
    "dx_fp_sqrt_host": [_P, _P, _P, _P, _L],
    "dx_g2_chunk_weight": [_I, _P, _P, _P, _P, _P, _P, _P, _L],
    "dx_g2_subgroup": [_I, _P, _P, _P, _L],
    "dx_limbs_canonical": [_I, _P, _P, _I, _P, _L],
    "dx_g1j_on_curve": [_I, _P, _P, _P, _L],
    "dx_rp_points_inl": [_P, _P, _P, _P, _P, _L, _I, _I],
    "dx_fold_steps_inl": [],
    "dx_rp_lines_inl": [_P, _P, _P, _P, _L, _L, _L],
    "dx_rp_accum_inl": [_P, _P, _P, _L, _I],
    "dx_rp_coeffs_inl": [_P, _P, _P, _L],
    "dx_rp_accum_p_inl": [_P, _P, _P, _P, _P, _L, _L, _I, _I],
    "dx_rp_verify_items": [_I, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _I],
    "dx_int_moments": [_I, _P, _P, _L, _I, _P, _L, _P, _I, _P, _P],
    "dx_sha256_rows": [_I, _P, _P, _L, _L, _L, _L, _P],
    "dx_sha256_segments": [_I, _P, _P, _L, _L, _L, _P],
    "dx_rp_points_glv": [_P, _P, _P, _P, _P, _P, _L, _I, _I, _I],
    "dx_g1_aff_to_uv": [_I, _P, _P, _L],
    "dx_rp_ncoeffs_inl": [_P, _P, _P, _P, _L],
    "dx_rp_accum_n_inl": [_P, _P, _P, _P, _P, _L, _L, _I, _I],
    "dx_ufold_coop_raw": [_P, _P, _P, _P, _P, _L, _L, _L],
    "dx_ufold_coop_steps": [],
    "dx_gt_frob8": [_I, _P, _P, _P, _L],
    "dx_gls6_entries": [],
    "dx_g2_gls6_table": [_I, _P, _P, _P, _P, _L],
    "dx_g2_gls6_mul": [_I, _P, _P, _P, _P, _P, _L],
    "dx_gt_gls6_table": [_I, _P, _P, _P, _P, _L],
    "dx_gt_gls6_pow": [_I, _P, _P, _P, _P, _P, _L],
    "dx_rp_prove_a_gls6": [_I, _P, _P, _P, _P, _P, _P, _P, _L, _I, _I],
    "dx_g2_joint_table": [_I, _P, _P, _P, _L],
    "dx_rp_u_joint": [_I, _P, _P, _P, _P, _L, _I, _I, _L, _P],
    "dx_g2_slice_sum": [_I, _P, _P, _P, _P, _P, _P, _L, _I, _L],
    "dx_g2_mul_small": [_I, _P, _P, _P, _P, _L],
    "dx_g2_horner": [_I, _P, _P, _P, _I, _I, _I, _L, _L],
    "dx_rp_msm_uv": [_I, _P, _P, _P, _L, _I, _L],
    "dx_msm_keys": [_I, _P, _P, _P, _L, _L, _I, _I, _P, _P],
    "dx_gls8_entries": [],
    "dx_g2_gls8_table": [_I, _P, _P, _P, _P, _L],
    "dx_gt_gls8_table": [_I, _P, _P, _P, _P, _L],
    "dx_g2_gls8_mul": [_I, _P, _P, _P, _P, _P, _L],
    "dx_rp_prove_a_gls8": [_I, _P, _P, _P, _P, _P, _P, _P, _L, _I, _I, _I],
    "dx_gt16_entries": [],
    "dx_gt16_table": [_I, _P, _P, _P],
}


def _declare(lib):
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int


def lib():
    return _load()


def loaded_path() -> str:
    _load()
    return LIB_PATH


# ----------------------------------------------------------------------------- helpers
_keep = threading.local()


def _ptr(t: torch.Tensor | None):
    """Raw pointer of a contiguous tensor for a native call.  The tensor is
    kept alive until the calling thread's next ``_call`` returns: a temporary
    such as ``_ptr(x.contiguous())`` would otherwise be freed before the call
    runs (on the host path the native code would then read freed memory)."""
    if t is None:
        return None
    assert t.is_contiguous(), "native ops need contiguous tensors"
    held = getattr(_keep, "held", None)
    if held is None:
        held = _keep.held = []
    held.append(t)
    return ctypes.c_void_p(t.data_ptr())


def _ctx(*ts):
    dev = None
    for t in ts:
        if t is not None:
            dev = t.device
            break
    for t in ts:
        if t is not None and t.device != dev:
            raise ValueError(f"native op mixes devices {dev} and {t.device}")
    if dev is not None and dev.type == "cuda":
        if _CHECK_DEVICE and torch.cuda.current_device() != dev.index:
            # DRYNX_CHECK_DEVICE=1 (the GPU suite): a thread launching on a GPU
            # that is not its current device was never pinned to the rank's
            raise AssertionError(f"native op on {dev} from a thread whose current device is "
                                 f"cuda:{torch.cuda.current_device()}")
        return 1, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    return 0, None


_CHECK_DEVICE = os.environ.get("DRYNX_CHECK_DEVICE", "0") == "1"


def _raw_call(name, *args) -> int:
    """A native call whose return code the caller interprets; releases the
    tensors ``_ptr`` held for it, like ``_call``."""
    try:
        return getattr(_load(), name)(*args)
    finally:
        _keep.held = []


def _call(name, *args):
    rc = _raw_call(name, *args)
    if rc != 0:
        raise RuntimeError(f"native op {name} failed (rc={rc})")


def _rows(t: torch.Tensor, width: int) -> int:
    assert t.dtype == torch.int32 and t.shape[-1] == width, (t.dtype, t.shape, width)
    return t.numel() // width


def empty_like_rows(ref: torch.Tensor, n: int, width: int) -> torch.Tensor:
    return torch.empty((n, width), dtype=torch.int32, device=ref.device)


# ----------------------------------------------------------------------------- field
def fp_to_mont(x: torch.Tensor) -> torch.Tensor:
    out = torch.empty_like(x)
    g, s = _ctx(x)
    _call("dx_fp_to_mont", g, s, _ptr(x), _ptr(out), _rows(x, 8))
    return out


def fp_from_mont(x: torch.Tensor) -> torch.Tensor:
    out = torch.empty_like(x)
    g, s = _ctx(x)
    _call("dx_fp_from_mont", g, s, _ptr(x), _ptr(out), _rows(x, 8))
    return out


FR_ADD, FR_SUB, FR_MUL, FR_NEG, FR_INV, FR_REDUCE = range(6)


def fr_arith(op: int, a: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """Row-wise Fr op of a [n, 8] with b: n rows, or k rows read periodically
    (row i uses b[i % k]; k = 1 broadcasts one scalar), canonical in and out."""
    n = _rows(a, 8)
    out = torch.empty_like(a)
    bb = b.contiguous() if b is not None else None
    nb = _rows(bb, 8) if bb is not None else 0
    bcast = nb if (bb is not None and nb != n) else 0
    assert bcast == 0 or n % nb == 0, (n, nb)
    g, s = _ctx(a, bb)
    _call("dx_fr_arith", g, s, op, _ptr(a), _ptr(bb), _ptr(out), n, bcast)
    return out


def fr_dot_rows(a: torch.Tensor, b: torch.Tensor | None, groups: int, b_periodic: bool = False,
                chunk: int = 32) -> torch.Tensor:
    """Per-group Fr sums of a[g*m + k] * b(g, k) -> [groups, 8] (canonical).
    b: None (plain sums), [groups*m, 8] (per row) or [m, 8] (b_periodic)."""
    n = _rows(a, 8)
    m = n // groups
    assert m * groups == n and m > 0
    if b is not None:
        assert _rows(b, 8) == (m if b_periodic else n)
    cur, bb = a.contiguous(), None if b is None else b.contiguous()
    while True:
        n_chunks = (m + chunk - 1) // chunk
        out = torch.empty((groups * n_chunks, 8), dtype=torch.int32, device=a.device)
        g, s = _ctx(cur, bb)
        _call("dx_fr_dot_chunks", g, s, _ptr(cur), _ptr(bb), int(b_periodic), _ptr(out), groups, m, chunk)
        cur, bb, m = out, None, n_chunks
        if m == 1:
            return cur


def fr_seg_sum(a: torch.Tensor, offs: torch.Tensor) -> torch.Tensor:
    """Per-segment Fr sums of the rows of a: out[t] = sum a[offs[t]:offs[t+1]]
    (canonical; offs int64 [k+1] on a's device, non-decreasing, <= rows)."""
    k = offs.numel() - 1
    assert k >= 0 and offs.dtype == torch.int64
    out = torch.empty((k, 8), dtype=torch.int32, device=a.device)
    if k:
        offs = offs.to(a.device).contiguous()
        g, s = _ctx(a, offs, out)
        _call("dx_fr_seg_sum", g, s, _ptr(a.contiguous()), _ptr(offs), _ptr(out), k)
    return out

# ----------------------------------------------------------------------------- G1
def g1_fb_table(base_aff: torch.Tensor) -> torch.Tensor:
    """Comb table(s) [n_bases*8192, 16] for one or more affine G1 bases."""
    bases = base_aff.contiguous().view(-1, 16)
    nb = bases.shape[0]
    table = torch.empty((nb * 8192, 16), dtype=torch.int32, device=base_aff.device)
    work = torch.empty((nb * 256, 24), dtype=torch.int32, device=base_aff.device)
    g, s = _ctx(bases)
    _call("dx_g1_fb_table", g, s, _ptr(bases), _ptr(work), _ptr(table), nb)
    return table


def g1_fb_mul(table: torch.Tensor, scalars: torch.Tensor) -> torch.Tensor:
    n = _rows(scalars, 8)
    out = torch.empty((n, 24), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(table, scalars)
    _call("dx_g1_fb_mul", g, s, _ptr(table), _ptr(scalars), _ptr(out), n)
    return out


def g1_fb_mul_idx(tables: torch.Tensor, tab_idx: torch.Tensor, scalars: torch.Tensor) -> torch.Tensor:
    """k_i * base_{tab_idx[i]} over stacked comb tables [n_bases*8192, 16]."""
    n = _rows(scalars, 8)
    assert tab_idx.dtype == torch.int32 and tab_idx.numel() == n
    out = torch.empty((n, 24), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(tables, tab_idx, scalars)
    _call("dx_g1_fb_mul_idx", g, s, _ptr(tables), _ptr(tab_idx), _ptr(scalars), _ptr(out), n)
    return out


def g1_fb_mul_i64(table: torch.Tensor, m: torch.Tensor) -> torch.Tensor:
    assert m.dtype == torch.int64
    n = m.numel()
    out = torch.empty((n, 24), dtype=torch.int32, device=m.device)
    g, s = _ctx(table, m)
    _call("dx_g1_fb_mul_i64", g, s, _ptr(table), _ptr(m.contiguous()), _ptr(out), n)
    return out


# rows up to which g1_mul runs two lanes per row (the latency form; tools/bench_g1mul.py)
G1_MUL_PAIR_ROWS = 1 << 14


def gt_t2_compress(a: torch.Tensor, out: torch.Tensor | None = None):
    """GT elements [n, 96] -> (c [n, 48] int32, ok [n] uint8): c = (1 + g) / h
    of f = g + h w (torus T2; csrc/kernels/dx_gt_t2.hip); ok = 1 where the
    decompression gives back exactly these limbs (canonical, unitary, h != 0).
    ``out``: a contiguous [n, 48] destination for c; then only ok is returned."""
    n = _rows(a, 96)
    c = torch.empty((n, 48), dtype=torch.int32, device=a.device) if out is None else out
    assert c.is_contiguous() and _rows(c, 48) == n
    ok = torch.empty((n,), dtype=torch.uint8, device=a.device)
    g, s = _ctx(a, c)
    _call("dx_gt_t2_compress", g, s, _ptr(a.contiguous()), _ptr(c), _ptr(ok), n)
    return ok if out is not None else (c, ok)


def gt_t2_decompress(c: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """[n, 48] torus-compressed GT elements -> [n, 96] (``out``: a contiguous
    destination of that shape, e.g. a slice of a payload being rebuilt)."""
    n = _rows(c, 48)
    out = torch.empty((n, 96), dtype=torch.int32, device=c.device) if out is None else out
    assert out.is_contiguous() and _rows(out, 96) == n
    g, s = _ctx(c, out)
    _call("dx_gt_t2_decompress", g, s, _ptr(c.contiguous()), _ptr(out), n)
    return out


def g2_x_compress(V: torch.Tensor, x_out: torch.Tensor | None = None, flag_out: torch.Tensor | None = None):
    """Affine G2 [n, 32] -> (x [n, 16], flag [n] int32: y parity | 2 * infinity,
    ok [n] uint8: canonical and on the twist, i.e. ``g2_x_decompress`` gives the
    same limbs back).  ``x_out`` / ``flag_out``: contiguous destinations."""
    n = _rows(V, 32)
    x = torch.empty((n, 16), dtype=torch.int32, device=V.device) if x_out is None else x_out
    f = torch.empty((n,), dtype=torch.int32, device=V.device) if flag_out is None else flag_out
    assert x.is_contiguous() and f.is_contiguous() and x.numel() == 16 * n and f.numel() == n
    ok = torch.empty((n,), dtype=torch.uint8, device=V.device)
    g, s = _ctx(V, x, f)
    _call("dx_g2_x_compress", g, s, _ptr(V.contiguous()), _ptr(x), _ptr(f), _ptr(ok), n)
    return x, f, ok


def g2_x_decompress(x: torch.Tensor, flag: torch.Tensor, out: torch.Tensor | None = None):
    """(x [n, 16], flag [n]) -> (affine G2 [n, 32], bad [n] uint8: no point
    with that x)."""
    n = _rows(x, 16)
    V = torch.empty((n, 32), dtype=torch.int32, device=x.device) if out is None else out
    assert V.is_contiguous() and V.numel() == 32 * n and flag.numel() == n
    bad = torch.empty((n,), dtype=torch.uint8, device=x.device)
    g, s = _ctx(x, flag, V)
    _call("dx_g2_x_decompress", g, s, _ptr(x.contiguous()), _ptr(flag.contiguous()), _ptr(V), _ptr(bad), n)
    return V, bad


def glv_split(scalars: torch.Tensor) -> torch.Tensor:
    """[n, 8] scalars -> [n, 9] int32 words: k1 (4), |k2| (4), k2 < 0 with
    k = k1 + k2 GLV_LAMBDA mod r (csrc/bn254/glv_split.h; host or device)."""
    n = _rows(scalars, 8)
    out = torch.empty((n, 9), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(scalars)
    _call("dx_glv_split", g, s, _ptr(scalars.contiguous()), _ptr(out), n)
    return out


def g1_mul(pts_jac: torch.Tensor, scalars: torch.Tensor) -> torch.Tensor:
    np_ = _rows(pts_jac, 24)
    nk = _rows(scalars, 8)
    n = max(np_, nk)
    assert np_ in (1, n) and nk in (1, n)
    out = torch.empty((n, 24), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(pts_jac, scalars)
    if g:  # gfx950: in-kernel GLV split, 128-step ladder (dx_g1_varmul.hip)
        rc = _raw_call("dx_g1_mul_glv256", s, _ptr(pts_jac), _ptr(scalars), _ptr(_glv_const("beta", out.device)),
                       _ptr(out), n, int(np_ == 1 and n > 1), int(nk == 1 and n > 1), int(n <= G1_MUL_PAIR_ROWS))
        if rc:
            raise RuntimeError(f"dx_g1_mul_glv256 failed rc={rc}")
        return out
    _call("dx_g1_mul", g, s, _ptr(pts_jac), _ptr(scalars), _ptr(out), n, int(np_ == 1 and n > 1),
          int(nk == 1 and n > 1))
    return out


def g1_add(a: torch.Tensor, b: torch.Tensor, subtract: bool = False) -> torch.Tensor:
    n = _rows(a, 24)
    nb = _rows(b, 24)
    assert nb in (1, n)
    out = torch.empty((n, 24), dtype=torch.int32, device=a.device)
    g, s = _ctx(a, b)
    _call("dx_g1_add", g, s, _ptr(a), _ptr(b), _ptr(out), n, int(subtract), int(nb == 1 and n > 1))
    return out


def g1_to_affine(jac: torch.Tensor) -> torch.Tensor:
    n = _rows(jac, 24)
    out = torch.empty((n, 16), dtype=torch.int32, device=jac.device)
    g, s = _ctx(jac)
    _call("dx_g1_to_affine", g, s, _ptr(jac), _ptr(out), n)
    return out


def g1_from_affine(aff: torch.Tensor) -> torch.Tensor:
    n = _rows(aff, 16)
    out = torch.empty((n, 24), dtype=torch.int32, device=aff.device)
    g, s = _ctx(aff)
    _call("dx_g1_from_affine", g, s, _ptr(aff), _ptr(out), n)
    return out


def g1_eq(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    n = _rows(a, 24)
    assert _rows(b, 24) == n
    out = torch.empty((n,), dtype=torch.uint8, device=a.device)
    g, s = _ctx(a, b)
    _call("dx_g1_eq", g, s, _ptr(a), _ptr(b), _ptr(out), n)
    return out


def g1_on_curve(aff: torch.Tensor) -> torch.Tensor:
    n = _rows(aff, 16)
    out = torch.empty((n,), dtype=torch.uint8, device=aff.device)
    g, s = _ctx(aff)
    _call("dx_g1_on_curve", g, s, _ptr(aff), _ptr(out), n)
    return out


def limbs_canonical(x: torch.Tensor, fr: bool = False) -> torch.Tensor:
    """uint8 per 8-limb row: row < p (Fp, Montgomery coordinates) or < r (Fr)."""
    n = _rows(x, 8)
    out = torch.empty((n,), dtype=torch.uint8, device=x.device)
    g, s = _ctx(x)
    _call("dx_limbs_canonical", g, s, _ptr(x.contiguous()), int(fr), _ptr(out), n)
    return out


def g1j_on_curve(jac: torch.Tensor) -> torch.Tensor:
    n = _rows(jac, 24)
    out = torch.empty((n,), dtype=torch.uint8, device=jac.device)
    g, s = _ctx(jac)
    _call("dx_g1j_on_curve", g, s, _ptr(jac.contiguous()), _ptr(out), n)
    return out


def g2_subgroup(aff: torch.Tensor) -> torch.Tensor:
    """uint8 per affine twist point: on the curve and in G2 (psi(Q) == [6u^2] Q)."""
    n = _rows(aff, 32)
    out = torch.empty((n,), dtype=torch.uint8, device=aff.device)
    g, s = _ctx(aff)
    _call("dx_g2_subgroup", g, s, _ptr(aff.contiguous()), _ptr(out), n)
    return out


def gt_cyclotomic(a: torch.Tensor) -> torch.Tensor:
    """uint8 per Fp12: non-zero and in the cyclotomic subgroup (x^(p^4) x == x^(p^2))."""
    n = _rows(a, 96)
    out = torch.empty((n,), dtype=torch.uint8, device=a.device)
    g, s = _ctx(a)
    _call("dx_gt_cyclotomic", g, s, _ptr(a.contiguous()), _ptr(out), n)
    return out


def gt_membership(a: torch.Tensor) -> torch.Tensor:
    """[n] uint8: a_i in the prime-order GT, for a_i in the cyclotomic subgroup
    (x^p == x^(6u^2): one Frobenius against two cyclotomic u-ladders)."""
    n = _rows(a, 96)
    out = torch.empty((n,), dtype=torch.uint8, device=a.device)
    g, s = _ctx(a)
    _call("dx_gt_membership", g, s, _ptr(a.contiguous()), _ptr(out), n)
    return out


def g1_sum(x: torch.Tensor, chunk: int = 64) -> torch.Tensor:
    """Sum over axis 0 of x[n_items, n_groups, 24] (Jacobian) -> [n_groups, 24].

    Multi-pass chunked reduction: each pass has n_groups * ceil(items/chunk)
    independent threads, so wide vectors and deep reductions both fill the GPU.
    """
    assert x.dim() == 3 and x.shape[-1] == 24
    n_items, n_groups = x.shape[0], x.shape[1]
    cur = x.contiguous()
    if n_items == 0:
        from ..crypto.bn254 import g1_infinity_jac

        return g1_infinity_jac(n_groups, x.device)
    while n_items > 1:
        ch = max(2, min(chunk, n_items)) if n_groups >= 4096 else max(2, min(8, n_items))
        n_chunks = (n_items + ch - 1) // ch
        out = torch.empty((n_chunks, n_groups, 24), dtype=torch.int32, device=x.device)
        g, s = _ctx(cur)
        _call("dx_g1_sum_chunks", g, s, _ptr(cur), _ptr(out), n_items, n_groups, ch)
        cur, n_items = out, n_chunks
    return cur[0]


# ----------------------------------------------------------------------------- ElGamal
def elgamal_encrypt(tabB, tabP, m: torch.Tensor, r: torch.Tensor):
    n = m.numel()
    assert m.dtype == torch.int64 and _rows(r, 8) == n
    K = torch.empty((n, 24), dtype=torch.int32, device=m.device)
    C = torch.empty((n, 24), dtype=torch.int32, device=m.device)
    g, s = _ctx(tabB, tabP, m, r)
    _call("dx_elgamal_encrypt", g, s, _ptr(tabB), _ptr(tabP), _ptr(m.contiguous()), _ptr(r), _ptr(K), _ptr(C), n)
    return K, C


def bsgs_build(tabB: torch.Tensor, m_baby: int, cap: int):
    assert cap & (cap - 1) == 0 and cap >= 2 * m_baby
    keys = torch.zeros((cap,), dtype=torch.int64, device=tabB.device)
    vals = torch.zeros((cap,), dtype=torch.int32, device=tabB.device)
    g, s = _ctx(tabB)
    _call("dx_bsgs_build", g, s, _ptr(tabB), m_baby, _ptr(keys), _ptr(vals), cap)
    return keys, vals


def bsgs_solve(targets_jac, giant_aff, keys, vals, m_baby: int, n_giant: int, offset: int):
    n = _rows(targets_jac, 24)
    out = torch.empty((n,), dtype=torch.int64, device=targets_jac.device)
    found = torch.empty((n,), dtype=torch.uint8, device=targets_jac.device)
    g, s = _ctx(targets_jac, giant_aff, keys, vals)
    _call("dx_bsgs_solve", g, s, _ptr(targets_jac), _ptr(giant_aff), _ptr(keys), _ptr(vals), keys.numel(), m_baby,
          n_giant, offset, _ptr(out), _ptr(found), n)
    return out, found


# ----------------------------------------------------------------------------- G2
def g2_fb_table(base_aff: torch.Tensor) -> torch.Tensor:
    """Comb table(s) [n_bases*8192, 32] for one or more affine G2 bases."""
    bases = base_aff.contiguous().view(-1, 32)
    nb = bases.shape[0]
    table = torch.empty((nb * 8192, 32), dtype=torch.int32, device=base_aff.device)
    work = torch.empty((nb * 256, 48), dtype=torch.int32, device=base_aff.device)
    g, s = _ctx(bases)
    _call("dx_g2_fb_table", g, s, _ptr(bases), _ptr(work), _ptr(table), nb)
    return table


def g2_fb_mul(tables: torch.Tensor, scalars: torch.Tensor, tab_idx: torch.Tensor | None = None) -> torch.Tensor:
    n = _rows(scalars, 8)
    out = torch.empty((n, 32), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(tables, scalars, tab_idx)
    _call("dx_g2_fb_mul", g, s, _ptr(tables), _ptr(tab_idx), _ptr(scalars), _ptr(out), n)
    return out


FB4_ENTRIES = 960  # 64 windows x 15 non-zero digits


def g2_fb4_table(base_aff: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """4-bit comb table(s) [n_bases*960, 32] (120 KiB per base).  ``out``: a
    preallocated slice of a larger table tensor to fill in place."""
    bases = base_aff.contiguous().view(-1, 32)
    nb = bases.shape[0]
    table = out if out is not None else torch.empty((nb * FB4_ENTRIES, 32), dtype=torch.int32, device=bases.device)
    assert table.shape == (nb * FB4_ENTRIES, 32) and table.is_contiguous()
    work = torch.empty((nb * 64, 48), dtype=torch.int32, device=bases.device)
    g, s = _ctx(bases, table)
    _call("dx_g2_fb4_table", g, s, _ptr(bases), _ptr(work), _ptr(table), nb)
    return table


def g2_fb4_mul(tables: torch.Tensor, scalars: torch.Tensor, tab_idx: torch.Tensor | None = None) -> torch.Tensor:
    n = _rows(scalars, 8)
    out = torch.empty((n, 32), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(tables, scalars, tab_idx)
    _call("dx_g2_fb4_mul", g, s, _ptr(tables), _ptr(tab_idx), _ptr(scalars), _ptr(out), n)
    return out


GLS6_ENTRIES = 1386  # 22 six-bit windows x 63 non-zero digits (csrc/kernels/dx_gls.hip)


def g2_gls6_table(base_aff: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """GLS-2 6-bit fixed-base table(s) [n_bases*1386, 32] (177 KiB per base)."""
    bases = base_aff.contiguous().view(-1, 32)
    nb = bases.shape[0]
    table = out if out is not None else torch.empty((nb * GLS6_ENTRIES, 32), dtype=torch.int32, device=bases.device)
    assert table.shape == (nb * GLS6_ENTRIES, 32) and table.is_contiguous()
    work = torch.empty((nb * 22, 48), dtype=torch.int32, device=bases.device)
    g, s = _ctx(bases, table)
    _call("dx_g2_gls6_table", g, s, _ptr(bases), _ptr(work), _ptr(table), nb)
    return table


def g2_gls6_mul(tables: torch.Tensor, scalars: torch.Tensor, tab_idx: torch.Tensor | None = None) -> torch.Tensor:
    """k * A (affine) with k = k0 + k1 lambda2, psi(k1 A) + k0 A from one table."""
    n = _rows(scalars, 8)
    out = torch.empty((n, 32), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(tables, scalars, tab_idx)
    _call("dx_g2_gls6_mul", g, s, _ptr(tables), _ptr(tab_idx), _ptr(scalars), _ptr(out), n)
    return out


def gt_gls6_table(bases: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """GLS-2 6-bit fixed-base table(s) [n_bases*1386, 96] of GT elements (532 KiB per base)."""
    bases = bases.contiguous()
    nb = _rows(bases, 96)
    table = out if out is not None else torch.empty((nb * GLS6_ENTRIES, 96), dtype=torch.int32, device=bases.device)
    assert table.shape == (nb * GLS6_ENTRIES, 96) and table.is_contiguous()
    work = torch.empty((nb * 22, 96), dtype=torch.int32, device=bases.device)
    g, s = _ctx(bases, table)
    _call("dx_gt_gls6_table", g, s, _ptr(bases), _ptr(work), _ptr(table), nb)
    return table


def gt_gls6_pow(tables: torch.Tensor, scalars: torch.Tensor, tab_idx: torch.Tensor | None = None) -> torch.Tensor:
    n = _rows(scalars, 8)
    out = torch.empty((n, 96), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(tables, scalars, tab_idx)
    _call("dx_gt_gls6_pow", g, s, _ptr(tables), _ptr(tab_idx), _ptr(scalars), _ptr(out), n)
    return out


GLS8_ENTRIES = 2176  # 17 signed byte windows x 128 digits (csrc/kernels/dx_gls8.hip)


def g2_gls8_table(base_aff: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """GLS-2 signed 8-bit fixed-base table(s) [n_bases*2176, 32] (272 KiB per base)."""
    bases = base_aff.contiguous().view(-1, 32)
    nb = bases.shape[0]
    table = out if out is not None else torch.empty((nb * GLS8_ENTRIES, 32), dtype=torch.int32, device=bases.device)
    assert table.shape == (nb * GLS8_ENTRIES, 32) and table.is_contiguous()
    work = torch.empty((nb * 17, 48), dtype=torch.int32, device=bases.device)
    g, s = _ctx(bases, table)
    _call("dx_g2_gls8_table", g, s, _ptr(bases), _ptr(work), _ptr(table), nb)
    return table


def gt_gls8_table(bases: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """GLS-2 signed 8-bit fixed-base table(s) [n_bases*2176, 96] of GT elements (816 KiB per base)."""
    bases = bases.contiguous()
    nb = _rows(bases, 96)
    table = out if out is not None else torch.empty((nb * GLS8_ENTRIES, 96), dtype=torch.int32, device=bases.device)
    assert table.shape == (nb * GLS8_ENTRIES, 96) and table.is_contiguous()
    work = torch.empty((nb * 17, 96), dtype=torch.int32, device=bases.device)
    g, s = _ctx(bases, table)
    _call("dx_gt_gls8_table", g, s, _ptr(bases), _ptr(work), _ptr(table), nb)
    return table


def g2_gls8_mul(tables: torch.Tensor, scalars: torch.Tensor, tab_idx: torch.Tensor | None = None) -> torch.Tensor:
    """k * A (affine) from the signed 8-bit GLS-2 table of A: 34 mixed additions."""
    n = _rows(scalars, 8)
    assert tab_idx is None or (tab_idx.dtype == torch.int32 and tab_idx.numel() == n)
    out = torch.empty((n, 32), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(tables, scalars, tab_idx)
    _call("dx_g2_gls8_mul", g, s, _ptr(tables), _ptr(tab_idx), _ptr(scalars), _ptr(out), n)
    return out


_gt16: dict = {}


def gt16_table(device) -> torch.Tensor:
    """gT with signed 16-bit windows: [17 * 32768, 96], gT^(d 2^(16w)) (214 MB,
    built once per device; csrc/kernels/dx_gls8.hip)."""
    key = str(torch.device(device))
    if key not in _gt16:
        from ..crypto import bn254 as _bn
        from ..crypto import oracle as _O

        g = _O.pairing(_O.G1_GEN, _O.G2_GEN)
        pows = []
        for _ in range(17):
            pows.append(g)
            for _ in range(16):
                g = g * g
        pow2 = _bn.gt_tensor(pows, device)
        n = _load().dx_gt16_entries()
        table = torch.empty((n, 96), dtype=torch.int32, device=pow2.device)
        gg, s = _ctx(pow2, table)
        _call("dx_gt16_table", gg, s, _ptr(pow2), _ptr(table))
        _gt16[key] = table
    return _gt16[key]


def g2_mul(pts_aff: torch.Tensor, scalars: torch.Tensor) -> torch.Tensor:
    n = _rows(scalars, 8)
    np_ = _rows(pts_aff, 32)
    assert np_ in (1, n)
    out = torch.empty((n, 32), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(pts_aff, scalars)
    _call("dx_g2_mul", g, s, _ptr(pts_aff), _ptr(scalars), _ptr(out), n, int(np_ == 1 and n > 1))
    return out


def g2_on_curve(aff: torch.Tensor) -> torch.Tensor:
    n = _rows(aff, 32)
    out = torch.empty((n,), dtype=torch.uint8, device=aff.device)
    g, s = _ctx(aff)
    _call("dx_g2_on_curve", g, s, _ptr(aff), _ptr(out), n)
    return out


# ----------------------------------------------------------------------------- pairing / GT
def miller_loop(P_aff: torch.Tensor, Q_aff: torch.Tensor) -> torch.Tensor:
    n = _rows(P_aff, 16)
    assert _rows(Q_aff, 32) == n
    out = torch.empty((n, 96), dtype=torch.int32, device=P_aff.device)
    g, s = _ctx(P_aff, Q_aff)
    _call("dx_miller_loop", g, s, _ptr(P_aff), _ptr(Q_aff), _ptr(out), n)
    return out


def final_exp(f: torch.Tensor) -> torch.Tensor:
    n = _rows(f, 96)
    out = torch.empty_like(f)
    g, s = _ctx(f)
    _call("dx_final_exp", g, s, _ptr(f), _ptr(out), n)
    return out


def pairing(P_aff: torch.Tensor, Q_aff: torch.Tensor) -> torch.Tensor:
    n = _rows(P_aff, 16)
    assert _rows(Q_aff, 32) == n
    out = torch.empty((n, 96), dtype=torch.int32, device=P_aff.device)
    g, s = _ctx(P_aff, Q_aff)
    _call("dx_pairing", g, s, _ptr(P_aff), _ptr(Q_aff), _ptr(out), n)
    return out


_CHUNK_WORDS = 4096


def batched_copy(pairs: list) -> None:
    """``dst.copy_(src)`` for many (src, dst) pairs of one device in ONE
    launch of 16 KB chunks (csrc/kernels/dx_copy.hip); both contiguous, the
    same byte size, a multiple of 4 bytes."""
    pairs = [(s_, d_) for s_, d_ in pairs if s_.numel()]
    if not pairs:
        return
    dev = pairs[0][1].device
    desc = np.empty((len(pairs), 4), dtype=np.int64)
    c0 = 0
    for i, (s_, d_) in enumerate(pairs):
        nb = s_.numel() * s_.element_size()
        assert s_.is_contiguous() and d_.is_contiguous() and s_.device == dev and d_.device == dev
        assert nb == d_.numel() * d_.element_size() and nb % 4 == 0, (s_.shape, d_.shape)
        w = nb // 4
        desc[i] = (s_.data_ptr(), d_.data_ptr(), w, c0)
        c0 += -(-w // _CHUNK_WORDS)
    ht = torch.from_numpy(desc)
    if dev.type == "cuda":
        no_capture("batched_copy")
    dd = ht.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else ht
    g, st = _ctx(pairs[0][1])
    for s_, d_ in pairs:  # held until the call returns
        _ptr(s_), _ptr(d_)
    _call("dx_batched_copy", g, st, _ptr(dd), _ptr(ht), len(pairs), c0)


COPY_OUT_BLOCKS = 32


def copy_to_host(pairs: list, host_base: torch.Tensor, blocks: int = COPY_OUT_BLOCKS) -> None:
    """``dst.copy_(src)`` for (device src, slice of the pinned host buffer
    ``host_base``) pairs in ONE launch of a ``blocks``-workgroup persistent
    grid on the current stream (csrc/kernels/dx_copy.hip copy_out_kernel):
    PCIe-bound like the runtime's blit copy, but on a few CUs instead of
    thousands of waves beside the compute kernels.  4-byte multiples."""
    pairs = [(s_, d_) for s_, d_ in pairs if s_.numel()]
    if not pairs:
        return
    dev = pairs[0][0].device
    assert dev.type == "cuda" and host_base.is_pinned() and host_base.is_contiguous()
    hb = host_base.data_ptr()
    dbase = ctypes.c_int64(0)
    rc = _load().dx_host_device_ptr(ctypes.c_void_p(hb), ctypes.cast(ctypes.pointer(dbase), ctypes.c_void_p))
    if rc:
        raise RuntimeError("pinned buffer has no device mapping")
    hend = hb + host_base.numel() * host_base.element_size()
    desc = np.empty((len(pairs), 4), dtype=np.int64)
    c0 = 0
    for i, (s_, d_) in enumerate(pairs):
        nb = s_.numel() * s_.element_size()
        assert s_.is_contiguous() and d_.is_contiguous() and s_.device == dev and d_.device.type == "cpu"
        assert nb == d_.numel() * d_.element_size() and nb % 4 == 0 and s_.data_ptr() % 4 == 0
        assert hb <= d_.data_ptr() and d_.data_ptr() + nb <= hend and (d_.data_ptr() - hb) % 4 == 0
        w = nb // 4
        desc[i] = (s_.data_ptr(), dbase.value + (d_.data_ptr() - hb), w, c0)
        c0 += -(-w // _CHUNK_WORDS)
    ht = torch.from_numpy(desc)
    no_capture("copy_to_host")
    dd = ht.pin_memory().to(dev, non_blocking=True)
    st = torch.cuda.current_stream(dev).cuda_stream
    for s_, _ in pairs:
        _ptr(s_)
    _call("dx_copy_out", 1, st, _ptr(dd), _ptr(ht), len(pairs), c0, int(blocks))


def _strided_rows(ts: list):
    """[G, *shape] strided view over G equally shaped contiguous blocks that
    sit at a constant byte step in ONE storage, else None."""
    t0 = ts[0]
    # many small blocks only (thousands of one-record DPs): a few large ones
    # copy faster through the batched 16 KB-chunk kernel
    if len(ts) < 256 or not all(t.is_contiguous() and t.shape == t0.shape and t.dtype == t0.dtype for t in ts):
        return None
    st = t0.untyped_storage().data_ptr()
    if any(t.untyped_storage().data_ptr() != st for t in ts):
        return None
    es = t0.element_size()
    step = ts[1].data_ptr() - t0.data_ptr()
    if step % es or step < t0.numel() * es:
        return None
    p0 = t0.data_ptr()
    if any(t.data_ptr() != p0 + g * step for g, t in enumerate(ts)):
        return None
    return t0.as_strided((len(ts), t0.numel()), (step // es, 1))


def cat_rows(groups: list) -> list:
    """``[torch.cat(g) for g in groups]`` (dim 0) with every copy in ONE
    ``batched_copy`` launch.  A one-tensor group is returned as is (no copy);
    groups whose element bytes are not a multiple of 4 use torch.cat."""
    outs, pairs = [], []
    for g_ in groups:
        if len(g_) == 1:
            outs.append(g_[0])
            continue
        t0 = g_[0]
        if any(t.numel() * t.element_size() % 4 for t in g_):
            outs.append(torch.cat(g_))
            continue
        sv = _strided_rows(g_)
        if sv is not None:
            # equally shaped blocks at a constant stride in one storage (the
            # fields of thousands of one-proof bundles packed as rows of one
            # tensor): ONE strided copy, not one copy descriptor per block
            outs.append(sv.clone(memory_format=torch.contiguous_format).view((-1,) + tuple(t0.shape[1:])))
            continue
        out = torch.empty((sum(t.shape[0] for t in g_),) + tuple(t0.shape[1:]), dtype=t0.dtype, device=t0.device)
        o = 0
        for t in g_:
            assert t.dtype == t0.dtype and tuple(t.shape[1:]) == tuple(t0.shape[1:])
            pairs.append((t.contiguous(), out[o: o + t.shape[0]]))
            o += t.shape[0]
        outs.append(out)
    batched_copy(pairs)
    return outs


def rows_all(flags: list, n: int) -> torch.Tensor:
    """uint8 [n]: row p passes iff every flag array (uint8 / bool, n * k_a
    entries, row-major) is non-zero on its k_a entries of row p -- one
    wavefront per row (csrc/kernels/dx_copy.hip), no bool conversions or
    reductions."""
    fl = [f.reshape(-1).contiguous() for f in flags]
    fl = [f.view(torch.uint8) if f.dtype == torch.bool else f for f in fl]
    assert all(f.dtype == torch.uint8 and f.numel() % max(n, 1) == 0 for f in fl)
    out = torch.empty((n,), dtype=torch.uint8, device=fl[0].device)
    if n == 0:
        return out
    for i in range(0, len(fl), 16):
        part = fl[i: i + 16]
        ptrs = np.asarray([f.data_ptr() for f in part], dtype=np.int64)
        ks = np.asarray([f.numel() // n for f in part], dtype=np.int64)
        g, s = _ctx(out)
        for f in part:
            _ptr(f)
        o = out if i == 0 else torch.empty_like(out)
        _call("dx_rows_all", g, s, ptrs.ctypes.data, ks.ctypes.data, len(part), n, _ptr(o))
        if i:
            out &= o
    return out


def gt_mul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    n = _rows(a, 96)
    out = torch.empty_like(a)
    g, s = _ctx(a, b)
    _call("dx_gt_mul", g, s, _ptr(a), _ptr(b), _ptr(out), n)
    return out


def gt_inv(a: torch.Tensor) -> torch.Tensor:
    """Row-wise inverse in Fp12*."""
    n = _rows(a, 96)
    out = torch.empty_like(a)
    g, s = _ctx(a)
    _call("dx_gt_inv", g, s, _ptr(a.contiguous()), _ptr(out), n)
    return out


def gt_pow(a: torch.Tensor, scalars: torch.Tensor) -> torch.Tensor:
    n = _rows(scalars, 8)
    na = _rows(a, 96)
    out = torch.empty((n, 96), dtype=torch.int32, device=a.device)
    g, s = _ctx(a, scalars)
    _call("dx_gt_pow", g, s, _ptr(a), _ptr(scalars), _ptr(out), n, int(na == 1 and n > 1))
    return out


def gt_eq(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    n = _rows(a, 96)
    out = torch.empty((n,), dtype=torch.uint8, device=a.device)
    g, s = _ctx(a, b)
    _call("dx_gt_eq", g, s, _ptr(a), _ptr(b), _ptr(out), n)
    return out


def gt_fb_table(bases: torch.Tensor) -> torch.Tensor:
    nb = _rows(bases, 96)
    table = torch.empty((nb * 8192, 96), dtype=torch.int32, device=bases.device)
    work = torch.empty((nb * 256, 96), dtype=torch.int32, device=bases.device)
    g, s = _ctx(bases)
    _call("dx_gt_fb_table", g, s, _ptr(bases.contiguous()), _ptr(work), _ptr(table), nb)
    return table


def gt_fb_pow(tables: torch.Tensor, scalars: torch.Tensor, tab_idx: torch.Tensor | None = None) -> torch.Tensor:
    n = _rows(scalars, 8)
    out = torch.empty((n, 96), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(tables, scalars, tab_idx)
    _call("dx_gt_fb_pow", g, s, _ptr(tables), _ptr(tab_idx), _ptr(scalars), _ptr(out), n)
    return out


def gt_fb4_table(bases: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """4-bit comb table(s) [n_bases*960, 96] (360 KiB per base)."""
    bases = bases.contiguous()
    nb = _rows(bases, 96)
    table = out if out is not None else torch.empty((nb * FB4_ENTRIES, 96), dtype=torch.int32, device=bases.device)
    assert table.shape == (nb * FB4_ENTRIES, 96) and table.is_contiguous()
    work = torch.empty((nb * 64, 96), dtype=torch.int32, device=bases.device)
    g, s = _ctx(bases, table)
    _call("dx_gt_fb4_table", g, s, _ptr(bases), _ptr(work), _ptr(table), nb)
    return table


def gt_fb4_pow(tables: torch.Tensor, scalars: torch.Tensor, tab_idx: torch.Tensor | None = None) -> torch.Tensor:
    n = _rows(scalars, 8)
    out = torch.empty((n, 96), dtype=torch.int32, device=scalars.device)
    g, s = _ctx(tables, scalars, tab_idx)
    _call("dx_gt_fb4_pow", g, s, _ptr(tables), _ptr(tab_idx), _ptr(scalars), _ptr(out), n)
    return out


def gt_prod(x: torch.Tensor, chunk: int = 16) -> torch.Tensor:
    """Product over axis 0 of x[n_items, n_groups, 96] -> [n_groups, 96]."""
    assert x.dim() == 3 and x.shape[-1] == 96
    n_items, n_groups = x.shape[0], x.shape[1]
    cur = x.contiguous()
    while n_items > 1:
        ch = max(2, min(chunk, n_items))
        n_chunks = (n_items + ch - 1) // ch
        out = torch.empty((n_chunks, n_groups, 96), dtype=torch.int32, device=x.device)
        g, s = _ctx(cur)
        _call("dx_gt_prod_chunks", g, s, _ptr(cur), _ptr(out), n_items, n_groups, ch)
        cur, n_items = out, n_chunks
    return cur[0]


# ----------------------------------------------------------------------------- logistic-regression GEMM (K13)
def lr_gd_k2(a0, S, w0, N: float, lam: float, step: float, max_iter: int, C) -> list:
    """FindMinimumWeights for k = 2 on the host (csrc/kernels/dx_lr.hip
    dx_lr_gd_k2; float64 numpy arrays in, the minimum weights out).  The
    ctypes call releases the GIL for the whole descent."""
    a0 = np.ascontiguousarray(a0, dtype=np.float64)
    S = np.ascontiguousarray(S, dtype=np.float64)
    w0 = np.ascontiguousarray(w0, dtype=np.float64)
    d1 = a0.shape[0]
    out = np.empty(d1, dtype=np.float64)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = _load().dx_lr_gd_k2(p(a0), p(S), p(w0), d1, float(N), float(lam), float(step), int(max_iter), float(C[0]),
                             float(C[1]), float(C[2]), p(out))
    if rc:
        raise RuntimeError(f"dx_lr_gd_k2 failed rc={rc}")
    return out.tolist()


def random_scalars(n: int, device) -> torch.Tensor:
    """n uniform nonzero Fr scalars [n, 8] (plain limbs): ChaCha20 keyed with
    256 fresh bits of os.urandom per call, one block per scalar (dx_hash.hip)."""
    import numpy as _np

    device = torch.device(device)
    out = torch.empty((max(0, n), 8), dtype=torch.int32, device=device)
    if n <= 0:
        return out
    key = _np.frombuffer(os.urandom(32), dtype="<u4").copy()
    g, s = _ctx(out)
    _call("dx_random_scalars", g, s, key.ctypes.data_as(ctypes.c_void_p), 0, _ptr(out), n)
    return out


def hash_to_g1(seed: bytes, start: int, n: int, device) -> torch.Tensor:
    """[n, 16] affine G1 points h_start .. h_{start+n-1} derived from a 32-byte
    seed by try-and-increment (dx_hash.hip; unknown discrete logarithms)."""
    from ..crypto import oracle as _O

    device = torch.device(device)
    out = torch.empty((max(0, n), 16), dtype=torch.int32, device=device)
    if n <= 0:
        return out
    sd = np.frombuffer(seed, dtype=">u4").astype("<u4").copy()  # seed words as big-endian message words
    e = np.frombuffer(((_O.P + 1) // 4).to_bytes(32, "little"), dtype="<u4").copy()
    g, s = _ctx(out)
    _call("dx_hash_to_g1", g, s, sd.ctypes.data_as(ctypes.c_void_p), e.ctypes.data_as(ctypes.c_void_p), start,
          _ptr(out), n)
    return out


def fp_sqrt_host(vals: list) -> list:
    """[(sqrt or None)] of Python ints mod p (p = 3 mod 4: a^((p+1)/4)), one
    native host batch."""
    from ..crypto import oracle as _O

    n = len(vals)
    if n == 0:
        return []
    a = np.frombuffer(b"".join((int(v) % _O.P).to_bytes(32, "little") for v in vals), dtype="<u4").copy()
    e = np.frombuffer(((_O.P + 1) // 4).to_bytes(32, "little"), dtype="<u4").copy()
    y = np.empty(8 * n, dtype="<u4")
    ok = np.empty(n, dtype=np.uint8)
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    if _load().dx_fp_sqrt_host(p(a), p(e), p(y), p(ok), n):
        raise RuntimeError("dx_fp_sqrt_host failed")
    yb = y.tobytes()
    return [int.from_bytes(yb[32 * i: 32 * i + 32], "little") if ok[i] else None for i in range(n)]


def prg_scalars(key: bytes, n: int, device) -> torch.Tensor:
    """n Fr scalars from ChaCha20 keyed by a 32-byte ``key`` (deterministic:
    Fiat-Shamir challenge vectors expanded on the device)."""
    device = torch.device(device)
    out = torch.empty((max(0, n), 8), dtype=torch.int32, device=device)
    if n <= 0:
        return out
    k = np.frombuffer(key[:32], dtype="<u4").copy()
    g, s = _ctx(out)
    _call("dx_random_scalars", g, s, k.ctypes.data_as(ctypes.c_void_p), 0, _ptr(out), n)
    return out


def sha256_chunks(data: torch.Tensor, chunk: int) -> torch.Tensor:
    """[k, 8] big-endian SHA-256 words of every `chunk`-byte slice of the raw
    bytes of a contiguous tensor (k = ceil(nbytes / chunk), >= 1)."""
    data = data.contiguous()
    nbytes = data.numel() * data.element_size()
    k = max(1, (nbytes + chunk - 1) // chunk)
    out = torch.empty((k, 8), dtype=torch.int32, device=data.device)
    g, s = _ctx(data)
    _call("dx_sha256_chunks", g, s, _ptr(data), nbytes, chunk, _ptr(out))
    return out


def sha256_segments(tensors: list, chunk: int) -> list:
    """``sha256_chunks`` of many contiguous tensors (same device) in ONE
    launch -> list of [k_i, 8] views of one output tensor."""
    if not tensors:
        return []
    dev = tensors[0].device
    ts = [t.contiguous() for t in tensors]
    nbytes = [t.numel() * t.element_size() for t in ts]
    ks = [max(1, (b + chunk - 1) // chunk) for b in nbytes]
    first = np.concatenate([[0], np.cumsum(ks)[:-1]]).astype(np.int64)
    desc = np.empty((len(ts), 3), dtype=np.int64)
    desc[:, 0] = [t.data_ptr() for t in ts]
    desc[:, 1] = nbytes
    desc[:, 2] = first
    total = int(sum(ks))
    out = torch.empty((total, 8), dtype=torch.int32, device=dev)
    d = _upload(desc, dev)
    g, s = _ctx(out)
    # (the descriptor and any contiguous copies are allocated on this stream:
    # the caching allocator reuses them only behind this launch)
    _call("dx_sha256_segments", g, s, _ptr(d), len(ts), total, chunk, _ptr(out))
    return [out[a: a + k] for a, k in zip(first.tolist(), ks)]


INT_MOMENTS_MAX_COLS = 64


def no_capture(what: str):
    """Host-to-device copies from temporary host buffers must not be recorded
    into a HIP graph (a replay would read freed host memory)."""
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        raise RuntimeError(f"{what}: host upload inside a HIP graph capture")


def _upload(a: np.ndarray, device) -> torch.Tensor:
    t = torch.from_numpy(np.ascontiguousarray(a))
    if torch.device(device).type == "cuda":
        no_capture("upload")
        return t.pin_memory().to(device, non_blocking=True)
    return t


def int_moments(Z: torch.Tensor, seg_rows, pairs) -> torch.Tensor:
    """K14 (csrc/kernels/dx_moments.hip): exact int64 ``out[g, p] = sum over the
    rows of segment g of Z[i, a_p] * Z[i, b_p]`` (mod 2^64), column index
    ``C = Z.shape[1]`` standing for a constant 1.  ``seg_rows`` are the host-known
    row counts of the consecutive segments (one per DP); ``pairs`` a [P, 2]
    int sequence.  One launch for all segments."""
    assert Z.dtype == torch.int64 and Z.dim() == 2 and Z.stride(1) == 1
    C = Z.shape[1]
    pr = np.asarray(pairs, dtype=np.int16).reshape(-1, 2)
    if C > INT_MOMENTS_MAX_COLS or pr.size == 0 or pr.min() < 0 or pr.max() > C:
        raise ValueError(f"int_moments: {C} columns, pairs out of range")
    counts = np.asarray(seg_rows, dtype=np.int64)
    G, P = len(counts), pr.shape[0]
    if counts.sum() != Z.shape[0]:
        raise ValueError(f"int_moments: segments cover {counts.sum()} rows, Z has {Z.shape[0]}")
    out = torch.zeros((G, P), dtype=torch.int64, device=Z.device)
    # tiles: row ranges of one segment, sized so a big DP spreads over ~2k
    # workgroups and each tile still streams >= 64 rows
    per_tile = -(-int(counts.sum()) // 2048)
    chunk = max(64, (per_tile + 63) // 64 * 64)
    per = np.maximum(1, -(-counts // chunk)) * (counts > 0)
    seg = np.repeat(np.arange(G, dtype=np.int64), per)
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.int64)
    first = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(np.int64)
    k = np.arange(len(seg), dtype=np.int64) - np.repeat(first, per)
    r0 = np.repeat(starts, per) + k * chunk
    r1 = np.minimum(r0 + chunk, np.repeat(starts + counts, per))
    n_tiles = len(seg)
    if n_tiles == 0:
        return out
    Zc = Z.contiguous()
    tiles = _upload(np.stack([seg, r0, r1], axis=1), Z.device)
    pairs_t = _upload(pr, Z.device)
    g, s = _ctx(Zc)
    partial = None if g else torch.empty((n_tiles, P), dtype=torch.int64)
    _call("dx_int_moments", g, s, _ptr(Zc), Zc.stride(0), C, _ptr(tiles), n_tiles, _ptr(pairs_t), P, _ptr(out),
          _ptr(partial))
    return out


def sha256_rows(data: torch.Tensor, chunk: int) -> torch.Tensor:
    """[rows, k, 8] big-endian SHA-256 words of every `chunk`-byte slice of
    every row of a contiguous 2-D tensor (k = ceil(row bytes / chunk), >= 1)."""
    assert data.dim() == 2 and data.is_contiguous()
    rows = data.shape[0]
    row_bytes = data.shape[1] * data.element_size()
    k = max(1, (row_bytes + chunk - 1) // chunk)
    out = torch.empty((rows, k, 8), dtype=torch.int32, device=data.device)
    g, s = _ctx(data)
    _call("dx_sha256_rows", g, s, _ptr(data), rows, row_bytes, row_bytes, chunk, _ptr(out))
    return out


def lr_moments(X: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """sum_i w_i X_i X_i^T on the fp64-MFMA kernel (GPU tensors only)."""
    assert X.is_cuda and X.dtype == torch.float64 and X.dim() == 2 and X.shape[1] <= 48
    N, D = X.shape
    steps = (N + 3) // 4
    n_blocks = int(max(1, min(2048, (steps + 15) // 16)))
    partial = torch.empty((n_blocks, 48, 48), dtype=torch.float64, device=X.device)
    _, s = _ctx(X)
    rc = _raw_call("dx_lr_moments", s, _ptr(X), _ptr(w.to(torch.float64).contiguous()), N, D, _ptr(partial), n_blocks)
    if rc != 0:
        raise RuntimeError(f"dx_lr_moments failed rc={rc}")
    return partial.sum(0)[:D, :D]


def lr_encode(X: torch.Tensor, y: torch.Tensor, mean: torch.Tensor, sd: torch.Tensor, wa: float, wb: float):
    """Fused DP encoder on the fp64-MFMA kernel (GPU tensors only): with
    xa_i = [1, (X_i - mean)/sd], returns (sum_i (2y_i-1) xa_i  [D],
    sum_i (wa*y_i + wb) xa_i xa_i^T  [D, D]), D = X.shape[1] + 1 <= 47."""
    tot = lr_encode_many([X], [y], mean, sd, wa, wb)[0]
    D = X.shape[1] + 1
    return tot[D, :D], tot[:D, :D]


def _lr_blocks(N: int) -> int:
    steps = (N + 3) // 4
    return int(max(1, min(1024, (steps + 15) // 16)))


def lr_encode_many(Xs: list, ys: list, mean, sd, wa: float, wb: float) -> torch.Tensor:
    """``lr_encode`` of several DPs' records with the same standardisation:
    one encoder launch per DP into one partial slab, then ONE reduction
    launch (dx_lr_reduce, fixed summation order: a DP's totals are the same
    bits alone or batched) -> [n, 48, 48] totals (level 1 in row D)."""
    X0 = Xs[0]
    dev = X0.device
    dx = X0.shape[1]
    if dx + 1 >= 48:
        raise ValueError(f"lr_encode supports at most 46 features (got {dx})")
    mean = torch.as_tensor(mean, dtype=torch.float64).to(dev).contiguous()
    sd = torch.as_tensor(sd, dtype=torch.float64).to(dev).contiguous()
    assert mean.numel() == dx and sd.numel() == dx
    nbs = [_lr_blocks(X.shape[0]) for X in Xs]
    nb = max(nbs)
    alloc = torch.empty if all(b == nb for b in nbs) else torch.zeros  # unused blocks must add nothing
    partial = alloc((len(Xs), nb, 48, 48), dtype=torch.float64, device=dev)
    _, s = _ctx(X0)
    keep = []
    for i, (X, y) in enumerate(zip(Xs, ys)):
        assert X.is_cuda and X.dtype == torch.float64 and X.dim() == 2 and X.stride(1) == 1 and X.shape[1] == dx
        N = X.shape[0]
        y = y.to(device=dev, dtype=torch.float64).contiguous()
        assert y.numel() == N
        keep.append(y)
        rc = _raw_call("dx_lr_encode", s, _ptr(X), X.stride(0), N, dx, _ptr(mean), _ptr(sd), _ptr(y), float(wa),
                       float(wb), _ptr(partial[i]), nbs[i])
        if rc != 0:
            raise RuntimeError(f"dx_lr_encode failed rc={rc}")
    out = torch.empty((len(Xs), 48, 48), dtype=torch.float64, device=dev)
    rc = _raw_call("dx_lr_reduce", s, _ptr(partial), nb, 48 * 48, len(Xs), _ptr(out))
    if rc != 0:
        raise RuntimeError(f"dx_lr_reduce failed rc={rc}")
    return out


# ----------------------------------------------------------------------------- range proofs (K15/K16)
def rp_prove_a(negsB_aff, V_aff, t_sc, gt_table, S: int, L: int) -> torch.Tensor:
    n = _rows(V_aff, 32)
    out = torch.empty((n, 96), dtype=torch.int32, device=V_aff.device)
    g, s = _ctx(negsB_aff, V_aff, t_sc, gt_table)
    _call("dx_rp_prove_a", g, s, _ptr(negsB_aff), _ptr(V_aff), _ptr(t_sc), _ptr(gt_table), _ptr(out), n, S, L)
    return out


def rp_prove_a_tab(gphi_tables, tab_idx, e_sc, t_sc, gt_table, S: int, L: int, wbits: int = 8) -> torch.Tensor:
    """wbits = 8: gphi_tables in the 8-bit comb layout; 4: the 4-bit layout
    (gt_fb4_table); 6: the GLS-2 6-bit layout (gt_gls6_table); 7: the GLS-2
    signed 8-bit layout (gt_gls8_table)."""
    assert wbits in (4, 6, 7, 8)
    n = _rows(e_sc, 8)
    out = torch.empty((n, 96), dtype=torch.int32, device=e_sc.device)
    g, s = _ctx(gphi_tables, tab_idx, e_sc, t_sc, gt_table)
    if wbits == 7:
        assert tab_idx.dtype == torch.int32 and tab_idx.numel() == n and n % (S * L) == 0
        t16 = gt16_table(e_sc.device) if e_sc.is_cuda else None                # gT^t in 17 products
        _call("dx_rp_prove_a_gls8", g, s, _ptr(gphi_tables), _ptr(tab_idx), _ptr(e_sc), _ptr(t_sc),
              _ptr(t16 if t16 is not None else gt_table), _ptr(out), n, S, L, int(t16 is not None))
        return out
    if wbits == 6:
        _call("dx_rp_prove_a_gls6", g, s, _ptr(gphi_tables), _ptr(tab_idx), _ptr(e_sc), _ptr(t_sc), _ptr(gt_table),
              _ptr(out), n, S, L)
        return out
    _call("dx_rp_prove_a_tab", g, s, _ptr(gphi_tables), _ptr(tab_idx), _ptr(e_sc), _ptr(t_sc), _ptr(gt_table),
          _ptr(out), n, S, L, wbits)
    return out


def rp_challenges(C_aff: torch.Tensor, b_words: torch.Tensor, y_words: torch.Tensor,
                  cols: torch.Tensor) -> torch.Tensor:
    """Range-proof challenges SHA3-512(B || C_p || Y_col) mod r -> [n, 8]
    canonical scalars (dx_keccak.hip).  b_words [16] and y_words [n_cols, 16]
    are the 64-byte point encodings viewed as little-endian int32 words."""
    n = _rows(C_aff, 16)
    assert cols.dtype == torch.int32 and cols.numel() == n and b_words.numel() == 16
    out = torch.empty((n, 8), dtype=torch.int32, device=C_aff.device)
    g, s = _ctx(C_aff, b_words, y_words, cols)
    _call("dx_rp_challenges", g, s, _ptr(C_aff), _ptr(b_words), _ptr(y_words), _ptr(cols), _ptr(out), n)
    return out


def rp_verify_items(ZB_jac, Y_jac, rho, V_aff, a, S: int, L: int):
    n = _rows(V_aff, 32)
    f = torch.empty((n, 96), dtype=torch.int32, device=V_aff.device)
    gg = torch.empty((n, 96), dtype=torch.int32, device=V_aff.device)
    g, s = _ctx(ZB_jac, Y_jac, rho, V_aff, a)
    _call("dx_rp_verify_items", g, s, _ptr(ZB_jac), _ptr(Y_jac), _ptr(rho), _ptr(V_aff), _ptr(a), _ptr(f), _ptr(gg),
          n, S, L)
    return f, gg


def rp_verify_products(ZB_jac, Y_jac, rho, V_aff, a, S: int, L: int):
    """(prod_it ML_it, prod_it a_it^rho_it) as two [1, 96] HOST tensors.
    GPU: the Miller values fold per 64-item workgroup in LDS (dx_rp_verify_fold)
    and the a^rho product is a bucket multi-exponentiation (gt_multi_exp64);
    host: per-item values + product tree."""
    g, s = _ctx(ZB_jac, Y_jac, rho, V_aff, a)
    if not g:
        f, gg = rp_verify_items(ZB_jac, Y_jac, rho, V_aff, a, S, L)
        return gt_prod(f.view(-1, 1, 96), chunk=4).view(1, 96), gt_prod(gg.view(-1, 1, 96), chunk=4).view(1, 96)
    plan = _multi_exp64_plan(rho)  # index work first: its one host sync does not wait for the Miller fold
    fb = rp_verify_fold(ZB_jac, Y_jac, rho, V_aff, S, L)
    G = _multi_exp64_run(a, plan)
    return _finish_prod_on_host(fb), G


def rp_verify_fold(ZB_jac, Y_jac, rho, V_aff, S: int, L: int) -> torch.Tensor:
    """Launch the fused Miller fold (GPU, asynchronous): [ceil(n/64), 96]
    per-workgroup Miller products on the current stream."""
    n = _rows(V_aff, 32)
    _, s = _ctx(ZB_jac, Y_jac, rho, V_aff)
    fb = torch.empty(((n + 63) // 64, 96), dtype=torch.int32, device=V_aff.device)
    rc = _raw_call("dx_rp_verify_fold", s, _ptr(ZB_jac), _ptr(Y_jac), _ptr(rho), _ptr(V_aff), _ptr(fb), n, S, L)
    if rc:
        raise RuntimeError(f"dx_rp_verify_fold failed rc={rc}")
    return fb


# inl: tower force-inlined into the fold kernels (12.4M Miller loops/s on one
# MI355X vs 10.0M for ni, the out-of-line tower; tools/fold_bench.py)
FOLD_VARIANT = "inl"  # dx_fold_inl.hip (force-inlined tower functions; the out-of-line build lost its A/B)


def rp_fold_points(ZB_jac: torch.Tensor, Y_jac: torch.Tensor, rho: torch.Tensor, S: int, L: int,
                   variant: str | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """GPU: P_it = affine(rho_it (ZB[p*L+j] - Y[p*S+i])), it = (p*S+i)*L + j,
    one fused launch -> [n, 16] (n = rows of rho), or into ``out``."""
    v = variant or FOLD_VARIANT
    n = _rows(rho, 8)
    assert _rows(ZB_jac, 24) * S == n and _rows(Y_jac, 24) * L == n and ZB_jac.is_cuda
    P = out if out is not None else torch.empty((n, 16), dtype=torch.int32, device=rho.device)
    assert P.shape == (n, 16) and P.is_contiguous()
    _, s = _ctx(ZB_jac, Y_jac, rho)
    rc = _raw_call(f"dx_rp_points_{v}", s, _ptr(ZB_jac.contiguous()), _ptr(Y_jac.contiguous()), _ptr(rho),
                                                  _ptr(P), n, S, L)
    if rc:
        raise RuntimeError(f"dx_rp_points_{v} failed rc={rc}")
    return P


def rp_fold_lines(P_aff: torch.Tensor, V_aff: torch.Tensor, variant: str | None = None,
                  period: int | None = None) -> torch.Tensor:
    """Phase 1 of the two-phase Miller fold (GPU): the sparse line values of
    every item's Miller loop evaluated at its P -> flat int32 image
    [steps * 12 * n * 4] (csrc/kernels/fold_body.h).  ``period``: item it
    pairs P[it] with V[it % period] (several verifiers' batches, each padded
    to ``period`` rows, in one launch)."""
    v = variant or FOLD_VARIANT
    n = _rows(P_aff, 16)
    nv = _rows(V_aff, 32)
    period = period or n
    assert nv <= period and n % period == 0 and P_aff.is_cuda
    steps = getattr(_load(), f"dx_fold_steps_{v}")()
    lines = torch.empty((steps * 12 * n * 4,), dtype=torch.int32, device=P_aff.device)
    _, s = _ctx(P_aff, V_aff)
    rc = _raw_call(f"dx_rp_lines_{v}", s, _ptr(P_aff), _ptr(V_aff), _ptr(lines), n, period, nv)
    if rc:
        raise RuntimeError(f"dx_rp_lines_{v} failed rc={rc}")
    return lines


def rp_fold_accum(lines: torch.Tensor, n: int, K: int = 4, variant: str | None = None) -> torch.Tensor:
    """Phase 2: per-workgroup products of the Miller values of 64*K items,
    K items per lane sharing one accumulator -> [ceil(n / (64 K)), 96]."""
    v = variant or FOLD_VARIANT
    fb = torch.empty(((n + 64 * K - 1) // (64 * K), 96), dtype=torch.int32, device=lines.device)
    _, s = _ctx(lines)
    rc = _raw_call(f"dx_rp_accum_{v}", s, _ptr(lines), _ptr(fb), n, K)
    if rc:
        raise RuntimeError(f"dx_rp_accum_{v} failed rc={rc}")
    return fb


# GLV batch weights (csrc/kernels/dx_glv.hip): rho = a + b * GLV_LAMBDA mod r with
# a, b 32-bit; phi(x, y) = (GLV_BETA x, y) = [GLV_LAMBDA] on G1; x^GLV_LAMBDA =
# x^(p^8) on GT.  Both constants are checked against the oracle in the tests.
GLV_BETA = 0x59E26BCEA0D48BACD4F263F1ACDB5C4F5763473177FFFFFE
GLV_LAMBDA = 0xB3C4D79D41A917585BFC41088D8DAAA78B17EA66B99C90DD
_glv_consts: dict = {}


def _glv_const(kind: str, device) -> torch.Tensor:
    from ..crypto import bn254 as _bn

    key = (kind, str(device))
    if key not in _glv_consts:
        if kind == "beta":
            v = _bn.to_tensor(_bn.ints_to_limbs([_bn.mont(GLV_BETA)]), device)
        else:
            v = _bn.to_tensor(_bn.ints_to_limbs([GLV_LAMBDA]), device)
        _glv_consts[key] = _bn.publish(v.contiguous())
    return _glv_consts[key]


def prg_glv(key: bytes, n: int, device):
    """``glv_weights(n, device, raw=prg_scalars(key, n, device))`` in ONE
    launch (csrc/kernels/dx_hash.hip dx_prg_glv) -> (ab [n, 2], rho [n, 8])."""
    device = torch.device(device)
    ab = torch.empty((max(0, n), 2), dtype=torch.int32, device=device)
    rho = torch.empty((max(0, n), 8), dtype=torch.int32, device=device)
    if n <= 0:
        return ab, rho
    k = np.frombuffer(key[:32], dtype="<u4").copy()
    lam = np.asarray(_lambda_limbs(), dtype=np.uint32)
    g, s = _ctx(ab)
    _call("dx_prg_glv", g, s, k.ctypes.data_as(ctypes.c_void_p), 0, lam.ctypes.data_as(ctypes.c_void_p), _ptr(ab),
          _ptr(rho), n)
    return ab, rho


def prg_bits(key: bytes, n: int, bits: int, device) -> torch.Tensor:
    """``coins.mask_bits(prg_scalars(key, n, device), bits)`` in ONE launch."""
    device = torch.device(device)
    out = torch.empty((max(0, n), 8), dtype=torch.int32, device=device)
    if n <= 0:
        return out
    k = np.frombuffer(key[:32], dtype="<u4").copy()
    g, s = _ctx(out)
    _call("dx_prg_bits", g, s, k.ctypes.data_as(ctypes.c_void_p), 0, int(bits), _ptr(out), n)
    return out


def _lambda_limbs() -> list:
    from ..crypto import bn254 as _bn

    return [int(x) for x in _bn.ints_to_limbs([GLV_LAMBDA]).reshape(-1)]


def glv_weights(n: int, device, raw: torch.Tensor | None = None):
    """n GLV batch weights: (ab [n, 2] int32 = the 32-bit halves (a, b),
    rho [n, 8] = a + b * GLV_LAMBDA as canonical scalars); ``raw``: [n, 8]
    uniform scalars to take the halves from (a verifier's own coins)."""
    from ..crypto import bn254 as _bn

    if raw is None:
        raw = _bn.random_scalars(n, device)
    ab = raw[:, :2].contiguous()
    a = torch.zeros_like(raw)
    b = torch.zeros_like(raw)
    a[:, 0] = ab[:, 0]
    b[:, 0] = ab[:, 1]
    rho = fr_arith(FR_ADD, a, fr_arith(FR_MUL, b, _glv_const("lambda", device)))
    return ab, rho


def g1_mul_glv(pts_jac: torch.Tensor, ab: torch.Tensor) -> torch.Tensor:
    """(a_i + b_i GLV_LAMBDA) P_i for 32-bit halves ab [n, 2] (``glv_weights``)
    -> Jacobian [n, 24]: 32 doublings of a joint 2-bit-window ladder over
    (P, phi(P)) instead of 64 (csrc/kernels/dx_glv.hip).  GPU; on the host
    the full scalars go through ``g1_mul``."""
    n = _rows(ab, 2)
    np_ = _rows(pts_jac, 24)
    assert np_ in (1, n)
    if not ab.is_cuda:
        a = torch.zeros((n, 8), dtype=torch.int32)
        b = torch.zeros((n, 8), dtype=torch.int32)
        a[:, 0], b[:, 0] = ab[:, 0], ab[:, 1]
        rho = fr_arith(FR_ADD, a, fr_arith(FR_MUL, b, _glv_const("lambda", "cpu")))
        return g1_mul(pts_jac, rho)
    out = torch.empty((n, 24), dtype=torch.int32, device=ab.device)
    _, s = _ctx(pts_jac, ab)
    rc = _raw_call("dx_g1_mul_glv", s, _ptr(pts_jac.contiguous()), _ptr(ab.contiguous()),
                   _ptr(_glv_const("beta", ab.device)), _ptr(out), n, int(np_ == 1 and n > 1))
    if rc:
        raise RuntimeError(f"dx_g1_mul_glv failed rc={rc}")
    return out


def rp_fold_points_glv(ZB_jac: torch.Tensor, Y_jac: torch.Tensor, ab: torch.Tensor, S: int, L: int,
                       out: torch.Tensor | None = None, uv: bool = False) -> torch.Tensor:
    """G1 side of the fold with GLV weights: affine((a + b lambda)(ZB - Y)) per
    item (or, ``uv``, its (x/y, 1/y) form for the normalised fold), one launch
    -> [n, 16] (GPU only)."""
    n = _rows(ab, 2)
    assert ab.dtype == torch.int32 and _rows(ZB_jac, 24) * S == n and _rows(Y_jac, 24) * L == n and ZB_jac.is_cuda
    P = out if out is not None else torch.empty((n, 16), dtype=torch.int32, device=ab.device)
    assert P.shape == (n, 16) and P.is_contiguous()
    _, s = _ctx(ZB_jac, Y_jac, ab)
    _call("dx_rp_points_glv", s, _ptr(ZB_jac.contiguous()), _ptr(Y_jac.contiguous()), _ptr(ab.contiguous()),
          _ptr(_glv_const("beta", ab.device)), _ptr(P), n, S, L, int(uv))
    return P


def g1_aff_to_uv_(aff: torch.Tensor) -> torch.Tensor:
    """In place: affine (x, y) rows -> (x/y, 1/y) (infinity stays zeros)."""
    g, s = _ctx(aff)
    _call("dx_g1_aff_to_uv", g, s, _ptr(aff), _rows(aff, 16))
    return aff


def rp_fold_ncoeffs(V_aff: torch.Tensor, variant: str | None = None) -> torch.Tensor:
    """Normalised shared-V line image: per V and step (c1/c0, c3/c0) ->
    flat int32 [steps * 8 * m * 4] (fold mode 4, csrc/kernels/fold_body.h)."""
    v = variant or FOLD_VARIANT
    m = _rows(V_aff, 32)
    assert V_aff.is_cuda and V_aff.is_contiguous()
    steps = getattr(_load(), f"dx_fold_steps_{v}")()
    img = torch.empty((steps * 8 * m * 4,), dtype=torch.int32, device=V_aff.device)
    scratch = torch.empty((2 * steps * 4 * m * 4,), dtype=torch.int32, device=V_aff.device)
    _, s = _ctx(V_aff)
    rc = _raw_call(f"dx_rp_ncoeffs_{v}", s, _ptr(V_aff), _ptr(img), _ptr(scratch), m)
    if rc:
        raise RuntimeError(f"dx_rp_ncoeffs_{v} failed rc={rc}")
    return img


def rp_fold_accum_n(img: torch.Tensor, UV: torch.Tensor, V_aff: torch.Tensor, period: int, G: int, K: int = 4,
                    variant: str | None = None) -> torch.Tensor:
    """Normalised shared-V accumulation: G verifiers' (u, v) point images
    against one normalised line image -> [G * period / (64 K), 96]."""
    v = variant or FOLD_VARIANT
    m = _rows(V_aff, 32)
    assert _rows(UV, 16) == G * period and period >= m and period % (64 * K * FOLD_P_ALIGN) == 0
    steps = getattr(_load(), f"dx_fold_steps_{v}")()
    assert img.numel() == steps * 8 * m * 4
    fb = torch.empty((G * period // (64 * K), 96), dtype=torch.int32, device=UV.device)
    _, s = _ctx(img, UV, V_aff)
    rc = _raw_call(f"dx_rp_accum_n_{v}", s, _ptr(img), _ptr(UV), _ptr(V_aff), _ptr(fb), m, period, G, K)
    if rc:
        raise RuntimeError(f"dx_rp_accum_n_{v} failed rc={rc}")
    return fb


def rp_fold_accum_coop_raw(coef: torch.Tensor, P_aff: torch.Tensor, V_aff: torch.Tensor, period: int,
                           G: int) -> torch.Tensor:
    """``rp_fold_accum_coop`` over the RAW line coefficients (``rp_fold_coeffs``,
    no normalising pass) and affine points P -> [G * period / 64, 96].  GPU only."""
    m = _rows(V_aff, 32)
    n = G * period
    assert _rows(P_aff, 16) == n and period >= m and period % 64 == 0
    assert coef.numel() == _load().dx_ufold_coop_steps() * 12 * m * 4
    f = torch.empty((n, 96), dtype=torch.int32, device=P_aff.device)
    _, s = _ctx(coef, P_aff, V_aff)
    rc = _raw_call("dx_ufold_coop_raw", s, _ptr(coef), _ptr(P_aff), _ptr(V_aff), _ptr(f), m, period, n)
    if rc:
        raise RuntimeError(f"dx_ufold_coop_raw failed rc={rc}")
    x = f.view(64, n // 64, 96)  # written lane-major by the kernel: item t at row (t % 64, t // 64)
    while x.shape[0] > 1:
        x = _gt_prod_level(x, 8)
    return x.view(n // 64, 96)


def gt_frob8(a: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """a^(p^8) per row (= a^GLV_LAMBDA on GT); ``out``: a contiguous
    destination of a's shape (e.g. the second half of a stacked image)."""
    out = torch.empty_like(a) if out is None else out
    assert out.is_contiguous() and out.shape == a.shape
    g, s = _ctx(a)
    _call("dx_gt_frob8", g, s, _ptr(a.contiguous()), _ptr(out), _rows(a, 96))
    return out


def rp_fold_coeffs(V_aff: torch.Tensor, variant: str | None = None) -> torch.Tensor:
    """Shared-V phase 1: the line coefficients of every V's Miller loop (no P)
    -> flat int32 image [steps * 12 * m * 4]; several verifiers folding the
    same proofs share it (``rp_fold_accum_p`` evaluates at their P)."""
    v = variant or FOLD_VARIANT
    m = _rows(V_aff, 32)
    assert V_aff.is_cuda and V_aff.is_contiguous()
    steps = getattr(_load(), f"dx_fold_steps_{v}")()
    coef = torch.empty((steps * 12 * m * 4,), dtype=torch.int32, device=V_aff.device)
    _, s = _ctx(V_aff)
    rc = _raw_call(f"dx_rp_coeffs_{v}", s, _ptr(V_aff), _ptr(coef), m)
    if rc:
        raise RuntimeError(f"dx_rp_coeffs_{v} failed rc={rc}")
    return coef


FOLD_P_ALIGN = 8  # verifier blocks are padded to 64 K * 8 items (XCD-paired block mapping)


def rp_fold_accum_p(coef: torch.Tensor, P_aff: torch.Tensor, V_aff: torch.Tensor, period: int, G: int, K: int = 4,
                    variant: str | None = None) -> torch.Tensor:
    """Shared-V phase 2: G verifiers' point images (P[v * period + q], q < m)
    folded against one coefficient image -> [G * period / (64 K), 96]
    partial products, verifier-major."""
    v = variant or FOLD_VARIANT
    m = _rows(V_aff, 32)
    assert _rows(P_aff, 16) == G * period and period >= m and period % (64 * K * FOLD_P_ALIGN) == 0
    steps = getattr(_load(), f"dx_fold_steps_{v}")()
    assert coef.numel() == steps * 12 * m * 4
    fb = torch.empty((G * period // (64 * K), 96), dtype=torch.int32, device=P_aff.device)
    _, s = _ctx(coef, P_aff, V_aff)
    rc = _raw_call(f"dx_rp_accum_p_{v}", s, _ptr(coef), _ptr(P_aff), _ptr(V_aff), _ptr(fb), m, period, G, K)
    if rc:
        raise RuntimeError(f"dx_rp_accum_p_{v} failed rc={rc}")
    return fb


def gt_slice_prod(src: torch.Tensor, idx, start: torch.Tensor, length: torch.Tensor) -> torch.Tensor:
    """out[s] = prod_k src[idx[start[s] + k]] (or src[start[s] + k]), k < length[s].
    (A latency-hidden 1-wave/SIMD variant with the gathers issued one
    product ahead measured the same, 3.62 vs 3.71 ms on 3.4M factors, and
    was dropped.)"""
    n = start.numel()
    out = torch.empty((n, 96), dtype=torch.int32, device=src.device)
    g, s = _ctx(src, idx, start, length)
    _call("dx_gt_slice_prod", g, s, _ptr(src), _ptr(idx), _ptr(start), _ptr(length), _ptr(out), n)
    return out


_ME_C = 8          # window bits
_ME_W = 64 // _ME_C
_ME_SLICE = 8      # entries per thread in each segmented-product pass


def _segment_passes(counts):
    """Slice plans that reduce contiguous per-bucket runs of `counts` entries
    to one product per bucket, <= _ME_SLICE factors per thread per pass (a
    lone GPU lane runs an Fp12 chain latency-bound, so chains stay short and
    each pass is wide).  Returns [(start, len), ...] numpy arrays per pass."""
    import numpy as _np

    passes = []
    c = _np.asarray(counts, dtype=_np.int64)
    while c.size and c.max() > 1:
        n_sl = (c + _ME_SLICE - 1) // _ME_SLICE
        first = _np.cumsum(c) - c
        b = _np.repeat(_np.arange(c.size), n_sl)
        k = _np.arange(b.size) - (_np.cumsum(n_sl) - n_sl)[b]
        start = first[b] + k * _ME_SLICE
        ln = _np.minimum(c[b] - k * _ME_SLICE, _ME_SLICE)
        passes.append((start, ln))
        c = n_sl
    return passes


def _multi_exp64_plan(rho: torch.Tensor):
    """Bucket plan of prod_i a_i^{rho_i} for 64-bit exponents (limbs 0, 1 of rho)."""
    return _bucket_plan(rho, _ME_W)


def _sort_buckets(keys: torch.Tensor, items: torch.Tensor, nb: int):
    """Sort the (key, item) entries of a bucket plan by key (torch's onesweep
    radix sort: on gfx950 faster than a direct rocPRIM pairs sort over the
    keys' bits, and it interferes least with the kernels running beside the
    plan, profiles/r4/ab_plan_sort.txt) and find every bucket's run
    (csrc/kernels/dx_plan.hip) -> (sorted items, per-bucket counts on the
    host: the plan's one device-to-host copy)."""
    i2, first, end = _sorted_runs(keys, items, nb)
    return i2, (end - first).cpu().numpy().astype(np.int64)


def _sorted_runs(keys: torch.Tensor, items: torch.Tensor, nb: int):
    """(items sorted by key, first[nb], end[nb]): every bucket's run in the
    sorted entries, on the keys' device (empty buckets: first = end = 0).
    (An atomic counting sort measured +22 ms on a 1-GPU inbox's 60M entries:
    the radix sort stays.)"""
    dev = keys.device
    k2, order = torch.sort(keys)
    i2 = items.index_select(0, order)
    bounds = torch.zeros((2, nb), dtype=torch.int64, device=dev)
    g, s = _ctx(k2)
    _call("dx_bucket_bounds", g, s, _ptr(k2), keys.numel(), nb, _ptr(bounds[0]), _ptr(bounds[1]))
    return i2, bounds[0], bounds[1]


def _segment_passes_dev(counts, dev, first_slice: int | None = None):
    """``_segment_passes`` with the per-slice (start, len) arrays written on
    the device by one thread per bucket (csrc/kernels/dx_plan.hip
    dx_slice_plan): only the per-bucket counts (at most a few hundred
    thousand) go through the host; the millions of slice descriptors of a wide
    multi-exponentiation are never built by numpy or torch index kernels.
    ``first_slice``: entries per thread in the first pass (later passes use
    _ME_SLICE)."""
    import numpy as _np

    passes = []
    c = _np.asarray(counts, dtype=_np.int64)
    while c.size and c.max() > 1:
        sl = first_slice if (first_slice and not passes) else _ME_SLICE
        n_sl = (c + sl - 1) // sl
        total = int(n_sl.sum())
        meta = _np.stack([_np.cumsum(c) - c, c, _np.cumsum(n_sl) - n_sl])
        m_dev = _upload(meta, dev)
        start = torch.empty(total, dtype=torch.int64, device=dev)
        ln = torch.empty(total, dtype=torch.int32, device=dev)
        g, s = _ctx(m_dev)
        _call("dx_slice_desc", g, s, _ptr(m_dev[0]), _ptr(m_dev[1]), _ptr(m_dev[2]), sl, c.size, total, _ptr(start),
              _ptr(ln))
        passes.append((start, ln))
        c = n_sl
    return passes


def _segment_passes_dev_torch(counts, dev, first_slice: int | None = None):
    """``_segment_passes`` with the per-slice (start, len) arrays built on the
    device: only the per-bucket counts (at most a few thousand) live on the
    host, the millions of slice descriptors of a wide multi-exponentiation
    never cross PCIe and never run through numpy.  ``first_slice``: entries
    per thread in the first pass (later passes use _ME_SLICE)."""
    import numpy as _np

    passes = []
    c = _np.asarray(counts, dtype=_np.int64)
    while c.size and c.max() > 1:
        sl = first_slice if (first_slice and not passes) else _ME_SLICE
        n_sl = (c + sl - 1) // sl
        total = int(n_sl.sum())
        ct = _upload(c, dev)
        nt_ = _upload(n_sl, dev)
        first = torch.cumsum(ct, 0) - ct
        b = torch.repeat_interleave(torch.arange(c.size, device=dev), nt_, output_size=total)
        k = torch.arange(total, device=dev) - (torch.cumsum(nt_, 0) - nt_)[b]
        start = first[b] + k * sl
        ln = torch.minimum(ct[b] - k * sl, torch.full_like(k, sl)).to(torch.int32)
        passes.append((start.contiguous(), ln.contiguous()))
        c = n_sl
    return passes


def _group_arg(group, n: int, dev):
    """(explicit int32 group tensor or None, group stride): an int ``group``
    means entry t belongs to group t // group (no per-entry tensor)."""
    if group is None:
        return None, 0
    if isinstance(group, int):
        return None, group
    assert group.numel() == n
    return group.to(device=dev, dtype=torch.int32).contiguous(), 0


def _bucket_plan(k: torch.Tensor, W: int, group: torch.Tensor | None = None, n_groups: int = 1, c: int = 8):
    """Bucket plan of a multi-scalar product over the low W c-bit windows of
    the scalars k [n, 8]: window w, digit d -> bucket (w << c) + d (plus
    g * (W << c) for entries of group g when `group` is given); entries sorted
    by bucket, then segmented passes down to one value per non-empty bucket.
    One host sync (the counts); ``_device_layout`` plans need none."""
    dev = k.device
    n = k.shape[0]
    nb = (W << c) * n_groups
    assert n * W < 2 ** 31 and nb < 2 ** 31 - 1
    keys = torch.empty(n * W, dtype=torch.int32, device=dev)
    item = torch.empty(n * W, dtype=torch.int32, device=dev)
    grp, gstride = _group_arg(group, n, dev)
    g, s = _ctx(k, keys)
    _call("dx_msm_keys", g, s, _ptr(k.contiguous()), _ptr(grp), gstride, n, c, W, _ptr(keys),  # dx_rpmsm.hip
          _ptr(item))
    item, counts = _sort_buckets(keys, item, nb)   # zero digits carry a sentinel key that sorts last
    it = item[: int(counts.sum())].to(torch.int64)                  # drop the zero-digit sentinels
    bk = np.flatnonzero(counts)
    passes = _segment_passes_dev(counts[bk], dev)
    # bucket digits and scatter slots, staged now so the run needs no host->device copy
    mask = (1 << c) - 1
    sc = torch.zeros((bk.size, 8), dtype=torch.int32)
    sc[:, 0] = torch.from_numpy((bk & mask).astype("int32"))
    slot = torch.from_numpy((bk & mask) * W + (bk >> c))
    return {"item": it, "passes": passes, "bk": bk, "single": not passes,
            "digit_sc": _upload(sc.numpy(), dev), "slot": _upload(slot.numpy(), dev), "W": W, "c": c}


def _multi_exp64_run(a: torch.Tensor, plan) -> torch.Tensor:
    """Finish prod a_i^{rho_i}: segmented passes -> bucket values B_{w,d} ->
    B^d (GPU), then per-window products and the 8-window Horner combination
    on the host (short serial Fp12 chains: one host core beats one GPU lane)."""
    dev = a.device
    bk = plan["bk"]
    if bk.size == 0:
        return gt_one("cpu").clone()
    cur = a.index_select(0, plan["item"]).contiguous() if plan["single"] else None
    for k, (st, ln) in enumerate(plan["passes"]):
        cur = gt_slice_prod(a if k == 0 else cur, plan["item"] if k == 0 else None, st, ln)
    bkp = gt_pow(cur, plan["digit_sc"])
    W, c = plan.get("W", _ME_W), plan.get("c", _ME_C)
    win = gt_one(dev).repeat((1 << c) * W, 1)
    win[plan["slot"]] = bkp
    win = win.view(1 << c, W, 96)
    if dev.type == "cuda":
        while win.shape[0] > 32:
            win = _gt_prod_level(win, 8)
    S_w = gt_prod(win.cpu(), chunk=4)                                  # [W, 96] on the host
    acc = S_w[W - 1: W].contiguous()
    for w in range(W - 2, -1, -1):
        acc = gt_pow(acc, _pow2_scalar(c))
        acc = gt_mul(acc, S_w[w: w + 1].contiguous())
    return acc


def multi_exp_plan(k: torch.Tensor, group, n_groups: int, W: int = _ME_W, c: int = 8):
    """The bucket plan of ``multi_exp_grouped`` alone (its one host sync)."""
    return _bucket_plan(k, W, group, n_groups, c)


def multi_exp_grouped(a: torch.Tensor, k: torch.Tensor, group, n_groups: int, W: int = _ME_W, c: int = 8,
                      plan: dict | None = None, item_split: tuple | None = None):
    """Launch G independent multi-exponentiations prod_{i: group_i = g} a[i % n]^k_i
    (n = rows of a, k [m, 8] with m a multiple of n, low W c-bit windows of
    each exponent; ``group`` an int32 tensor or an int stride) as ONE bucket
    plan (one host sync for all groups, e.g. the batch weights of several
    verifying nodes).  Returns a handle for ``multi_exp_grouped_finish``;
    device passes are queued on the current stream.
    ``item_split`` = (s, q): entry i < s uses a[i % n], entry i >= s uses
    a[(i - s) % q] (two exponent blocks over different row periods)."""
    n = a.shape[0]
    if plan is None:
        plan = _bucket_plan(k, W, group, n_groups, c)
    it = plan["item"]
    if item_split is not None:
        sp, q = item_split
        plan["item"] = torch.where(it < sp, it % n, (it - sp) % q).contiguous()
    else:
        plan["item"] = (it % n).contiguous()
    bk = plan["bk"]
    h = {"G": n_groups, "W": W, "c": c, "win": None}
    if bk.size == 0:
        return h
    cur = a.index_select(0, plan["item"]).contiguous() if plan["single"] else None
    for i, (st, ln) in enumerate(plan["passes"]):
        cur = gt_slice_prod(a if i == 0 else cur, plan["item"] if i == 0 else None, st, ln)
    _me_windows(h, cur, bk, n_groups, W, c, a.device)
    return h


def _me_windows(h: dict, cur, bk, n_groups: int, W: int, c: int, dev):
    """Bucket values -> B^d (GPU) scattered into per-(group, window) rows,
    reduced on the device down to <= 32 rows each (``multi_exp_grouped_finish``
    ends on the host)."""
    digit_sc = torch.zeros((bk.size, 8), dtype=torch.int32)
    digit_sc[:, 0] = torch.from_numpy((bk & ((1 << c) - 1)).astype("int32"))
    bkp = gt_pow(cur, _upload(digit_sc.numpy(), dev))
    D = 1 << c
    g, w, d = bk // (W * D), (bk >> c) % W, bk & (D - 1)
    slot = _upload(d * (n_groups * W) + g * W + w, dev)
    win = gt_one(dev).repeat(D * n_groups * W, 1)
    win[slot] = bkp
    win = win.view(D, n_groups * W, 96)
    if torch.device(dev).type == "cuda":  # 8-way device levels down to <= 32 rows per (group, window)
        while win.shape[0] > 32:
            win = _gt_prod_level(win, 8)
    h["win"] = win
    h["G"] = n_groups


def multi_exp_grouped_finish(h) -> torch.Tensor:
    """[G, 96] host results: per-window products and the Horner steps on the host."""
    G, W = h["G"], h["W"]
    if h["win"] is None:
        return gt_one("cpu").repeat(G, 1)
    S_w = gt_prod(h["win"].cpu(), chunk=64).view(G, W, 96)  # host: one chain per (group, window)
    acc = S_w[:, W - 1].contiguous()
    sh = _pow2_scalar(h.get("c", _ME_C)).expand(G, 8).contiguous()
    for w in range(W - 2, -1, -1):
        acc = gt_mul(gt_pow(acc, sh), S_w[:, w].contiguous())
    return acc


# ----------------------------------------------------------------------------- device-resident bucket plans
# The bucket plans above take ONE host sync each (the per-bucket counts decide
# the slice passes).  A device-resident plan fixes its layout from the plan's
# SHAPE instead: every bucket owns a number of lanes set by its window's
# expected run (uniform digits: the batch weights are uniform), each lane
# takes an equal share of the bucket's actual run (csrc/kernels/dx_plan.hip
# dx_lane_slices), the multi-lane buckets reduce by a fixed tree and the
# bucket weighting runs over a fixed set of buckets.  Nothing goes through the
# host, so every pass is queued at once behind the sort.

_DPLANS: dict = {}
_PLAN_LIMIT = 32


def _layout_tensors(lay: dict):
    for k, v in lay.items():
        if isinstance(v, torch.Tensor):
            yield v
        elif k == "passes":
            for st, ln in v:
                yield st
                yield ln


def _mark_use(lay: dict, dev):
    """A cached layout is read by kernels of whatever stream the caller is on;
    its tensors were allocated on the stream that built it.  Every new user
    stream is recorded on them (``record_stream``), so when the cache evicts
    the layout the caching allocator hands its blocks out again only after
    every such stream has passed its last use -- without this an eviction
    while another stream's kernels still read the layout let the building
    stream reuse the memory under them (profiles/r6/graph_fault.md).  A HIP
    graph being captured keeps the layout itself (``capture_keep``): a
    captured launch reads it at every replay, long after any eviction."""
    keep = getattr(_CAPTURE, "keep", None)
    if keep is not None:
        keep.append(lay)
    if dev.type != "cuda":
        return
    s = torch.cuda.current_stream(dev)
    seen = lay.setdefault("_streams", set())
    if s.stream_id not in seen:
        seen.add(s.stream_id)
        for t in _layout_tensors(lay):
            t.record_stream(s)


_CAPTURE = threading.local()


class capture_keep:
    """Inside a HIP graph capture on this thread: collects every cached device
    object the captured launches read (``_mark_use``) into ``self.items``;
    the graph must hold them for its lifetime."""

    def __enter__(self):
        self.prev = getattr(_CAPTURE, "keep", None)
        self.items = []
        _CAPTURE.keep = self.items
        return self

    def __exit__(self, *a):
        _CAPTURE.keep = self.prev
        return False


def _device_layout(groups: tuple, W: int, c: int, sl: int, dev) -> dict:
    """Static layout of a device-resident plan (cached per shape).
    ``groups`` = ((entries, scalar bits), ...) per group.  Window w of a group
    with b = min(c, bits - w c) > 0 bits uses the buckets of digits 1 .. 2^b - 1,
    each with ceil(entries / (2^b sl)) lanes; every other bucket keeps one lane
    and must stay empty (``overflow`` counts entries that land there)."""
    dev = torch.device(dev)
    key = (groups, W, c, sl, str(dev))
    lay = _DPLANS.get(key)
    if lay is not None:
        _mark_use(lay, dev)
        return lay
    D = 1 << c
    nb = len(groups) * W * D
    lanes = np.ones(nb, dtype=np.int64)
    used = np.zeros(nb, dtype=bool)
    for g, (rows, bits) in enumerate(groups):
        for w in range(W):
            bw = min(c, int(bits) - w * c)
            if bw <= 0:
                continue
            base, hi = (g * W + w) * D, 1 << bw
            used[base + 1: base + hi] = True
            lanes[base + 1: base + hi] = max(1, -(-int(rows) // (hi * sl)))
    off = np.cumsum(lanes) - lanes
    L = int(lanes.sum())
    lane_bucket = np.repeat(np.arange(nb), lanes)
    lane_j = np.arange(L) - off[lane_bucket]
    multi = np.flatnonzero(lanes > 1)
    passes = []
    if multi.size:
        # first level over the multi-lane buckets' lanes (in place in the lane
        # array), then the usual segmented passes over the compacted results
        c_ = lanes[multi]
        n_sl = -(-c_ // _ME_SLICE)
        b = np.repeat(np.arange(multi.size), n_sl)
        k = np.arange(b.size) - (np.cumsum(n_sl) - n_sl)[b]
        passes.append((off[multi][b] + k * _ME_SLICE, np.minimum(c_[b] - k * _ME_SLICE, _ME_SLICE)))
        passes += _segment_passes(n_sl)
    up = lambda a, dt: _upload(np.asarray(a).astype(dt), dev)  # noqa: E731
    ubk = np.flatnonzero(used)
    lay = {"nb": nb, "n_lanes": L, "W": W, "c": c, "used": ubk,
           "lane_bucket": up(lane_bucket, np.int32), "lane_j": up(lane_j, np.int32), "lanes": up(lanes, np.int32),
           "first_lane": up(off, np.int64), "multi": up(multi, np.int64),
           "passes": [(up(st, np.int64), up(ln, np.int32)) for st, ln in passes],
           "used_t": up(ubk, np.int64), "unused_t": up(np.flatnonzero(~used), np.int64)}
    if dev.type == "cuda":  # uploaded on this stream; readers on others must not see it half-copied
        torch.cuda.current_stream(dev).synchronize()
    while len(_DPLANS) > _PLAN_LIMIT:  # least recently built first (see ``_mark_use`` for why that is safe)
        _DPLANS.pop(next(iter(_DPLANS)))
    _DPLANS[key] = lay
    _mark_use(lay, dev)
    return lay


def _device_runs(k: torch.Tensor, group, n_groups: int, W: int, c: int):
    """Bucket keys of every (entry, window) and their runs in key order, on
    the device: (items sorted by key, first[nb], end[nb])."""
    dev = k.device
    n = k.shape[0]
    nb = (W << c) * n_groups
    assert n * W < 2 ** 31 and nb < 2 ** 31 - 1
    keys = torch.empty(n * W, dtype=torch.int32, device=dev)
    items = torch.empty(n * W, dtype=torch.int32, device=dev)
    grp, gstride = _group_arg(group, n, dev)
    g, s = _ctx(k, keys)
    _call("dx_msm_keys", g, s, _ptr(k.contiguous()), _ptr(grp), gstride, n, c, W, _ptr(keys), _ptr(items))
    return _sorted_runs(keys, items, nb)


def _device_slices(first: torch.Tensor, end: torch.Tensor, lay: dict):
    L = lay["n_lanes"]
    st = torch.empty(L, dtype=torch.int64, device=first.device)
    ln = torch.empty(L, dtype=torch.int32, device=first.device)
    g, s = _ctx(first, st)
    _call("dx_lane_slices", g, s, _ptr(first), _ptr(end), _ptr(lay["lane_bucket"]), _ptr(lay["lane_j"]),
          _ptr(lay["lanes"]), L, _ptr(st), _ptr(ln))
    return st, ln


def _device_reduce(part: torch.Tensor, lay: dict, slice_op) -> torch.Tensor:
    """Per-lane partials -> one value per USED bucket (``lay["used"]`` order)."""
    B = part.index_select(0, lay["first_lane"])
    if lay["passes"]:
        cur = None
        for i, (st, ln) in enumerate(lay["passes"]):
            cur = slice_op(part if i == 0 else cur, st, ln)
        B.index_copy_(0, lay["multi"], cur)
    return B.index_select(0, lay["used_t"])


def _overflow(first, end, lay) -> torch.Tensor:
    """Entries in buckets outside the layout (scalars wider than declared): a device scalar."""
    return (end - first).index_select(0, lay["unused_t"]).sum()


def check_overflow(h: dict):
    """Raise if a device-resident plan dropped entries (checked once the
    results are read back, so it costs no extra host sync)."""
    ov = h.get("overflow")
    if ov is not None and int(ov) != 0:
        raise RuntimeError(f"device bucket plan: {int(ov)} entries fell outside the declared scalar widths")


def gt_chunk_weight(B: torch.Tensor, d: torch.Tensor, start: torch.Tensor, length: torch.Tensor,
                    base: torch.Tensor) -> torch.Tensor:
    """out[ch] = prod_{i in chunk ch} B[i]^d[i] over digit-sorted GT buckets
    (chunk: start/length rows whose digits lie in [base, base + L)) -- running
    products instead of one power per bucket."""
    n = start.numel()
    out = torch.empty((n, 96), dtype=torch.int32, device=B.device)
    g, s = _ctx(B, d, start, length, base)
    _call("dx_gt_chunk_weight", g, s, _ptr(B.contiguous()), _ptr(d.contiguous()), _ptr(start), _ptr(length),
          _ptr(base), _ptr(out), n)
    return out


def me_window(groups: tuple, lo: int = 8, hi: int = 16) -> tuple:
    """(W, c) of a GT multi-exponentiation over ``groups`` = ((entries,
    exponent bits), ...): c minimises the bucket products (entries x windows)
    plus ~3 products per bucket for the running-product weights -> 16-bit
    windows for a whole 1-GPU inbox (2 windows per 32-bit GLV half instead of
    3), 11 bits for a pool slice."""
    def cost(c):
        return sum(r * -(-b // c) for r, b in groups) + 3 * sum(-(-b // c) for _, b in groups) * (1 << c)
    c = min(range(lo, hi + 1), key=cost)
    return max(-(-b // c) for _, b in groups), c


def multi_exp_device(a: torch.Tensor, k: torch.Tensor, group, groups: tuple, W: int | None = None,
                     c: int | None = None, item_split: tuple | None = None) -> dict:
    """``multi_exp_grouped`` with a device-resident plan (no host sync):
    ``groups`` = ((entries, exponent bits), ...) per group (window from
    ``me_window`` unless given).  -> the handle of ``multi_exp_grouped_finish``."""
    dev = a.device
    n = a.shape[0]
    G = len(groups)
    if c is None:
        W, c = me_window(tuple(groups))
    items, first, end = _device_runs(k, group, G, W, c)
    it = items.to(torch.int64)
    if item_split is not None:
        sp, q = item_split
        it = torch.where(it < sp, it % n, (it - sp) % q)
    else:
        it = it % n
    lay = _device_layout(tuple(groups), W, c, _ME_SLICE, dev)
    st, ln = _device_slices(first, end, lay)
    part = gt_slice_prod(a, it.contiguous(), st, ln)
    B = _device_reduce(part, lay, lambda src, s_, l_: gt_slice_prod(src, None, s_, l_))
    h = {"G": G, "W": W, "c": c, "win": None, "overflow": _overflow(first, end, lay)}
    if "gtw" not in lay:
        lay["gtw"] = _g2_weight_plan(lay["used"], c, dev)
    wp = lay["gtw"]
    cur = gt_chunk_weight(B, wp["d"], *wp["chunks"])                     # running products per chunk
    for st, ln in wp["gpasses"]:
        cur = gt_slice_prod(cur, None, st, ln)                            # chunks -> (group, window)
    win = gt_one(dev).repeat(G * W, 1)
    win.index_copy_(0, wp["gws"], cur)
    h["win"] = win.view(1, G * W, 96)
    return h


def g2_msm_device(P_aff: torch.Tensor, k: torch.Tensor, group, groups: tuple, c: int = 13,
                  bits: int = 254) -> tuple:
    """``g2_msm_launch`` + ``g2_msm_run`` with a device-resident plan (no host
    sync): out[g] = sum_{t: group_t = g} k_t P[t % m] -> ([G * W, 48] window
    sums, handle for ``g2_msm_finish``)."""
    dev = P_aff.device
    m = _rows(P_aff, 32)
    G = len(groups)
    W = -(-bits // c)
    items, first, end = _device_runs(k, group, G, W, c)
    lay = _device_layout(tuple(groups), W, c, 32, dev)
    st, ln = _device_slices(first, end, lay)
    part = g2_slice_sum(P_aff, items, st, ln, True, m)
    B = _device_reduce(part, lay, lambda src, s_, l_: g2_slice_sum(src, None, s_, l_, False))
    if "g2w" not in lay:
        lay["g2w"] = _g2_weight_plan(lay["used"], c, dev)
    S = torch.zeros((G * W, 48), dtype=torch.int32, device=dev)
    _g2_weigh(B, lay["g2w"], S)
    return S, {"G": G, "W": W, "c": c, "overflow": _overflow(first, end, lay)}


def g1_msm_device(P_jac: torch.Tensor, k: torch.Tensor, group, groups: tuple, bits: int = 256) -> dict:
    """``g1_msm_launch`` with a device-resident plan (8-bit windows, no host
    sync) -> the handle of ``g1_msm_finish``."""
    dev = P_jac.device
    G = len(groups)
    W = (bits + 7) // 8
    items, first, end = _device_runs(k, group, G, W, 8)
    lay = _device_layout(tuple(groups), W, 8, _ME_SLICE, dev)
    st, ln = _device_slices(first, end, lay)
    part = g1_slice_sum(P_jac.contiguous(), items.to(torch.int64), st, ln)
    B = _device_reduce(part, lay, lambda src, s_, l_: g1_slice_sum(src, None, s_, l_))
    h = {"n_groups": G, "W": W, "S_w": None, "overflow": _overflow(first, end, lay)}
    if "g1w" not in lay:
        bk = lay["used"]
        sc = np.zeros((bk.size, 8), dtype=np.int32)
        sc[:, 0] = bk % 256
        gws, counts = np.unique(bk // 256, return_counts=True)
        lay["g1w"] = (_upload(sc, dev), [(_upload(st_, dev), _upload(ln_.astype("int32"), dev))
                                         for st_, ln_ in _segment_passes(counts)], gws)
    sc, wpasses, gws = lay["g1w"]
    cur = g1_mul(B, sc)                                                  # d * B_{g,w,d}
    for st_, ln_ in wpasses:
        cur = g1_slice_sum(cur, None, st_, ln_)
    h["S_w"], h["gws"] = cur, gws
    return h


def g1_slice_sum(src: torch.Tensor, idx, start: torch.Tensor, length: torch.Tensor) -> torch.Tensor:
    """out[s] = sum_k src[idx[start[s] + k]] (or src[start[s] + k]), k < length[s] (Jacobian)."""
    n = start.numel()
    out = torch.empty((n, 24), dtype=torch.int32, device=src.device)
    g, s = _ctx(src, idx, start, length)
    _call("dx_g1_slice_sum", g, s, _ptr(src), _ptr(idx), _ptr(start), _ptr(length), _ptr(out), n)
    return out


def g1_msm(P_jac: torch.Tensor, k: torch.Tensor, bits: int = 256) -> torch.Tensor:
    """sum_i k_i P_i (Pippenger bucket method, 8-bit windows) -> [1, 24] HOST
    Jacobian point.  Buckets accumulate in wide segmented passes on the device
    (no per-point 256-step doubling chain: the cost is ~bits/8 additions per
    point), bucket weights d*B_{w,d} are one short variable-base launch, and
    the 32-window Horner combination runs on the host pool."""
    return g1_msm_grouped(P_jac, k, None, 1, bits)


def g1_msm_grouped(P_jac: torch.Tensor, k: torch.Tensor, group: torch.Tensor | None, n_groups: int,
                   bits: int = 256) -> torch.Tensor:
    """G independent MSMs in one bucket pass: out[g] = sum_{i: group_i = g}
    k_i P_i -> [n_groups, 24] HOST Jacobian points.  Only non-zero 8-bit
    digits enter a bucket, so a 64-bit weight costs 8 bucket additions, not
    32: batch verifiers keep the short random weights in their own group and
    apply the shared full-size factor (a challenge) to the group's sum on the
    host, instead of multiplying it into every per-element scalar."""
    return g1_msm_finish(g1_msm_launch(P_jac, k, group, n_groups, bits))


def g1_msm_plan(k: torch.Tensor, group, n_groups: int, bits: int = 256):
    """The bucket plan of ``g1_msm_launch`` alone (its one host sync), so a
    caller can take every plan's sync before queueing any heavy pass."""
    if not k.shape[0]:
        return None
    return _bucket_plan(k, (bits + 7) // 8, group, n_groups)


def g1_msm_launch(P_jac: torch.Tensor, k: torch.Tensor, group: torch.Tensor | None, n_groups: int,
                  bits: int = 256, plan: dict | None = None) -> dict:
    """First half of g1_msm_grouped: the bucket plan (one host sync on k,
    unless ``plan`` comes from ``g1_msm_plan``) and every device pass, queued
    on the current stream.  g1_msm_finish waits for them and runs the Horner
    steps on the host."""
    assert P_jac.shape[0] == k.shape[0]
    assert group is None or isinstance(group, int) or group.numel() == k.shape[0]
    dev = P_jac.device
    W = (bits + 7) // 8
    h = {"n_groups": n_groups, "W": W, "S_w": None}
    if P_jac.shape[0] == 0:
        return h
    if plan is None:
        plan = _bucket_plan(k, W, group, n_groups)
    bk = plan["bk"]
    if bk.size == 0:
        return h
    P_jac = P_jac.contiguous()
    cur = P_jac.index_select(0, plan["item"]).contiguous() if plan["single"] else None
    for i, (st, ln) in enumerate(plan["passes"]):
        cur = g1_slice_sum(P_jac if i == 0 else cur, plan["item"] if i == 0 else None, st, ln)
    _g1_windows(h, cur, bk, dev)
    return h


def _g1_windows(h: dict, cur, bk, dev):
    """Bucket sums -> d * B_{g,w,d} (one short variable-base launch) ->
    per-(group, window) sums on the device (``g1_msm_finish`` ends on the host)."""
    sc = torch.zeros((bk.size, 8), dtype=torch.int32)
    sc[:, 0] = torch.from_numpy((bk % 256).astype("int32"))
    weighted = g1_mul(cur, _upload(sc.numpy(), dev))                     # d * B_{g,w,d}
    # per-(group, window) sums: buckets are sorted by key = (g*W + w)*256 + d,
    # so each (group, window) is a contiguous run
    gws, counts = np.unique(bk // 256, return_counts=True)
    cur = weighted
    for st, ln in _segment_passes(counts):
        cur = g1_slice_sum(cur, None, _upload(st, dev), _upload(ln.astype("int32"), dev))
    h["S_w"], h["gws"] = cur, gws


def g1_msm_finish(h: dict) -> torch.Tensor:
    from ..crypto.bn254 import g1_infinity_jac

    out = g1_infinity_jac(h["n_groups"], "cpu")
    if h["S_w"] is None:
        return out
    W, gws = h["W"], h["gws"]
    S_w = h["S_w"].cpu()                                                 # [len(gws), 24]
    G = h["n_groups"]
    # Horner over the windows, all groups at once: acc = 2^8 acc + S_{g,w}.
    # ~8 doublings per window and group, instead of one up-to-248-doubling
    # multiplication 2^{8w} S_{g,w} per (group, window)
    rows = g1_infinity_jac(G * W, "cpu")
    rows[torch.from_numpy(gws.astype(np.int64))] = S_w
    rows = rows.view(G, W, 24)
    top = int((gws % W).max())
    out = torch.empty((G, 24), dtype=torch.int32)
    src = rows[:, : top + 1].contiguous()  # held: the host call reads it
    rc = _raw_call("dx_g1_horner_host", _ptr(src), _ptr(out), G, top + 1, 8)
    if rc:
        raise RuntimeError(f"dx_g1_horner_host failed rc={rc}")
    return out


# ----------------------------------------------------------------------------- G2 MSM (verifier mode "msm")
# csrc/kernels/dx_rpmsm.hip: range-proof batch verification by bilinearity
G2_JOINT_ENTRIES = 15


def g2_joint_table(V_aff: torch.Tensor) -> torch.Tensor:
    """Per V: the 15 affine points da V + db [lambda] V ((da, db) in [0, 3]^2,
    not both 0) -> [m * 15, 32]; the U-combination kernel's window table."""
    m = _rows(V_aff, 32)
    out = torch.empty((m * G2_JOINT_ENTRIES, 32), dtype=torch.int32, device=V_aff.device)
    g, s = _ctx(V_aff)
    _call("dx_g2_joint_table", g, s, _ptr(V_aff.contiguous()), _ptr(out), m)
    return out


def rp_u_joint(table: torch.Tensor, ab: torch.Tensor, n_groups: int, G: int, L: int, out: torch.Tensor,
               pad: int, pos: torch.Tensor | None = None) -> torch.Tensor:
    """out[v*pad + q] = affine(sum_j (a + b lambda)_{v, q*L+j} V_{q*L+j}) for every
    verifier v < G and group q < n_groups (ab [G * n_groups * L, 2] int32);
    ``pos`` (int64 [G * n_groups], rows of ``out``): the row of (v, q) instead."""
    assert _rows(table, 32) == n_groups * L * G2_JOINT_ENTRIES and _rows(ab, 2) == G * n_groups * L
    assert out.is_contiguous() and pad >= n_groups
    if pos is None:
        assert _rows(out, 32) >= (G - 1) * pad + n_groups
    else:
        assert pos.dtype == torch.int64 and pos.numel() == G * n_groups and pos.device == out.device
    g, s = _ctx(table, ab, out)
    # a small batch (a pool helper's 1/W slice) splits each combination over
    # 2 or 4 threads so the launch still fills the chip (~2 waves per SIMD)
    n = G * n_groups
    sp = 1 if (not g or n >= 131072) else (2 if n >= 65536 else 4)
    sp = min(sp, L)
    if sp > 1:
        tmp = torch.empty((n * sp, 48), dtype=torch.int32, device=out.device)
        _call("dx_rp_u_joint_split", g, s, _ptr(table), _ptr(ab.contiguous()), _ptr(out), n_groups, G, L, pad, sp,
              _ptr(tmp), _ptr(pos))
        return out
    _call("dx_rp_u_joint", g, s, _ptr(table), _ptr(ab.contiguous()), _ptr(out), n_groups, G, L, pad, _ptr(pos))
    return out


def g2_slice_sum(src: torch.Tensor, idx, start: torch.Tensor, length: torch.Tensor, src_aff: bool,
                 idx_mod: int = 0) -> torch.Tensor:
    """out[s] = sum_k src[idx[start[s] + k] % idx_mod] (or src[start[s] + k]),
    k < length[s], from affine (mixed additions) or Jacobian G2 rows -> Jacobian [n, 48]."""
    n = start.numel()
    assert src.shape[-1] == (32 if src_aff else 48) and (idx is None or idx.dtype == torch.int32)
    assert start.dtype == torch.int64 and length.dtype == torch.int32
    out = torch.empty((n, 48), dtype=torch.int32, device=src.device)
    g, s = _ctx(src, idx, start, length)
    _call("dx_g2_slice_sum", g, s, _ptr(src), _ptr(idx), _ptr(start), _ptr(length), _ptr(out), n, int(src_aff),
          int(idx_mod))
    return out


G2_CHUNK = 32  # digit range of one running-sum chunk of Pippenger buckets


def g2_chunk_weight(B_jac: torch.Tensor, d: torch.Tensor, start: torch.Tensor, length: torch.Tensor,
                    base: torch.Tensor) -> torch.Tensor:
    """out[ch] = sum_{i in chunk ch} d[i] B[i] over digit-sorted Jacobian
    buckets (chunk: start/length rows whose digits lie in [base, base +
    G2_CHUNK)) -- running sums instead of one multiplication per bucket."""
    n = start.numel()
    assert B_jac.shape[-1] == 48 and d.dtype == torch.int32 and start.dtype == torch.int64
    assert length.dtype == torch.int32 and base.dtype == torch.int32 and base.numel() == n
    out = torch.empty((n, 48), dtype=torch.int32, device=B_jac.device)
    g, s = _ctx(B_jac, d, start, length, base)
    _call("dx_g2_chunk_weight", g, s, _ptr(B_jac.contiguous()), _ptr(d.contiguous()), _ptr(start), _ptr(length),
          _ptr(base), _ptr(out), n)
    return out


def g2_mul_small(jac: torch.Tensor, d: torch.Tensor) -> torch.Tensor:
    """d[i] * jac[i] (Jacobian G2, 0 <= d < 2^31)."""
    n = _rows(jac, 48)
    assert d.dtype == torch.int32 and d.numel() == n
    out = torch.empty_like(jac)
    g, s = _ctx(jac, d)
    _call("dx_g2_mul_small", g, s, _ptr(jac.contiguous()), _ptr(d.contiguous()), _ptr(out), n)
    return out


def g2_msm_launch(P_aff: torch.Tensor, k: torch.Tensor, group: torch.Tensor | None, n_groups: int,
                  c: int = 13, bits: int = 254, first_slice: int = 32):
    """Bucket plan of G independent G2 MSMs out[g] = sum_{t: group_t = g}
    k_t P[t % m] (m = rows of P_aff, k [n, 8] with n a multiple of m; group:
    int32 tensor, or an int stride s meaning group_t = t // s):
    c-bit windows; int32 keys (g, w, d) built by one kernel (zero digits get
    a sentinel that sorts last), one radix sort over the keys' bits
    (csrc/kernels/dx_plan.hip), per-bucket runs by their boundaries -- ONE
    host sync (the counts).  ``g2_msm_run`` queues the device passes."""
    dev = P_aff.device
    n, m = k.shape[0], _rows(P_aff, 32)
    W = -(-bits // c)
    nb = (W << c) * n_groups
    assert n % m == 0 and n < 2 ** 31 and nb < 2 ** 31 - 1
    keys = torch.empty(n * W, dtype=torch.int32, device=dev)
    items = torch.empty(n * W, dtype=torch.int32, device=dev)
    grp, gstride = _group_arg(group, n, dev)
    g, s = _ctx(k, keys)
    _call("dx_msm_keys", g, s, _ptr(k.contiguous()), _ptr(grp), gstride, n, c, W, _ptr(keys), _ptr(items))
    items, counts = _sort_buckets(keys, items, nb)             # the one host sync
    bk = np.flatnonzero(counts)
    h = {"G": n_groups, "W": W, "c": c, "m": m, "bk": bk, "item": items[: int(counts.sum())]}
    if bk.size:
        passes = _segment_passes_dev(counts[bk], dev, first_slice)
        if not passes:  # every bucket holds one entry
            passes = [(torch.arange(bk.size, device=dev), torch.ones(bk.size, dtype=torch.int32, device=dev))]
        h["passes"] = passes
        h.update(_g2_weight_plan(bk, c, dev))
    return h


def _g2_chunk(n_buckets: int) -> int:
    """Digit range of a bucket-weight chunk: 32 (about two additions per
    bucket) while that still gives ~16k chunk lanes, shorter for a small
    plan (a 1/8 pool slice: 8, i.e. 4x the lanes with a third of the chain)."""
    ch = G2_CHUNK
    while ch > 4 and n_buckets // ch < 16384:
        ch //= 2
    return ch


def _g2_weight_plan(bk, c: int, dev) -> dict:
    """Bucket weights by running sums (G2) / running products (GT) over
    chunks of an aligned digit range (csrc/kernels/dx_rpmsm.hip
    chunk_weight_one, dx_range.hip gt_chunk_weight_coop), then per-window
    sums of the chunk results, for the sorted bucket keys ``bk``."""
    chunk = _g2_chunk(bk.size)
    dig = bk & ((1 << c) - 1)
    gw = bk >> c
    ck = gw * ((1 << c) // chunk + 1) + dig // chunk
    first = np.flatnonzero(np.r_[True, ck[1:] != ck[:-1]])
    clen = np.diff(np.r_[first, bk.size])
    gwf = gw[first]                                  # sorted: run lengths instead of np.unique's sort
    gstart = np.flatnonzero(np.r_[True, gwf[1:] != gwf[:-1]])
    gws, gcounts = gwf[gstart], np.diff(np.r_[gstart, gwf.size])
    return {"d": _upload(dig.astype("int32"), dev),
            "chunks": (_upload(first.astype(np.int64), dev), _upload(clen.astype(np.int32), dev),
                       _upload(((dig[first] // chunk) * chunk).astype(np.int32), dev)),
            "gws": _upload(gws.astype(np.int64), dev), "gpasses": _segment_passes_dev(gcounts, dev)}


def _g2_weigh(cur, wp: dict, S: torch.Tensor) -> torch.Tensor:
    cur = g2_chunk_weight(cur, wp["d"], *wp["chunks"])
    for st, ln in wp["gpasses"]:
        cur = g2_slice_sum(cur, None, st, ln, False)
    S.index_copy_(0, wp["gws"], cur)
    return S


def g2_msm_run(P_aff: torch.Tensor, h: dict) -> torch.Tensor:
    """Device passes of a ``g2_msm_launch`` plan, queued on the current stream:
    bucket sums, weights d B_d, per-(group, window) sums -> [G * W, 48]
    Jacobian window sums (``g2_msm_finish`` combines them)."""
    G, W = h["G"], h["W"]
    S = torch.zeros((G * W, 48), dtype=torch.int32, device=P_aff.device)   # Jacobian infinity = Z 0
    if h["bk"].size:
        cur = None
        for i, (st, ln) in enumerate(h["passes"]):
            cur = g2_slice_sum(P_aff if i == 0 else cur, h["item"] if i == 0 else None, st, ln, i == 0,
                               h["m"] if i == 0 else 0)
        _g2_weigh(cur, h, S)
    return S


def g2_msm_finish(S: torch.Tensor, h: dict, out_aff: torch.Tensor | None = None, stride: int = 1,
                  offset: int = 0) -> torch.Tensor:
    """Horner over the windows, one lane per group (W*c doublings), on the
    tensor's device: out_aff[g * stride + offset] = affine(out[g]).  On the
    host (CPU tensors) a core runs this serial chain ~5x faster than one GPU lane."""
    G, W, c = h["G"], h["W"], h["c"]
    if out_aff is None:
        out_aff = torch.zeros((G, 32), dtype=torch.int32, device=S.device)
    g, s = _ctx(S, out_aff)
    _call("dx_g2_horner", g, s, _ptr(S.contiguous()), _ptr(out_aff), G, W, c, stride, offset)
    return out_aff


def rp_msm_uv(Y_jac: torch.Tensor, UV: torch.Tensor, n_groups: int, G: int, pad: int) -> torch.Tensor:
    """UV[v*pad + q] = (x/y, 1/y) of -Y_q (q < n_groups) and of B (q = n_groups)."""
    assert _rows(Y_jac, 24) == n_groups and _rows(UV, 16) >= (G - 1) * pad + n_groups + 1 and pad > n_groups
    g, s = _ctx(Y_jac, UV)
    _call("dx_rp_msm_uv", g, s, _ptr(Y_jac.contiguous()), _ptr(UV), n_groups, G, pad)
    return UV


_gt_one_cache: dict = {}


def gt_one(device) -> torch.Tensor:
    """Fp12 one (Montgomery limbs: c0.c0.c0 = R mod p)."""
    key = str(device)
    if key not in _gt_one_cache:
        import numpy as _np

        from ..crypto import bn254 as _bn

        t = _np.zeros((1, 96), dtype=_np.uint32)
        t[0, :8] = _bn.ints_to_limbs([_bn.mont(1)])[0]
        _gt_one_cache[key] = _bn.publish(_bn.to_tensor(t, device))
    return _gt_one_cache[key]


def _pow2_scalar(c: int) -> torch.Tensor:
    t = torch.zeros((1, 8), dtype=torch.int32)
    t[0, c // 32] = 1 << (c % 32)
    return t


def _finish_prod_on_host(parts: torch.Tensor) -> torch.Tensor:
    """Product of [n, 96] GT partials: 8-way GPU levels while n > 256, then the
    rest on the host pool (a lone GPU lane runs an Fp12 chain latency-bound,
    ~30x slower than one host core).  Returns a [1, 96] HOST tensor."""
    cur = parts.view(-1, 1, 96)
    while cur.shape[0] > 256:
        cur = _gt_prod_level(cur, 8)
    return gt_prod(cur.cpu(), chunk=4).view(1, 96)


def _gt_prod_level(x: torch.Tensor, ch: int) -> torch.Tensor:
    n_items, n_groups = x.shape[0], x.shape[1]
    n_chunks = (n_items + ch - 1) // ch
    out = torch.empty((n_chunks, n_groups, 96), dtype=torch.int32, device=x.device)
    g, s = _ctx(x)
    _call("dx_gt_prod_chunks", g, s, _ptr(x.contiguous()), _ptr(out), n_items, n_groups, ch)
    return out
