#!/usr/bin/env python3
"""Microbenchmark + check of the range-verification Miller fold variants on
one GPU: the fused per-item kernel (dx_rp_verify_fold) vs the two-phase fold
(lines + K-item multi-Miller accumulation, out-of-line / inlined tower).
Prints one JSON line per variant with ms and Miller loops/s."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from drynx_amd import native as nt  # noqa: E402
from drynx_amd.crypto import bn254 as bn  # noqa: E402


VARIANTS = os.environ.get("FOLD_VARIANTS", "inl").split(",")


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best, out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 993_600
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    k1 = bn.random_scalars(n, dev)
    k2 = bn.random_scalars(n, dev)
    P = nt.g1_to_affine(nt.g1_fb_mul(bn.base_table(dev), k1))
    V = nt.g2_fb_mul(bn.base2_table(dev), k2)
    # reference value on a small prefix: FE(prod ML) via per-item Miller loops
    m = 4096
    ref = nt.final_exp(nt._finish_prod_on_host(nt.miller_loop(P[:m].contiguous(), V[:m].contiguous())))
    for v in VARIANTS:
        for K in (1, 2, 4, 8):
            fb = nt.rp_fold_accum(nt.rp_fold_lines(P[:m].contiguous(), V[:m].contiguous(), v), m, K, v)
            got = nt.final_exp(nt._finish_prod_on_host(fb))
            assert bool(nt.gt_eq(got, ref).all()), (v, K)
    print(json.dumps({"check": "ok", "items": m}), flush=True)
    # the fused kernel (with its own rho * (ZB - Y) point work): rho = 1, Y = 0
    ZB = nt.g1_from_affine(P)
    Y = bn.g1_infinity_jac(n, dev)
    rho = torch.zeros((n, 8), dtype=torch.int32, device=dev)
    rho[:, 0] = 1
    if os.environ.get("FOLD_FUSED", "0") == "1":
        t, _ = timed(lambda: nt.rp_verify_fold(ZB, Y, rho, V, 1, 1))
        print(json.dumps({"variant": "fused", "n": n, "ms": round(1e3 * t, 2), "ml_per_s": round(n / t)}), flush=True)
    for v in VARIANTS:
        tl, lines = timed(lambda: nt.rp_fold_lines(P, V, v))
        for K in (1, 2, 4, 8):
            ta, _ = timed(lambda: nt.rp_fold_accum(lines, n, K, v))
            print(json.dumps({"variant": v, "K": K, "n": n, "lines_ms": round(1e3 * tl, 2),
                              "accum_ms": round(1e3 * ta, 2),
                              "ml_per_s": round(n / (tl + ta))}), flush=True)
        del lines
        torch.cuda.empty_cache()
        # shared-V: one coefficient image, G verifiers' points evaluated in the accumulation
        G = int(os.environ.get("FOLD_G", "3"))
        tc, coef = timed(lambda: nt.rp_fold_coeffs(V, v))
        for K in (4, 8):
            per = 64 * K * nt.FOLD_P_ALIGN
            pad = -(-n // per) * per
            PG = torch.zeros((G * pad, 16), dtype=torch.int32, device=dev)
            for g in range(G):
                PG[g * pad: g * pad + n] = P
            ta, _ = timed(lambda: nt.rp_fold_accum_p(coef, PG, V, pad, G, K, v))
            print(json.dumps({"variant": v + "-sharedV", "G": G, "K": K, "n": n, "coeffs_ms": round(1e3 * tc, 2),
                              "accum_ms": round(1e3 * ta, 2), "ml_per_s": round(G * n / (tc + ta))}), flush=True)
            del PG
        del coef
        torch.cuda.empty_cache()
        # normalised lines (fold mode 4): (c1/c0, c3/c0) per V, (x/y, 1/y) per point
        tn, img = timed(lambda: nt.rp_fold_ncoeffs(V, v))
        for K in (4, 8):
            per = 64 * K * nt.FOLD_P_ALIGN
            pad = -(-n // per) * per
            UV = torch.zeros((G * pad, 16), dtype=torch.int32, device=dev)
            uv1 = nt.g1_aff_to_uv_(P.clone())
            for g in range(G):
                UV[g * pad: g * pad + n] = uv1
            ta, _ = timed(lambda: nt.rp_fold_accum_n(img, UV, V, pad, G, K, v))
            print(json.dumps({"variant": v + "-normalised", "G": G, "K": K, "n": n, "coeffs_ms": round(1e3 * tn, 2),
                              "accum_ms": round(1e3 * ta, 2), "ml_per_s": round(G * n / (tn + ta))}), flush=True)
            del UV
        del img
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
