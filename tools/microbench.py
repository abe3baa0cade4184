"""Kernel throughput microbenchmarks (GPU): items/s for the hot BN254 kernels."""
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from drynx_amd import native as nt  # noqa: E402
from drynx_amd.crypto import bn254 as bn  # noqa: E402
from drynx_amd.crypto import oracle as O  # noqa: E402


def tm(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    return best


def main():
    dev = torch.device("cuda", 0)
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    res = {}
    n = 1 << 20
    k = bn.random_scalars(n, dev)
    tab = bn.base_table(dev)
    res["g1_fb_mul_per_s"] = n / tm(lambda: nt.g1_fb_mul(tab, k))
    J = bn.g1_jac_tensor([O.g1_mul(7, O.G1_GEN)], dev)
    m = 1 << 17
    res["g1_var_mul_per_s"] = m / tm(lambda: nt.g1_mul(J, k[:m].contiguous()))
    m = 1 << 15 * scale
    Q = bn.g2_aff_tensor([O.G2_GEN], dev)
    res["g2_var_mul_per_s"] = m / tm(lambda: nt.g2_mul(Q, k[:m].contiguous()))
    P = nt.g1_to_affine(nt.g1_fb_mul(tab, k[:m].contiguous()))
    Qs = nt.g2_fb_mul(bn.base2_table(dev), k[:m].contiguous())
    res["miller_loop_per_s"] = m / tm(lambda: nt.miller_loop(P, Qs))
    f = nt.miller_loop(P, Qs)
    res["final_exp_per_s"] = m / tm(lambda: nt.final_exp(f))
    res["pairing_per_s"] = m / tm(lambda: nt.pairing(P, Qs))
    g = nt.final_exp(f)
    res["gt_pow256_per_s"] = m / tm(lambda: nt.gt_pow(g, k[:m].contiguous()))
    print(json.dumps({k_: round(v, 1) for k_, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
