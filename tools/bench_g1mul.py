"""Latency of native.g1_mul (GLV kernel, csrc/kernels/dx_g1_varmul.hip) in
its two-lanes-per-row and one-lane-per-row forms at the sizes the protocol
uses (decryption / key switching ~2k-12k rows, range-proof challenges more).
Sets ``native.G1_MUL_PAIR_ROWS`` to force each form; one line per (n, form)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from drynx_amd import native as nt  # noqa: E402
from drynx_amd.crypto import bn254 as bn  # noqa: E402


def main():
    dev = "cuda"
    keep = nt.G1_MUL_PAIR_ROWS
    for n in (2112, 12480, 32768, 65536, 131072, 262144):
        P = nt.g1_fb_mul(bn.base_table(dev), bn.random_scalars(n, dev))
        K = bn.random_scalars(n, dev)
        res = {}
        for pair in (True, False):
            nt.G1_MUL_PAIR_ROWS = n if pair else 0
            res[pair] = nt.g1_mul(P, K)
            torch.cuda.synchronize()
            reps = 5
            t0 = time.perf_counter()
            for _ in range(reps):
                nt.g1_mul(P, K)
            torch.cuda.synchronize()
            print(f"n={n:7d} {'pair  ' if pair else 'single'} {(time.perf_counter() - t0) / reps * 1e3:8.3f} ms",
                  flush=True)
        assert bool(nt.g1_eq(res[True], res[False]).all())
    nt.G1_MUL_PAIR_ROWS = keep


if __name__ == "__main__":
    main()
