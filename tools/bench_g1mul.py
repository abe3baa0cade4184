"""Latency of native.g1_mul (GLV 128-step kernel vs the window-3 256-step one)
at the sizes the protocol uses (decryption / key switching ~2k-12k rows,
range-proof challenges larger).  Prints one line per (n, kernel)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from drynx_amd import native as nt  # noqa: E402
from drynx_amd.crypto import bn254 as bn  # noqa: E402


def main():
    dev = "cuda"
    for n in (2112, 12480, 65536, 262144):
        P = nt.g1_fb_mul(bn.base_table(dev), bn.random_scalars(n, dev))
        K = bn.random_scalars(n, dev)
        for glv in (True, False):
            nt.G1_MUL_GLV = glv
            nt.g1_mul(P, K)
            torch.cuda.synchronize()
            reps = 5
            t0 = time.perf_counter()
            for _ in range(reps):
                nt.g1_mul(P, K)
            torch.cuda.synchronize()
            print(f"n={n:7d} {'glv ' if glv else 'win3'} {(time.perf_counter() - t0) / reps * 1e3:8.3f} ms", flush=True)
    nt.G1_MUL_GLV = True


if __name__ == "__main__":
    main()
