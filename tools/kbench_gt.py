#!/usr/bin/env python3
"""Microbenchmark: GT product chains (the verifier multi-exponentiation's
bucket accumulation) -- dx_gt_slice_prod vs the latency-hidden dx_gt_chain.
Shapes of one headline query: ~3.4M gathered Fp12 factors in slices of <= 8
from a 2M-row array (1M a_ij and their Frobenius images)."""
import json
import sys
import time

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from drynx_amd import native as nt  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    rows, total, sl = 2_000_000, 3_400_000, 8
    src = torch.randint(0, 1 << 30, (rows, 96), generator=g, device=dev, dtype=torch.int32)
    idx = torch.randint(0, rows, (total,), generator=g, device=dev, dtype=torch.int64)
    n = total // sl
    start = torch.arange(n, device=dev, dtype=torch.int64) * sl
    length = torch.full((n,), sl, device=dev, dtype=torch.int32)
    out = {}
    for name, chain in (("slice_prod", False), ("chain", True), ("slice_prod", False), ("chain", True)):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(3):
            r = nt.gt_slice_prod(src, idx, start, length, chain=chain)
        torch.cuda.synchronize()
        out.setdefault(name, []).append(round((time.perf_counter() - t) / 3 * 1e3, 2))
        out[name + "_res"] = r
    same = bool(torch.equal(out.pop("slice_prod_res"), out.pop("chain_res")))
    print(json.dumps({"ms": out, "equal": same, "slices": n, "factors": total}))


if __name__ == "__main__":
    main()
