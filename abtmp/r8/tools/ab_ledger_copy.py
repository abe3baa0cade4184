"""A/B diagnostic: what the ledger's device-to-host payload copy costs the
headline.  Runs bench.py's main with the node's ``_host_bytes`` replaced by
a producer that hands the ledger zero bytes of the same sizes from a
reused pinned buffer (no device-to-host copy, same disk writes).  The
result is INVALID as a benchmark (the stored payloads are zeros); it only
bounds how much the copy -- a runtime blit kernel on the CUs, overlapping the
verification -- slows the query.  Usage: python tools/ab_ledger_copy.py <bench.py args>
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from drynx_amd.services.service import DrynxNode  # noqa: E402

_buf = {}


def _no_copy(self, tensors):
    sizes = [t.numel() for t in tensors]
    need = sum(sizes)
    b = _buf.get("b")
    if b is None or b.numel() < need:
        b = _buf["b"] = torch.zeros(need, dtype=torch.uint8, pin_memory=torch.cuda.is_available())

    def produce():
        mv = memoryview(b.numpy())
        out, o = [], 0
        for n in sizes:
            out.append(mv[o: o + n])
            o += n
        return out
    return produce


DrynxNode._host_bytes = _no_copy
if __name__ == "__main__":
    bench.main()
