"""Host cost of small host->device uploads while the GPU queue is busy.

Queues ~50 ms of matmuls on the current stream, then times N uploads of a
small int32 tensor done three ways: pinned + non_blocking (bn254.h2d),
pageable blocking, pageable non_blocking.  Prints host ms per upload."""
import time

import torch


def busy(dev):
    a = torch.randn(4096, 4096, device=dev)
    for _ in range(40):
        a = a @ a
        a = a / a.norm()
    return a


def main():
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)
    small = [torch.arange(8 * (i + 1), dtype=torch.int32) for i in range(16)]
    ways = {
        "pinned_nb": lambda t: t.pin_memory().to(dev, non_blocking=True),
        "pageable_block": lambda t: t.to(dev),
        "pageable_nb": lambda t: t.to(dev, non_blocking=True),
    }
    for rep in range(2):
        for name, f in ways.items():
            torch.cuda.synchronize()
            t_busy = time.perf_counter()
            busy(dev)
            t0 = time.perf_counter()
            for t in small:
                f(t)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(f"rep{rep} {name:15s} host {1e3 * (t1 - t0) / len(small):7.3f} ms/upload  "
                  f"queue {1e3 * (t0 - t_busy):6.2f} ms  drain {1e3 * (t2 - t1):6.2f} ms", flush=True)


if __name__ == "__main__":
    main()
