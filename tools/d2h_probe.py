"""Which engine moves a large device-to-host copy: the ledger's ~540 MB of
range payloads per query showed up as a 10.7 ms __amd_rocclr_copyBuffer
kernel (a blit on the CUs) in the serialized span table.  Copies 512 MB into
(a) a torch pinned tensor (torch's caching host allocator), (b) a numpy
buffer page-locked with hipHostRegister, (c) hipHostMalloc memory, each with
hipMemcpyAsync on a side stream, and prints the wall time per copy; run it
under ``rocprofv3 --kernel-trace --memory-copy-trace`` to see whether a
copyBuffer kernel or an SDMA copy did the work."""
import ctypes
import time

import numpy as np
import torch


def main():
    dev = torch.device("cuda", 0)
    n = 512 << 20
    src = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
    hip = ctypes.CDLL("libamdhip64.so")
    st = torch.cuda.Stream(dev)
    D2H = 2

    def timed(name, dst_ptr, reps=3):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rc = hip.hipMemcpyAsync(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(n),
                                    D2H, ctypes.c_void_p(st.cuda_stream))
            assert rc == 0, rc
            st.synchronize()
            ts.append(1e3 * (time.perf_counter() - t))
        print(f"{name:28s} {min(ts):7.2f} ms  ({n / min(ts) / 1e6:.1f} GB/s)", flush=True)

    pinned = torch.empty((n,), dtype=torch.uint8, pin_memory=True)
    timed("torch pin_memory", pinned.data_ptr())
    buf = np.empty(n, dtype=np.uint8)
    assert hip.hipHostRegister(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(n), 0) == 0
    timed("hipHostRegister(numpy)", buf.ctypes.data)
    hip.hipHostUnregister(ctypes.c_void_p(buf.ctypes.data))
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(n), 0) == 0
    timed("hipHostMalloc(default)", p.value)
    hip.hipHostFree(p)
    p2 = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p2), ctypes.c_size_t(n), 0x4) == 0  # hipHostMallocWriteCombined
    timed("hipHostMalloc(writecomb)", p2.value)
    hip.hipHostFree(p2)
    # torch's own path (what the ledger uses)
    torch.cuda.synchronize()
    t = time.perf_counter()
    with torch.cuda.stream(st):
        pinned.copy_(src, non_blocking=True)
    st.synchronize()
    print(f"{'torch copy_ non_blocking':28s} {1e3 * (time.perf_counter() - t):7.2f} ms", flush=True)


if __name__ == "__main__":
    main()
