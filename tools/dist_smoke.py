"""The RCCL data plane + gloo control planes of DistComm in ONE rank
(DRYNX_FORCE_DIST=1): process-group init with a device id, gloo groups next
to the nccl one, all_to_all_single on HBM tensors with unknown and known
receive sizes, object broadcast / all-gather on the control group and on a
side plane, barrier.  A one-GPU box cannot hold two RCCL ranks (RCCL refuses
two ranks on one device), so this is the multi-GPU code path's API surface
as far as one GPU can exercise it.
Run: DRYNX_FORCE_DIST=1 torchrun --nproc-per-node 1 --master-addr 127.0.0.1 tools/dist_smoke.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from drynx_amd.parallel.comm import DistComm, init_distributed, make_comm  # noqa: E402


def main():
    init_distributed()
    comm = make_comm()
    assert isinstance(comm, DistComm), type(comm)
    assert comm.backend == ("nccl" if torch.cuda.is_available() else "gloo")
    t = torch.arange(1000, dtype=torch.int32, device=comm.device).view(250, 4)
    got = comm.exchange({0: t})
    assert torch.equal(got[0].view(250, 4), t)
    got = comm.exchange({0: t[:7]}, recv_sizes={0: 28})
    assert torch.equal(got[0], t[:7].reshape(-1))
    assert comm.exchange({}) == {}
    obj = {"survey": "s1", "big": 1 << 200, "t": torch.ones(3, dtype=torch.int64)}
    back = comm.broadcast_object(obj)
    assert back["big"] == 1 << 200
    assert comm.all_gather_object(("x", 5)) == [("x", 5)]
    pool = comm.plane("pool")
    assert pool.all_gather_object([1, 2]) == [[1, 2]]
    comm.barrier()
    pool.barrier()
    if comm.device.type == "cuda":
        torch.cuda.synchronize()
    print(f"dist smoke ok: backend {comm.backend}, device {comm.device}, sent {comm.bytes_sent} recv {comm.bytes_recv}",
          flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
