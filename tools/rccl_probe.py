"""Can two ranks share ONE GPU over RCCL (backend "nccl")?  all_reduce,
all_to_all_single with uneven splits, broadcast, all_gather_into_tensor.
Run: torchrun --nproc-per-node 2 tools/rccl_probe.py"""
import os

import torch
import torch.distributed as dist


def main():
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    dist.init_process_group("nccl")
    r, w = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", int(os.environ.get("RCCL_PROBE_DEVICE", "0")))
    torch.cuda.set_device(dev)
    x = torch.full((4,), r + 1.0, device=dev)
    dist.all_reduce(x)
    ins = [r * 10 + k for k in range(w)]
    send = torch.arange(sum(ins), device=dev, dtype=torch.int32) + 1000 * r
    recv_sizes = [k * 10 + r for k in range(w)]
    recv = torch.empty(sum(recv_sizes), device=dev, dtype=torch.int32)
    dist.all_to_all_single(recv, send, recv_sizes, ins)
    b = torch.tensor([r], device=dev)
    dist.broadcast(b, 0)
    g = torch.empty(w * 3, device=dev)
    dist.all_gather_into_tensor(g, torch.full((3,), float(r), device=dev))
    torch.cuda.synchronize()
    print(f"rank {r}: all_reduce {x.tolist()} a2a {recv.numel()} bcast {b.item()} gather {g.tolist()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
