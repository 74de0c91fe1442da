"""Probe: can two RCCL ranks (two processes) share one GPU? (decides how the library's RCCL exchange
is tested on a one-GPU box)."""
import os
import sys
import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    x = torch.full((4,), rank + 1, dtype=torch.int64, device=dev)
    dist.all_reduce(x)
    y = torch.zeros(2 * 4, dtype=torch.int64, device=dev)
    dist.all_to_all_single(y, torch.arange(8, dtype=torch.int64, device=dev) + 100 * rank)
    torch.cuda.synchronize()
    print("rank", rank, "allreduce", x.tolist(), "a2a", y.tolist(), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
