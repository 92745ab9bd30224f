#!/usr/bin/env python3
"""Rehearsal probe: can two ranks share ONE GPU over RCCL (torch.distributed "nccl" and libdppo's
own communicator)?  Launch with
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        tools/probe/rccl_same_gpu.py
"""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "diamond-ppo_amd"))


def main():
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    t = torch.full((4,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    print(f"rank {rank}: torch all_reduce -> {t.tolist()}", flush=True)
    from diamond import _native as N
    h = N.Handle(0, N.Dims(128, 64, 4, 2, 0, 64, 1, 1, 2, rank))
    obj = [N.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    h.comm_init(2, rank, obj[0])
    print(f"rank {rank}: libdppo comm ok", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
