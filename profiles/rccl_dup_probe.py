"""Probe: can two processes share the one GPU of a gpurun box through RCCL (torch.distributed
'nccl' = RCCL)?  If so, the library's RCCL transport can be exercised at 2 ranks on one card.
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 profiles/rccl_dup_probe.py
"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=rank, world_size=int(os.environ["WORLD_SIZE"]), device_id=torch.device("cuda:0"))
t = torch.full((4,), float(rank + 1), device="cuda:0")
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce -> {t.tolist()}", flush=True)
dist.destroy_process_group()
