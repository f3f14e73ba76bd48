"""Probe: can two RCCL ranks share one GPU on this pool's box? (rehearsal only)"""
import os
import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
x = torch.full((4,), float(rank + 1), device="cuda")
dist.all_reduce(x)
torch.cuda.synchronize()
print(f"rank {rank} all_reduce -> {x.tolist()}", flush=True)
dist.destroy_process_group()
