"""Probe: can two ranks share one GPU under the nccl (RCCL) backend?  (The multi-GPU bench path's
device all-reduce can then be exercised on a one-GPU box.)  Run under torchrun --nproc-per-node 2."""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda:0"))
t = torch.full((576,), rank + 1, dtype=torch.int64, device="cuda:0")
dist.all_reduce(t)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce ok, t[0] = {int(t[0])}", flush=True)
dist.barrier()
dist.destroy_process_group()
