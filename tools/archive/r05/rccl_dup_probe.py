"""Probe: can two RCCL ranks share ONE GPU on this image?  (If so, the
bench's nccl paths at N = 2 can be rehearsed on a one-GPU box.)  Run as
torch.distributed.run --nproc-per-node 2; prints one line per rank."""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
try:
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    t = torch.ones(4, device="cuda") * (rank + 1)
    dist.all_reduce(t)
    torch.cuda.synchronize()
    print(f"rank {rank}: all_reduce ok {t.tolist()}", flush=True)
    dist.destroy_process_group()
except Exception as e:  # noqa: BLE001 -- the probe's answer
    print(f"rank {rank}: FAILED {type(e).__name__}: {str(e)[:300]}", flush=True)
