"""Probe: can RCCL (torch 'nccl' backend) run two ranks on ONE GPU?  If it can, the sharded step's RCCL
path (async all_to_all handles, device all_reduce) is testable on a one-GPU box.  Launch:
  python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 \
      profiles/probe/rccl_two_ranks_one_gpu.py"""
import os
import sys

import torch
import torch.distributed as dist

rank = int(os.environ['RANK'])
torch.cuda.set_device(0)
try:
    dist.init_process_group('nccl', device_id=torch.device('cuda', 0))
    x = torch.full((4,), float(rank + 1), device='cuda')
    dist.all_reduce(x)
    outs = [torch.empty(2, device='cuda') for _ in range(2)]
    ins = [torch.full((2,), float(10 * rank + j), device='cuda') for j in range(2)]
    h = dist.all_to_all(outs, ins, async_op=True)
    h.wait()
    torch.cuda.synchronize()
    print(f'rank {rank}: all_reduce {x.tolist()} all_to_all {[o.tolist() for o in outs]}', flush=True)
    dist.destroy_process_group()
except Exception as e:   # report, do not hang
    print(f'rank {rank}: RCCL two-ranks-one-GPU failed: {type(e).__name__}: {e}', flush=True)
    sys.exit(3)
