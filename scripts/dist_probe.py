"""Probe: can two ranks share one GPU over the "nccl" (RCCL) backend?

Run under torch.distributed.run with --nproc-per-node 2 on a one-GPU box.
Every rank uses cuda:0 and exercises the collectives bench.py uses at N > 1
(scatter, barrier, all_reduce MAX, gather, all_gather_into_tensor).  Used
only to decide whether bench.py's multi-rank path can be rehearsed on one GPU.
"""
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group(os.environ.get("PROBE_BACKEND", "nccl"), device_id=dev)
mine = torch.zeros(3, dtype=torch.int64, device=dev)
parts = [torch.full((3,), r, dtype=torch.int64, device=dev) for r in range(world)] if rank == 0 else None
dist.scatter(mine, parts, src=0)
dist.barrier()
t = torch.tensor([float(rank)], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
y = torch.full((4, 8), float(rank), device=dev)
outs = [torch.empty_like(y) for _ in range(world)] if rank == 0 else None
dist.gather(y, outs, dst=0)
big = torch.empty(world * 5, device=dev)
dist.all_gather_into_tensor(big, torch.full((5,), float(rank), device=dev))
torch.cuda.synchronize()
print(f"rank {rank}: scatter {mine.tolist()} max {t.item()} allgather {big.tolist()}"
      + (f" gather {[float(o[0, 0]) for o in outs]}" if rank == 0 else ""), flush=True)
dist.destroy_process_group()
