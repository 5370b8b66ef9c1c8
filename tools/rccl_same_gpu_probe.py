"""Probe: can two RCCL ranks share one GPU on this pool's boxes?  (If so,
the frame driver's RCCL path can be rehearsed with 2 ranks on one MI355X.)
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_same_gpu_probe.py
"""
import os
import time

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
x = torch.full((4,), rank + 1, dtype=torch.int32, device=dev)
dist.all_reduce(x, op=dist.ReduceOp.MAX)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce -> {x.tolist()}", flush=True)
buf = torch.full((1 << 20,), rank, dtype=torch.uint8, device=dev)
gl = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
dist.gather(buf, gather_list=gl, dst=0)
torch.cuda.synchronize()
if rank == 0:
    print("gather ok:", [int(g[0]) for g in gl], flush=True)
dist.barrier()
t0 = time.perf_counter()
for _ in range(200):
    dist.all_reduce(x[:1], op=dist.ReduceOp.MAX)
torch.cuda.synchronize()
print(f"rank {rank}: all_reduce latency {(time.perf_counter() - t0) / 200 * 1e6:.1f} us", flush=True)
dist.destroy_process_group()
