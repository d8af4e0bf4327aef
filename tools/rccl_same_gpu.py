"""Probe: can RCCL ("nccl" backend) run two ranks on ONE GPU?  If it can, the bench's RCCL paths (barrier, max-over-ranks
all-reduce, the gather mode's batch_isend_irecv) can be exercised on a 1-GPU box.  Run under torch.distributed.run:
  python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
      tools/rccl_same_gpu.py
Prints one JSON line per rank."""
import json
import os

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
world = int(os.environ["WORLD_SIZE"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
out = {"rank": rank, "world": world}
try:
    dist.init_process_group("nccl", device_id=dev)
    x = torch.full((1024,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    torch.cuda.synchronize()
    out["all_reduce"] = float(x[0].item())
    peer = (rank + 1) % world
    src = (rank - 1) % world
    s = torch.full((1 << 20,), rank, dtype=torch.uint8, device=dev)
    r = torch.empty_like(s)
    ops = [dist.P2POp(dist.isend, s, peer), dist.P2POp(dist.irecv, r, src)]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    torch.cuda.synchronize()
    out["p2p_ok"] = bool((r == src).all().item())
    dist.barrier()
    out["status"] = "ok"
except Exception as e:  # record what RCCL says
    out["status"] = "error"
    out["error"] = f"{type(e).__name__}: {str(e)[:400]}"
print(json.dumps(out), flush=True)
if dist.is_initialized():
    dist.destroy_process_group()
