"""GPU box check of the multi-GPU collectives bench.py uses at N > 1, on however many ranks
torch.distributed.run starts (1 on a one-GPU box): RCCL ("nccl") process group bound to the
rank's device, barrier, int64 SUM all-reduce of a histogram-shaped tensor (dptok.dist) and the
float64 MAX all-reduce of the step time."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dp-tokenization_amd")]
import torch
import torch.distributed as dist
from dptok import dist as ddist

rank, world, local = ddist.rank_world()
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
dev = torch.device("cuda", local)
h = torch.arange(266, dtype=torch.int64, device=dev) * (rank + 1)
if dist.get_world_size() > 1:
    ddist.allreduce_histogram(h)
else:
    dist.all_reduce(h, op=dist.ReduceOp.SUM)
dist.barrier()
t = torch.tensor([0.5 + rank], dtype=torch.float64, device=dev)
dist.all_reduce(t, op=dist.ReduceOp.MAX)
want = torch.arange(266, dtype=torch.int64) * sum(r + 1 for r in range(world))
assert torch.equal(h.cpu(), want), h[:4]
assert float(t.item()) == 0.5 + world - 1
print("rank", rank, "world", world, "nccl all-reduce int64 SUM / float64 MAX ok", flush=True)
dist.destroy_process_group()
