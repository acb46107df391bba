"""Probe (not collected): bench.replica_check on identical CUDA tensors over gloo, 2 ranks on one GPU."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402

dist.init_process_group("gloo")
torch.cuda.set_device(0)


class N:
    pass


n = N()
n.params = torch.randn(694803, generator=torch.Generator().manual_seed(0)).cuda()
print(dist.get_rank(), "cuda identical ->", bench.replica_check(n, dist), flush=True)
v = torch.tensor([1.0 + dist.get_rank(), 5.0], dtype=torch.float64, device="cuda")
lo, hi = v.clone(), v.clone()
dist.all_reduce(lo, op=dist.ReduceOp.MIN)
dist.all_reduce(hi, op=dist.ReduceOp.MAX)
print(dist.get_rank(), "min", lo.tolist(), "max", hi.tolist(), flush=True)
dist.destroy_process_group()
