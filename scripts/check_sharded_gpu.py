"""Multi-rank parity of sharded_two_hop on the GPU: every rank builds the same global graph,
keeps its user block, runs the sharded fwd+bwd with HIP hops + the real all-reduce, and
compares its rows with the single-device hgconv2 of the whole graph."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraph_diffusion_for_recommendation_amd import Incidence, hgconv2  # noqa: E402
from hypergraph_diffusion_for_recommendation_amd.sharded import (ShardedIncidence,  # noqa: E402
                                                                   sharded_two_hop)

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dev = torch.device(f"cuda:{int(os.environ['LOCAL_RANK']) % torch.cuda.device_count()}")
torch.cuda.set_device(dev)
backend = os.environ.get("HGD_DIST_BACKEND", "nccl")
dist.init_process_group(backend, **({"device_id": dev} if backend == "nccl" else {}))
U, I, E, d = 50_000, 7_000, 600_000, 64
g = torch.Generator(device=dev).manual_seed(0)
u = torch.randint(0, U, (E,), device=dev, generator=g)
i = torch.randint(0, I, (E,), device=dev, generator=g)
key = torch.unique(u * I + i)
rows, cols = key // I, key % I
X = torch.randn(U, d, device=dev, generator=g)
dY = torch.randn(U, d, device=dev, generator=g)
full = Incidence.from_coo(torch.stack([rows, cols]), None, (U, I), device=dev)
Xf = X.clone().requires_grad_(True)
Yf = hgconv2(full, Xf)
(dXf,) = torch.autograd.grad(Yf, Xf, dY)
per = U // world
lo, hi = rank * per, (U if rank == world - 1 else (rank + 1) * per)
sel = (rows >= lo) & (rows < hi)
loc = Incidence.from_coo(torch.stack([rows[sel] - lo, cols[sel]]), None, (hi - lo, I), device=dev)
sh = ShardedIncidence(loc, n_chunks=3)
Xl = X[lo:hi].clone().requires_grad_(True)
Yl = sharded_two_hop(sh, Xl)
(dXl,) = torch.autograd.grad(Yl, Xl, dY[lo:hi])
ey = ((Yl - Yf[lo:hi]).abs().max() / Yf.abs().max()).item()
ed = ((dXl - dXf[lo:hi]).abs().max() / dXf.abs().max()).item()
print(f"rank {rank}: rows [{lo},{hi}) max rel err Y {ey:.2e} dX {ed:.2e}", flush=True)
assert ey < 1e-5 and ed < 1e-5
dist.barrier()
dist.destroy_process_group()
