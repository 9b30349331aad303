"""RCCL as the sharded path initialises it (sharded.init_process_group: backend "nccl" = RCCL,
communicator kernels on a high-priority stream), exercised at one rank on the one-GPU box: the
asynchronous all-reduce the slice pipeline queues behind each hop-1 chunk, and the sharded conv
with those options against the single-GPU conv. N > 1 over xGMI runs on the driver's 8-GPU node
(bench.py --gpus N)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def rccl_one_rank():
    from hypergraph_diffusion_for_recommendation_amd.sharded import init_process_group
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    init_process_group(dev, "nccl", rank=0, world_size=1)
    try:
        yield dev
    finally:
        dist.destroy_process_group()


def test_high_priority_async_all_reduce(rccl_one_rank):
    dev = rccl_one_rank
    x = torch.arange(1 << 20, dtype=torch.float32, device=dev)
    ref = x.clone()
    works = [dist.all_reduce(x[a:a + (1 << 18)], async_op=True) for a in range(0, 1 << 20, 1 << 18)]
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    assert torch.equal(x, ref)


def test_sharded_conv_under_rccl_matches_local(rccl_one_rank):
    import numpy as np

    from hypergraph_diffusion_for_recommendation_amd import Incidence, hgconv2
    from hypergraph_diffusion_for_recommendation_amd.sharded import (ShardedIncidence,
                                                                       sharded_two_hop)
    from oracle import hgd_oracle as O
    dev = rccl_one_rank
    U, I = 3000, 700
    rows, cols = O.synthetic_incidence(U, I, 30000, seed=4)
    idx = torch.from_numpy(np.stack([rows, cols])).to(dev)
    sh, u0, u1 = ShardedIncidence.from_global(idx, U, I, device=dev, n_chunks=4, slice_width=32)
    assert (u0, u1) == (0, U)
    inc = Incidence.from_coo(idx, None, (U, I), device=dev)
    g = torch.Generator(device=dev).manual_seed(3)
    X = torch.randn(U, 64, device=dev, generator=g)
    dY = torch.randn(U, 64, device=dev, generator=g)
    Xs = X.clone().requires_grad_(True)
    Ys = sharded_two_hop(sh, Xs)
    (dXs,) = torch.autograd.grad(Ys, Xs, dY)
    Xl = X.clone().requires_grad_(True)
    Yl = hgconv2(inc, Xl)
    (dXl,) = torch.autograd.grad(Yl, Xl, dY)
    # the same hops in column slices: every output element is the same edge-ordered sum, so
    # this is expected bitwise; the bound is the suite's 1e-5 relative one
    torch.testing.assert_close(Ys, Yl, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(dXs, dXl, rtol=1e-5, atol=1e-6)
