"""The direct xGMI peer transport (csrc/p2p.hip, sharded.P2PExchange) rehearsed on the one-GPU
box: N processes share cuda:0 (the IPC-mapped buffers of a peer on the same device are the same
memory; over xGMI each peer is another GPU), gloo carries only the setup (IPC handles) and the
comparison. Covered: the two-shot reduce equals the rank-ordered sum bit for bit on every rank,
ragged block splits (count not a multiple of 4·N), the two slot sets alternating over several
exchanges, the sharded conv on the p2p transport against the single-GPU conv of the global graph,
and a bounded wait: a peer that never signals makes the exchange time out and report, instead of
hanging the device."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    return dev


def _partial(rank, count, rnd):
    g = torch.Generator().manual_seed(1000 * rnd + rank)
    return torch.randn(count, generator=g)


def _allreduce_worker(rank, world, port, counts, outdir):
    dev = _init(rank, world, port)
    try:
        from hypergraph_diffusion_for_recommendation_amd.sharded import P2PExchange
        ex = P2PExchange(max(counts), 4, dev, timeout_s=60.0)
        side = torch.cuda.Stream(dev)
        bad = []
        for rnd, count in enumerate(counts):
            k = rnd % 4
            send = ex.slot(k, 1, count)
            send.copy_(_partial(rank, count, rnd).to(dev).view(1, count))
            out = torch.full((count,), float("nan"), device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            ex.allreduce(k, count, out, side.cuda_stream)
            torch.cuda.current_stream(dev).wait_stream(side)
            ref = _partial(0, count, rnd).clone()
            for q in range(1, world):  # the kernel's order: ranks ascending, fp32
                ref += _partial(q, count, rnd)
            got = out.cpu()
            if not torch.equal(got, ref):
                bad.append((rnd, count, float((got - ref).abs().max())))
        ex.check()
        torch.save(bad, os.path.join(outdir, f"r{rank}.pt"))
        ex.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_p2p_allreduce_is_the_rank_ordered_sum(dev, tmp_path, world):
    counts = [4, 1 << 16, 12_345 * 4, (1 << 20) + 36, 8]
    mp.start_processes(_allreduce_worker, args=(world, _free_port(), counts, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    for r in range(world):
        assert torch.load(str(tmp_path / f"r{r}.pt"), weights_only=True) == [], r


def _conv_worker(rank, world, port, outdir):
    dev = _init(rank, world, port)
    try:
        from hypergraph_diffusion_for_recommendation_amd.sharded import (ShardedIncidence,
                                                                           sharded_two_hop)
        from oracle import hgd_oracle as O
        U, I, d = 20_000, 3_000, 64
        rows, cols = O.synthetic_incidence(U, I, 200_000, seed=5)
        idx = torch.from_numpy(np.stack([rows, cols])).to(dev)
        sh, u0, u1 = ShardedIncidence.from_global(idx, U, I, device=dev, slice_width=32,
                                                  transport="p2p")
        g = torch.Generator().manual_seed(6)
        X = torch.randn(U, d, generator=g)
        G = torch.randn(U, d, generator=g)
        outs = []
        for _ in range(3):  # both slot sets, reused
            x = X[u0:u1].to(dev).requires_grad_(True)
            y = sharded_two_hop(sh, x)
            (dx,) = torch.autograd.grad(y, x, G[u0:u1].to(dev))
            outs.append((y.detach().cpu(), dx.cpu()))
        sh._p2p.check()
        torch.save({"u0": u0, "u1": u1, "outs": outs}, os.path.join(outdir, f"r{rank}.pt"))
        sh.close()
    finally:
        dist.destroy_process_group()


def test_sharded_conv_on_p2p_matches_single_gpu(dev, tmp_path):
    from hypergraph_diffusion_for_recommendation_amd import Incidence, hgconv2
    from oracle import hgd_oracle as O
    world = 2
    mp.start_processes(_conv_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    U, I, d = 20_000, 3_000, 64
    rows, cols = O.synthetic_incidence(U, I, 200_000, seed=5)
    inc = Incidence.from_coo(torch.from_numpy(np.stack([rows, cols])).to(dev), None, (U, I),
                             device=dev)
    g = torch.Generator().manual_seed(6)
    X = torch.randn(U, d, generator=g).to(dev).requires_grad_(True)
    G = torch.randn(U, d, generator=g).to(dev)
    Y = hgconv2(inc, X)
    (dX,) = torch.autograd.grad(Y, X, G)
    with torch.no_grad():
        mag, dmag = hgconv2(inc, X.abs()), hgconv2(inc, G.abs())
    parts = [torch.load(str(tmp_path / f"r{r}.pt"), weights_only=True) for r in range(world)]
    assert parts[0]["u0"] == 0 and parts[-1]["u1"] == U
    for p in parts:
        a, b = p["u0"], p["u1"]
        for y, dx in p["outs"]:
            assert torch.equal(y, p["outs"][0][0]) and torch.equal(dx, p["outs"][0][1])
            for got, ref, m in ((y, Y[a:b], mag[a:b]), (dx, dX[a:b], dmag[a:b])):
                err = (got.to(dev) - ref).abs()
                assert bool((err <= 1e-5 * m + 1e-30).all()), float((err / (m + 1e-30)).max())


def _timeout_worker(rank, world, port, outdir):
    dev = _init(rank, world, port)
    try:
        from hypergraph_diffusion_for_recommendation_amd._native import HGDNativeError
        from hypergraph_diffusion_for_recommendation_amd.sharded import P2PExchange
        ex = P2PExchange(1024, 2, dev, timeout_s=1.0)
        msg = "no error"
        if rank == 0:  # rank 1 never exchanges: rank 0's wait must give up after ~1 s
            out = torch.empty(1024, device=dev)
            ex.allreduce(0, 1024, out, torch.cuda.current_stream(dev).cuda_stream)
            ex.allreduce(1, 1024, out, torch.cuda.current_stream(dev).cuda_stream)  # a no-op now
            torch.cuda.synchronize(dev)
            try:
                ex.check()
            except HGDNativeError as e:
                msg = str(e)
        with open(os.path.join(outdir, f"r{rank}.txt"), "w") as f:
            f.write(msg)
        dist.barrier()
        ex.close()
    finally:
        dist.destroy_process_group()


def test_p2p_wait_is_bounded(dev, tmp_path):
    mp.start_processes(_timeout_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2,
                       join=True, start_method="spawn")
    msg = (tmp_path / "r0.txt").read_text()
    assert "timed out waiting for rank 1" in msg, msg
