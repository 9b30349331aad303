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


def _allreduce_worker(rank, world, port, counts, outdir, seg_mb=0):
    dev = _init(rank, world, port)
    try:
        from hypergraph_diffusion_for_recommendation_amd import _native as nat
        from hypergraph_diffusion_for_recommendation_amd.sharded import P2PExchange
        nat.check(nat.load().hgd_set_tuning(10, seg_mb), "hgd_set_tuning")  # P2P_SEGMENT_MB
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
        ex.poll()
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


def test_p2p_allreduce_over_several_segments(dev, tmp_path):
    """1 MiB segments: the 4 send + 4 reduced slots of 400 KB each live two to a segment, so the exchange addresses slots across four separately imported allocations (the
    layout that keeps each import under the size at which hipIpcOpenMemHandle stalled)."""
    world = 3
    counts = [100_000, 4, 99_996, 65_536, 100_000, 40]
    mp.start_processes(_allreduce_worker,
                       args=(world, _free_port(), counts, str(tmp_path), 1),
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
            out = torch.zeros(1024, device=dev)
            ex.allreduce(0, 1024, out, torch.cuda.current_stream(dev).cuda_stream)
            out2 = torch.zeros(1024, device=dev)
            ex.allreduce(1, 1024, out2, torch.cuda.current_stream(dev).cuda_stream)  # NaN now
            ex.wait(timeout_s=30.0)
            polled = "no error"
            try:
                ex.poll()  # host-visible flag, no sync
            except HGDNativeError as e:
                polled = str(e)
            try:
                ex.check()
            except HGDNativeError as e:
                msg = str(e)
            # a failed exchange never passes for data: every element of both outputs is NaN
            nan_out = bool(torch.isnan(out).all()) and bool(torch.isnan(out2).all())
            msg = f"{msg}|poll: {polled}|nan: {nan_out}"
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
    check, polled, nan = msg.split("|")
    assert "timed out waiting for rank 1" in check, msg
    assert "timed out waiting for rank 1" in polled, msg
    assert nan == "nan: True", msg


def _native_conv_worker(rank, world, port, outdir):
    """The sharded conv through the C ABI over a peer-exchange communicator
    (hgd_comm_create_p2p, hgd_incidence_globalize_columns, hgd_conv2hop_forward / _backward)
    against the Python ShardedIncidence on transport 'p2p', same shard, same inputs."""
    import ctypes
    dev = _init(rank, world, port)
    try:
        from hypergraph_diffusion_for_recommendation_amd import _native as nat
        from hypergraph_diffusion_for_recommendation_amd.sharded import (P2PExchange,
                                                                           ShardedIncidence,
                                                                           sharded_two_hop)
        from oracle import hgd_oracle as O
        lib = nat.load()
        U, I, d = 20_000, 3_000, 96  # d = 96: three 32-column slices, six slots
        rows, cols = O.synthetic_incidence(U, I, 200_000, seed=5)
        idx = torch.from_numpy(np.stack([rows, cols])).to(dev)
        sh, u0, u1 = ShardedIncidence.from_global(idx, U, I, device=dev, transport="p2p")
        g = torch.Generator().manual_seed(6)
        X = torch.randn(U, d, generator=g)[u0:u1].to(dev)
        G = torch.randn(U, d, generator=g)[u0:u1].to(dev)
        st = torch.cuda.current_stream(dev).cuda_stream
        # the native objects: the same local CSR, its own exchange and communicator
        inc = sh.inc
        h = ctypes.c_void_p()
        nat.check(lib.hgd_incidence_create(inc.csr.rowptr.data_ptr(), inc.csr.col.data_ptr(),
                                           None, inc.n_rows, I, inc.nnz, ctypes.byref(h), st),
                  "hgd_incidence_create")
        ex = P2PExchange(I * 32, 6, dev)
        comm = ctypes.c_void_p()
        nat.check(lib.hgd_comm_create_p2p(ex.h, world, rank, ctypes.byref(comm)),
                  "hgd_comm_create_p2p")
        nat.check(lib.hgd_incidence_globalize_columns(h, comm, st), "globalize")
        q = ctypes.c_void_p()
        nat.check(lib.hgd_incidence_scale(h, 1, 1, ctypes.byref(q)), "scale")  # cols, MEAN
        q_nat = torch.empty(I, device=dev)
        hip = ctypes.CDLL("libamdhip64.so")
        assert hip.hipMemcpy(ctypes.c_void_p(q_nat.data_ptr()), q, ctypes.c_size_t(4 * I), 3) == 0
        res = {"scale_equal": bool(torch.equal(q_nat, sh.q))}
        ws = torch.empty(lib.hgd_conv2hop_workspace_size(h, d, 0), dtype=torch.uint8, device=dev)
        same = []
        for _ in range(3):  # both slot sets of both transports, reused
            x = X.clone().requires_grad_(True)
            y = sharded_two_hop(sh, x)
            (dx,) = torch.autograd.grad(y, x, G)
            Y = torch.empty(inc.n_rows, d, device=dev)
            M = torch.empty(I, d, device=dev)
            nat.check(lib.hgd_conv2hop_forward(h, 2, 1, 2, X.data_ptr(), d, d, Y.data_ptr(), d, 0,
                                               0.0, M.data_ptr(), None, comm, ws.data_ptr(),
                                               ws.numel(), st), "hgd_conv2hop_forward")
            dX = torch.empty(inc.n_rows, d, device=dev)
            nat.check(lib.hgd_conv2hop_backward(h, 2, 1, 2, G.data_ptr(), d, d, None, 0, 0.0,
                                                dX.data_ptr(), d, comm, ws.data_ptr(), ws.numel(),
                                                st), "hgd_conv2hop_backward")
            torch.cuda.synchronize(dev)
            same.append(bool(torch.equal(Y, y.detach())) and bool(torch.equal(dX, dx)))
        res["conv_equal"] = same
        # hgd_exchange_allreduce over the peer exchange: the rank-ordered sum, bitwise
        buf = _partial(rank, 4096, 7).to(dev)
        nat.check(lib.hgd_exchange_allreduce(comm, buf.data_ptr(), 4096, st), "allreduce")
        ref = _partial(0, 4096, 7).clone()
        for r in range(1, world):
            ref += _partial(r, 4096, 7)
        res["allreduce_equal"] = bool(torch.equal(buf.cpu(), ref))
        ex.check()
        sh._p2p.check()
        torch.save(res, os.path.join(outdir, f"r{rank}.pt"))
        lib.hgd_comm_destroy(comm)
        lib.hgd_incidence_destroy(h)
        dist.barrier()
        ex.close()
        sh.close()
    finally:
        dist.destroy_process_group()


def test_native_conv2hop_over_p2p_equals_python_p2p_conv(dev, tmp_path):
    world = 2
    mp.start_processes(_native_conv_worker, args=(world, _free_port(), str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    for r in range(world):
        res = torch.load(str(tmp_path / f"r{r}.pt"), weights_only=True)
        assert res == {"scale_equal": True, "conv_equal": [True] * 3,
                       "allreduce_equal": True}, (r, res)


def _sharded_with_p2p(dev, items=1 << 20, d=64):
    """A one-rank ShardedIncidence whose peer transport is up (4 slots of items·d floats)."""
    from hypergraph_diffusion_for_recommendation_amd import Incidence
    from hypergraph_diffusion_for_recommendation_amd.sharded import ShardedIncidence
    idx = torch.tensor([[0, 1, 2, 3], [0, 5, items - 1, 7]], device=dev)
    sh = ShardedIncidence(Incidence.from_coo(idx, None, (4, items), device=dev))
    return sh, sh.p2p(d)


def _free_bytes(dev):
    import gc
    gc.collect()
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    return torch.cuda.mem_get_info(dev)[0]


def test_p2p_segments_of_a_dropped_exchange_go_with_the_next_collective_close(dev):
    """A ShardedIncidence dropped without close() keeps its exported segments mapped (a peer's
    exchange kernel may still read them), and the next collective close() in the process frees
    them with its own: hipMemGetInfo gains back both exchanges' slots. No global keeps the
    dropped exchange's Python objects alive. (Deltas at 0.8 of the slot bytes: other tests'
    garbage collected in between moves the absolute free figure by tens of MB.)"""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd import sharded
    items, d = 1 << 20, 64
    slots_bytes = 4 * items * d * 4  # 2 send + 2 reduced slots of 256 MB
    free0 = _free_bytes(dev)
    live0 = nat.live_views()
    a0 = sharded.abandoned_p2p()
    sh, ex = _sharded_with_p2p(dev, items, d)
    ex.slot(0, items, d).fill_(1.0)
    free1 = _free_bytes(dev)
    assert free0 - free1 >= 0.8 * slots_bytes, (free0, free1)
    del sh, ex
    free2 = _free_bytes(dev)
    assert abs(free2 - free1) < 0.2 * slots_bytes, (free1, free2)  # still mapped
    assert sharded.abandoned_p2p() == a0 + 1 and nat.live_views() == live0
    sh2, _ = _sharded_with_p2p(dev, items, d)
    free3 = _free_bytes(dev)
    sh2.close()  # collective (one rank): frees its own segments and the dropped exchange's
    free4 = _free_bytes(dev)
    assert free4 - free3 >= 1.6 * slots_bytes, (free3, free4)
    assert sharded.abandoned_p2p() == 0


def test_p2p_slot_view_held_past_close_stays_valid(dev):
    """close() makes the exchange unusable, but a slot view handed out before it keeps its memory
    alive (never a view of freed memory); the memory goes at the first safe point after the last
    view's storage (never inside torch's storage release)."""
    items, d = 1 << 20, 64
    slots_bytes = 4 * items * d * 4
    sh, ex = _sharded_with_p2p(dev, items, d)
    v = ex.slot(1, items, d)[10:20]  # a view of the view: the storage outlives the slot tensor
    free_open = _free_bytes(dev)
    sh.close()
    with pytest.raises(RuntimeError, match="closed"):
        ex.slot(1, items, d)
    free_closed = _free_bytes(dev)
    assert free_closed - free_open < 0.2 * slots_bytes  # still mapped: v points at live memory
    v.fill_(3.0)
    assert bool((v == 3.0).all())
    del v
    from hypergraph_diffusion_for_recommendation_amd import sharded
    assert sharded.release_pending_p2p() >= 1  # the deleter only queued it: a safe point frees
    assert _free_bytes(dev) - free_closed >= 0.8 * slots_bytes
    del sh, ex
