"""CPU, world_size 2 over gloo: the user-row sharded 2-hop conv (sharded.py) — global item-degree
all-reduce, chunked async all-reduce of item partial sums, local second hop — reproduces the
unsharded operator. The per-shard hop itself is replaced by a CPU stand-in built on the oracle
(only this test does that; the product path has no CPU hop)."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import hgd_oracle as O

U_PER, I, NNZ_PER, D = 60, 25, 500, 8


class _CPUCsr:
    def __init__(self, rowptr, col, n_rows, n_cols):
        self.rowptr = torch.from_numpy(rowptr)
        self.col = torch.from_numpy(col.astype(np.int32))
        self.n_rows, self.n_cols, self.nnz = n_rows, n_cols, len(col)


class _CPUIncidence:
    """Interface-compatible stand-in for Incidence (scale / edge_values / csr / csc)."""

    def __init__(self, rows, cols, n_rows, n_cols):
        rowptr, col, _, _ = O.csr_from_coo(rows, cols, n_rows)
        colptr, rows_t, _, _ = O.transpose_csr(rowptr, col, n_cols)
        self.csr = _CPUCsr(rowptr, col, n_rows, n_cols)
        self.csc = _CPUCsr(colptr, rows_t, n_cols, n_rows)
        self.n_rows, self.n_cols, self.val = n_rows, n_cols, None

    def scale(self, side, kind):
        if kind is None:
            return None
        o = self.csr if side == "row" else self.csc
        deg = (o.rowptr[1:] - o.rowptr[:-1]).numpy()
        return torch.from_numpy(O.degree_scale(deg, {"mean": -1.0, "sym": -0.5}[kind])).float()

    def edge_values(self, orient, kind):
        s = self.scale("col" if orient == "csr" else "row", kind)
        if s is None:
            return None
        o = self.csr if orient == "csr" else self.csc
        return s[o.col.long()]


def _cpu_spmm(csr, X, val=None, row_scale=None, epilogue=0, slope=0.0, out=None, row_begin=0,
              row_end=None):
    row_end = csr.n_rows if row_end is None else row_end
    Y = O.spmm_csr(csr.rowptr.numpy(), csr.col.numpy(), X.detach().numpy(),
                   None if val is None else val.numpy(),
                   None if row_scale is None else row_scale.numpy())
    if out is None:
        out = torch.zeros(csr.n_rows, X.shape[1])
    out[row_begin:row_end] = torch.from_numpy(Y[row_begin:row_end]).float()
    return out


def _graph(rank):
    rows, cols = O.synthetic_incidence(U_PER, I, NNZ_PER, seed=100 + rank)
    return rows, cols


def _worker(rank, world, port, outdir, scales):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hypergraph_diffusion_for_recommendation_amd import sharded
    sharded.spmm_csr = _cpu_spmm  # CPU stand-in for the HIP hop (test only)
    rows, cols = _graph(rank)
    P, Q, R = scales
    sh = sharded.ShardedIncidence(_CPUIncidence(rows, cols, U_PER, I), n_chunks=3, P=P, Q=Q, R=R,
                                   slice_width=4)
    rng = np.random.default_rng(rank)
    X = torch.from_numpy(rng.standard_normal((U_PER, D)).astype(np.float32))
    dY = torch.from_numpy(rng.standard_normal((U_PER, D)).astype(np.float32))
    X.requires_grad_(True)
    Y = sharded.sharded_two_hop(sh, X)
    (dX,) = torch.autograd.grad(Y, X, dY)
    np.savez(os.path.join(outdir, f"r{rank}.npz"), X=X.detach().numpy(), dY=dY.numpy(),
             Y=Y.detach().numpy(), dX=dX.numpy(), n_chunks=len(sh.bounds))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SCALES = [("sym", "mean", "sym"),   # hgconv2 (data/graph.py:28-42)
          ("mean", "mean", None)]   # the ED-HNN vertex/edge means (layers2/EquivSetConv2.py:88-93)


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("scales", SCALES, ids=["hgconv2", "mean2hop"])
def test_sharded_two_hop_matches_global(world, scales):
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_worker, args=(world, _free_port(), td, scales), nprocs=world,
                           join=True, start_method="spawn")
        parts = [np.load(os.path.join(td, f"r{r}.npz")) for r in range(world)]
    assert all(int(p["n_chunks"]) == 3 for p in parts)
    P, Q, R = scales
    rows = np.concatenate([_graph(r)[0] + r * U_PER for r in range(world)])
    cols = np.concatenate([_graph(r)[1] for r in range(world)])
    shape = (world * U_PER, I)
    X = np.concatenate([p["X"] for p in parts])
    dY = np.concatenate([p["dY"] for p in parts])
    Y = O.two_hop(rows, cols, None, shape, X, P, Q, R)
    dX = O.two_hop_backward(rows, cols, None, shape, Y, dY, P, Q, R)
    got_Y = np.concatenate([p["Y"] for p in parts])
    got_dX = np.concatenate([p["dX"] for p in parts])
    mag = O.two_hop(rows, cols, None, shape, np.abs(X), P, Q, R)
    dmag = O.two_hop_backward(rows, cols, None, shape, Y, np.abs(dY), P, Q, R)
    assert np.all(np.abs(got_Y - Y) <= 1e-5 * mag + 1e-12)
    assert np.all(np.abs(got_dX - dX) <= 1e-5 * dmag + 1e-12)


# --- strong scaling: ONE global graph, degree-balanced user ranges (bench.py --scaling strong) ---
U_G, I_G, NNZ_G = 150, 40, 1200


def _strong_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hypergraph_diffusion_for_recommendation_amd import sharded
    sharded.spmm_csr = _cpu_spmm  # CPU stand-in for the HIP hop (test only)
    rows, cols = O.synthetic_incidence(U_G, I_G, NNZ_G, seed=7, zipf=1.0)
    idx = torch.from_numpy(np.stack([rows, cols]).astype(np.int64))
    u0, u1, loc = sharded.shard_rows_of_sorted_coo(idx, U_G, world, rank)
    sh = sharded.ShardedIncidence(
        _CPUIncidence(loc[0].numpy(), loc[1].numpy(), u1 - u0, I_G), P="sym", Q="mean", R="sym",
        slice_width=4, n_chunks=2)
    rng = np.random.default_rng(0)
    Xg = rng.standard_normal((U_G, D)).astype(np.float32)
    dYg = rng.standard_normal((U_G, D)).astype(np.float32)
    X = torch.from_numpy(Xg[u0:u1].copy()).requires_grad_(True)
    Y = sharded.sharded_two_hop(sh, X)
    (dX,) = torch.autograd.grad(Y, X, torch.from_numpy(dYg[u0:u1].copy()))
    np.savez(os.path.join(outdir, f"r{rank}.npz"), Y=Y.detach().numpy(), dX=dX.numpy(),
             u=np.array([u0, u1]), nnz=loc.shape[1])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_strong_sharding_of_one_global_graph(world):
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_strong_worker, args=(world, _free_port(), td), nprocs=world,
                           join=True, start_method="spawn")
        parts = [np.load(os.path.join(td, f"r{r}.npz")) for r in range(world)]
    rows, cols = O.synthetic_incidence(U_G, I_G, NNZ_G, seed=7, zipf=1.0)
    # the user ranges tile [0, U) and every global nonzero lands on exactly one rank
    us = [tuple(p["u"]) for p in parts]
    assert us[0][0] == 0 and us[-1][1] == U_G and all(a[1] == b[0] for a, b in zip(us, us[1:]))
    assert sum(int(p["nnz"]) for p in parts) == len(rows)
    shape = (U_G, I_G)
    rng = np.random.default_rng(0)
    X = rng.standard_normal((U_G, D)).astype(np.float32)
    dY = rng.standard_normal((U_G, D)).astype(np.float32)
    Y = O.two_hop(rows, cols, None, shape, X, "sym", "mean", "sym")
    dX = O.two_hop_backward(rows, cols, None, shape, Y, dY, "sym", "mean", "sym")
    mag = O.two_hop(rows, cols, None, shape, np.abs(X), "sym", "mean", "sym")
    dmag = O.two_hop_backward(rows, cols, None, shape, Y, np.abs(dY), "sym", "mean", "sym")
    got_Y = np.concatenate([p["Y"] for p in parts])
    got_dX = np.concatenate([p["dX"] for p in parts])
    assert np.all(np.abs(got_Y - Y) <= 1e-5 * mag + 1e-12)
    assert np.all(np.abs(got_dX - dX) <= 1e-5 * dmag + 1e-12)


def _dropout_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hypergraph_diffusion_for_recommendation_amd.sharded_encoders import (_rank_generators,
                                                                              _SplitDropout)
    rep, loc = _rank_generators("cpu", 5, None)
    drop = _SplitDropout(0.5, rep, loc).train()
    x = torch.ones(400, 8)
    y = drop(x, 300)  # 300 local user rows, 100 replicated item rows
    np.save(os.path.join(outdir, f"r{rank}.npy"), y.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_split_dropout_local_masks_differ_across_ranks():
    """User rows of different ranks get independent dropout masks (per-rank generator); the
    replicated item rows get the same mask on every rank (shared-seed masks made
    users u0+j of every rank keep or drop together)."""
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_dropout_worker, args=(2, _free_port(), td), nprocs=2, join=True,
                           start_method="spawn")
        a, b = (np.load(os.path.join(td, f"r{r}.npy")) for r in range(2))
    assert set(np.unique(a)) <= {0.0, 2.0}
    assert not np.array_equal(a[:300], b[:300])
    assert np.array_equal(a[300:], b[300:])
    frac = (a[:300] > 0).mean()
    assert 0.4 < frac < 0.6
