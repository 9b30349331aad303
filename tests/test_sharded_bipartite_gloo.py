"""CPU, gloo, world sizes 2 and 3: the model-side user-row sharded operators (sharded.py,
SURVEY.md §8e "HCCF specifics") reproduce the global operators on the reference's bipartite
graphs — the GCN hop on norm_adj (HCCF.py:193-199), HGCNConv (HGNN_HD4.py:450-462), the ED-HNN
mean pair on ui_adj (EquivSetConv2.py:88-93), a globally-masked drop-edge hop (HCCF.py:213-226)
and HGNNLayer's dense H·(Hᵀ·X) (HCCF.py:201-211) — forward values and gradients, under the
partial-gradient convention for replicated item rows (Σ over ranks = the global gradient).

The per-shard hop and the small dense products are replaced by CPU stand-ins built on the
float64 oracle (test only; the product path has no CPU hop). Structure slicing (block_coo),
symmetric-transpose views, global-degree scales, the chunked async all-reduces and the autograd
wiring are the product code."""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import hgd_oracle as O

U, I, NNZ, D, K = 37, 23, 260, 8, 16
KEEP = 0.7


class _Csr:
    def __init__(self, rowptr, col, n_rows, n_cols):
        self.rowptr = torch.from_numpy(np.asarray(rowptr, dtype=np.int64))
        self.col = torch.from_numpy(np.asarray(col, dtype=np.int32))
        self.n_rows, self.n_cols, self.nnz = n_rows, n_cols, len(col)
        self.device = torch.device("cpu")


class _Inc:
    """Stand-in for Incidence: CSR + CSC (stable, rows ascending per column), val / val_t,
    perm_t (CSC position → CSR position) and a CPU drop()."""

    def __init__(self, csr, csc, val, val_t):
        self.csr, self.csc, self.val, self.val_t = csr, csc, val, val_t
        self.n_rows, self.n_cols, self.nnz = csr.n_rows, csr.n_cols, csr.nnz
        self.device = torch.device("cpu")
        self.perm_t = None
        self.coo_sorted = True

    @classmethod
    def from_coo(cls, idx, vals, shape, device=None, **kw):
        rows, cols = idx[0].numpy(), idx[1].numpy()
        v = None if vals is None else vals.numpy().astype(np.float32)
        rowptr, col, vs, _ = O.csr_from_coo(rows, cols, shape[0], v)
        colptr, row_t, vt, perm = O.transpose_csr(rowptr, col, shape[1], vs)
        inc = cls(_Csr(rowptr, col, shape[0], shape[1]), _Csr(colptr, row_t, shape[1], shape[0]),
                  None if vs is None else torch.from_numpy(vs),
                  None if vt is None else torch.from_numpy(vt))
        inc.perm_t = torch.from_numpy(perm.astype(np.int32))
        return inc

    def drop(self, mask, keep):
        m = mask.numpy().astype(bool)
        rp = self.csr.rowptr.numpy()
        rows = np.repeat(np.arange(self.n_rows), np.diff(rp))[m]
        cols = self.csr.col.numpy()[m]
        v = (self.val.numpy()[m] / np.float32(keep)).astype(np.float32)
        return _Inc.from_coo(torch.from_numpy(np.stack([rows, cols])), torch.from_numpy(v),
                             (self.n_rows, self.n_cols))


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


def _cpu_fold(base, scale, col, nnz):
    s = scale[col.long()]
    return s if base is None else base * s


def _leaky(z, epi, slope):
    return torch.where(z > 0, z, z * slope)


def _leaky_bwd(ref, dy, epi, slope):
    return torch.where(ref > 0, dy, dy * slope)


def _graph():
    u, i = O.synthetic_incidence(U, I, NNZ, seed=5)
    ui = O.bipartite_adjacency(u, i, U, I)
    norm = O.normalize_graph_mat(ui)
    return ui.tocsr(), norm.tocsr()


def _coo(mat):
    mat = mat.tocsr()
    mat.sort_indices()
    idx, v = O.coo_of(mat)
    return torch.from_numpy(idx), torch.from_numpy(v)


def _bounds(world):
    cuts = np.linspace(0, U, world + 1).astype(int)
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def _inputs():
    rng = np.random.default_rng(11)
    X = rng.standard_normal((U + I, D)).astype(np.float32)
    H = rng.standard_normal((U, K)).astype(np.float32)
    Xd = rng.standard_normal((U, D)).astype(np.float32)
    return X, H, Xd


def _grads(world):
    """Per-rank upstream gradients: user rows owned by the rank, item rows a per-rank partial."""
    rng = np.random.default_rng(12)
    G = rng.standard_normal((U + I, D)).astype(np.float32)
    Gi = [rng.standard_normal((I, D)).astype(np.float32) for _ in range(world)]
    return G, Gi


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hypergraph_diffusion_for_recommendation_amd import sharded as S
    # CPU stand-ins for the device kernels (test only)
    S.spmm_csr, S._fold = _cpu_spmm, _cpu_fold
    S._epilogue_apply, S._epilogue_backward = _leaky, _leaky_bwd
    S._tn = lambda A, B: A.t() @ B
    S._nn = lambda A, M: A @ M
    S._nt = lambda A, M: A @ M.t()
    S.Incidence = _Inc

    ui, norm = _graph()
    u0, u1 = _bounds(world)[rank]
    X, H, Xd = _inputs()
    G, Gi = _grads(world)
    Xl = np.concatenate([X[u0:u1], X[U:]])
    Gl = torch.from_numpy(np.concatenate([G[u0:u1], Gi[rank]]))
    res = {}

    def shard(mat, symmetric):
        idx, v = _coo(mat)
        b_idx, b_val, c_idx, c_val, sel_b, sel_c = S.block_coo(idx, v, U, u0, u1)
        B = _Inc.from_coo(b_idx, b_val, (u1 - u0, I))
        C = None if symmetric else _Inc.from_coo(c_idx, c_val, (I, u1 - u0))
        sh = S.ShardedBipartite(B, C, n_chunks=3)
        sh.sel_b, sh.sel_c = sel_b, sel_c
        return sh

    def run(name, fn):
        x = torch.from_numpy(Xl.copy()).requires_grad_(True)
        y = fn(x)
        (dx,) = torch.autograd.grad(y, x, Gl)
        res[name + "_Y"] = y.detach().numpy()
        res[name + "_dX"] = dx.numpy()

    sh_norm = shard(norm, True)
    sh_norm_full = shard(norm, False)  # the same operator with C_g stored explicitly
    sh_ui = shard(ui, True)
    run("gcn", lambda x: S.sharded_gcn_hop(sh_norm, x))
    run("gcn_c", lambda x: S.sharded_gcn_hop(sh_norm_full, x))
    run("hgcn", lambda x: S.sharded_hgcn_conv(sh_norm, x, act=True, slope=0.5))
    run("mean2", lambda x: S.sharded_mean_two_hop(sh_ui, x))
    mask = torch.from_numpy(np.random.default_rng(3).random(norm.nnz) + KEEP >= 1.0)
    sh_drop = sh_norm.drop_global(KEEP, mask)
    run("drop", lambda x: S.bipartite_hop(sh_drop, x))
    res["drop_symmetric"] = np.array(sh_drop.symmetric)
    res["n_chunks"] = np.array(len(sh_norm.bounds))
    # dense learned hypergraph: user rows of H and X on this rank
    h = torch.from_numpy(H[u0:u1].copy()).requires_grad_(True)
    xd = torch.from_numpy(Xd[u0:u1].copy()).requires_grad_(True)
    yd = S.sharded_dense_two_hop(h, xd)
    dh, dxd = torch.autograd.grad(yd, (h, xd), torch.from_numpy(G[u0:u1]))
    res.update(dense_Y=yd.detach().numpy(), dense_dH=dh.numpy(), dense_dX=dxd.numpy())
    # all_reduce_sum: forward sum, backward sum
    z = torch.full((4,), float(rank + 1), requires_grad=True)
    s = S.all_reduce_sum(z)
    (dz,) = torch.autograd.grad(s, z, torch.full((4,), float(rank + 1)))
    res.update(ars_Y=s.detach().numpy(), ars_dX=dz.numpy())
    np.savez(os.path.join(outdir, f"r{rank}.npz"), mask=mask.numpy(), **res)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _close(got, ref, mag):
    assert got.shape == ref.shape
    bad = np.abs(got - ref) > 1e-5 * mag + 1e-12
    assert not bad.any(), f"max err {np.abs(got - ref).max():.3e}"


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_bipartite_ops_match_global(world):
    with tempfile.TemporaryDirectory() as td:
        mp.start_processes(_worker, args=(world, _free_port(), td), nprocs=world, join=True,
                           start_method="spawn")
        parts = [dict(np.load(os.path.join(td, f"r{r}.npz"))) for r in range(world)]
    ui, norm = _graph()
    X, H, Xd = _inputs()
    G, Gi = _grads(world)
    Gt = G.astype(np.float64).copy()
    Gt[U:] = np.sum(Gi, axis=0)  # the true item gradient = Σ of the ranks' partials
    bounds = _bounds(world)
    A = norm.toarray().astype(np.float64)
    B = ui.toarray().astype(np.float64)
    deg = B.sum(1)
    S = np.diag(np.where(deg > 0, 1.0 / np.maximum(deg, 1), 0.0))
    mask = parts[0]["mask"]
    coo = norm.tocoo()  # same row-major order as _coo (sorted CSR)
    Ad = np.zeros_like(A)
    keep = mask.astype(bool)
    np.add.at(Ad, (coo.row[keep], coo.col[keep]),
              (coo.data[keep] / np.float32(KEEP)).astype(np.float32))
    X64 = X.astype(np.float64)

    def check(name, Y, dX, magY, magdX):
        for r, (u0, u1) in enumerate(bounds):
            p = parts[r]
            n = u1 - u0
            _close(p[name + "_Y"][:n], Y[u0:u1], magY[u0:u1])
            _close(p[name + "_Y"][n:], Y[U:], magY[U:])
            _close(p[name + "_dX"][:n], dX[u0:u1], magdX[u0:u1])
        _close(sum(p[name + "_dX"][u1 - u0:] for p, (u0, u1) in zip(parts, bounds)), dX[U:],
               magdX[U:])

    aA, aX, aG = np.abs(A), np.abs(X64), np.abs(Gt)
    for name in ("gcn", "gcn_c"):
        check(name, A @ X64, A.T @ Gt, aA @ aX, aA.T @ aG)
    Z = A @ (A @ X64)
    dZ = np.where(Z > 0, Gt, 0.5 * Gt)
    check("hgcn", np.where(Z > 0, Z, 0.5 * Z), A.T @ (A.T @ dZ), aA @ (aA @ aX),
          aA.T @ (aA.T @ aG))
    M = S @ B
    check("mean2", M @ (M @ X64), M.T @ (M.T @ Gt), M @ (M @ aX), M.T @ (M.T @ aG))
    aD = np.abs(Ad)
    check("drop", Ad @ X64, Ad.T @ Gt, aD @ aX, aD.T @ aG)
    assert not parts[0]["drop_symmetric"]
    assert all(int(p["n_chunks"]) == 3 for p in parts)
    # dense two-hop over the whole user set
    H64, Xd64, Gu = H.astype(np.float64), Xd.astype(np.float64), G[:U].astype(np.float64)
    Mh = H64.T @ Xd64
    dM = H64.T @ Gu
    Yd, dH, dXd = H64 @ Mh, Gu @ Mh.T + Xd64 @ dM.T, H64 @ dM
    aH = np.abs(H64)
    magM = aH.T @ np.abs(Xd64)
    magdM = aH.T @ np.abs(Gu)
    for r, (u0, u1) in enumerate(bounds):
        p = parts[r]
        _close(p["dense_Y"], Yd[u0:u1], (aH @ magM)[u0:u1])
        _close(p["dense_dX"], dXd[u0:u1], (aH @ magdM)[u0:u1])
        _close(p["dense_dH"], dH[u0:u1],
               (np.abs(Gu) @ magM.T + np.abs(Xd64) @ magdM.T)[u0:u1])
    tot = world * (world + 1) / 2
    for p in parts:
        assert np.all(p["ars_Y"] == tot) and np.all(p["ars_dX"] == tot)


def test_block_coo_slices_the_blocks():
    ui, norm = _graph()
    from hypergraph_diffusion_for_recommendation_amd.sharded import block_coo
    idx, v = _coo(norm)
    u0, u1 = 5, 19
    b_idx, b_val, c_idx, c_val, sel_b, sel_c = block_coo(idx, v, U, u0, u1)
    A = norm.toarray()
    Bd = np.zeros((u1 - u0, I), np.float32)
    Bd[b_idx[0].numpy(), b_idx[1].numpy()] = b_val.numpy()
    Cd = np.zeros((I, u1 - u0), np.float32)
    Cd[c_idx[0].numpy(), c_idx[1].numpy()] = c_val.numpy()
    assert np.array_equal(Bd, A[u0:u1, U:]) and np.array_equal(Cd, A[U:, u0:u1])
    assert np.array_equal(Cd, Bd.T)
    # row-major order kept (sel ascending) and the positions index the global COO
    assert torch.all(sel_b[1:] > sel_b[:-1]) and torch.all(sel_c[1:] > sel_c[:-1])
    assert torch.equal(v[sel_b], b_val) and torch.equal(v[sel_c], c_val)


def test_block_coo_of_a_row_unsorted_coo_is_in_csr_order():
    """A shuffled COO (not the row-major order of tocoo()): each block comes out row-sorted, and
    sel_b / sel_c still index the input, so a global drop-edge mask sliced through them lines
    up with the blocks' CSR order (sharded.drop_global)."""
    from hypergraph_diffusion_for_recommendation_amd.sharded import block_coo
    ui, norm = _graph()
    idx, v = _coo(norm)
    perm = torch.randperm(idx.shape[1], generator=torch.Generator().manual_seed(0))
    idx_s, v_s = idx[:, perm], v[perm]
    u0, u1 = 3, 17
    b_idx, b_val, c_idx, c_val, sel_b, sel_c = block_coo(idx_s, v_s, U, u0, u1)
    for blk in (b_idx, c_idx):
        assert torch.all(blk[0, 1:] >= blk[0, :-1])
    assert torch.equal(v_s[sel_b], b_val) and torch.equal(v_s[sel_c], c_val)
    assert torch.equal(idx_s[0, sel_b] - u0, b_idx[0]) and torch.equal(idx_s[1, sel_c] - u0,
                                                                       c_idx[1])
    A = norm.toarray()
    Bd = np.zeros((u1 - u0, I), np.float32)
    Bd[b_idx[0].numpy(), b_idx[1].numpy()] = b_val.numpy()
    assert np.array_equal(Bd, A[u0:u1, U:])
