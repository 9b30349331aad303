"""Generates the golden vectors in tests/golden/*.npz from the CPU oracle.

Every fixture is produced by oracle/hgd_oracle.py (float64 numpy restatement of the reference,
file:line cited there) and cross-checked here against oracle/ref_cpu.py, which calls the same
torch-CPU library functions the reference calls (torch.sparse.mm, index_reduce 'mean' for
torch_scatter's mean, torch.rand for the drop-edge mask). The reference itself could not be
imported in this container, so these vectors pin our restatement, not the
reference's own outputs — parity is "unpinned" in that sense.

    python tests/golden/make_golden.py      # rewrites the .npz files (deterministic)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import hgd_oracle as O  # noqa: E402
from oracle import ref_cpu  # noqa: E402


def _check(a, b, mag, what):
    err = np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64))
    assert np.all(err <= 1e-5 * np.asarray(mag) + 1e-12), (what, float(err.max()))


def toy_hgconv2():
    """3 users × 2 items, H = [[1,0],[1,1],[0,1]]: closed form checked by hand.
    d_v = (1,2,1), d_e = (2,2). T = D_v^-1/2 H D_e^-1 Hᵀ D_v^-1/2 =
    [[1/2, 1/(2√2), 0], [1/(2√2), 1/2, 1/(2√2)], [0, 1/(2√2), 1/2]]."""
    rows = np.array([0, 1, 1, 2])
    cols = np.array([0, 0, 1, 1])
    X = np.array([[1.0, 2.0], [3.0, -1.0], [0.5, 4.0]], dtype=np.float32)
    s = 1.0 / (2.0 * np.sqrt(2.0))
    T = np.array([[0.5, s, 0.0], [s, 0.5, s], [0.0, s, 0.5]])
    Y_hand = T @ X.astype(np.float64)
    Y = O.two_hop(rows, cols, None, (3, 2), X, "sym", "mean", "sym")
    assert np.allclose(Y, Y_hand, rtol=0, atol=1e-15), "toy hgconv2 known answer"
    Hd = np.zeros((3, 2))
    Hd[rows, cols] = 1
    import scipy.sparse as sp
    T2 = O.normalize_graph_mat_hyper(sp.csr_matrix(Hd)).toarray()
    assert np.allclose(T2, T, atol=1e-15), "normalize_graph_mat_hyper known answer"
    return dict(rows=rows, cols=cols, shape=np.array([3, 2]), X=X, Y=Y)


def interactions(rng, n_users, n_items, n):
    """A training list in file order (with repeats), remapped like data/ui_graph.py:43-68."""
    raw_u = rng.integers(1000, 1000 + n_users, size=n)
    raw_i = rng.integers(50, 50 + n_items, size=n)
    user, item = O.remap_ids(zip(raw_u.tolist(), raw_i.tolist()))
    u = np.array([user[x] for x in raw_u])
    i = np.array([item[x] for x in raw_i])
    return u, i, len(user), len(item)


def hgcn_fixture(rng):
    """HGCNConv on norm_adj (ui_graph.py:134-148 → graph.py:11-25 → torch_interface.py:8-12),
    act=True with LeakyReLU(0.5) (HGNN_HD4.py:455-460), fwd + bwd; plus the GCNLayer hop."""
    u, i, U, I = interactions(rng, 40, 30, 400)
    A = O.normalize_graph_mat(O.bipartite_adjacency(u, i, U, I))
    idx, vals = O.coo_of(A)
    N = U + I
    X = rng.standard_normal((N, 16)).astype(np.float32)
    dY = rng.standard_normal((N, 16)).astype(np.float32)
    Z = O.two_hop(idx[0], idx[1], vals, (N, N), X)
    Y = O.epilogue(Z, "leaky_relu", 0.5)
    dX = O.two_hop_backward(idx[0], idx[1], vals, (N, N), Z, dY, epi="leaky_relu", slope=0.5)
    G = O.spmm_coo(idx[0], idx[1], vals, N, X)
    # cross-check with torch.sparse.mm + autograd
    adj = ref_cpu.coo_tensor(idx[0], idx[1], vals, (N, N))
    Xt = torch.from_numpy(X).requires_grad_(True)
    Yt = ref_cpu.hgcn_conv(adj, Xt, act=True, slope=0.5)
    (dXt,) = torch.autograd.grad(Yt, Xt, torch.from_numpy(dY))
    mag = O.two_hop(idx[0], idx[1], np.abs(vals), (N, N), np.abs(X))
    _check(Yt.detach().numpy(), Y, mag, "hgcn fwd vs torch")
    dmag = O.two_hop(idx[0], idx[1], np.abs(vals), (N, N), np.abs(dY))
    _check(dXt.numpy(), dX, dmag, "hgcn bwd vs torch")
    Gt = torch.sparse.mm(adj, torch.from_numpy(X)).numpy()
    _check(Gt, G, O.spmm_coo(idx[0], idx[1], np.abs(vals), N, np.abs(X)), "gcn vs torch")
    return dict(user=u, item=i, n_users=np.array(U), n_items=np.array(I), indices=idx,
                values=vals, X=X, dY=dY, Y=Y, dX=dX, G=G)


def edhnn_fixture(rng):
    """ED-HNN mean pair on V/E = nonzero(ui_adj > 0) (EquivSetGNN2.py:105-133,
    EquivSetConv2.py:88-93) and the EquivSetConv block with W = Linear(LayerNorm(·))."""
    u, i, U, I = interactions(rng, 30, 25, 250)
    N = U + I
    dense = O.bipartite_adjacency(u, i, U, I).toarray()
    V, E = O.nonzero_threshold(dense)
    X = rng.standard_normal((N, 8)).astype(np.float32)
    Y = O.equivset_mean_2hop(X, V, E, N)
    Yt = ref_cpu.equivset_mean_2hop(torch.from_numpy(X), torch.from_numpy(V),
                                    torch.from_numpy(E), N).numpy()
    _check(Yt, Y, O.equivset_mean_2hop(np.abs(X), V, E, N), "edhnn vs torch")
    ln_w = rng.standard_normal(8).astype(np.float32)
    ln_b = rng.standard_normal(8).astype(np.float32)
    lin_w = rng.standard_normal((8, 8)).astype(np.float32)
    lin_b = rng.standard_normal(8).astype(np.float32)
    conv = O.equivset_conv(X, V, E, X, 0.0, ln_w, ln_b, lin_w, lin_b)
    return dict(V=V, E=E, N=np.array(N), dense=dense.astype(np.float32), X=X, Y=Y, ln_w=ln_w,
                ln_b=ln_b, lin_w=lin_w, lin_b=lin_b, conv=conv)


def dropedge_fixture(rng):
    """SpAdjDropEdge with the mask drawn exactly like HCCF.py:223 (torch.manual_seed(7))."""
    u, i, U, I = interactions(rng, 25, 20, 200)
    A = O.normalize_graph_mat(O.bipartite_adjacency(u, i, U, I))
    idx, vals = O.coo_of(A)
    keep = 0.7
    torch.manual_seed(7)
    mask = ((torch.rand(vals.shape[0]) + keep).floor()).type(torch.bool).numpy()
    new_idx, new_vals = O.dropedge(idx, vals, mask, keep)
    t_idx = torch.from_numpy(idx)[:, torch.from_numpy(mask)]
    t_vals = torch.from_numpy(vals)[torch.from_numpy(mask)] / keep
    assert np.array_equal(t_idx.numpy(), new_idx)
    assert np.array_equal(t_vals.numpy().view(np.uint32), new_vals.view(np.uint32))
    return dict(indices=idx, values=vals, mask=mask, keep=np.array(keep, np.float32),
                new_indices=new_idx, new_values=new_vals)


def structure_fixture(rng):
    """Unsorted COO with duplicates → CSR (stable) and CSC (rows ascending per column)."""
    rows = rng.integers(0, 30, size=300)
    cols = rng.integers(0, 20, size=300)
    vals = rng.standard_normal(300).astype(np.float32)
    rowptr, col, v, _ = O.csr_from_coo(rows, cols, 30, vals)
    colptr, rows_t, vt, _ = O.transpose_csr(rowptr, col, 20, v)
    heavy, cptr, ch = O.split_plan(rowptr, 12, 4)
    return dict(rows=rows, cols=cols, vals=vals, rowptr=rowptr, col=col, val=v, colptr=colptr,
                rows_t=rows_t, val_t=vt, heavy=heavy, heavy_cptr=cptr, chunk_heavy=ch)


def hgconv2_fixture():
    rows, cols = O.synthetic_incidence(500, 120, 4000, seed=0)
    rng = np.random.default_rng(3)
    X = rng.standard_normal((500, 32)).astype(np.float32)
    dY = rng.standard_normal((500, 32)).astype(np.float32)
    Y = O.two_hop(rows, cols, None, (500, 120), X, "sym", "mean", "sym")
    dX = O.two_hop_backward(rows, cols, None, (500, 120), Y, dY, "sym", "mean", "sym")
    H = ref_cpu.coo_tensor(rows, cols, None, (500, 120))
    Yt, dXt = ref_cpu.hgconv2_fwd_bwd(H, torch.from_numpy(X), torch.from_numpy(dY))
    _check(Yt.numpy(), Y, O.two_hop(rows, cols, None, (500, 120), np.abs(X), "sym", "mean",
                                     "sym"), "hgconv2 vs torch")
    _check(dXt.numpy(), dX, O.two_hop(rows, cols, None, (500, 120), np.abs(dY), "sym", "mean",
                                       "sym"), "hgconv2 bwd vs torch")
    return dict(rows=rows, cols=cols, shape=np.array([500, 120]), X=X, dY=dY, Y=Y, dX=dX)


def hccf_fixture(rng):
    """HCCFEncoder.forward at keep_rate=1, dropout off (HCCF.py:173-191)."""
    u, i, U, I = interactions(rng, 30, 24, 240)
    A = O.normalize_graph_mat(O.bipartite_adjacency(u, i, U, I))
    idx, vals = O.coo_of(A)
    d, K = 16, 8
    E_u = (rng.standard_normal((U, d)) * 0.1).astype(np.float32)
    E_i = (rng.standard_normal((I, d)) * 0.1).astype(np.float32)
    W_u = (rng.standard_normal((d, K)) * 0.1).astype(np.float32)
    W_i = (rng.standard_normal((d, K)) * 0.1).astype(np.float32)
    ue, ie, gcns, hyps = O.hccf_forward(idx[0], idx[1], vals, U + I, E_u, E_i, W_u, W_i, 2)
    return dict(indices=idx, values=vals, n_users=np.array(U), n_items=np.array(I), E_u=E_u,
                E_i=E_i, W_u=W_u, W_i=W_i, user_emb=ue, item_emb=ie, gcn0=gcns[0],
                gcn1=gcns[1], hyp0=hyps[0], hyp1=hyps[1])


def main():
    rng = np.random.default_rng(2024)
    fixtures = {
        "toy_hgconv2": toy_hgconv2(),
        "hgcn_conv": hgcn_fixture(rng),
        "edhnn": edhnn_fixture(rng),
        "dropedge": dropedge_fixture(rng),
        "structure": structure_fixture(rng),
        "hgconv2": hgconv2_fixture(),
        "hccf": hccf_fixture(rng),
    }
    for name, arrs in fixtures.items():
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **arrs)
        print(f"wrote {path} ({os.path.getsize(path)} bytes)")


if __name__ == "__main__":
    main()
