"""GPU: the drop-in layer modules against CPU restatements of the reference modules."""
import copy

import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O
from oracle import ref_cpu
from tests import _ref64 as R
from tests._util import random_coo

pytestmark = pytest.mark.gpu

EDHNN_ARGS = {  # LocalAwareEncoder.init_edhnn_config, HGNN_HD4.py:371-388
    'MLP_hidden': 32, 'MLP1_num_layers': 0, 'MLP2_num_layers': 0, 'MLP3_num_layers': 1,
    'MLP_num_layers': 0, 'restart_alpha': 0.0, 'aggregate': 'mean', 'dropout': 0.5,
    'normalization': 'ln', 'input_norm': True, 'All_num_layers': 1, 'activation': 'relu',
    'input_dropout': 0.6, 'AllSet_input_norm': True}


def _ui(rng, U, I, n):
    u, i = random_coo(rng, U, I, n)
    return O.bipartite_adjacency(u, i, U, I)


def test_equivset_gnn_eval_matches_reference(dev):
    from hypergraph_diffusion_for_recommendation_amd.layers import EquivSetGNN
    rng = np.random.default_rng(0)
    ui = _ui(rng, 120, 80, 900)
    N = ui.shape[0]
    dense = torch.tensor(ui.todense(), dtype=torch.float32)  # the reference passes this (CPU)
    torch.manual_seed(0)
    m = EquivSetGNN(32, EDHNN_ARGS, dense).to(dev).eval()
    x = torch.randn(N, 32)
    y = m(x.to(dev), dense, N)
    # float64 CPU restatement with the same parameters; every row within 1e-5 (tests/_ref64.py)
    mc = copy.deepcopy(m).cpu().double().eval()
    nz = torch.nonzero(dense > 0)
    V, E = nz[:, 0], nz[:, 1]
    h = torch.relu(mc.lin_in(x.double()))
    h = ref_cpu.equivset_conv(h, V, E, h, mc.conv.W1, None, mc.conv.W, 0.0, "mean")
    ref = torch.relu(h)
    R.check_rows(y, ref, "EquivSetGNN")
    Vg, Eg = m.generate_V_E(N, dense)
    assert torch.equal(Vg.cpu(), V) and torch.equal(Eg.cpu(), E)


@pytest.mark.parametrize("aggr", ["mean", "add"])
@pytest.mark.parametrize("mlp2", [0, 1])
def test_equivset_conv_paths(dev, aggr, mlp2):
    from hypergraph_diffusion_for_recommendation_amd.layers import EquivSetConv
    rng = np.random.default_rng(5 + mlp2)
    ui = _ui(rng, 70, 50, 500)
    N = ui.shape[0]
    nz = torch.nonzero(torch.tensor(ui.todense()) > 0)
    V, E = nz[:, 0].contiguous(), nz[:, 1].contiguous()
    torch.manual_seed(1)
    conv = EquivSetConv(16, 16, mlp1_layers=1, mlp2_layers=mlp2, mlp3_layers=1, aggr=aggr,
                        alpha=0.3, normalization='ln', input_norm=True).to(dev).eval()
    X = torch.randn(N, 16)
    X0 = torch.randn(N, 16)
    Xg = X.to(dev).requires_grad_(True)
    y = conv(Xg, V.to(dev), E.to(dev), X0.to(dev))
    y.sum().backward()
    cc = copy.deepcopy(conv).cpu().double().eval()
    Xc = X.double().requires_grad_(True)
    ref = ref_cpu.equivset_conv(Xc, V, E, X0.double(), cc.W1, cc.W2, cc.W, 0.3, aggr)
    ref.sum().backward()
    R.check_rows(y, ref, "EquivSetConv")
    R.check_rows(Xg.grad, Xc.grad, "d X")


def test_spadj_dropedge_layer_bit_exact(dev):
    from hypergraph_diffusion_for_recommendation_amd.layers import GCNLayer, SpAdjDropEdge
    rng = np.random.default_rng(3)
    A = O.normalize_graph_mat(_ui(rng, 90, 60, 800))
    idx, vals = O.coo_of(A)
    adj = torch.sparse_coo_tensor(torch.from_numpy(idx), torch.from_numpy(vals), A.shape)
    torch.manual_seed(11)
    out = SpAdjDropEdge()(adj.to(dev), 0.7)
    torch.manual_seed(11)
    mask = ((torch.rand(vals.shape[0]) + 0.7).floor()).type(torch.bool)
    ref_idx, ref_vals = O.dropedge(idx, vals, mask.numpy(), 0.7)
    assert np.array_equal(out._indices().cpu().numpy(), ref_idx)
    assert np.array_equal(out._values().cpu().numpy().view(np.uint32), ref_vals.view(np.uint32))
    X = rng.standard_normal((A.shape[0], 16)).astype(np.float32)
    y = GCNLayer(0.5)(out, torch.from_numpy(X).to(dev)).cpu().numpy()
    ref = O.spmm_coo(ref_idx[0], ref_idx[1], ref_vals, A.shape[0], X)
    mag = O.spmm_coo(ref_idx[0], ref_idx[1], np.abs(ref_vals), A.shape[0], np.abs(X))
    assert np.all(np.abs(y - ref) <= 1e-5 * mag + 1e-30)
    assert SpAdjDropEdge()(adj, 1.0) is adj


def test_hgnn_layer_dense(dev):
    from hypergraph_diffusion_for_recommendation_amd.layers import HGNNLayer
    H = torch.randn(100, 8, device=dev)
    X = torch.randn(100, 16, device=dev)
    y = HGNNLayer(0.5)(H, X)
    Hd, Xd = H.double(), X.double()
    ref = Hd @ (Hd.T @ Xd)
    mag = Hd.abs() @ (Hd.abs().T @ Xd.abs())  # Σ|terms| of the two products
    assert ((y.double() - ref).abs() <= 1e-5 * mag).all()


@pytest.mark.parametrize("mlp2", [0, 1])
def test_spmm_form_equivset_gnn(dev, mlp2):
    """SpMM-form ED-HNN (model/layers/EquivSetGNN.py / EquivSetConv.py) vs a CPU restatement
    with torch.sparse.mm HGCNConv, eval mode, fwd + grad."""
    from hypergraph_diffusion_for_recommendation_amd.edhnn_spmm import EquivSetGNN
    rng = np.random.default_rng(7 + mlp2)
    A = O.normalize_graph_mat(_ui(rng, 70, 50, 600))
    N = A.shape[0]
    idx, vals = O.coo_of(A)
    adj = torch.sparse_coo_tensor(torch.from_numpy(idx), torch.from_numpy(vals), A.shape)
    args = dict(EDHNN_ARGS, MLP_hidden=16, MLP2_num_layers=mlp2, MLP1_num_layers=0)
    torch.manual_seed(2)
    m = EquivSetGNN(16, args).to(dev).eval()
    x = torch.randn(N, 16)
    xg = x.to(dev).requires_grad_(True)
    y = m(xg, adj.to(dev), N)
    y.square().sum().backward()
    mc = copy.deepcopy(m).cpu().double().eval()
    adj64 = adj.double()
    xc = x.double().requires_grad_(True)
    h = torch.relu(mc.lin_in(xc))
    c = mc.conv
    Xve = c.W1(h)
    Xe = c.lns[0](ref_cpu.hgcn_conv(adj64, Xve, act=True, slope=0.2)) + Xve
    Xev = Xe if c.W2 is None else c.W2(torch.cat([h, Xe], -1))
    Xv = c.lns[1](ref_cpu.hgcn_conv(adj64, Xev, act=True, slope=0.2)) + Xev
    ref = torch.relu(c.W((1 - c.alpha) * Xv + c.alpha * h))
    ref.square().sum().backward()
    R.check_rows(y, ref, "SpMM-form EquivSetGNN")
    R.check_rows(xg.grad, xc.grad, "d x")


def test_hgcnconv_dense_adjacency_dhcf(dev):
    """DHCF passes a dense [U, I] interaction matrix to HGCNConv (DHCF.py:124-140)."""
    from hypergraph_diffusion_for_recommendation_amd.layers import HGCNConv
    rng = np.random.default_rng(9)
    U, I, d = 60, 45, 16
    Ad = (rng.random((U, I)) < 0.1).astype(np.float32)
    X = rng.standard_normal((U, d)).astype(np.float32)
    A = torch.from_numpy(Ad).to(dev)
    Xg = torch.from_numpy(X).to(dev).requires_grad_(True)
    y = HGCNConv(0.3)(A, Xg, act=True)
    y.sum().backward()
    At = torch.from_numpy(Ad).double()
    Xc = torch.from_numpy(X).double().requires_grad_(True)
    ref = torch.nn.functional.leaky_relu(At @ (At.T @ Xc), 0.3)
    ref.sum().backward()
    R.check_rows(y, ref, "HGCNConv(dense A)")
    R.check_rows(Xg.grad, Xc.grad, "d X")
    r, c = np.nonzero(Ad)
    inc = A._hgd_incidence
    np.testing.assert_array_equal(inc.csr.col.cpu().numpy(), c)


def test_equivset_fused_epilogue_matches_unfused(dev):
    """fused_epilogue True (hgd_spmm_fused) vs False (the reference's separate ops) for both
    ED-HNN forms, fwd + parameter grads, training-mode dropout off."""
    from hypergraph_diffusion_for_recommendation_amd import edhnn_spmm
    from hypergraph_diffusion_for_recommendation_amd.layers import EquivSetGNN
    rng = np.random.default_rng(11)
    A = O.normalize_graph_mat(_ui(rng, 80, 60, 700))
    N = A.shape[0]
    idx, vals = O.coo_of(A)
    adj = torch.sparse_coo_tensor(torch.from_numpy(idx), torch.from_numpy(vals), A.shape).to(dev)
    H = torch.from_numpy((np.asarray(A.todense()) > 0).astype(np.float32)).to(dev)
    args = dict(EDHNN_ARGS, MLP_hidden=32, MLP2_num_layers=0, dropout=0.0, input_dropout=0.0,
                restart_alpha=0.3)
    x = torch.randn(N, 32, device=dev)
    for build, call in (
            (lambda: edhnn_spmm.EquivSetGNN(32, args), lambda m, xx: m(xx, adj, N)),
            (lambda: EquivSetGNN(32, args, H), lambda m, xx: m(xx, H, N))):
        torch.manual_seed(4)
        m = build().to(dev)
        outs = []
        for fused in (True, False):
            m.conv.fused_epilogue = fused
            m.zero_grad()
            xx = x.clone().requires_grad_(True)
            y = call(m, xx)
            y.square().sum().backward()
            outs.append([y.detach(), xx.grad] + [p.grad.clone() for p in m.parameters()
                                                  if p.grad is not None])
        for a, b in zip(*outs):
            s = b.abs().max().item() + 1e-6
            assert (a - b).abs().max().item() <= 5e-5 * s


@pytest.mark.parametrize("n,K,d", [(31_668, 32, 64), (1000, 16, 32), (77, 48, 128)])
def test_hgnn_layer_dense_two_hop(dev, n, K, d):
    """HGNNLayer (HCCF.py:201-211) on the MFMA kernels vs float64: output and grads of H, X."""
    from hypergraph_diffusion_for_recommendation_amd.layers import HGNNLayer
    torch.manual_seed(n)
    H = (torch.randn(n, K) * 0.2).to(dev).requires_grad_(True)
    X = torch.randn(n, d).to(dev).requires_grad_(True)
    dY = torch.randn(n, d).to(dev)
    Y = HGNNLayer(0.5)(H, X)
    gH, gX = torch.autograd.grad(Y, (H, X), dY)
    Hd = H.detach().double().cpu().requires_grad_(True)
    Xd = X.detach().double().cpu().requires_grad_(True)
    Yd = Hd @ (Hd.T @ Xd)
    rH, rX = torch.autograd.grad(Yd, (Hd, Xd), dY.double().cpu())
    # |err| <= 1e-5 · Σ|terms| element-wise, Σ|terms| from the same products on |·|:
    #   Y = H·(Hᵀ·X)                  -> |H|·(|H|ᵀ·|X|)
    #   dX = H·(Hᵀ·dY)                -> |H|·(|H|ᵀ·|dY|)
    #   dH = dY·Mᵀ + X·dMᵀ, M = HᵀX,  -> |dY|·(|H|ᵀ|X|)ᵀ + |X|·(|H|ᵀ|dY|)ᵀ
    #        dM = HᵀdY                   (the inner reductions' own terms expanded)
    aH, aX, adY = Hd.abs().detach(), Xd.abs().detach(), dY.double().cpu().abs()
    mag = aH @ (aH.T @ aX)
    assert ((Y.detach().double().cpu() - Yd.detach()).abs() <= 1e-5 * mag + 1e-300).all()
    mag_dX = aH @ (aH.T @ adY)
    mag_dH = adY @ (aH.T @ aX).T + aX @ (aH.T @ adY).T
    for g, r, m, what in ((gH, rH, mag_dH, "dH"), (gX, rX, mag_dX, "dX")):
        err = (g.double().cpu() - r).abs()
        assert (err <= 1e-5 * m + 1e-300).all(), (what, float((err / m).max()))


@pytest.mark.parametrize("nu,ni,K,d", [(31_668, 38_048, 32, 64), (300, 1000, 16, 32),
                                        (5, 77, 48, 128)])
def test_dense_two_hop_pair(dev, nu, ni, K, d):
    """HCCF's user + item HGNNLayer pair of a layer as one grouped op
    (functional.dense_two_hop_pair: hgd_gemm_tn / hgd_gemm_rows over both halves, output and
    table gradient in place) vs float64: output, dX and both dH at the 1e-5·Σ|terms| bound."""
    from hypergraph_diffusion_for_recommendation_amd.functional import dense_two_hop_pair
    torch.manual_seed(nu + ni)
    Hu = (torch.randn(nu, K) * 0.2).to(dev).requires_grad_(True)
    Hi = (torch.randn(ni, K) * 0.2).to(dev).requires_grad_(True)
    X = torch.randn(nu + ni, d).to(dev).requires_grad_(True)
    dY = torch.randn(nu + ni, d).to(dev)
    Y = dense_two_hop_pair(Hu, Hi, X, nu)
    gHu, gHi, gX = torch.autograd.grad(Y, (Hu, Hi, X), dY)
    adY = dY.double().cpu().abs()
    for H, gH, sl in ((Hu, gHu, slice(0, nu)), (Hi, gHi, slice(nu, nu + ni))):
        Hd = H.detach().double().cpu()
        Xd = X.detach().double().cpu()[sl]
        dYd = dY.double().cpu()[sl]
        Yd = Hd @ (Hd.T @ Xd)
        rX = Hd @ (Hd.T @ dYd)
        rH = dYd @ (Hd.T @ Xd).T + Xd @ (Hd.T @ dYd).T
        aH, aX, ad = Hd.abs(), Xd.abs(), adY[sl]
        checks = ((Y.detach().double().cpu()[sl], Yd, aH @ (aH.T @ aX), "Y"),
                  (gX.double().cpu()[sl], rX, aH @ (aH.T @ ad), "dX"),
                  (gH.double().cpu(), rH, ad @ (aH.T @ aX).T + aX @ (aH.T @ ad).T, "dH"))
        for got, ref, mag, what in checks:
            err = (got - ref).abs()
            assert (err <= 1e-5 * mag + 1e-300).all(), (what, float((err / mag).max()))


def test_equivset_gnn_fresh_learned_hypergraph_each_call(dev):
    """HCCF_diffusion.py:205-206 feeds EquivSetGNN a NEW dense learned hypergraph
    (dropout(E·W) [n, K]) every call: each call must use that call's nonzero pattern, even when the
    allocator / Python hand the new tensor the address / id() of a freed predecessor."""
    from hypergraph_diffusion_for_recommendation_amd.layers import EquivSetGNN
    args = dict(EDHNN_ARGS, MLP_hidden=16, dropout=0.0, input_dropout=0.0)
    torch.manual_seed(0)
    m = EquivSetGNN(16, args).to(dev).eval()
    n, K = 300, 32
    x = torch.randn(n, 16, device=dev)
    for step in range(4):
        g = torch.Generator(device=dev).manual_seed(step)
        H = torch.randn(n, K, device=dev, generator=g)  # new tensor, likely the same address
        y = m(x, H, n)
        r, c = torch.nonzero(H > 0, as_tuple=True)
        # this call's pattern, float64 (α = 0): mean over each hyperedge, then over each vertex
        md = copy.deepcopy(m).cpu().double()
        hd = torch.relu(md.lin_in(x.cpu().double()))
        me = R.mean_operator(c.cpu().numpy(), r.cpu().numpy(), K, n)
        mv = R.mean_operator(r.cpu().numpy(), c.cpu().numpy(), n, K)
        ref64 = md.act(md.conv.W(torch.sparse.mm(mv, torch.sparse.mm(me, md.conv.W1(hd)))))
        R.check_rows(y, ref64, f"call {step}")
        del H
