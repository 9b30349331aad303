"""GPU: the CF/KG encoders of the KG carriers (HGNN_cp / KHGRec SelfAwareEncoder and
RelationalAwareEncoder, HD's ED-HNN SelfAwareEncoder) against CPU restatements with the
reference's torch calls and the same parameters (deep-copied modules on the host):

* SelfAwareEncoder (HGNN_cp.py:394-411): per layer lns[k](leaky(A·(Aᵀ·x))) + res on an
  edge-dropped (non-symmetric) A, no activation on the last layer — forward and, with the
  UGformer off (no dropout left in the encoder), the gradients of the input and every parameter;
  with the UGformer on, forward in eval mode.
* RelationalAwareEncoder (HGNN_cp.py:426-446) on a rectangular adjacency, forward + backward.
* SelfAwareEncoderHD (HD.py:461-487): edhnn_layers[0] for layers 0..L-2, edhnn_layers[1] for the
  last, each on V/E = nonzero(norm_adj > 0) plus the layer-0 residual, eval mode.

The restatements run in float64 (deep-copied modules cast to double). Bound: tests/_ref64.check_rows
— every row (an embedding, a gradient row, a whole γ/β gradient vector) within 1e-5 of that row's
largest |ref|, no absolute floor; 1e-4 with the UGformer (its attention is the library's
float32 kernel on our side, float64 on the reference side)."""
import copy
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O
from oracle import ref_cpu
from tests import _ref64 as R
from tests._util import random_coo

pytestmark = pytest.mark.gpu


def _graph(seed, U=60, I=45, nnz=400):
    rng = np.random.default_rng(seed)
    u, i = random_coo(rng, U, I, nnz)
    ui = O.bipartite_adjacency(u, i, U, I)
    A = O.normalize_graph_mat(ui)
    return SimpleNamespace(n_users=U, n_items=I, norm_adj=A, ui_adj=ui)


def _dropped_cpu(A, keep, seed):
    """A sparse COO with a fixed subset of edges kept and scaled by 1/keep (a SpAdjDropEdge
    draw, HCCF.py:217-226, fixed so both sides see the same matrix)."""
    idx, vals = O.coo_of(A)
    m = np.random.default_rng(seed).random(len(vals)) < keep
    return ref_cpu.coo_tensor(idx[0][m], idx[1][m], np.asarray(vals)[m] / keep, A.shape)


def _close(got, ref, tol=R.TOL, what="value"):
    R.check_rows(torch.as_tensor(got), torch.as_tensor(ref), what, tol)


def _ln(x, ln):
    return torch.nn.functional.layer_norm(x, (x.shape[1],), ln.weight, ln.bias, ln.eps)


def _self_aware_ref(ec, x, adj, res):
    """HGNN_cp.py:394-411 with torch.sparse.mm."""
    for k in range(ec.layers):
        if ec.use_self_att:
            x = ec.ugformer_layers[k](x.unsqueeze(1)).squeeze(1)
        last = k == ec.layers - 1
        x = _ln(ref_cpu.hgcn_conv(adj, x, act=not last, slope=ec.leaky), ec.lns[k]) + res
    return x


def test_self_aware_encoder_fwd_bwd(dev):
    from hypergraph_diffusion_for_recommendation_amd.encoders import SelfAwareEncoder
    data = _graph(3)
    d = 16
    torch.manual_seed(0)
    enc = SelfAwareEncoder(data, d, d, 3, 0.1, 0.2, device=dev, use_self_att=False)
    with torch.no_grad():
        for ln in enc.lns:  # non-trivial affine so the γ/β gradients are checked
            ln.weight.uniform_(0.5, 1.5)
            ln.bias.uniform_(-0.2, 0.2)
    adj_c = _dropped_cpu(data.norm_adj, 0.7, seed=5)
    ego = torch.randn(data.n_users + data.n_items, d)
    w = torch.randn_like(ego)
    xg = ego.to(dev).requires_grad_(True)
    ue, ie = enc(xg, adj_c.to(dev))
    (torch.cat([ue, ie]) * w.to(dev)).sum().backward()

    ec = copy.deepcopy(enc).cpu().double()
    for p in ec.parameters():
        p.grad = None
    xc = ego.double().requires_grad_(True)
    ref = _self_aware_ref(ec, xc, adj_c.double(), xc)
    (ref * w.double()).sum().backward()
    _close(torch.cat([ue, ie]).detach().cpu(), ref.detach())
    _close(xg.grad.cpu(), xc.grad)
    n_checked = 0
    for (n, p), (_, pc) in zip(enc.named_parameters(), ec.named_parameters()):
        if pc.grad is not None:
            assert p.grad is not None, n
            _close(p.grad.cpu(), pc.grad, what=f"d {n}")
            n_checked += 1
    assert n_checked == 2 * 3  # γ and β of every layer's LayerNorm


def test_self_aware_encoder_ugformer_eval(dev):
    from hypergraph_diffusion_for_recommendation_amd.encoders import SelfAwareEncoder
    data = _graph(4)
    d = 16
    torch.manual_seed(1)
    enc = SelfAwareEncoder(data, d, d, 2, 0.1, 0.2, device=dev).eval()
    assert enc.use_self_att  # HGNN_cp's default
    adj_c = _dropped_cpu(data.norm_adj, 1.0, seed=0)
    ego = torch.randn(data.n_users + data.n_items, d)
    with torch.no_grad():
        ue, ie = enc(ego.to(dev), adj_c.to(dev))
        ref = _self_aware_ref(copy.deepcopy(enc).cpu().double().eval(), ego.double(),
                              adj_c.double(), ego.double())
    _close(torch.cat([ue, ie]).cpu(), ref, tol=1e-4)


def test_relational_aware_encoder(dev):
    from hypergraph_diffusion_for_recommendation_amd.encoders import RelationalAwareEncoder
    rng = np.random.default_rng(7)
    n_ent, n_cols, d = 90, 40, 16
    r, c = random_coo(rng, n_ent, n_cols, 500)
    vals = (rng.random(len(r)) + 0.1).astype(np.float32)
    kg_c = ref_cpu.coo_tensor(r, c, vals, (n_ent, n_cols))
    torch.manual_seed(2)
    enc = RelationalAwareEncoder(0.2, 0.1, 2, d).to(dev)
    x = torch.randn(n_ent, d)
    w = torch.randn_like(x)
    xg = x.to(dev).requires_grad_(True)
    out = enc(xg, kg_c.to(dev), None)
    (out * w.to(dev)).sum().backward()
    ec = copy.deepcopy(enc).cpu().double()
    xc = x.double().requires_grad_(True)
    y = xc
    for k in range(2):
        y = _ln(ref_cpu.hgcn_conv(kg_c.double(), y, act=k != 1, slope=0.2), ec.lns[k]) + xc
    (y * w.double()).sum().backward()
    _close(out.detach().cpu(), y.detach())
    _close(xg.grad.cpu(), xc.grad)


def test_self_aware_encoder_hd_eval(dev):
    from hypergraph_diffusion_for_recommendation_amd.encoders import SelfAwareEncoderHD
    data = _graph(5)
    d = 16
    torch.manual_seed(3)
    enc = SelfAwareEncoderHD(data, d, d, 3, 0.3, 0.2, device=dev).eval()
    ego = torch.randn(data.n_users + data.n_items, d)
    with torch.no_grad():
        ue, ie = enc(ego.to(dev), enc.sparse_norm_adj)
    ec = copy.deepcopy(enc).cpu().double().eval()
    idx, vals = O.coo_of(data.norm_adj)
    adj = ref_cpu.coo_tensor(idx[0], idx[1], vals, data.norm_adj.shape).coalesce().double()
    keep = adj._values() > 0  # nonzero(norm_adj > 0), row-major
    V, E = adj._indices()[0][keep], adj._indices()[1][keep]
    x = ego = ego.double()
    with torch.no_grad():
        for k in range(3):
            blk = ec.edhnn_layers[0 if k != 2 else 1]
            h = torch.relu(torch.nn.functional.linear(x, blk.lin_in.weight, blk.lin_in.bias))
            h = ref_cpu.equivset_conv(h, V, E, h, blk.conv.W1, None, blk.conv.W, 0.0, "mean")
            x = torch.relu(h) + ego
    _close(torch.cat([ue, ie]).cpu(), x)
