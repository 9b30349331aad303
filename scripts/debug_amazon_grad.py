"""Localises a gradient mismatch of the LocalAwareEncoder at the Amazon shape: each device
component (Linear, LayerNorm, mean two-hop, fused HGCN two-hop + LN + residual) forward and
backward against float64 torch, at d = 128 and the same sizes; prints the worst row ratio."""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import hgd_oracle as O  # noqa: E402
from tests import _ref64 as R  # noqa: E402
from hypergraph_diffusion_for_recommendation_amd import functional as FN  # noqa: E402
from hypergraph_diffusion_for_recommendation_amd.incidence import Incidence  # noqa: E402
from hypergraph_diffusion_for_recommendation_amd.layers import LayerNorm, Linear  # noqa: E402

dev = torch.device("cuda:0")
U, I, nnz = 52_643, 91_599, 2_240_000
d = int(sys.argv[1]) if len(sys.argv) > 1 else 128
N = U + I
rows, cols = O.synthetic_incidence(U, I, nnz, seed=30)
ui = O.bipartite_adjacency(rows, cols, U, I)
A = O.normalize_graph_mat(ui)
g = torch.Generator().manual_seed(0)
X = torch.randn(N, d, generator=g) * 0.1
G = torch.randn(N, d, generator=g)


def report(name, got, ref):
    try:
        r = R.check_rows(got, ref, name, tol=1.0)
    except AssertionError as e:
        print(name, "FAIL", e)
        return
    print(f"{name:40s} worst row ratio {r:.3e}", flush=True)


def run(name, fn_dev, fn_ref, extra_params=()):
    x = X.to(dev).requires_grad_(True)
    y = fn_dev(x)
    y.backward(G.to(dev))
    xr = X.double().requires_grad_(True)
    yr = fn_ref(xr)
    gr = torch.autograd.grad(yr, [xr] + [p for _, p in extra_params], G.double())
    report(name + " fwd", y, yr)
    report(name + " dX", x.grad, gr[0])
    for (pname, _), gp in zip(extra_params, gr[1:]):
        report(f"{name} d{pname}", pname_dev[pname].grad, gp)


torch.manual_seed(1)
lin = Linear(d, d).to(dev)
ln = LayerNorm(d).to(dev)
with torch.no_grad():
    ln.weight.uniform_(0.5, 1.5)
    ln.bias.uniform_(-0.2, 0.2)
Wr = lin.weight.detach().cpu().double().requires_grad_(True)
br = lin.bias.detach().cpu().double().requires_grad_(True)
lwr = ln.weight.detach().cpu().double().requires_grad_(True)
lbr = ln.bias.detach().cpu().double().requires_grad_(True)
pname_dev = {"W": lin.weight, "b": lin.bias, "gamma": ln.weight, "beta": ln.bias}

run("linear", lambda x: lin(x), lambda x: F.linear(x, Wr, br), [("W", Wr), ("b", br)])
lin.zero_grad()
run("linear+relu", lambda x: lin(x, relu=True), lambda x: F.relu(F.linear(x, Wr, br)),
    [("W", Wr), ("b", br)])
run("layernorm", lambda x: ln(x), lambda x: F.layer_norm(x, (d,), lwr, lbr, 1e-5),
    [("gamma", lwr), ("beta", lbr)])
ln.zero_grad()

c = ui.tocsr().copy()
c.sort_indices()
coo = c.tocoo()
V, E = torch.from_numpy(coo.row.astype(np.int64)), torch.from_numpy(coo.col.astype(np.int64))
inc = Incidence.from_index_lists(V.to(dev), E.to(dev), N, N)
me, mv = R.ui_mean_operators(ui, N)
run("mean2hop", lambda x: FN.mean2hop(inc, x),
    lambda x: torch.sparse.mm(mv, torch.sparse.mm(me, x)))

Ac = A.tocoo()
idx = torch.from_numpy(np.stack([Ac.row, Ac.col]).astype(np.int64))
val = torch.from_numpy(Ac.data.astype(np.float32))
torch.manual_seed(5)
di, dv = R.drop_edge_reference(idx, val, 0.8)
adj = R.sparse(di, dv, (N, N))
adj_t = adj.t().coalesce()
incA = Incidence.from_coo(di.to(dev), dv.to(dev), (N, N))
res = torch.randn(N, d, generator=g)
run("hgcn two-hop", lambda x: FN.two_hop(incA, x),
    lambda x: torch.sparse.mm(adj, torch.sparse.mm(adj_t, x)))
ln.zero_grad()
run("hgcn two-hop + LN + res (fused)",
    lambda x: FN.two_hop_fused(incA, x, norm=ln, res1=x, res1_scale=1.0),
    lambda x: F.layer_norm(torch.sparse.mm(adj, torch.sparse.mm(adj_t, x)), (d,), lwr, lbr,
                           1e-5) + x, [("gamma", lwr), ("beta", lbr)])
