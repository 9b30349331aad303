"""torch-CPU restatement of the reference path — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

Uses the very library calls the reference makes (paths relative to
/root/reference/HD_SELFRec), so it doubles as the ``cpu_baseline`` (kind "port") of bench.py
and as a second, independent cross-check of ``oracle/hgd_oracle.py``:

* COO built like TorchGraphInterface.convert_sparse_mat_to_tensor (base/torch_interface.py:8-12)
* hops with ``torch.sparse.mm`` (GCNLayer HCCF.py:199; HGCNConv HGNN_HD4.py:459-462, which
  re-derives ``adj.t()`` per call)
* torch_scatter's mean restated as ``index_reduce_(..., 'mean', include_self=False)``
  (EquivSetConv2.py:89,93 — torch_scatter itself is not installed here)
* backward by autograd, as in the reference training loop (HCCF.py:93-96).

Never imported by the product package.
"""
from __future__ import annotations

import torch


def coo_tensor(rows, cols, vals, shape):
    i = torch.stack([torch.as_tensor(rows, dtype=torch.int64),
                     torch.as_tensor(cols, dtype=torch.int64)])
    v = (torch.ones(i.shape[1], dtype=torch.float32) if vals is None
         else torch.as_tensor(vals, dtype=torch.float32))
    return torch.sparse_coo_tensor(i, v, tuple(shape))


def degree_scale(idx, n, power, weights=None):
    deg = torch.zeros(n, dtype=torch.float32)
    deg.index_add_(0, torch.as_tensor(idx, dtype=torch.int64),
                   torch.ones(len(idx)) if weights is None else weights)
    s = torch.pow(deg, power)
    s[torch.isinf(s)] = 0.0
    return s


def hgconv2(H: torch.Tensor, X: torch.Tensor, dv=None, de=None) -> torch.Tensor:
    """D_v^-1/2·H·D_e^-1·Hᵀ·D_v^-1/2·X with torch.sparse.mm (data/graph.py:28-42 operator);
    H is a sparse COO [V, E]. Autograd flows to X."""
    Hi = H._indices()
    if dv is None:
        dv = degree_scale(Hi[0], H.shape[0], -0.5)
    if de is None:
        de = degree_scale(Hi[1], H.shape[1], -1.0)
    M = torch.sparse.mm(H.t(), X * dv[:, None]) * de[:, None]
    return torch.sparse.mm(H, M) * dv[:, None]


def hgcn_conv(adj: torch.Tensor, X: torch.Tensor, act=True, slope=0.5) -> torch.Tensor:
    """HGCNConv.forward (HGNN_HD4.py:455-462): leaky(A·(Aᵀ·X)) or no activation."""
    Y = torch.sparse.mm(adj, torch.sparse.mm(adj.t(), X))
    return torch.nn.functional.leaky_relu(Y, slope) if act else Y


def scatter_mean(src: torch.Tensor, index: torch.Tensor, dim_size=None) -> torch.Tensor:
    n = dim_size if dim_size is not None else int(index.max()) + 1
    out = torch.zeros((n, src.shape[1]), dtype=src.dtype)
    return out.index_reduce_(0, index, src, "mean", include_self=False)


def equivset_mean_2hop(X: torch.Tensor, V: torch.Tensor, E: torch.Tensor, N: int):
    """EquivSetConv2.forward core (layers2/EquivSetConv2.py:88-93)."""
    Xe = scatter_mean(X[V], E)
    return scatter_mean(Xe[E], V, dim_size=N)


def hgconv2_fwd_bwd(H: torch.Tensor, X: torch.Tensor, dY: torch.Tensor):
    """One fwd+bwd of the benchmarked op on CPU; returns (Y, dX)."""
    X = X.detach().requires_grad_(True)
    Y = hgconv2(H, X)
    (dX,) = torch.autograd.grad(Y, X, dY)
    return Y.detach(), dX


def equivset_conv(X, vertex, edges, X0, W1, W2, W, alpha, aggr="mean"):
    """EquivSetConv.forward (layers2/EquivSetConv2.py:85-100) with torch ops on CPU; W1/W2/W are
    callables (W2 None = the ``X[..., in_features:]`` slice of mlp2_layers = 0)."""
    N = X.shape[-2]

    def scatter(src, index, dim_size=None):
        n = dim_size if dim_size is not None else int(index.max()) + 1
        out = torch.zeros((n, src.shape[1]), dtype=src.dtype)
        if aggr == "mean":
            return out.index_reduce_(0, index, src, "mean", include_self=False)
        return out.index_add_(0, index, src)

    Xve = W1(X)[..., vertex, :]
    Xe = scatter(Xve, edges)
    Xev = Xe[..., edges, :]
    cat = torch.cat([X[..., vertex, :], Xev], -1)
    Xev = cat[..., X.shape[-1]:] if W2 is None else W2(cat)
    Xv = scatter(Xev, vertex, dim_size=N)
    X = (1 - alpha) * Xv + alpha * X0
    return W(X)


def contrast_loss(embeds1: torch.Tensor, embeds2: torch.Tensor, nodes: torch.Tensor, temp):
    """contrastLoss (util/loss_torch.py:103-110) with the reference's own torch calls; run in
    float64 on the host it is the oracle for hgd_infonce_* (values and, via autograd, grads)."""
    F = torch.nn.functional
    embeds1 = F.normalize(embeds1 + 1e-8, p=2)
    embeds2 = F.normalize(embeds2 + 1e-8, p=2)
    pck1 = embeds1[nodes]
    pck2 = embeds2[nodes]
    nume = torch.exp(torch.sum(pck1 * pck2, dim=-1) / temp)
    deno = torch.exp(pck1 @ pck2.T / temp).sum(-1) + 1e-8
    return -torch.log(nume / deno).mean()


# ---------------------------------------------------------------------------------------------
# HCCF training step with the reference's own torch calls (device-agnostic; GPU tests run it on
# the device as the plugin-level oracle) — model/graph/HCCF.py:61-97, 163-226, util/loss_torch.py
# ---------------------------------------------------------------------------------------------
def bpr_loss(user_emb, pos_item_emb, neg_item_emb):
    """util/loss_torch.py:5-9."""
    pos_score = torch.mul(user_emb, pos_item_emb).sum(dim=1)
    neg_score = torch.mul(user_emb, neg_item_emb).sum(dim=1)
    return torch.mean(-torch.log(10e-6 + torch.sigmoid(pos_score - neg_score)))


def sp_adj_drop_edge(adj, keep_rate):
    """SpAdjDropEdge.forward (HCCF.py:217-226): CPU torch.rand(nnz) mask, kept values / keep."""
    if keep_rate == 1.0:
        return adj
    vals = adj._values()
    idxs = adj._indices()
    mask = ((torch.rand(vals.size()) + keep_rate).floor()).type(torch.bool)
    return torch.sparse_coo_tensor(idxs[:, mask.to(idxs.device)],
                                   vals[mask.to(vals.device)] / keep_rate, adj.shape)


class HCCFEncoderRef(torch.nn.Module):
    """HCCFEncoder.forward (HCCF.py:173-191) with torch.sparse.mm / torch.mm, parameter names
    of the reference (and of encoders.HCCFEncoder, so a state_dict moves between them)."""

    def __init__(self, n_users, n_items, latent, hyper_dim, n_layers, drop_rate, sparse_adj):
        super().__init__()
        self.n_users, self.n_layers = n_users, n_layers
        self.adj = sparse_adj
        dev = sparse_adj.device
        self.embedding_dict = torch.nn.ParameterDict({
            'user_emb': torch.nn.Parameter(torch.empty(n_users, latent, device=dev)),
            'item_emb': torch.nn.Parameter(torch.empty(n_items, latent, device=dev)),
            'user_w': torch.nn.Parameter(torch.empty(latent, hyper_dim, device=dev)),
            'item_w': torch.nn.Parameter(torch.empty(latent, hyper_dim, device=dev)),
        })
        self.drop_out = torch.nn.Dropout(drop_rate)

    def forward(self, keep_rate=0.5):
        nu = self.n_users
        e = self.embedding_dict
        hidden = [torch.cat([e['user_emb'], e['item_emb']], 0)]
        gcn_hidden, hgnn_hidden = [], []
        hyper_uu = e['user_emb'] @ e['user_w']
        hyper_ii = e['item_emb'] @ e['item_w']
        for _ in range(self.n_layers):
            gcn = torch.sparse.mm(sp_adj_drop_edge(self.adj, keep_rate), hidden[-1])
            hu = self.drop_out(hyper_uu)
            hi = self.drop_out(hyper_ii)
            hyper_u = torch.mm(hu, torch.mm(hu.T, hidden[-1][:nu]))
            hyper_i = torch.mm(hi, torch.mm(hi.T, hidden[-1][nu:]))
            gcn_hidden.append(gcn)
            hgnn_hidden.append(torch.cat([hyper_u, hyper_i], 0))
            hidden.append(gcn + hgnn_hidden[-1])
        emb = sum(hidden)
        return emb[:nu], emb[nu:], gcn_hidden, hgnn_hidden


def hccf_losses(n_users, n_layers, ancs, poss, negs, gcn, hyper, temp, ss_rate):
    """HCCF.calcLosses (HCCF.py:61-70): BPR + ss_rate · Σ_layers InfoNCE(users) + InfoNCE(items)
    over torch.unique(emb.long()) node lists."""
    ssl = 0
    for i in range(n_layers):
        e1, e2 = gcn[i].detach(), hyper[i]
        ssl += contrast_loss(e1[:n_users], e2[:n_users], torch.unique(ancs.long()), temp) \
            + contrast_loss(e1[n_users:], e2[n_users:], torch.unique(poss.long()), temp)
    return bpr_loss(ancs, poss, negs), ssl * ss_rate
