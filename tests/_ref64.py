"""The reference encoders and losses restated in float64 with the reference's own torch calls
(TEST INFRASTRUCTURE; never imported by the product package). Paths relative to
/root/reference/HD_SELFRec:

* :func:`hccf_encoder`    HCCFEncoder.forward, model/graph/HCCF.py:173-191 (+ HGNNLayer :201-211)
* :func:`edhnn_block`     EquivSetGNN.forward, model/layers/layers2/EquivSetGNN2.py:83-103 with
                          EquivSetConv2.forward :85-100 (mean aggregation, W1 = identity, W2 =
                          the edge-half slice, W = MLP 'ln' InputNorm, MLP.py:109-117)
* :func:`local_aware`     LocalAwareEncoder.forward, model/graph/HGNN_HD4.py:390-405 with
                          HGCNConv :450-462
* :func:`hccf_diffusion`  HCCFEncoder.forward of model/graph/HCCF_diffusion.py:173-215
* :func:`bpr_loss`, :func:`contrast_loss`  util/loss_torch.py:5-9, :103-110

Dropout masks and drop-edge structures are inputs (drawn once, fed to both sides: the
:class:`FixedDropout` and :class:`DropRecorder` here wrap the GPU encoders), so a comparison is
of the arithmetic alone.

The encoder-level bound (:func:`check_rows`): every row — one user's / item's embedding, one row
of a gradient — within 1e-5 relative of that row's largest magnitude (north_star: "fp32
embeddings within 1e-5 relative"), with no absolute floor. Why rows and not the element-wise
Σ|terms| of the single-hop tests: carried through L layers of hops, Linear, ReLU and LayerNorm,
the worst-case Σ|terms| compounds multiplicatively (LayerNorm alone scales it by |x|/σ per
layer) — measured on a 3-layer ED-HNN stack it admitted 1.5e-2 relative error, a vacuous bound.
The row bound is the tighter test; tests/test_ref64.py shows the reference's own float32
evaluation meets it with margin and that an error of 2e-5 of a row's scale is caught.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

TOL = 1e-5


# ---------------------------------------------------------------------------------------------
# draws shared by both sides
# ---------------------------------------------------------------------------------------------
class FixedDropout(nn.Module):
    """nn.Dropout(p) whose k-th call (in training mode) uses the k-th mask of a CPU generator
    seeded with ``seed``; the masks are kept (``self.masks``) for the reference side."""

    def __init__(self, p: float, seed: int):
        super().__init__()
        self.p = float(p)
        self.gen = torch.Generator().manual_seed(int(seed))
        self.masks: List[torch.Tensor] = []

    def forward(self, x):
        if not self.training or self.p == 0.0:
            return x
        m = torch.empty(tuple(x.shape)).bernoulli_(1.0 - self.p, generator=self.gen)
        self.masks.append(m)
        return x * m.to(x.device, x.dtype) / (1.0 - self.p)


class DropRecorder(nn.Module):
    """Wraps an SpAdjDropEdge; keeps every output's (indices, values) on the host."""

    def __init__(self, inner):
        super().__init__()
        self.inner = inner
        self.outputs = []

    def begin_step(self):
        begin = getattr(self.inner, "begin_step", None)
        if begin is not None:
            begin()

    def forward(self, adj, keep):
        out = self.inner(adj, keep)
        if getattr(out, "parent", None) is not None and hasattr(out.csr, "mask"):
            # a masked view (SpAdjDropEdge(capture_safe)): the kept entries of the parent COO
            # (CSR order), values / keep in float32 — what the compacted output holds
            m = out.csr.mask.bool().cpu()
            idx, vals = adj._indices().cpu(), adj._values().cpu()
            self.outputs.append((idx[:, m], vals[m] / keep))
        else:
            self.outputs.append((out._indices().cpu(), out._values().cpu()))
        return out


def drop_edge_reference(indices: torch.Tensor, values: torch.Tensor, keep: float):
    """SpAdjDropEdge.forward (HCCF.py:217-226): the CPU torch.rand mask on the default generator
    (caller seeds it), kept entries in order, values / keep in float32."""
    mask = ((torch.rand(values.size()) + keep).floor()).type(torch.bool)
    return indices[:, mask], values[mask] / keep


class ReluMasks:
    """The device's ReLU decisions, recorded in call order (:meth:`wrap_linear` for the fused
    ``Linear(..., relu=True)``, :meth:`module` for an ``nn.ReLU``), replayed by the reference's
    :func:`relu`. A ReLU's derivative at a pre-activation within fp32 rounding of zero is
    decided by that rounding (the reference's own fp32 run could go either way), so the
    reference takes the device's mask — after checking that every element where it disagrees
    with the float64 sign lies within TOL of zero relative to its row (``flips`` counts them)."""

    def __init__(self):
        self.masks: List[torch.Tensor] = []
        self.pos = 0
        self.flips = 0

    def wrap_linear(self, lin):
        orig = lin.forward

        def forward(x, relu=False):
            y = orig(x, relu)
            if relu:
                self.masks.append((y > 0).detach().cpu())
            return y

        lin.forward = forward

    def module(self) -> nn.Module:
        rec = self

        class _Relu(nn.Module):
            def forward(self, x):
                y = torch.relu(x)
                rec.masks.append((y > 0).detach().cpu())
                return y

        return _Relu()

    def take(self, x: torch.Tensor) -> torch.Tensor:
        m = self.masks[self.pos]
        self.pos += 1
        v = x.detach()
        flipped = (v > 0) != m
        if bool(flipped.any()):
            scale = v.abs().amax(-1, keepdim=True).expand_as(v)
            assert bool((v[flipped].abs() <= TOL * scale[flipped]).all()), \
                "device ReLU mask differs from the reference at a clearly signed element"
            self.flips += int(flipped.sum())
        return m


def relu(x: torch.Tensor, masks: "ReluMasks" = None) -> torch.Tensor:
    if masks is None:
        return F.relu(x)
    return x * masks.take(x).to(x.dtype)


def sparse(indices, values, shape, dtype=torch.float64) -> torch.Tensor:
    i = torch.as_tensor(np.asarray(indices), dtype=torch.int64)
    v = torch.as_tensor(np.asarray(values)).to(dtype)
    return torch.sparse_coo_tensor(i, v, tuple(shape)).coalesce()


def mean_operator(rows, cols, n_rows, n_cols, dtype=torch.float64) -> torch.Tensor:
    """D_r^-1·B for a binary B[rows, cols]: torch_scatter's mean of the rows gathered by
    ``cols`` into ``rows`` (empty rows stay 0)."""
    rows = np.asarray(rows, dtype=np.int64)
    cols = np.asarray(cols, dtype=np.int64)
    deg = np.bincount(rows, minlength=n_rows).astype(np.float64)
    return sparse(np.stack([rows, cols]), 1.0 / deg[rows], (n_rows, n_cols), dtype)


def ui_mean_operators(ui_csr, n: int, dtype=torch.float64):
    """V/E = nonzero(ui_adj > 0) (HGNN_HD4.py:367-369, row-major) as the two scatter means over
    the [n, n] pattern: Xe = scatter_mean(X[V], E), Xv = scatter_mean(Xe[E], V, dim_size=n)."""
    c = ui_csr.tocsr().copy()
    c.sort_indices()
    c.eliminate_zeros()
    coo = c.tocoo()
    V, E = coo.row.astype(np.int64), coo.col.astype(np.int64)
    return mean_operator(E, V, n, n, dtype), mean_operator(V, E, n, n, dtype)


def leaves(module: nn.Module, dtype=torch.float64) -> Dict[str, torch.Tensor]:
    """float64 (or ``dtype``) CPU copies of a module's parameters, requiring grad."""
    return {k: p.detach().cpu().to(dtype).requires_grad_(True)
            for k, p in module.named_parameters()}


# ---------------------------------------------------------------------------------------------
# encoders
# ---------------------------------------------------------------------------------------------
def hccf_encoder(P: Dict[str, torch.Tensor], adjs: List[torch.Tensor],
                 masks: List[torch.Tensor], keep_h: float, n_users: int, n_layers: int):
    """HCCF.py:173-191: per layer the GCN hop on the edge-dropped adjacency plus HGNNLayer's
    ``H·(Hᵀ·X)`` (:201-211) with H = dropout(E·W) for users and items; ``masks`` in call order
    (users then items, per layer)."""
    Eu, Ei = P["embedding_dict.user_emb"], P["embedding_dict.item_emb"]
    Wu, Wi = P["embedding_dict.user_w"], P["embedding_dict.item_w"]
    hidden = [torch.cat([Eu, Ei], 0)]
    gcn_l, hyp_l = [], []
    huu, hii = Eu @ Wu, Ei @ Wi
    for layer in range(n_layers):
        h = hidden[-1]
        gcn = torch.sparse.mm(adjs[layer], h)
        hu = huu * masks[2 * layer].to(h.dtype) / keep_h
        hi = hii * masks[2 * layer + 1].to(h.dtype) / keep_h
        hyp_u = hu @ (hu.T @ h[:n_users])
        hyp_i = hi @ (hi.T @ h[n_users:])
        gcn_l.append(gcn)
        hyp_l.append(torch.cat([hyp_u, hyp_i], 0))
        hidden.append(gcn + hyp_l[-1])
    emb = sum(hidden)
    return emb[:n_users], emb[n_users:], gcn_l, hyp_l


class Probe:
    """Records, per weight of the reference forward, every use's input and (grad-retaining)
    output, so that after ``backward`` (not ``autograd.grad``: the outputs' ``.grad`` must be
    populated) the weight gradient's bound can be formed from the reduction it is
    (:func:`check_weight_grad`). A weight shared between calls (HCCF_diffusion's one ED-HNN
    block, called for users and items in every layer) keeps every use."""

    def __init__(self):
        self.uses: Dict[str, list] = {}

    def _add(self, name, entry_w, entry_b):
        self.uses.setdefault(name + ".weight", []).append(entry_w)
        self.uses.setdefault(name + ".bias", []).append(entry_b)

    def linear(self, name: str, x, y):
        y.retain_grad()
        self._add(name, ("linear_w", x, y), ("bias", x, y))

    def layer_norm(self, name: str, x, y, eps: float):
        y.retain_grad()
        xd = x.detach()
        mu = xd.mean(-1, keepdim=True)
        xh = (xd - mu) * torch.rsqrt(xd.var(-1, unbiased=False, keepdim=True) + eps)
        self._add(name, ("ln_w", xh, y), ("bias", xh, y))


def _lin(x, P, name, probe):
    y = F.linear(x, P[name + ".weight"], P[name + ".bias"])
    if probe is not None:
        probe.linear(name, x, y)
    return y


def _ln(x, P, name, eps, probe):
    y = F.layer_norm(x, (x.shape[-1],), P[name + ".weight"], P[name + ".bias"], eps)
    if probe is not None:
        probe.layer_norm(name, x, y, eps)
    return y


def edhnn_block(x, P, prefix: str, mean_e, mean_v, masks: List[torch.Tensor], keep: float,
                ln_eps: float, relu_masks: ReluMasks = None, probe: Probe = None):
    """EquivSetGNN2.forward (:83-103) for HGNN_HD4's edhnn_config: dropout → ReLU(lin_in) →
    dropout → EquivSetConv (Xe = mean over each hyperedge's vertices, Xv = mean over each
    vertex's hyperedges, α = 0, W = Linear(LayerNorm(·))) → ReLU → dropout. ``masks``: the
    block's three dropout masks in call order (empty in eval mode)."""
    def drop(t, k):
        return t * masks[k].to(t.dtype) / keep if masks else t

    x = drop(x, 0)
    x = relu(_lin(x, P, prefix + "lin_in", probe), relu_masks)
    x = drop(x, 1)
    xv = torch.sparse.mm(mean_v, torch.sparse.mm(mean_e, x))
    W = prefix + "conv.W."
    xn = _ln(xv, P, W + "normalizations.0", ln_eps, probe)
    x = relu(_lin(xn, P, W + "lins.0", probe), relu_masks)
    return drop(x, 2)


def local_aware(ego, P, n_layers: int, mean_e, mean_v, adj, masks: List[torch.Tensor],
                keep: float, ln_eps: float, prefix: str = "", relu_masks: ReluMasks = None,
                probe: Probe = None):
    """LocalAwareEncoder.forward (HGNN_HD4.py:390-405): layers 0..L-2 ED-HNN blocks on V/E =
    nonzero(ui_adj) plus the layer-0 residual; the last LN0(A·(Aᵀ·x)) + residual (HGCNConv
    act=False, :450-462)."""
    res = ego
    adj_t = adj.t().coalesce()
    for k in range(n_layers):
        if k != n_layers - 1:
            ego = edhnn_block(ego, P, f"{prefix}edhnn_layers.{k}.", mean_e, mean_v,
                              masks[3 * k:3 * k + 3], keep, ln_eps, relu_masks, probe) + res
        else:
            z = torch.sparse.mm(adj, torch.sparse.mm(adj_t, ego))
            ego = _ln(z, P, prefix + "lns.0", ln_eps, probe) + res
    return ego


def nonzero_mean_operators(H: torch.Tensor, n_nodes: int):
    dtype = H.dtype
    """V/E = nonzero(H > 0) of a dense [n, K] learned hypergraph (EquivSetGNN2.generate_V_E,
    row-major) as the scatter means over its K hyperedges and n vertices."""
    nz = torch.nonzero(H > 0)
    V, E = nz[:, 0].numpy(), nz[:, 1].numpy()
    K = H.shape[1]
    return mean_operator(E, V, K, n_nodes, dtype), mean_operator(V, E, n_nodes, K, dtype)


def hccf_diffusion(P, adjs, hyper_masks, keep_h: float, blk_masks, keep_b: float, n_users: int,
                   n_layers: int, ln_eps: float, relu_masks: ReluMasks = None,
                   probe: Probe = None):
    """HCCF_diffusion.py:173-215: per layer the GCN hop plus one shared ED-HNN block on the
    learned hypergraphs dropout(E·W) of users and of items (V/E = nonzero(H > 0); the block
    sees only their structure). ``blk_masks``: 3 per block call, users then items."""
    Eu, Ei = P["embedding_dict.user_emb"], P["embedding_dict.item_emb"]
    Wu, Wi = P["embedding_dict.user_w"], P["embedding_dict.item_w"]
    hidden = [torch.cat([Eu, Ei], 0)]
    gcn_l, hyp_l = [], []
    huu, hii = (Eu @ Wu).detach(), (Ei @ Wi).detach()
    n_i = Ei.shape[0]
    for layer in range(n_layers):
        h = hidden[-1]
        gcn = torch.sparse.mm(adjs[layer], h)
        Hu = huu * hyper_masks[2 * layer].to(h.dtype) / keep_h
        Hi = hii * hyper_masks[2 * layer + 1].to(h.dtype) / keep_h
        eu, vu = nonzero_mean_operators(Hu, n_users)
        ei, vi = nonzero_mean_operators(Hi, n_i)
        bu = blk_masks[6 * layer:6 * layer + 3]
        bi = blk_masks[6 * layer + 3:6 * layer + 6]
        hyp_u = edhnn_block(h[:n_users], P, "edhnnlayer.", eu, vu, bu, keep_b, ln_eps,
                            relu_masks, probe)
        hyp_i = edhnn_block(h[n_users:], P, "edhnnlayer.", ei, vi, bi, keep_b, ln_eps,
                            relu_masks, probe)
        gcn_l.append(gcn)
        hyp_l.append(torch.cat([hyp_u, hyp_i], 0))
        hidden.append(gcn + hyp_l[-1])
    emb = sum(hidden)
    return emb[:n_users], emb[n_users:], gcn_l, hyp_l


# ---------------------------------------------------------------------------------------------
# losses (util/loss_torch.py)
# ---------------------------------------------------------------------------------------------
def bpr_loss(user_emb, pos_item_emb, neg_item_emb):
    """loss_torch.py:5-9."""
    pos_score = torch.mul(user_emb, pos_item_emb).sum(dim=1)
    neg_score = torch.mul(user_emb, neg_item_emb).sum(dim=1)
    return torch.mean(-torch.log(10e-6 + torch.sigmoid(pos_score - neg_score)))


def contrast_loss(embeds1, embeds2, nodes, temp):
    """contrastLoss, loss_torch.py:103-110."""
    embeds1 = F.normalize(embeds1 + 1e-8, p=2)
    embeds2 = F.normalize(embeds2 + 1e-8, p=2)
    pck1 = embeds1[nodes]
    pck2 = embeds2[nodes]
    nume = torch.exp(torch.sum(pck1 * pck2, dim=-1) / temp)
    deno = torch.exp(pck1 @ pck2.T / temp).sum(-1) + 1e-8
    return -torch.log(nume / deno).mean()


# ---------------------------------------------------------------------------------------------
# comparison
# ---------------------------------------------------------------------------------------------
def check_rows(got, ref, what: str, tol: float = TOL) -> float:
    """Every row of ``got`` within ``tol`` of the same row of ``ref`` relative to that row's
    largest |ref| (a 1-D tensor is one row). Returns the worst row's ratio."""
    g = got.detach().to(device="cpu", dtype=torch.float64)
    r = ref.detach().to(device="cpu", dtype=torch.float64)
    assert g.shape == r.shape, (what, tuple(g.shape), tuple(r.shape))
    if g.numel() == 0:
        return 0.0
    if g.dim() == 1:
        g, r = g[None], r[None]
    g, r = g.reshape(g.shape[0], -1), r.reshape(r.shape[0], -1)
    err = (g - r).abs().amax(1)
    scale = r.abs().amax(1)
    zero = scale == 0
    assert bool((err[zero] == 0).all()), f"{what}: nonzero result in an all-zero reference row"
    ratio = torch.where(zero, torch.zeros_like(err), err / torch.where(zero, 1.0, scale))
    worst = float(ratio.max())
    if worst > tol:
        k = int(ratio.argmax())
        raise AssertionError(f"{what}: row {k} off by {float(err[k]):.3e} at scale "
                             f"{float(scale[k]):.3e} (ratio {worst:.3e} > {tol:g}); "
                             f"{int((ratio > tol).sum())} / {ratio.numel()} rows out")
    return worst


def check_weight_grad(got, ref, entries, what: str, tol: float = TOL) -> float:
    """A weight gradient is a reduction over the N rows of (upstream gradient, op input) pairs:
    dW = Σ_n dY_nᵀ·X_n (Linear), dγ = Σ_n dY_n ⊙ x̂_n (LayerNorm), db = dβ = Σ_n dY_n. Its
    operands are row-bounded (every row within TOL of its scale, :func:`check_rows`), and the
    reduction's own fp32 rounding is at most a few ulp of Σ|terms| (blocked / split-K sums).
    So the element-wise bound is TOL times the first-order propagation of the operands' row
    errors through the sum — Σ_n (‖dY_n‖∞·|X_n| + |dY_n|·‖X_n‖∞) — which is ≥ Σ|terms| of the
    reduction. ``entries``: the (kind, input, output) records of every use of the weight (a
    block shared between calls contributes each call's terms)."""
    bound = None
    for kind, x, y in entries:
        dy = y.grad.detach()
        ax = x.detach().abs()
        sdy = dy.abs().amax(-1, keepdim=True)
        sx = ax.amax(-1, keepdim=True)
        if kind == "linear_w":
            b = sdy.expand_as(dy).T @ ax + dy.abs().T @ sx.expand_as(ax)
        elif kind == "ln_w":
            b = (sdy * ax + dy.abs() * sx).sum(0)
        else:  # bias / β
            b = sdy.expand_as(dy).sum(0)
        bound = b if bound is None else bound + b
    g = got.detach().to(device="cpu", dtype=torch.float64)
    r = ref.detach().to(torch.float64)
    assert g.shape == r.shape == bound.shape, (what, g.shape, r.shape, bound.shape)
    err = (g - r).abs()
    ratio = float((err / bound).max())
    if ratio > tol:
        i = tuple(int(k) for k in (err > tol * bound).nonzero()[0])
        raise AssertionError(f"{what}: element {i} off by {float(err[i]):.3e}, reduction bound "
                             f"{float(tol * bound[i]):.3e} (ratio {ratio:.3e} > {tol:g})")
    return ratio
