"""CPU: calibration of the encoder-level parity bound (tests/_ref64.py check_rows) before any
GPU test relies on it. The reference encoders of tests/_ref64.py are evaluated in float32 — the
precision the reference itself runs in — and in float64:

* the float32 evaluation meets ``check_rows`` (every row within 1e-5 of its scale) for outputs
  and every gradient, so the bound does not demand more than fp32 arithmetic of the same
  operations delivers. Measured worst rows: forward embeddings ~5e-7 (a 20x margin); gradient
  rows ~1e-6 through the ED-HNN stack, but up to ~6.5e-6 through HCCF's BPR + InfoNCE losses
  and the learned-hypergraph products — fp32 gradient rows that sum many signed terms come
  within 1.5x of the bound, so 1e-5 is the tightest row bound fp32 arithmetic itself meets;
* an error of 2e-5 of one row's scale is rejected, so the bound is not vacuous;
* the weight gradients (reductions over all node rows) also meet ``check_weight_grad``.
"""
import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O
from tests import _ref64 as R

U, I, D = 90, 60, 16


def _graph():
    rows, cols = O.synthetic_incidence(U, I, 900, seed=0)
    ui = O.bipartite_adjacency(rows, cols, U, I)
    return ui, O.normalize_graph_mat(ui)


def _local_aware_params(rng, n_layers):
    P = {}
    for k in range(n_layers - 1):
        pre = f"edhnn_layers.{k}."
        P[pre + "lin_in.weight"] = rng.standard_normal((D, D)) / 4
        P[pre + "lin_in.bias"] = rng.standard_normal(D) / 4
        P[pre + "conv.W.normalizations.0.weight"] = 1 + rng.standard_normal(D) / 10
        P[pre + "conv.W.normalizations.0.bias"] = rng.standard_normal(D) / 10
        P[pre + "conv.W.lins.0.weight"] = rng.standard_normal((D, D)) / 4
        P[pre + "conv.W.lins.0.bias"] = rng.standard_normal(D) / 4
    P["lns.0.weight"] = 1 + rng.standard_normal(D) / 10
    P["lns.0.bias"] = rng.standard_normal(D) / 10
    return P


def _local_aware(dtype, n_layers=3):
    rng = np.random.default_rng(1)
    ui, A = _graph()
    N = U + I
    P = {k: torch.from_numpy(v).to(dtype).requires_grad_(True)
         for k, v in _local_aware_params(rng, n_layers).items()}
    ego = torch.from_numpy(rng.standard_normal((N, D)) / 8).to(dtype).requires_grad_(True)
    mean_e, mean_v = R.ui_mean_operators(ui, N, dtype)
    idx, vals = O.coo_of(A)
    adj = R.sparse(idx, vals, (N, N), dtype)
    g = torch.Generator().manual_seed(3)
    masks = [torch.empty(N, D).bernoulli_(0.5, generator=g) for _ in range(3 * (n_layers - 1))]
    probe = R.Probe()
    out = R.local_aware(ego, P, n_layers, mean_e, mean_v, adj, masks, 0.5, 1e-5, probe=probe)
    G = torch.randn(N, D, generator=g, dtype=torch.float64).to(dtype)
    out.backward(G)
    grads = {"ego": ego.grad, **{k: v.grad for k, v in P.items()}}
    return out.detach(), grads, probe


def _hccf(dtype, n_layers=2, K=8):
    rng = np.random.default_rng(2)
    _, A = _graph()
    N = U + I
    E = {"embedding_dict.user_emb": rng.standard_normal((U, D)) / 8,
         "embedding_dict.item_emb": rng.standard_normal((I, D)) / 8,
         "embedding_dict.user_w": rng.standard_normal((D, K)) / 3,
         "embedding_dict.item_w": rng.standard_normal((D, K)) / 3}
    P = {k: torch.from_numpy(v).to(dtype).requires_grad_(True) for k, v in E.items()}
    idx, vals = O.coo_of(A)
    g = torch.Generator().manual_seed(4)
    adjs = []
    for _ in range(n_layers):
        keep = torch.rand(len(vals), generator=g) < 0.7
        adjs.append(R.sparse(idx[:, keep.numpy()], vals[keep.numpy()] / np.float32(0.7), (N, N),
                             dtype))
    masks = [torch.empty(n, K).bernoulli_(0.8, generator=g)
             for _ in range(n_layers) for n in (U, I)]
    ue, ie, gcn, hyp = R.hccf_encoder(P, adjs, masks, 0.8, U, n_layers)
    u = torch.randint(0, U, (64,), generator=g)
    i = torch.randint(0, I, (64,), generator=g)
    j = torch.randint(0, I, (64,), generator=g)
    loss = R.bpr_loss(ue[u], ie[i], ie[j])
    nodes = torch.arange(0, U, 4)
    for k in range(n_layers):
        loss = loss + 0.1 * R.contrast_loss(gcn[k][:U].detach(), hyp[k][:U], nodes, 1.0)
    names = list(P)
    grads = torch.autograd.grad(loss, [P[k] for k in names])
    return torch.cat([ue, ie]), loss, dict(zip(names, grads))


def test_fp32_local_aware_meets_the_row_bound():
    o64, g64, probe = _local_aware(torch.float64)
    o32, g32, _ = _local_aware(torch.float32)
    worst = R.check_rows(o32, o64, "forward")
    for k in g64:
        worst = max(worst, R.check_rows(g32[k], g64[k], f"d {k}"))
    print(f"fp32 LocalAware worst row ratio {worst:.2e}")
    assert worst < 5e-6
    # the weight gradients' reduction bound (check_weight_grad) holds too, with a wide margin
    wr = max(R.check_weight_grad(g32[k], g64[k], probe.uses[k], f"d {k}") for k in probe.uses)
    print(f"fp32 LocalAware worst weight-gradient reduction ratio {wr:.2e}")
    assert wr < 1e-6


def test_fp32_hccf_with_losses_meets_the_row_bound():
    o64, l64, g64 = _hccf(torch.float64)
    o32, l32, g32 = _hccf(torch.float32)
    assert R.check_rows(o32, o64, "forward") < 2e-6
    assert abs(float(l32) - float(l64)) <= R.TOL * abs(float(l64))
    worst = max(R.check_rows(g32[k], g64[k], f"d {k}") for k in g64)
    print(f"fp32 HCCF worst gradient row ratio {worst:.2e}")


def test_row_bound_rejects_an_error_above_it():
    o64, _, _ = _local_aware(torch.float64)
    bad = o64.detach().clone()
    bad[7, 3] += 2e-5 * bad[7].abs().max()
    with pytest.raises(AssertionError):
        R.check_rows(bad, o64, "perturbed")
    R.check_rows(o64 + 0.5e-5 * o64.abs().amax(1, keepdim=True), o64, "within")
