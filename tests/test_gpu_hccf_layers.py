"""GPU: HCCF's layer loop as one op (functional.hccf_layers, model/graph/HCCF.py:173-191) and the
three store extensions it rides on.

* hgd_sum_slices is bitwise the chain of adds ``sum(hidden)`` makes;
* hgd_spmm_masked_fused over an edge-dropped view stores the bare hop through act_out bitwise
  equal to hgd_spmm_masked, hop + res1 + res2 (res2 aliasing the output) bitwise equal to the
  adds, and the second output sum_out = Y + sum_res;
* HCCFEncoder with the fused loop gives bitwise the forward of the per-layer module graph
  (same hops, same products, same add and sum orders) and the same gradients up to the order
  of autograd's accumulations, for the capture-safe masked drop-edge and the reference's CPU
  drop-edge stream, with nn dropout on. Parity against the float64 reference at the configs'
  shapes is tests/test_gpu_config_parity.py (which runs this fused path).
"""
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O

pytestmark = pytest.mark.gpu


def _norm_adj(U, I, nnz, seed):
    rows, cols = O.synthetic_incidence(U, I, nnz, seed=seed)
    return O.normalize_graph_mat(O.bipartite_adjacency(rows, cols, U, I))


def test_sum_slices_is_the_chain_of_adds(dev):
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    g = torch.Generator(device=dev).manual_seed(0)
    for S, n in ((1, 64), (4, 1000 * 64), (4, 4099), (3, 5)):
        stride = (n + 3) // 4 * 4
        P = torch.randn(S, stride, device=dev, generator=g)
        out = torch.empty(n, device=dev)
        nat.check(nat.load().hgd_sum_slices(P.data_ptr(), S, stride, n, out.data_ptr(),
                                            torch.cuda.current_stream().cuda_stream), "sum")
        ref = P[0, :n].clone()
        for s in range(1, S):
            ref = ref + P[s, :n]
        assert torch.equal(out, ref), (S, n)


def test_masked_fused_hop_stores(dev):
    from hypergraph_diffusion_for_recommendation_amd.encoders import sparse_tensor_of
    from hypergraph_diffusion_for_recommendation_amd.functional import _res_epilogue
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_csr
    from hypergraph_diffusion_for_recommendation_amd.layers import SpAdjDropEdge
    A = _norm_adj(900, 1300, 20_000, seed=3)
    adj = sparse_tensor_of(A, dev)
    torch.manual_seed(5)
    view = SpAdjDropEdge(device_rng=True, capture_safe=True)(adj, 0.6)
    N = A.shape[0]
    for d in (32, 64, 128):
        X = torch.randn(N, d, device=dev)
        res = torch.randn(N, d, device=dev)
        for csr, val in ((view.csr, view.val), (view.csc, view.val_t)):
            plain = spmm_csr(csr, X, val=val)
            act = torch.empty_like(plain)
            y = spmm_csr(csr, X, val=val, ex=_res_epilogue(res, act_out=act))
            assert torch.equal(act, plain), d
            assert torch.equal(y, plain + res), d
            # in place: res2 is the output buffer itself; second output y + sres
            r2 = torch.randn(N, d, device=dev)
            buf = r2.clone()
            sres = torch.randn(N, d, device=dev)
            sout = torch.empty_like(buf)
            spmm_csr(csr, X, val=val, ex=_res_epilogue(res, res2=buf, sum_res=sres,
                                                       sum_out=sout), out=buf)
            assert torch.equal(buf, (plain + res) + r2), d
            assert torch.equal(sout, buf + sres), d


def _encoder(dev, A, U, I, d, L, capture_safe, fused):
    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFEncoder
    data = SimpleNamespace(n_users=U, n_items=I, norm_adj=A)
    kw = dict(lrate=1e-3, lr_decay=0.9, max_epoch=1, batch_size=256, reg=0.01,
              embedding_size=d, hyper_dim=32, drop_rate=0.25, p=0.3, n_layers=L)
    torch.manual_seed(0)
    enc = HCCFEncoder(kw, data, device=dev).train()
    enc.fused_layers = fused
    if capture_safe:
        enc.edgeDropper.device_rng = True
        enc.edgeDropper.capture_safe = True
    return enc


def _run(enc, dev, U, I, seed):
    """Forward + a loss touching every output (the sum, every gcn_k — not detached here, so its
    gradient path is exercised too — and every hgnn_k through the paired InfoNCE), backward."""
    from hypergraph_diffusion_for_recommendation_amd.functional import (contrast_loss_pair,
                                                                         unique_long_n)
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)
    ue, ie, gcn, hyp = enc(keep_rate=0.7)
    g = torch.Generator(device=dev).manual_seed(seed)
    N = U + I
    W = torch.randn(N, ue.shape[1], device=dev, generator=g)
    loss = (torch.cat([ue, ie]) * W).sum()
    uid = torch.randint(0, U, (300,), device=dev, generator=g)
    pid = torch.randint(0, I, (300,), device=dev, generator=g)
    (un, uc), (pn, pc) = unique_long_n(uid), unique_long_n(pid)
    for k, (e1, e2) in enumerate(zip(gcn, hyp)):
        loss = loss + 0.3 * contrast_loss_pair(e1.detach(), e2, U, un, pn, 0.5, uc, pc)
        loss = loss + 1e-3 * (e1 * W).sum() * (k + 1)
    loss.backward()
    grads = {k: p.grad.clone() for k, p in enc.named_parameters()}
    return [ue.detach(), ie.detach()] + [t.detach() for t in gcn + hyp], float(loss), grads


@pytest.mark.parametrize("capture_safe", [True, False])
@pytest.mark.parametrize("L", [1, 3])
def test_fused_layers_match_module_graph(dev, capture_safe, L):
    U, I, d = 1500, 2200, 64
    A = _norm_adj(U, I, 40_000, seed=11)
    outs = {}
    for fused in (False, True):
        enc = _encoder(dev, A, U, I, d, L, capture_safe, fused)
        outs[fused] = _run(enc, dev, U, I, seed=7)
    (o0, l0, g0), (o1, l1, g1) = outs[False], outs[True]
    for a, b in zip(o0, o1):
        assert torch.equal(a, b)  # same kernels, same sums in the same order
    assert abs(l0 - l1) <= 1e-6 * abs(l0)
    for k in g0:
        a, b = g0[k], g1[k]
        scale = float(a.abs().max())
        err = float((a - b).abs().max())
        assert err <= 1e-5 * scale, (k, err, scale)


@pytest.mark.parametrize("capture_safe", [True, False])
@pytest.mark.parametrize("L", [1, 3])
def test_fused_hyper_dropouts_are_the_module_dropouts(dev, capture_safe, L):
    """functional.hyper_dropouts (the 2L hypergraph dropouts as one node, the backward summed in
    one hgd_masked_scale_sum launch) against one nn.Dropout node per layer and table: outputs,
    loss and every parameter gradient bitwise equal — the same masks from the device generator,
    and the same sums in autograd's accumulation order."""
    U, I, d = 1500, 2200, 64
    A = _norm_adj(U, I, 40_000, seed=12)
    outs = {}
    for fused in (False, True):
        enc = _encoder(dev, A, U, I, d, L, capture_safe, True)
        enc.fused_dropouts = fused
        outs[fused] = _run(enc, dev, U, I, seed=9)
    (o0, l0, g0), (o1, l1, g1) = outs[False], outs[True]
    for a, b in zip(o0, o1):
        assert torch.equal(a, b)
    assert l0 == l1
    for k in g0:
        assert torch.equal(g0[k], g1[k]), (k, float((g0[k] - g1[k]).abs().max()))


@pytest.mark.parametrize("d,K", [(64, 32), (32, 32), (128, 64)])
def test_table_projections_match_float64(dev, d, K):
    """functional.table_projections ([E_u·W_u, E_i·W_i] grouped, HCCF.py:178-179) against
    float64: outputs and every gradient within 1e-5 of each row's scale (Σ|terms|), and two runs
    bitwise equal."""
    from hypergraph_diffusion_for_recommendation_amd.functional import table_projections
    shapes = ((31_668, d), (38_048, d))
    runs = []
    for _ in range(2):
        g = torch.Generator(device=dev).manual_seed(d + K)
        Es = [torch.randn(s, device=dev, generator=torch.Generator(device=dev).manual_seed(s[0]))
              .requires_grad_(True) for s in shapes]
        Ws = [(0.1 * torch.randn(d, K, device=dev, generator=torch.Generator(device=dev)
                                 .manual_seed(s[0] + 1))).requires_grad_(True) for s in shapes]
        Hs = table_projections(Es, Ws)
        dHs = [torch.randn(H.shape, device=dev, generator=g) for H in Hs]
        torch.autograd.backward(Hs, dHs)
        runs.append((Es, Ws, Hs, dHs))
    (E0, W0, H0, _), (E1, W1, H1, dH1) = runs
    for a, b in zip(H0 + [e.grad for e in E0] + [w.grad for w in W0],
                    H1 + [e.grad for e in E1] + [w.grad for w in W1]):
        assert torch.equal(a, b)
    for E, W, H, dH in zip(E1, W1, H1, dH1):
        E64, W64, dH64 = E.detach().double(), W.detach().double(), dH.double()
        checks = ((H, E64 @ W64, E64.abs() @ W64.abs()),
                  (E.grad, dH64 @ W64.t(), dH64.abs() @ W64.abs().t()),
                  (W.grad, E64.t() @ dH64, E64.abs().t() @ dH64.abs()))
        for got, ref, mag in checks:
            err = (got.double() - ref).abs()
            assert bool((err <= 1e-5 * mag.max(1, keepdim=True).values + 1e-30).all()), \
                float((err / (mag + 1e-30)).max())


def test_fused_layers_eval_and_no_grad(dev):
    """keep_rate 1 (the eval forward, HCCF.py:103) under no_grad: same tables as the loop."""
    U, I, d = 700, 900, 32
    A = _norm_adj(U, I, 10_000, seed=2)
    res = []
    for fused in (False, True):
        enc = _encoder(dev, A, U, I, d, 2, True, fused).eval()
        with torch.no_grad():
            ue, ie, gcn, hyp = enc(keep_rate=1)
        res.append([ue, ie] + gcn + hyp)
    for a, b in zip(*res):
        assert torch.equal(a, b)
    assert np.isfinite(res[1][0].cpu().numpy()).all()


@pytest.mark.parametrize("d", [12, 16, 32, 64, 128, 256])
def test_bpr_loss_rows_matches_torch(dev, d):
    """functional.bpr_loss_rows (hgd_bpr_*) against util/loss_torch.py:5-9 on the gathers of
    HCCF.py:84-86 in float64: loss within 1e-6 relative, the table gradient row-bound
    (1e-5 · Σ|terms| of each row), the gathered rows bitwise; a small table makes most rows
    repeat within the batch (the summed-duplicates path); two runs are bitwise equal."""
    g = torch.Generator(device=dev).manual_seed(d)
    for U, I, B in ((300, 500, 4096), (31_668, 38_048, 4096), (5, 3, 64)):
        uid = torch.randint(0, U, (B,), device=dev, generator=g)
        pid = torch.randint(0, I, (B,), device=dev, generator=g)
        nid = torch.randint(0, I, (B,), device=dev, generator=g)
        _check_bpr_rows(dev, g, d, U, I, uid, pid, nid)


@pytest.mark.parametrize("d", [12, 64, 256])
def test_bpr_loss_rows_skewed_batch(dev, d):
    """A skewed catalogue's batch (bench_plugin_epoch's Zipf-1.2 items: one item is the positive
    of ~18 % of the rows, far more repeats than a row's LDS list holds): the same bounds and
    determinism on the list-scan path. (Its speed — the round-3 fallback took 45 ms per call
    here — is a benchmark's business: scripts/bench_plugin_epoch.py's Zipf epoch.)"""
    g = torch.Generator(device=dev).manual_seed(100 + d)
    U, I, B = 31_668, 38_048, 4096
    uid = torch.randint(0, U, (B,), device=dev, generator=g)
    pid = torch.randint(0, I, (B,), device=dev, generator=g)
    hot = torch.rand(B, device=dev, generator=g) < 0.18
    pid = torch.where(hot, torch.zeros_like(pid), pid)           # item 0: ~740 positives
    nid = torch.randint(0, I, (B,), device=dev, generator=g)
    nid[: B // 8] = 1                                             # item 1: 512 negatives
    uid[B // 2: B // 2 + 300] = 7                                 # user 7: 300 anchors
    _check_bpr_rows(dev, g, d, U, I, uid, pid, nid)


@pytest.mark.parametrize("d", [12, 64, 256])
def test_bpr_loss_rows_repeat_counts_around_the_list_bound(dev, d):
    """Rows repeated 7, 8, 9, 10, 64 and 65 times (the walked lists end at 8; more goes to the
    one-workgroup-per-row kernel), an item that is both a positive and a negative, and a batch
    of 5,000 (its 15,000 positions cross the heavy kernel's 4,096-position windows inside the
    positives): the same bounds and determinism."""
    g = torch.Generator(device=dev).manual_seed(7 + d)
    U, I, B = 2_000, 3_000, 5_000
    uid = torch.randint(0, U, (B,), device=dev, generator=g)
    pid = torch.randint(0, I, (B,), device=dev, generator=g)
    nid = torch.randint(0, I, (B,), device=dev, generator=g)
    at = 0
    for row, reps in ((11, 7), (12, 8), (13, 9), (14, 10), (15, 64), (16, 65)):
        uid[at:at + reps] = row
        pid[at + 100:at + 100 + reps] = row
        nid[at + 3000:at + 3000 + reps] = row + 1000
        at += reps
    nid[4000:4040] = 16  # item 16: 65 positives and 40 negatives
    _check_bpr_rows(dev, g, d, U, I, uid, pid, nid)


def _check_bpr_rows(dev, g, d, U, I, uid, pid, nid):
    from hypergraph_diffusion_for_recommendation_amd.functional import bpr_loss_rows
    B = uid.numel()
    E = (0.3 * torch.randn(U + I, d, device=dev, generator=g)).requires_grad_(True)
    ue, ie = torch.split(E, [U, I])
    outs = []
    for _ in range(2):
        loss, anc, pos = bpr_loss_rows(ue, ie, uid, pid, nid)
        (gE,) = torch.autograd.grad(2.5 * loss, E)
        outs.append((loss.detach(), anc, pos, gE))
    assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[1]))
    loss, anc, pos, gE = outs[0]
    assert torch.equal(anc, E.detach()[uid]) and torch.equal(pos, E.detach()[U + pid])
    E64 = E.detach().double().cpu().requires_grad_(True)
    u64, i64 = torch.split(E64, [U, I])
    a, p, n = u64[uid.cpu()], i64[pid.cpu()], i64[nid.cpu()]
    ps, ns = (a * p).sum(1), (a * n).sum(1)
    ref = torch.mean(-torch.log(1e-5 + torch.sigmoid(ps - ns)))
    (gR,) = torch.autograd.grad(2.5 * ref, E64)
    assert abs(float(loss) - float(ref)) <= 1e-6 * abs(float(ref)), (float(loss), float(ref))
    # Σ|terms| of each gradient row: the same chain on |·| (|coef| ≤ 1/B · 2.5)
    a_, p_, n_ = a.detach().abs(), p.detach().abs(), n.detach().abs()
    mag = torch.zeros_like(E64)
    w = 2.5 / B
    mag.index_add_(0, uid.cpu(), w * (p_ + n_))
    mag.index_add_(0, U + pid.cpu(), w * a_)
    mag.index_add_(0, U + nid.cpu(), w * a_)
    err = (gE.double().cpu() - gR).abs()
    assert bool((err <= 1e-5 * mag + 1e-30).all()), float((err / (mag + 1e-30)).max())
