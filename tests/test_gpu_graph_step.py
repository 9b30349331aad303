"""GPU: the capture-safe pieces of a HIP-graph training step (graphs.py) and the captured HCCF
step itself.

* the device drop-edge mask drawn from a device seed (hgd_bernoulli_mask_dev) equals its host
  restatement (oracle device_keep_mask) bit for bit, and the capacity-sized dropped structure
  (Incidence.drop(capacity=True)) holds exactly the kept entries of the compacted one, with a
  zeroed tail, and hops over it identically;
* unique_long_n (device count) equals torch.unique(x.long()); contrast_loss with a device
  count equals the float64 reference (row bound, tests/_ref64.py);
* HCCF steps replayed from a captured graph take bitwise the same steps as the same capture-safe
  step run eagerly (same seeds, nn dropout off), and the eager capture-safe step matches the
  float64 reference (loss 1e-5 relative, gradient rows 1e-5);
* the HCCF_diffusion step (ED-HNN block on the dense learned hypergraph, its dropouts on the
  library RNG seeded from torch's device generator) replayed from a graph equals the same steps
  run eagerly — dropouts on;
* the HCCF plugin trains end to end in graph mode (hgd_graph).
"""
import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O
from tests import _ref64 as R

pytestmark = pytest.mark.gpu


def _graph(U, I, nnz, seed):
    rows, cols = O.synthetic_incidence(U, I, nnz, seed=seed)
    ui = O.bipartite_adjacency(rows, cols, U, I)
    return O.normalize_graph_mat(ui)


def test_device_seed_mask_and_capacity_drop(dev):
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd.encoders import sparse_tensor_of
    from hypergraph_diffusion_for_recommendation_amd.functional import spmm
    A = _graph(700, 900, 12_000, seed=1)
    adj = sparse_tensor_of(A, dev)
    parent = adj._hgd_incidence
    seed = torch.tensor([123456789], dtype=torch.int64, device=dev)
    mask = torch.empty(parent.nnz, dtype=torch.uint8, device=dev)
    nat.check(nat.load().hgd_bernoulli_mask_dev(seed.data_ptr(), parent.nnz, 0.7, mask.data_ptr(),
                                                torch.cuda.current_stream().cuda_stream), "m")
    ref_mask = O.device_keep_mask(123456789, parent.nnz, 0.7)
    assert np.array_equal(mask.cpu().numpy().astype(bool), ref_mask)
    cap = parent.drop(mask, 0.7, capacity=True)
    exact = parent.drop(mask, 0.7)
    k = exact.nnz
    assert cap.nnz == parent.nnz and int(cap.csr.rowptr[-1]) == k
    for a, b in ((cap.csr.rowptr, exact.csr.rowptr), (cap.csc.rowptr, exact.csc.rowptr)):
        assert torch.equal(a, b)
    for a, b in ((cap.csr.col, exact.csr.col), (cap.val, exact.val),
                 (cap.csc.col, exact.csc.col), (cap.val_t, exact.val_t)):
        assert torch.equal(a[:k], b) and not a[k:].any()
    # the kept entries are the reference COO filtered by the mask, values / keep in float32
    idx, vals = O.coo_of(A)
    ri, rv = O.dropedge(idx, vals, ref_mask, 0.7)
    rows = torch.repeat_interleave(torch.arange(A.shape[0]), exact.csr.rowptr.diff().cpu())
    assert np.array_equal(rows.numpy(), ri[0]) and np.array_equal(
        exact.csr.col.cpu().numpy(), ri[1])
    assert np.array_equal(exact.val.cpu().numpy().view(np.uint32), rv.view(np.uint32))
    X = torch.randn(A.shape[0], 32, device=dev, requires_grad=True)
    y1 = spmm(cap, X)
    y2 = spmm(exact, X)
    assert torch.equal(y1, y2)
    g = torch.randn_like(y1)
    assert torch.equal(torch.autograd.grad(y1, X, g)[0], torch.autograd.grad(y2, X, g)[0])


def test_paired_device_mask_is_the_csc_permutation(dev):
    """hgd_bernoulli_mask_dev_pair: the CSR-order mask equals hgd_bernoulli_mask_dev's and the
    CSC-order one equals it gathered through perm_t, bit for bit (the capture-safe drop's two
    masks from one draw)."""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd.encoders import sparse_tensor_of
    A = _graph(800, 1100, 15_000, seed=9)
    parent = sparse_tensor_of(A, dev)._hgd_incidence
    seed = torch.tensor([987654321], dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    m = torch.empty(parent.nnz, dtype=torch.uint8, device=dev)
    mt = torch.empty_like(m)
    ref = torch.empty_like(m)
    lib = nat.load()
    nat.check(lib.hgd_bernoulli_mask_dev_pair(seed.data_ptr(), parent.perm_t.data_ptr(),
                                              parent.nnz, 0.6, m.data_ptr(), mt.data_ptr(), st),
              "pair")
    nat.check(lib.hgd_bernoulli_mask_dev(seed.data_ptr(), parent.nnz, 0.6, ref.data_ptr(), st),
              "single")
    assert torch.equal(m, ref)
    assert torch.equal(mt, ref[parent.perm_t.long()])


@pytest.mark.parametrize("d", [64, 32, 7, 256])
def test_masked_view_hops_equal_compacted(dev, d):
    """Incidence.masked (hgd_spmm_masked: the dropped matrix as a view of its parent) against
    the compacted structure of the same mask (Incidence.drop): without split rows every hop is
    bit-identical (kept edges summed in edge order), forward (CSR) and backward (CSC, the mask
    gathered through perm_t), for the float4 widths, a scalar width (d = 7) and a multi-pass one
    (d = 256); the two-hop A·(Aᵀ·X) of HGCNConv too."""
    from hypergraph_diffusion_for_recommendation_amd.encoders import sparse_tensor_of
    from hypergraph_diffusion_for_recommendation_amd.functional import spmm, two_hop
    A = _graph(900, 1300, 20_000, seed=5)
    parent = sparse_tensor_of(A, dev)._hgd_incidence
    assert parent.csr.n_heavy == 0 and parent.csc.n_heavy == 0
    mask = torch.from_numpy(O.device_keep_mask(99, parent.nnz, 0.6).astype(np.uint8)).to(dev)
    view = parent.masked(mask, 0.6)
    exact = parent.drop(mask, 0.6)
    X = torch.randn(A.shape[0], d, device=dev, requires_grad=True)
    g = torch.randn(A.shape[0], d, device=dev)
    for tr in (False, True):
        yv, ye = spmm(view, X, transpose=tr), spmm(exact, X, transpose=tr)
        assert torch.equal(yv, ye)
        assert torch.equal(torch.autograd.grad(yv, X, g)[0], torch.autograd.grad(ye, X, g)[0])
    zv, ze = two_hop(view, X, None, None, None), two_hop(exact, X, None, None, None)
    assert torch.equal(zv, ze)
    assert torch.equal(torch.autograd.grad(zv, X, g)[0], torch.autograd.grad(ze, X, g)[0])
    with pytest.raises(NotImplementedError):
        view.scale("row", "sym")


def test_masked_view_with_split_rows(dev):
    """Rows longer than the split threshold keep the parent's split plan under a mask: chunk
    partials of the parent's 512-edge chunks (kept edges only), so sums agree with the compacted
    structure's to fp32 rounding of a different association (1e-5 of Σ|terms|), and with the
    float64 restatement of the dropped matrix."""
    from hypergraph_diffusion_for_recommendation_amd import Incidence
    from hypergraph_diffusion_for_recommendation_amd.functional import spmm
    rng = np.random.default_rng(3)
    rows = np.concatenate([np.zeros(6000, np.int64), rng.integers(1, 400, 8000)])
    cols = np.concatenate([np.arange(6000), rng.integers(0, 6000, 8000)])
    vals = rng.random(rows.size).astype(np.float32) + 0.5
    key = np.unique(rows * 6000 + cols, return_index=True)[1]
    rows, cols, vals = rows[key], cols[key], vals[key]
    inc = Incidence.from_coo(torch.from_numpy(np.stack([rows, cols])), torch.from_numpy(vals),
                             (400, 6000), device=dev)
    assert inc.csr.n_heavy >= 1
    m = (rng.random(rows.size) < 0.5).astype(np.uint8)
    view = inc.masked(torch.from_numpy(m), 0.5)
    X = torch.randn(6000, 64, device=dev)
    got = spmm(view, X).double().cpu().numpy()
    kv = (vals[m == 1] / np.float32(0.5)).astype(np.float64)
    Xd = X.double().cpu().numpy()
    ref = np.zeros((400, 64))
    mag = np.zeros((400, 64))
    np.add.at(ref, rows[m == 1], kv[:, None] * Xd[cols[m == 1]])
    np.add.at(mag, rows[m == 1], np.abs(kv[:, None] * Xd[cols[m == 1]]))
    assert np.all(np.abs(got - ref) <= 1e-5 * mag + 1e-30)


def test_unique_long_n_and_counted_contrast_loss(dev):
    from hypergraph_diffusion_for_recommendation_amd.functional import (contrast_loss,
                                                                         unique_long_n)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(4096, 8, device=dev, generator=g) * 40
    nodes, count = unique_long_n(x)
    ref = torch.unique(x.long())
    k = int(count)
    assert k == ref.numel() and torch.equal(nodes[:k], ref) and not nodes[k:].any()
    n, d = 300, 32
    e1 = torch.randn(n, d, device=dev, generator=g)
    e2 = torch.randn(n, d, device=dev, generator=g).requires_grad_(True)
    nodes, count = unique_long_n(torch.randint(-n, n, (512,), device=dev, generator=g))
    loss = contrast_loss(e1, e2, nodes, 0.5, count)
    (ge2,) = torch.autograd.grad(loss, e2)
    live = nodes[:int(count)].cpu()
    live = torch.where(live < 0, live + n, live)
    e2r = e2.detach().cpu().double().requires_grad_(True)
    lr = R.contrast_loss(e1.cpu().double(), e2r, live, 0.5)
    (gr,) = torch.autograd.grad(lr, e2r)
    assert abs(float(loss.detach()) - float(lr.detach())) <= 1e-5 * abs(float(lr.detach()))
    R.check_rows(ge2, gr, "d e2")


def _hccf(dev, drop_rate, seed=3):
    from types import SimpleNamespace

    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFEncoder
    U, I = 1500, 1200
    A = _graph(U, I, 30_000, seed=2)
    data = SimpleNamespace(n_users=U, n_items=I, norm_adj=A)
    kw = dict(lrate=1e-3, lr_decay=0.9, max_epoch=1, batch_size=256, reg=0.01,
              embedding_size=32, hyper_dim=32, drop_rate=drop_rate, p=0.3, n_layers=2)
    torch.manual_seed(seed)
    enc = HCCFEncoder(kw, data, device=dev)
    enc.edgeDropper.device_rng = True
    enc.edgeDropper.capture_safe = True
    return enc, U, I


def test_contrast_loss_pair_equals_two_calls(dev):
    """contrast_loss_pair (one op over both halves of the tables, one zeroed gradient table)
    against the two contrast_loss calls of HCCF.py:65-66 it replaces: the same loss bitwise and
    the same table gradients (each row is written by one half's scatter only)."""
    from hypergraph_diffusion_for_recommendation_amd.functional import (contrast_loss,
                                                                         contrast_loss_pair,
                                                                         unique_long_n)
    g = torch.Generator(device=dev).manual_seed(11)
    U, N, d = 700, 1900, 64
    E1 = torch.randn(N, d, device=dev, generator=g)
    E2 = torch.randn(N, d, device=dev, generator=g)
    un, uc = unique_long_n(torch.randint(-40, 400, (300,), device=dev, generator=g))
    pn, pc = unique_long_n(torch.randint(0, 1200, (500,), device=dev, generator=g))
    a = E2.clone().requires_grad_(True)
    la = contrast_loss_pair(E1, a, U, un, pn, 0.3, uc, pc)
    la.backward()
    b = E2.clone().requires_grad_(True)
    lb = contrast_loss(E1[:U], b[:U], un, 0.3, uc) + contrast_loss(E1[U:], b[U:], pn, 0.3, pc)
    lb.backward()
    assert torch.equal(la, lb)
    assert torch.equal(a.grad, b.grad)


@pytest.mark.parametrize("L", [1, 3, 5])
def test_contrast_loss_layers_equals_per_layer_pairs(dev, L):
    """contrast_loss_layers (all 2·L InfoNCE terms of a step in one launch per kernel, up to four
    layers per group) against the per-layer contrast_loss_pair loop it replaces: every layer's
    table gradient bitwise, the summed loss within one rounding of each addend (the group
    sums the 2·L term losses in one reduction)."""
    from hypergraph_diffusion_for_recommendation_amd.functional import (contrast_loss_layers,
                                                                         contrast_loss_pair,
                                                                         unique_long_n)
    g = torch.Generator(device=dev).manual_seed(20 + L)
    U, N, d = 700, 1900, 64
    E1s = [torch.randn(N, d, device=dev, generator=g) for _ in range(L)]
    E2s = [torch.randn(N, d, device=dev, generator=g) for _ in range(L)]
    un, uc = unique_long_n(torch.randint(-40, 400, (300,), device=dev, generator=g))
    pn, pc = unique_long_n(torch.randint(0, 1200, (500,), device=dev, generator=g))
    a = [e.clone().requires_grad_(True) for e in E2s]
    la = contrast_loss_layers(E1s, a, U, un, pn, 0.3, uc, pc)
    la.backward()
    b = [e.clone().requires_grad_(True) for e in E2s]
    terms = [contrast_loss_pair(e1, e2, U, un, pn, 0.3, uc, pc) for e1, e2 in zip(E1s, b)]
    lb = sum(terms)
    lb.backward()
    assert abs(float(la) - float(lb)) <= 4 * L * 1.2e-7 * sum(abs(float(t)) for t in terms)
    for x, y in zip(a, b):
        assert torch.equal(x.grad, y.grad)


def _step_fn(enc, opt, U, temp=1.0, cl=0.01):
    from hypergraph_diffusion_for_recommendation_amd.functional import (bpr_loss_rows,
                                                                         contrast_loss_layers,
                                                                         unique_long_n)

    def step(u, i, j):
        ue, ie, gcn, hyp = enc(keep_rate=0.7)
        bpr, anc, pos = bpr_loss_rows(ue, ie, u, i, j)  # the plugin's fused BPR
        (un, uc), (pn, pc) = unique_long_n(anc), unique_long_n(pos)
        ssl = contrast_loss_layers([t.detach() for t in gcn], hyp, U, un, pn, temp, uc, pc)
        loss = bpr + ssl * cl
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss
    return step


def test_captured_hccf_steps_equal_eager_steps(dev):
    from hypergraph_diffusion_for_recommendation_amd.graphs import CapturedStep
    g = torch.Generator(device=dev).manual_seed(7)
    batches = [tuple(torch.randint(0, n, (256,), device=dev, generator=g) for n in (1500, 1200,
                                                                                     1200))
               for _ in range(5)]
    runs = []
    for captured in (False, True):
        enc, U, I = _hccf(dev, drop_rate=0.0)
        lr = torch.tensor(1e-3, device=dev)
        opt = torch.optim.Adam(enc.parameters(), lr=lr, capturable=True, fused=True)
        step = _step_fn(enc, opt, U)
        torch.manual_seed(11)  # the drop-edge seed counter's start
        losses = [float(step(*batches[0]))]
        if captured:
            cap = CapturedStep(step, batches[1])
            losses += [float(cap(*b)) for b in batches[1:]]
        else:
            losses += [float(step(*b)) for b in batches[1:]]
        torch.cuda.synchronize()
        runs.append((losses, {k: v.detach().clone() for k, v in enc.state_dict().items()}))
    (l0, s0), (l1, s1) = runs
    assert l0 == l1, (l0, l1)
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k


def test_capture_safe_step_matches_reference(dev):
    """One eager capture-safe HCCF step (device mask, masked drop-edge views, counted InfoNCE)
    against the float64 reference with the same drop-edge matrices."""
    enc, U, I = _hccf(dev, drop_rate=0.0)
    N = U + I
    drops = []

    class Recording(torch.nn.Module):  # keeps each dropped matrix's live COO (eager test only)
        def __init__(self, inner):
            super().__init__()
            self.inner = inner

        def forward(self, adj, keep):
            child = self.inner(adj, keep)  # a masked view of the parent (Incidence.masked)
            m = child.csr.mask.bool().cpu()
            rows = torch.repeat_interleave(torch.arange(N), child.csr.rowptr.diff().cpu())
            # vals[mask] / keepRate in float32, as the reference's SpAdjDropEdge (HCCF.py:224)
            drops.append((torch.stack([rows[m], child.csr.col.cpu().long()[m]]),
                          child.val.cpu()[m] / keep))
            return child

    enc.edgeDropper = Recording(enc.edgeDropper)
    opt = torch.optim.SGD(enc.parameters(), lr=0.0)
    before = R.leaves(enc)
    g = torch.Generator(device=dev).manual_seed(5)
    u, i, j = (torch.randint(0, n, (256,), device=dev, generator=g) for n in (U, I, I))
    torch.manual_seed(13)
    loss = _step_fn(enc, opt, U)(u, i, j)
    adjs = [R.sparse(di, dv, (N, N)) for di, dv in drops]
    ueR, ieR, gR, hR = R.hccf_encoder(before, adjs, [torch.ones(U, 32), torch.ones(I, 32)] * 2,
                                      1.0, U, 2)
    anc, pos, neg = ueR[u.cpu()], ieR[i.cpu()], ieR[j.cpu()]
    un, pn = torch.unique(anc.long()), torch.unique(pos.long())
    ssl = 0
    for layer in range(2):
        e1, e2 = gR[layer].detach(), hR[layer]
        ssl = ssl + R.contrast_loss(e1[:U], e2[:U], un, 1.0) + \
            R.contrast_loss(e1[U:], e2[U:], pn, 1.0)
    lossR = R.bpr_loss(anc, pos, neg) + ssl * 0.01
    assert abs(float(loss) - float(lossR)) <= 1e-5 * abs(float(lossR))
    names = list(before)
    grads = torch.autograd.grad(lossR, [before[k] for k in names])
    params = dict(enc.named_parameters())
    for k, gr in zip(names, grads):
        R.check_rows(params[k].grad, gr, f"d {k}")


def test_captured_hccf_diffusion_steps_equal_eager_steps(dev):
    """HCCF_diffusion(hgd_graph=True)'s step: replays draw the ED-HNN dropout seeds from torch's
    device generator inside the graph (the same philox offsets eager launches consume) and the
    drop-edge masks from the device seed counter, so replayed and eager steps agree bitwise."""
    from types import SimpleNamespace

    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFDiffusionEncoder
    from hypergraph_diffusion_for_recommendation_amd.graphs import CapturedStep
    g = torch.Generator(device=dev).manual_seed(8)
    U, I = 1500, 1200
    batches = [tuple(torch.randint(0, n, (256,), device=dev, generator=g) for n in (U, I, I))
               for _ in range(5)]
    A = _graph(U, I, 30_000, seed=2)
    data = SimpleNamespace(n_users=U, n_items=I, norm_adj=A)
    kw = dict(lrate=1e-3, lr_decay=0.9, max_epoch=1, batch_size=256, reg=0.01,
              embedding_size=32, hyper_dim=32, drop_rate=0.0, p=0.3, n_layers=2)
    runs = []
    for captured in (False, True):
        torch.manual_seed(3)
        enc = HCCFDiffusionEncoder(kw, data, device=dev).train()
        enc.edgeDropper.device_rng = True
        enc.edgeDropper.capture_safe = True
        assert enc.edhnnlayer._fused_dropout_ok()
        lr = torch.tensor(1e-3, device=dev)
        opt = torch.optim.Adam(enc.parameters(), lr=lr, capturable=True, fused=True)
        step = _step_fn(enc, opt, U)
        torch.manual_seed(11)
        torch.cuda.manual_seed(12)
        losses = [float(step(*batches[0]))]
        if captured:
            cap = CapturedStep(step, batches[1])
            losses += [float(cap(*b)) for b in batches[1:]]
        else:
            losses += [float(step(*b)) for b in batches[1:]]
        torch.cuda.synchronize()
        runs.append((losses, {k: v.detach().clone() for k, v in enc.state_dict().items()}))
    (l0, s0), (l1, s1) = runs
    assert l0 == l1, (l0, l1)
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k


def test_captured_hccf_steps_on_the_reference_cpu_mask_stream(dev):
    """Graph mode on the reference's drop-edge stream (SpAdjDropEdge capture-safe, device_rng
    off): the eager steps draw each layer's torch.rand mask inline into the call's slot, the
    captured step's replays get theirs from refill() before each replay. Replayed and eager
    steps agree bitwise, and the CPU generator advances exactly as the reference's
    floor(torch.rand(nnz) + keep) draws would (HCCF.py:223)."""
    from hypergraph_diffusion_for_recommendation_amd.graphs import CapturedStep
    g = torch.Generator(device=dev).manual_seed(7)
    batches = [tuple(torch.randint(0, n, (256,), device=dev, generator=g) for n in (1500, 1200,
                                                                                     1200))
               for _ in range(5)]
    runs = []
    for captured in (False, True):
        enc, U, I = _hccf(dev, drop_rate=0.0)
        enc.edgeDropper.device_rng = False  # the reference's CPU stream, through the slots
        lr = torch.tensor(1e-3, device=dev)
        opt = torch.optim.Adam(enc.parameters(), lr=lr, capturable=True, fused=True)
        step = _step_fn(enc, opt, U)
        torch.manual_seed(11)
        losses = [float(step(*batches[0]))]
        if captured:
            enc.edgeDropper.host_fed(True)
            cap = CapturedStep(step, batches[1], before_replay=enc.edgeDropper.refill)
            losses += [float(cap(*b)) for b in batches[1:]]
        else:
            losses += [float(step(*b)) for b in batches[1:]]
        torch.cuda.synchronize()
        after = torch.rand(4)
        runs.append((losses, {k: v.detach().clone() for k, v in enc.state_dict().items()},
                     after))
        nnz = enc.edgeDropper._slots[0][0]
    (l0, s0, a0), (l1, s1, a1) = runs
    assert l0 == l1, (l0, l1)
    for k in s0:
        assert torch.equal(s0[k], s1[k]), k
    torch.manual_seed(11)
    for _ in range(5 * 2):  # 5 steps x 2 layers of the reference's draws
        ((torch.rand(nnz) + 0.7).floor()).type(torch.bool)
    ref_after = torch.rand(4)
    assert torch.equal(a0, ref_after) and torch.equal(a1, ref_after)
