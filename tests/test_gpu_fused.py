"""hgd_spmm_fused / hgd_row_epilogue_backward: the LayerNorm, residual
and restart-blend epilogue fused into the second hop's store, forward and backward, against the
float64 oracle (oracle.hgd_oracle.row_epilogue*, restating model/layers/EquivSetConv.py:86-107
and layers2/EquivSetConv2.py:96), and against the unfused device composition."""
import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O
from tests._util import assert_close, random_coo

pytestmark = pytest.mark.gpu


def _inc(r, c, vals, shape, dev, **kw):
    from hypergraph_diffusion_for_recommendation_amd import Incidence
    idx = torch.from_numpy(np.stack([r, c]).astype(np.int64))
    v = None if vals is None else torch.from_numpy(vals.astype(np.float32))
    return Incidence.from_coo(idx, v, shape, device=dev, **kw)


def _run(dev, d, act, slope, ln, n_res, split, seed, weighted=True, unaligned=False):
    from hypergraph_diffusion_for_recommendation_amd.functional import two_hop_fused
    rng = np.random.default_rng(seed)
    Nv, Ne = 300, 180
    r, c = random_coo(rng, Nv, Ne, 4000)
    r = np.concatenate([r, np.full(Ne, 7)])           # one long row (split plan)
    c = np.concatenate([c, np.arange(Ne)])
    key = np.unique(r * Ne + c)
    r, c = key // Ne, key % Ne
    vals = (rng.random(len(r)) + 0.1).astype(np.float32) if weighted else None
    kw = dict(split_threshold=32, split_chunk=16) if split else dict(split_threshold=0)
    inc = _inc(r, c, vals, (Nv, Ne), dev, **kw)
    P, Q, R = (None, None, None) if weighted else ("mean", "mean", None)
    X = rng.standard_normal((Nv, d)).astype(np.float32)
    res = [rng.standard_normal((Nv, d)).astype(np.float32) for _ in range(n_res)]
    dY = rng.standard_normal((Nv, d)).astype(np.float32)
    norm = None
    if ln:
        norm = torch.nn.LayerNorm(d).to(dev)
        with torch.no_grad():
            norm.weight.copy_(torch.from_numpy(rng.random(d).astype(np.float32) + 0.5))
            norm.bias.copy_(torch.from_numpy(rng.standard_normal(d).astype(np.float32)))
    scales = dict(out_scale=0.7, s1=1.0, s2=0.3)
    if unaligned:
        Xt = torch.zeros((Nv, d + 1), device=dev)[:, 1:]
        Xt.copy_(torch.from_numpy(X))
        Xt.requires_grad_(True)
    else:
        Xt = torch.from_numpy(X).to(dev).requires_grad_(True)
    rt = [torch.from_numpy(x).to(dev).requires_grad_(True) for x in res]
    Y = two_hop_fused(inc, Xt, P=P, Q=Q, R=R, epilogue=act, slope=slope, norm=norm,
                      out_scale=scales["out_scale"],
                      res1=rt[0] if n_res > 0 else None, res1_scale=scales["s1"],
                      res2=rt[1] if n_res > 1 else None, res2_scale=scales["s2"])
    params = [Xt] + rt + ([norm.weight, norm.bias] if ln else [])
    grads = torch.autograd.grad(Y, params, torch.from_numpy(dY).to(dev))
    return dict(inc=inc, r=r, c=c, vals=vals, shape=(Nv, Ne), P=P, Q=Q, R=R, X=X, res=res, dY=dY,
                norm=norm, Y=Y.detach().cpu().numpy(),
                grads=[g.detach().cpu().numpy() for g in grads], **scales)


def _check(o, act, slope, ln):
    r, c, vals, shape = o["r"], o["c"], o["vals"], o["shape"]
    P, Q, R = o["P"], o["Q"], o["R"]
    X = o["X"]
    Z = O.two_hop(r, c, vals, shape, X, P, Q, R)
    magz = O.two_hop(r, c, None if vals is None else np.abs(vals), shape, np.abs(X), P, Q, R)
    gamma = beta = None
    if ln:
        gamma = o["norm"].weight.detach().cpu().numpy().astype(np.float64)
        beta = o["norm"].bias.detach().cpu().numpy().astype(np.float64)
    res = o["res"]
    Yref, a = O.row_epilogue(Z, act, slope, ln, gamma, beta, 1e-5, o["out_scale"],
                             res[0] if res else None, o["s1"],
                             res[1] if len(res) > 1 else None, o["s2"])
    if ln:
        rstd = 1.0 / np.sqrt(a.var(-1, keepdims=True) + 1e-5)
        m = (magz + magz.mean(-1, keepdims=True)) * rstd * 4
        mag = o["out_scale"] * (m * np.abs(gamma) + np.abs(beta))
    else:
        mag = o["out_scale"] * magz
    for k, s in zip(range(len(res)), (o["s1"], o["s2"])):
        mag = mag + abs(s) * np.abs(res[k])
    assert_close(o["Y"], Yref, mag, what="fused fwd")
    # backward: dZ through the epilogue, then the two backward hops
    dZ, dg, db = O.row_epilogue_backward(Z, o["dY"], act, slope, ln, gamma, 1e-5, o["out_scale"])
    dX = O.two_hop_backward(r, c, vals, shape, None, dZ, P, Q, R, None)
    dy = o["out_scale"] * np.abs(o["dY"])
    if ln:
        ah = np.abs(a - a.mean(-1, keepdims=True)) * rstd
        gh = dy * np.abs(gamma)
        mdz = rstd * (gh + gh.mean(-1, keepdims=True) + ah * (gh * ah).mean(-1, keepdims=True)) * 8
        mdz = mdz + np.abs(dZ) * 8 * magz * rstd  # LN conditioning on the error of a
    else:
        mdz = dy
    if act == "leaky_relu":
        mdz = mdz * max(1.0, slope)
    dmag = O.two_hop_backward(r, c, None if vals is None else np.abs(vals), shape, None, mdz,
                              P, Q, R, None)
    g = o["grads"]
    assert_close(g[0], dX, dmag, what="fused dX")
    for k, s in zip(range(len(res)), (o["s1"], o["s2"])):
        np.testing.assert_array_equal(g[1 + k], (np.float32(s) * o["dY"]) if s != 1.0
                                      else o["dY"])
    if ln:
        k = 1 + len(res)
        assert_close(g[k], dg, (dy * ah).sum(0) * 8 + 1e-6, what="dgamma")
        assert_close(g[k + 1], db, dy.sum(0) * 2, what="dbeta")


@pytest.mark.parametrize("d", [1, 3, 16, 48, 64, 100, 128, 256])
@pytest.mark.parametrize("ln", [False, True])
def test_fused_epilogue_fwd_bwd(dev, d, ln):
    for i, (act, slope, n_res, split, weighted) in enumerate([
            ("leaky_relu", 0.2, 1, True, True),
            (None, 0.0, 2, False, False),
            ("relu", 0.0, 0, True, False),
            ("leaky_relu", 0.5, 2, False, True)]):
        o = _run(dev, d, act, slope, ln, n_res, split, seed=100 * d + 10 * i + ln,
                 weighted=weighted)
        _check(o, act, slope, ln)


@pytest.mark.parametrize("d", [5, 64])
def test_fused_epilogue_unaligned(dev, d):
    o = _run(dev, d, "leaky_relu", 0.2, True, 2, True, seed=d, unaligned=True)
    _check(o, "leaky_relu", 0.2, True)


def test_fused_epilogue_wide_d(dev):
    """d = 320 without LayerNorm runs two column passes; with LayerNorm it takes the unfused
    device composition (the fused store holds at most 256 columns per row)."""
    for ln in (False, True):
        o = _run(dev, 320, "leaky_relu", 0.2, ln, 2, True, seed=320 + ln)
        _check(o, "leaky_relu", 0.2, ln)


def test_fused_matches_unfused_composition(dev):
    """The fused op and the reference's op chain (two_hop → nn.LayerNorm → adds) on the device."""
    from hypergraph_diffusion_for_recommendation_amd import two_hop
    from hypergraph_diffusion_for_recommendation_amd.functional import two_hop_fused
    rng = np.random.default_rng(3)
    Nv, Ne, d = 500, 300, 64
    r, c = random_coo(rng, Nv, Ne, 8000)
    vals = (rng.random(len(r)) + 0.1).astype(np.float32)
    inc = _inc(r, c, vals, (Nv, Ne), dev)
    X = torch.from_numpy(rng.standard_normal((Nv, d)).astype(np.float32)).to(dev)
    R1 = torch.from_numpy(rng.standard_normal((Nv, d)).astype(np.float32)).to(dev)
    R2 = torch.from_numpy(rng.standard_normal((Nv, d)).astype(np.float32)).to(dev)
    dY = torch.from_numpy(rng.standard_normal((Nv, d)).astype(np.float32)).to(dev)
    torch.manual_seed(0)
    norm = torch.nn.LayerNorm(d).to(dev)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.normal_()
    al = 0.3

    def run(fused):
        xs = [t.clone().requires_grad_(True) for t in (X, R1, R2)]
        if fused:
            y = two_hop_fused(inc, xs[0], epilogue="leaky_relu", slope=0.5, norm=norm,
                              out_scale=1 - al, res1=xs[1], res1_scale=1 - al, res2=xs[2],
                              res2_scale=al)
        else:
            y = (1 - al) * (norm(two_hop(inc, xs[0], epilogue="leaky_relu", slope=0.5)) + xs[1]) \
                + al * xs[2]
        g = torch.autograd.grad(y, xs + [norm.weight, norm.bias], dY)
        return [y.detach()] + [t.detach() for t in g]

    f, u = run(True), run(False)
    names = ["Y", "dX", "dR1", "dR2", "dgamma", "dbeta"]
    for n, a, b in zip(names, f, u):
        scale = b.abs().max().item() + 1e-6
        assert (a - b).abs().max().item() <= 2e-5 * scale * (50 if n in ("dgamma", "dbeta")
                                                              else 1), n
    # deterministic: a second fused run is bitwise identical
    f2 = run(True)
    for n, a, b in zip(names, f, f2):
        assert torch.equal(a, b), n


def test_fused_rejects_bad_descriptor(dev):
    import ctypes
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    lib = nat.load()
    ex = nat.RowEpilogue(act=nat.EPI_LEAKY_RELU, slope=-0.1, out_scale=1.0)
    rowptr = torch.zeros(3, dtype=torch.int64, device=dev)
    Y = torch.empty((2, 8), device=dev)
    st = lib.hgd_spmm_fused(rowptr.data_ptr(), None, None, None, 2, 0, 0, 2, None, 8,
                            Y.data_ptr(), 8, 8, ctypes.byref(ex), None, None, 0, None)
    assert st == 1 and b"slope" in lib.hgd_get_last_error_string()
    ex = nat.RowEpilogue(layer_norm=1, ln_eps=1e-5, out_scale=1.0)
    Y = torch.empty((2, 300), device=dev)
    st = lib.hgd_spmm_fused(rowptr.data_ptr(), None, None, None, 2, 0, 0, 2, None, 300,
                            Y.data_ptr(), 300, 300, ctypes.byref(ex), None, None, 0, None)
    assert st == 3


@pytest.mark.parametrize("d", [3, 16, 64, 100, 256])
def test_layer_norm_module_matches_torch(dev, d):
    """layers.LayerNorm (hgd_row_epilogue_forward/backward) vs nn.LayerNorm in float64: output
    rows within 1e-5 of the row's scale (tests/_ref64.check_rows); everything else element-wise
    within 1e-5·Σ|terms| — dx_i = (g_i - mean(g) - x̂_i·mean(g⊙x̂)) / σ with g = γ⊙dY (the
    terms |g_i|, mean|g|, |x̂_i|·mean|g⊙x̂|, over σ: at d = 3 a row's dx is mostly cancellation,
    far below its terms), dγ_j = Σ_n dY_nj·x̂_nj and dβ_j = Σ_n dY_nj over the 5003 rows."""
    from hypergraph_diffusion_for_recommendation_amd.layers import LayerNorm
    from tests import _ref64 as R
    torch.manual_seed(d)
    ref = torch.nn.LayerNorm(d).to(dev)
    with torch.no_grad():
        ref.weight.uniform_(0.5, 1.5)
        ref.bias.normal_()
    ours = LayerNorm(d).to(dev)
    ours.load_state_dict(ref.state_dict())
    x = (torch.randn(5003, d, device=dev) * 3 + 1)
    dY = torch.randn(5003, d, device=dev)
    xx = x.clone().requires_grad_(True)
    y = ours(xx)
    gx, gw, gb = torch.autograd.grad(y, (xx, ours.weight, ours.bias), dY)
    ref64 = torch.nn.LayerNorm(d).double().cpu()
    ref64.load_state_dict({k: v.double().cpu() for k, v in ref.state_dict().items()})
    x64 = x.double().cpu().requires_grad_(True)
    y64 = ref64(x64)
    rx, rw, rb = torch.autograd.grad(y64, (x64, ref64.weight, ref64.bias), dY.double().cpu())
    R.check_rows(y, y64, "y")
    with torch.no_grad():
        xhat = (y64 - ref64.bias) / ref64.weight
        d64 = dY.double().cpu()
        sigma = (x64.var(1, unbiased=False, keepdim=True) + ref64.eps).sqrt()
        g = d64 * ref64.weight
        dx_terms = (g.abs() + g.abs().mean(1, keepdim=True)
                    + xhat.abs() * (g * xhat).abs().mean(1, keepdim=True)) / sigma
        for name, got, exp, terms in (("dx", gx, rx, dx_terms),
                                      ("dgamma", gw, rw, (d64 * xhat).abs().sum(0)),
                                      ("dbeta", gb, rb, d64.abs().sum(0))):
            err = (got.double().cpu() - exp).abs()
            assert bool((err <= 1e-5 * terms).all()), (name, float((err / terms).max()))


def test_row_epilogue_standalone_vs_oracle(dev):
    from hypergraph_diffusion_for_recommendation_amd.functional import row_epilogue
    rng = np.random.default_rng(8)
    n, d = 777, 64
    Z = rng.standard_normal((n, d)).astype(np.float32)
    R1 = rng.standard_normal((n, d)).astype(np.float32)
    dY = rng.standard_normal((n, d)).astype(np.float32)
    norm = torch.nn.LayerNorm(d).to(dev)
    with torch.no_grad():
        norm.weight.uniform_(0.5, 1.5)
        norm.bias.normal_()
    Zt = torch.from_numpy(Z).to(dev).requires_grad_(True)
    Y = row_epilogue(Zt, "leaky_relu", 0.2, norm, 0.6, torch.from_numpy(R1).to(dev), 0.4)
    (gZ,) = torch.autograd.grad(Y, Zt, torch.from_numpy(dY).to(dev))
    g = norm.weight.detach().cpu().numpy()
    b = norm.bias.detach().cpu().numpy()
    Yref, a = O.row_epilogue(Z, "leaky_relu", 0.2, True, g, b, 1e-5, 0.6, R1, 0.4)
    from tests import _ref64 as R
    R.check_rows(Y, torch.from_numpy(np.asarray(Yref)), "Y")  # 1e-5 of each row's scale
    dZ, _, _ = O.row_epilogue_backward(Z, dY, "leaky_relu", 0.2, True, g, 1e-5, 0.6)
    # dZ element-wise within 1e-5·Σ|terms| of the LayerNorm backward through the LeakyReLU:
    # (|G_i| + mean|G| + |x̂_i|·mean|G⊙x̂|)/σ · leaky'(z_i), G = 0.6·γ⊙dY
    a = np.where(Z > 0, Z, 0.2 * Z).astype(np.float64)
    mu = a.mean(1, keepdims=True)
    sig = np.sqrt(a.var(1, keepdims=True) + 1e-5)
    xh = (a - mu) / sig
    G = 0.6 * g.astype(np.float64) * dY.astype(np.float64)
    terms = (np.abs(G) + np.abs(G).mean(1, keepdims=True)
             + np.abs(xh) * np.abs(G * xh).mean(1, keepdims=True)) / sig
    terms *= np.where(Z > 0, 1.0, 0.2)
    assert np.all(np.abs(gZ.cpu().numpy() - dZ) <= 1e-5 * terms)
