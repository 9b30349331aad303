"""Forward + backward parity of the autograd hops against the float64 oracle."""
import zlib

import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O
from tests._util import assert_close, random_coo

pytestmark = pytest.mark.gpu


def _inc(rows, cols, vals, shape, dev, **kw):
    from hypergraph_diffusion_for_recommendation_amd import Incidence
    idx = torch.from_numpy(np.stack([rows, cols]).astype(np.int64))
    v = None if vals is None else torch.from_numpy(np.asarray(vals, dtype=np.float32))
    return Incidence.from_coo(idx, v, shape, device=dev, **kw)


def _mag_two_hop(r, c, vals, shape, X, P, Q, R):
    w = None if vals is None else np.abs(vals)
    return O.two_hop(r, c, w, shape, np.abs(X), P=P, Q=Q, R=R)


CASES = [
    # name, weighted, P, Q, R, epi, slope
    ("hgconv2", False, "sym", "mean", "sym", None, 0.0),
    ("mean2hop", False, "mean", "mean", None, None, 0.0),
    ("hgcnconv_act", True, None, None, None, "leaky_relu", 0.5),
    ("hgcnconv_noact", True, None, None, None, None, 0.0),
    ("weighted_sym", True, "wsym", "wmean", "wsym", "relu", 0.0),
    ("neg_slope", True, None, None, None, "leaky_relu", -0.3),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("d", [16, 64])
def test_two_hop_fwd_bwd(dev, case, d):
    from hypergraph_diffusion_for_recommendation_amd import two_hop
    name, weighted, P, Q, R, epi, slope = case
    rng = np.random.default_rng(zlib.crc32(name.encode()) % 1000 + d)
    Nv, Ne = 400, 250
    r, c = random_coo(rng, Nv, Ne, 6000)
    vals = (rng.random(len(r)).astype(np.float32) + 0.1) if weighted else None
    inc = _inc(r, c, vals, (Nv, Ne), dev, split_threshold=32, split_chunk=16)
    X = rng.standard_normal((Nv, d)).astype(np.float32)
    dY = rng.standard_normal((Nv, d)).astype(np.float32)
    Xt = torch.from_numpy(X).to(dev).requires_grad_(True)
    Y = two_hop(inc, Xt, P=P, Q=Q, R=R, epilogue=epi, slope=slope)
    (dX,) = torch.autograd.grad(Y, Xt, torch.from_numpy(dY).to(dev))
    ref = O.two_hop(r, c, vals, (Nv, Ne), X, P, Q, R, epi, slope)
    mag = _mag_two_hop(r, c, vals, (Nv, Ne), X, P, Q, R)
    assert_close(Y.detach().cpu().numpy(), ref, mag, what=f"{name} fwd")
    Z = O.two_hop(r, c, vals, (Nv, Ne), X, P, Q, R)  # pre-activation (sign test of the bwd)
    dref = O.two_hop_backward(r, c, vals, (Nv, Ne), Z, dY, P, Q, R, epi, slope)
    dmag = O.two_hop_backward(r, c, None if vals is None else np.abs(vals), (Nv, Ne),
                              np.ones_like(ref), np.abs(dY), P, Q, R, None)
    if epi == "leaky_relu":
        dmag = dmag * max(1.0, abs(slope))
    assert_close(dX.cpu().numpy(), dref, dmag, what=f"{name} bwd")


def test_mean2hop_equals_scatter_mean_chain(dev):
    """ED-HNN: V/E from nonzero(H > 0) → mean over E then mean over V (EquivSetConv2.py:88-93)."""
    from hypergraph_diffusion_for_recommendation_amd import Incidence, mean2hop
    rng = np.random.default_rng(0)
    N = 300
    Hd = (rng.random((N, N)) > 0.97).astype(np.float32)
    V, E = O.nonzero_threshold(Hd)
    X = rng.standard_normal((N, 32)).astype(np.float32)
    inc = Incidence.from_index_lists(torch.from_numpy(V), torch.from_numpy(E), N, device=dev)
    Y = mean2hop(inc, torch.from_numpy(X).to(dev))
    ref = O.equivset_mean_2hop(X, V, E, N)
    mag = O.equivset_mean_2hop(np.abs(X), V, E, N)
    assert_close(Y.cpu().numpy(), ref, mag, what="mean2hop")


@pytest.mark.parametrize("transpose", [False, True])
def test_spmm_autograd(dev, transpose):
    from hypergraph_diffusion_for_recommendation_amd import spmm
    rng = np.random.default_rng(17)
    R, C, d = 220, 180, 32
    r, c = random_coo(rng, R, C, 3000)
    vals = rng.standard_normal(len(r)).astype(np.float32)
    inc = _inc(r, c, vals, (R, C), dev)
    n_in = R if transpose else C
    n_out = C if transpose else R
    X = rng.standard_normal((n_in, d)).astype(np.float32)
    dY = rng.standard_normal((n_out, d)).astype(np.float32)
    Xt = torch.from_numpy(X).to(dev).requires_grad_(True)
    Y = spmm(inc, Xt, transpose=transpose)
    (dX,) = torch.autograd.grad(Y, Xt, torch.from_numpy(dY).to(dev))
    if transpose:
        ref = O.spmm_coo(c, r, vals, C, X)
        mag = O.spmm_coo(c, r, np.abs(vals), C, np.abs(X))
        dref = O.spmm_coo(r, c, vals, R, dY)
        dmag = O.spmm_coo(r, c, np.abs(vals), R, np.abs(dY))
    else:
        ref = O.spmm_coo(r, c, vals, R, X)
        mag = O.spmm_coo(r, c, np.abs(vals), R, np.abs(X))
        dref = O.spmm_coo(c, r, vals, C, dY)
        dmag = O.spmm_coo(c, r, np.abs(vals), C, np.abs(dY))
    assert_close(Y.detach().cpu().numpy(), ref, mag, what="spmm fwd")
    assert_close(dX.cpu().numpy(), dref, dmag, what="spmm bwd")


def test_hgconv2_large_adjoint_property(dev):
    """Size-independent property at a larger size: <Y1, T·X2> == <T·Y1, X2> (T symmetric)."""
    from hypergraph_diffusion_for_recommendation_amd import Incidence, hgconv2
    g = torch.Generator(device=dev).manual_seed(0)
    U, I, nnz, d = 200_000, 20_000, 2_000_000, 64
    u = torch.randint(0, U, (nnz,), device=dev, generator=g)
    i = torch.randint(0, I, (nnz,), device=dev, generator=g)
    key = torch.unique(u * I + i)
    inc = Incidence.from_coo(torch.stack([key // I, key % I]), None, (U, I), device=dev)
    X1 = torch.randn(U, d, device=dev, generator=g)
    X2 = torch.randn(U, d, device=dev, generator=g)
    a = (hgconv2(inc, X1).double() * X2.double()).sum()
    b = (X1.double() * hgconv2(inc, X2).double()).sum()
    assert abs(float(a - b)) <= 1e-5 * float(a.abs() + b.abs()) + 1e-3


@pytest.mark.parametrize("n,count", [(2, 1000), (4, 144_242 * 128 + 3), (8, 7)])
def test_sum_arrays_is_the_binary_chain(dev, n, count):
    """hgd_sum_arrays: bitwise ((a_0 + a_1) + a_2) + … (torch's fp32 adds in the same order),
    including a ragged tail past the float4 body and out aliasing a_0."""
    import ctypes
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    g = torch.Generator(device=dev).manual_seed(count + n)
    arrs = [torch.randn(count, device=dev, generator=g) for _ in range(n)]
    want = arrs[0].clone()
    for a in arrs[1:]:
        want = want + a
    ptrs = (ctypes.c_void_p * n)(*[a.data_ptr() for a in arrs])
    out = arrs[0]  # in place over a_0
    nat.check(nat.load().hgd_sum_arrays(ptrs, n, count, out.data_ptr(), nat.stream_handle(dev)),
              "hgd_sum_arrays")
    assert torch.equal(out, want)


def test_fan_gradient_is_the_sum_of_its_uses(dev):
    """functional.fan: n aliases of x; x.grad = Σ of the uses' gradients (one n-ary pass), equal
    to autograd's own accumulation within fp32 reassociation (1e-6 of Σ|terms|)."""
    from hypergraph_diffusion_for_recommendation_amd.functional import fan
    g = torch.Generator(device=dev).manual_seed(5)
    x0 = torch.randn(3000, 64, device=dev, generator=g)
    ws = [torch.randn(3000, 64, device=dev, generator=g) for _ in range(4)]

    def loss(uses):
        return sum((u * w).sum() * (k + 1) for k, (u, w) in enumerate(zip(uses, ws)))

    x = x0.clone().requires_grad_(True)
    uses = fan(x, 4)
    assert all(u.data_ptr() == x.data_ptr() for u in uses)
    loss(uses).backward()
    ref = sum(w.double() * (k + 1) for k, w in enumerate(ws))
    mag = sum(w.double().abs() * (k + 1) for k, w in enumerate(ws))
    assert ((x.grad.double() - ref).abs() <= 1e-6 * mag).all()
