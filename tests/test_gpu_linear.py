"""hgd_linear_* (f32 MFMA skinny Linear) against float64: forward with
bias/ReLU, backward-data with the ReLU mask, split-K backward-weight with the bias gradient;
ragged row counts, several feature widths, determinism, and argument checks."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O
from tests._util import assert_close

pytestmark = pytest.mark.gpu

SHAPES = [(1000, 64, 64), (37, 16, 48), (5000, 128, 128), (333, 48, 16), (70_001, 64, 64),
          (300_017, 64, 32), (1, 32, 32)]


@pytest.mark.parametrize("rows,in_f,out_f", SHAPES)
@pytest.mark.parametrize("relu", [False, True])
def test_linear_fwd_bwd(dev, rows, in_f, out_f, relu):
    from hypergraph_diffusion_for_recommendation_amd.functional import linear
    rng = np.random.default_rng(rows + in_f + out_f + relu)
    X = rng.standard_normal((rows, in_f)).astype(np.float32)
    W = (rng.standard_normal((out_f, in_f)) / np.sqrt(in_f)).astype(np.float32)
    b = rng.standard_normal(out_f).astype(np.float32)
    dY = rng.standard_normal((rows, out_f)).astype(np.float32)
    Xt = torch.from_numpy(X).to(dev).requires_grad_(True)
    Wt = torch.from_numpy(W).to(dev).requires_grad_(True)
    bt = torch.from_numpy(b).to(dev).requires_grad_(True)
    Y = linear(Xt, Wt, bt, relu=relu)
    gX, gW, gb = torch.autograd.grad(Y, (Xt, Wt, bt), torch.from_numpy(dY).to(dev))
    Z = O.linear(X, W, b)
    ref = np.maximum(Z, 0) if relu else Z
    mag = np.abs(X).astype(np.float64) @ np.abs(W).T + np.abs(b)
    assert_close(Y.detach().cpu().numpy(), ref, mag, what="linear fwd")
    m = (Z > 0) if relu else np.ones_like(Z, dtype=bool)
    # the kernel masks with its own fp32 output; skip elements whose sign is ambiguous in fp32
    ok = ~(relu & (np.abs(Z) <= 1e-5 * mag)).any(axis=1)
    dYm = np.where(m, dY, 0.0)
    dX = dYm @ W.astype(np.float64)
    dXmag = np.abs(dYm) @ np.abs(W).astype(np.float64)
    assert_close(gX.cpu().numpy()[ok], dX[ok], dXmag[ok], what="linear dX")
    if ok.all():
        dW = dYm.T @ X.astype(np.float64)
        dWmag = np.abs(dYm).T @ np.abs(X).astype(np.float64)
        assert_close(gW.cpu().numpy(), dW, dWmag, what="linear dW")
        assert_close(gb.cpu().numpy(), dYm.sum(0), np.abs(dYm).sum(0), what="linear db")


def test_linear_deterministic_and_no_bias(dev):
    from hypergraph_diffusion_for_recommendation_amd.functional import linear
    torch.manual_seed(0)
    X = torch.randn(123_457, 64, device=dev)
    W = torch.randn(64, 64, device=dev, requires_grad=True)
    dY = torch.randn(123_457, 64, device=dev)
    g1 = torch.autograd.grad(linear(X, W, None, relu=True), W, dY)[0]
    g2 = torch.autograd.grad(linear(X, W, None, relu=True), W, dY)[0]
    assert torch.equal(g1, g2)
    # accuracy without the ReLU (a mask taken from the fp32 forward flips a few near-zero rows
    # against a float64 forward): |err| <= 1e-5 · Σ|terms|
    g = torch.autograd.grad(linear(X, W, None), W, dY)[0].double()
    ref = dY.double().T @ X.double()
    mag = dY.double().abs().T @ X.double().abs()
    assert ((g - ref).abs() <= 1e-5 * mag).all()


def test_linear_other_shapes_use_library_gemm(dev):
    """Widths the kernels do not cover (not multiples of 16, > 128) still give the right answer."""
    from hypergraph_diffusion_for_recommendation_amd.functional import linear
    for in_f, out_f in ((20, 64), (64, 256), (64, 30)):
        X = torch.randn(100, in_f, device=dev)
        W = torch.randn(out_f, in_f, device=dev)
        ref = X.double() @ W.double().T
        mag = X.double().abs() @ W.double().abs().T
        assert ((linear(X, W, None).double() - ref).abs() <= 1e-5 * mag).all()


def test_linear_abi_checks(dev):
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    lib = nat.load()
    X = torch.zeros(8, 20, device=dev)
    W = torch.zeros(16, 20, device=dev)
    Y = torch.zeros(8, 16, device=dev)
    st = lib.hgd_linear_forward(X.data_ptr(), 20, 8, 20, W.data_ptr(), 20, 16, None, 0,
                                Y.data_ptr(), 16, None)
    assert st == 1 and b"multiple of 16" in lib.hgd_get_last_error_string()
    st = lib.hgd_linear_backward_weight(Y.data_ptr(), 16, None, 0, X.data_ptr(), 20, 8, 16, 32,
                                        W.data_ptr(), None, None, 0, None)
    assert st in (1, 4)
    # zero rows: gradients are written as zeros
    dW = torch.full((16, 32), 7.0, device=dev)
    db = torch.full((16,), 7.0, device=dev)
    st = lib.hgd_linear_backward_weight(None, 16, None, 0, None, 32, 0, 16, 32, dW.data_ptr(),
                                        db.data_ptr(), None, 0, None)
    torch.cuda.synchronize()
    assert st == 0 and dW.abs().sum().item() == 0 and db.abs().sum().item() == 0


@pytest.mark.parametrize("tiles,splitk", [(1, 1), (2, 0), (3, 1), (3, 0)])
def test_linear_kernel_forms(dev, tiles, splitk):
    """Every form of the split-bf16 products (HGD_TUNE_X3S_TILES: one or two column tiles per
    wave, producer waves; HGD_TUNE_X3_SPLITK: split-bf16 or f32 weight gradient) against float64,
    at both ED-HNN widths, masked and unmasked."""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    lib = nat.load()
    try:
        assert lib.hgd_set_tuning(9, tiles) == 0 and lib.hgd_set_tuning(8, splitk) == 0
        for rows, d in ((70_001, 64), (20_011, 128), (4_999, 96)):
            for relu in (False, True):
                test_linear_fwd_bwd(dev, rows, d, d, relu)
    finally:
        lib.hgd_set_tuning(9, 0)
        lib.hgd_set_tuning(8, 2)


@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("relu", [False, True])
def test_x3p_queue_form_equals_barrier_form(dev, d, relu):
    """k_splitk_x3p's queue form (HGD_TUNE_X3P_QUEUE = 1: three LDS buffers, full / empty
    counters instead of a workgroup barrier per stage) runs the same MFMAs in the same order as
    the barrier form: bitwise the same dW / db, ragged slices included, and within the float64
    bound."""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd.functional import linear
    lib = nat.load()
    g = torch.Generator(device=dev).manual_seed(d + relu)
    for rows in (144_242, 4_099, 20_011):
        X = torch.randn(rows, d, device=dev, generator=g)
        W = (torch.randn(d, d, device=dev, generator=g) / d ** 0.5).requires_grad_(True)
        b = torch.randn(d, device=dev, generator=g).requires_grad_(True)
        dY = torch.randn(rows, d, device=dev, generator=g)
        outs = []
        try:
            for q in (0, 1):
                assert lib.hgd_set_tuning(13, q) == 0
                outs.append(torch.autograd.grad(linear(X, W, b, relu=relu), (W, b), dY))
        finally:
            lib.hgd_set_tuning(13, 0)
        (gW0, gb0), (gW1, gb1) = outs
        assert torch.equal(gW0, gW1) and torch.equal(gb0, gb1), rows
        if not relu:
            ref = dY.double().T @ X.double()
            mag = dY.double().abs().T @ X.double().abs()
            assert ((gW1.double() - ref).abs() <= 1e-5 * mag).all()
