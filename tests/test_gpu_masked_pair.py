"""The masked hop's two-batch walk (hgd_spmm_masked, HGD_TUNE_MASK_PAIR = 2, the default: kept
entries packed by forward permutes; 1: by set-bit searches and pulls) against the one-batch walk
(0) and the compacted child (Incidence.drop): the same sums in the same edge
order, so bitwise — at every lane-group width (d = 16 … 256, including the one-batch fallback
below 8 lanes), keep rates from sparse to dense, rows longer than the split threshold (the split
plan's chunks walked the same way) and empty / fully dropped rows."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _graph(dev, n_rows, n_cols, nnz, heavy, seed):
    from hypergraph_diffusion_for_recommendation_amd.incidence import Incidence
    rng = np.random.default_rng(seed)
    r = rng.integers(0, n_rows, nnz)
    c = rng.integers(0, n_cols, nnz)
    if heavy:  # one row far past the split threshold, one empty row
        r = np.concatenate([r, np.zeros(60_000, dtype=np.int64)])
        c = np.concatenate([c, rng.integers(0, n_cols, 60_000)])
        r[r == 5] = 6
    key = np.unique(r * n_cols + c)
    r, c = key // n_cols, key % n_cols
    v = rng.random(len(r), dtype=np.float32) + 0.1
    idx = torch.from_numpy(np.stack([r, c]))
    return Incidence.from_coo(idx, torch.from_numpy(v), (n_rows, n_cols), device=dev)


@pytest.mark.parametrize("d", [16, 24, 32, 64, 128, 256])
@pytest.mark.parametrize("keep", [0.1, 0.5, 0.9])
@pytest.mark.parametrize("heavy", [False, True])
def test_masked_pair_walk_bitwise(dev, d, keep, heavy):
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_csr
    lib = nat.load()
    inc = _graph(dev, 3000, 2500, 90_000, heavy, seed=d)
    g = torch.Generator(device=dev).manual_seed(int(keep * 10) + d)
    mask = (torch.rand(inc.nnz, device=dev, generator=g) < keep).to(torch.uint8)
    X = torch.randn(inc.shape[1], d, device=dev, generator=g)
    Xt = torch.randn(inc.shape[0], d, device=dev, generator=g)
    view = inc.masked(mask, keep)
    outs = {}
    try:
        for pair in (2, 1, 0):
            nat.check(lib.hgd_set_tuning(15, pair), "hgd_set_tuning")
            outs[pair] = (spmm_csr(view.csr, X, view.val), spmm_csr(view.csc, Xt, view.val_t))
    finally:
        nat.check(lib.hgd_set_tuning(15, 2), "hgd_set_tuning")
    for pair in (1, 0):
        assert torch.equal(outs[2][0], outs[pair][0]) and torch.equal(outs[2][1], outs[pair][1])
    if not heavy:  # no split rows: the compacted child's hop is the same sums
        child = inc.drop(mask, keep)
        assert torch.equal(outs[2][0], spmm_csr(child.csr, X, child.val))
        assert torch.equal(outs[2][1], spmm_csr(child.csc, Xt, child.val_t))


@pytest.mark.parametrize("keep", [0.5, 0.25, 0.125, 0.3])
@pytest.mark.parametrize("pair", [2, 1, 0])
def test_masked_keep_reciprocal_is_the_division(dev, keep, pair):
    """HGD_TUNE_MASK_DIV: with keep a power of two the kept weight is val · (1 / keep), one
    multiply, instead of the IEEE val / keep — the same bits (one real value, rounded once), here
    over values from subnormal to near the float32 top; 0.3 takes the division either way."""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd.incidence import Incidence, spmm_csr
    lib = nat.load()
    rng = np.random.default_rng(7)
    n_rows, n_cols, nnz = 2000, 1500, 60_000
    key = np.unique(rng.integers(0, n_rows, nnz) * n_cols + rng.integers(0, n_cols, nnz))
    r, c = key // n_cols, key % n_cols
    v = (rng.random(len(r)) * 2.0 ** rng.integers(-140, 100, len(r))).astype(np.float32)
    inc = Incidence.from_coo(torch.from_numpy(np.stack([r, c])), torch.from_numpy(v),
                             (n_rows, n_cols), device=dev)
    g = torch.Generator(device=dev).manual_seed(11)
    mask = (torch.rand(inc.nnz, device=dev, generator=g) < keep).to(torch.uint8)
    X = torch.randn(n_cols, 64, device=dev, generator=g) * 1e-20
    view = inc.masked(mask, keep)
    outs = {}
    try:
        nat.check(lib.hgd_set_tuning(15, pair), "hgd_set_tuning")
        for div in (0, 1):
            nat.check(lib.hgd_set_tuning(16, div), "hgd_set_tuning")
            outs[div] = spmm_csr(view.csr, X, view.val)
    finally:
        nat.check(lib.hgd_set_tuning(16, 0), "hgd_set_tuning")
        nat.check(lib.hgd_set_tuning(15, 2), "hgd_set_tuning")
    assert torch.equal(outs[0], outs[1])
    child = inc.drop(mask, keep)  # the dropped COO's values divided on their own
    assert torch.equal(outs[0], spmm_csr(child.csr, X, child.val))
