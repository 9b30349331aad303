"""Parity of the hgd_spmm hop (HIP, gfx950) against the float64 oracle.

Every case goes through the C ABI (libhgd.so via ctypes). Tolerance: |got - ref| <= 1e-5·Σ|terms|
element-wise (tests/_util.py).
"""
import gc

import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O
from tests._util import assert_close, random_coo

pytestmark = pytest.mark.gpu


def _build(rows, cols, vals, shape, dev, **kw):
    from hypergraph_diffusion_for_recommendation_amd import Incidence
    idx = torch.from_numpy(np.stack([rows, cols]))
    v = None if vals is None else torch.from_numpy(vals.astype(np.float32))
    return Incidence.from_coo(idx, v, shape, device=dev, **kw)


@pytest.mark.parametrize("d", [1, 3, 4, 8, 16, 32, 48, 64, 96, 128, 256, 320])
@pytest.mark.parametrize("weighted", [False, True])
def test_spmm_dims(dev, d, weighted):
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    rng = np.random.default_rng(d * 7 + weighted)
    R, C = 173, 129
    r, c = random_coo(rng, R, C, 2500)
    vals = rng.standard_normal(len(r)).astype(np.float32) if weighted else None
    inc = _build(r, c, vals, (R, C), dev)
    X = rng.standard_normal((C, d)).astype(np.float32)
    scale = rng.random(R).astype(np.float32) if weighted else None
    Y = spmm_csr(inc.csr, torch.from_numpy(X).to(dev), val=inc.val,
                 row_scale=None if scale is None else torch.from_numpy(scale).to(dev))
    rowptr, col, v, _ = O.csr_from_coo(r, c, R, vals)
    ref = O.spmm_csr(rowptr, col, X, v, scale)
    mag = O.spmm_csr(rowptr, col, X, v, scale, absolute=True)
    assert_close(Y.cpu().numpy(), ref, mag, what=f"spmm d={d}")


@pytest.mark.parametrize("d", [8, 64, 128])
def test_spmm_transpose_hop(dev, d):
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    rng = np.random.default_rng(11 + d)
    R, C = 300, 77
    r, c = random_coo(rng, R, C, 4000)
    vals = rng.random(len(r)).astype(np.float32)
    inc = _build(r, c, vals, (R, C), dev)
    X = rng.standard_normal((R, d)).astype(np.float32)
    Y = spmm_csr(inc.csc, torch.from_numpy(X).to(dev), val=inc.val_t)
    ref = O.spmm_coo(c, r, vals, C, X)
    mag = O.spmm_coo(c, r, np.abs(vals), C, np.abs(X))
    assert_close(Y.cpu().numpy(), ref, mag, what="Aᵀ·X")


@pytest.mark.parametrize("d", [4, 32, 64, 256, 7])
@pytest.mark.parametrize("epi", [None, "leaky_relu", "relu"])
def test_spmm_split_rows_and_epilogue(dev, d, epi):
    """Long rows through the deterministic chunk split (threshold 16, chunk 8)."""
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    rng = np.random.default_rng(5 + d)
    R, C = 64, 500
    degs = np.array([0, 1, 15, 16, 17, 24, 400, 3] + list(rng.integers(0, 40, R - 8)))
    rows = np.repeat(np.arange(R), degs)
    cols = np.concatenate([rng.choice(C, size=k, replace=False) for k in degs])
    vals = rng.standard_normal(len(rows)).astype(np.float32)
    inc = _build(rows, cols, vals, (R, C), dev, split_threshold=16, split_chunk=8)
    heavy, cptr, ch = O.split_plan(np.concatenate([[0], np.cumsum(degs)]), 16, 8)
    assert inc.csr.n_heavy == len(heavy)
    ha, hc, chh = inc.csr._plan_arrays
    np.testing.assert_array_equal(ha.cpu().numpy(), heavy)
    np.testing.assert_array_equal(hc.cpu().numpy(), cptr)
    np.testing.assert_array_equal(chh.cpu().numpy(), ch)
    X = rng.standard_normal((C, d)).astype(np.float32)
    scale = rng.random(R).astype(np.float32)
    code = {None: nat.EPI_NONE, "leaky_relu": nat.EPI_LEAKY_RELU, "relu": nat.EPI_RELU}[epi]
    Y = spmm_csr(inc.csr, torch.from_numpy(X).to(dev), val=inc.val,
                 row_scale=torch.from_numpy(scale).to(dev), epilogue=code, slope=0.2)
    rowptr, col, v, _ = O.csr_from_coo(rows, cols, R, vals)
    ref = O.spmm_csr(rowptr, col, X, v, scale, epi=epi, slope=0.2)
    mag = O.spmm_csr(rowptr, col, X, v, scale, absolute=True)
    assert_close(Y.cpu().numpy(), ref, mag, what=f"split d={d} epi={epi}")


def test_spmm_row_range_and_empty(dev):
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    rng = np.random.default_rng(3)
    R, C, d = 100, 40, 64
    r, c = random_coo(rng, R, C, 600)
    inc = _build(r, c, None, (R, C), dev)
    X = torch.from_numpy(rng.standard_normal((C, d)).astype(np.float32)).to(dev)
    out = torch.full((R, d), 7.0, device=dev)
    spmm_csr(inc.csr, X, out=out, row_begin=30, row_end=55)
    rowptr, col, _, _ = O.csr_from_coo(r, c, R)
    ref = O.spmm_csr(rowptr, col, X.cpu().numpy())
    mag = O.spmm_csr(rowptr, col, X.cpu().numpy(), absolute=True)
    got = out.cpu().numpy()
    assert (got[:30] == 7.0).all() and (got[55:] == 7.0).all()
    assert_close(got[30:55], ref[30:55], mag[30:55], what="row range")
    # empty structure: all-zero output, no launch problems
    inc0 = _build(np.zeros(0, np.int64), np.zeros(0, np.int64), None, (5, 9), dev)
    Y0 = spmm_csr(inc0.csr, torch.ones(9, 16, device=dev))
    assert Y0.shape == (5, 16) and float(Y0.abs().sum()) == 0.0


def test_spmm_unaligned_view(dev):
    """A column slice (16-byte misaligned base) takes the scalar path and still matches."""
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    rng = np.random.default_rng(9)
    R, C = 50, 60
    r, c = random_coo(rng, R, C, 700)
    inc = _build(r, c, None, (R, C), dev)
    big = torch.from_numpy(rng.standard_normal((C, 70)).astype(np.float32)).to(dev)
    X = big[:, 1:65]
    Y = spmm_csr(inc.csr, X)
    rowptr, col, _, _ = O.csr_from_coo(r, c, R)
    Xn = X.cpu().numpy()
    assert_close(Y.cpu().numpy(), O.spmm_csr(rowptr, col, Xn),
                 O.spmm_csr(rowptr, col, Xn, absolute=True), what="unaligned")


def test_spmm_deterministic(dev):
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    rng = np.random.default_rng(21)
    R, C, d = 2000, 300, 64
    r, c = random_coo(rng, R, C, 60000)
    inc = _build(r, c, rng.random(len(r)).astype(np.float32), (R, C), dev, split_threshold=64,
                 split_chunk=16)
    X = torch.from_numpy(rng.standard_normal((C, d)).astype(np.float32)).to(dev)
    a = spmm_csr(inc.csc, torch.randn(R, d, device=dev), val=inc.val_t)
    Y1 = spmm_csr(inc.csr, X, val=inc.val)
    Y2 = spmm_csr(inc.csr, X, val=inc.val)
    assert torch.equal(Y1, Y2)
    assert a.shape == (C, d)


def test_spmm_rejects_bad_input(dev):
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    inc = _build(np.array([0, 1]), np.array([1, 0]), None, (2, 2), dev)
    with pytest.raises(ValueError):
        spmm_csr(inc.csr, torch.ones(3, 4, device=dev))
    with pytest.raises(TypeError):
        spmm_csr(inc.csr, torch.ones(2, 4, device=dev, dtype=torch.float64))
    with pytest.raises(RuntimeError):
        spmm_csr(inc.csr, torch.ones(2, 4))


@pytest.mark.parametrize("d", [8, 32, 48, 64, 128, 256, 320, 7])
@pytest.mark.parametrize("weighted", [False, True])
def test_spmm_segmented_kernel(dev, d, weighted):
    """The short-row segmented walk (HGD_PLAN_SEGMENTED) vs the oracle: empty rows, rows longer
    than a gather batch, a row count that is not a multiple of the group, sub-ranges."""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    rng = np.random.default_rng(31 + d + weighted)
    R, C = 1037, 211
    degs = rng.integers(0, 14, R)
    degs[::17] = 0
    degs[5] = 40
    degs[6] = 17
    rows = np.repeat(np.arange(R), degs)
    cols = rng.integers(0, C, len(rows))
    vals = rng.standard_normal(len(rows)).astype(np.float32) if weighted else None
    inc = _build(rows, cols, vals, (R, C), dev)
    inc.csr.configure_kernel(segmented=True)
    assert inc.csr.segmented
    X = rng.standard_normal((C, d)).astype(np.float32)
    scale = rng.random(R).astype(np.float32)
    rowptr, col, v, _ = O.csr_from_coo(rows, cols, R, vals)
    ref = O.spmm_csr(rowptr, col, X, v, scale, epi="leaky_relu", slope=0.1)
    mag = O.spmm_csr(rowptr, col, X, v, scale, absolute=True)
    Y = spmm_csr(inc.csr, torch.from_numpy(X).to(dev), val=inc.val,
                 row_scale=torch.from_numpy(scale).to(dev), epilogue=nat.EPI_LEAKY_RELU,
                 slope=0.1)
    assert_close(Y.cpu().numpy(), ref, mag, what=f"segmented d={d}")
    out = torch.full((R, d), 3.0, device=dev)
    spmm_csr(inc.csr, torch.from_numpy(X).to(dev), val=inc.val,
             row_scale=torch.from_numpy(scale).to(dev), epilogue=nat.EPI_LEAKY_RELU, slope=0.1,
             out=out, row_begin=100, row_end=901)
    got = out.cpu().numpy()
    assert (got[:100] == 3.0).all() and (got[901:] == 3.0).all()
    assert_close(got[100:901], ref[100:901], mag[100:901], what="segmented range")
    inc.csr.configure_kernel(segmented=False)
    Y2 = spmm_csr(inc.csr, torch.from_numpy(X).to(dev), val=inc.val,
                  row_scale=torch.from_numpy(scale).to(dev), epilogue=nat.EPI_LEAKY_RELU,
                  slope=0.1)
    assert torch.equal(Y, Y2)  # same per-row edge order → bitwise identical


def test_segmented_only_for_short_rows(dev):
    rng = np.random.default_rng(0)
    r, c = random_coo(rng, 5000, 100, 30000)  # avg degree 6 rows, 300 per column
    inc = _build(r, c, None, (5000, 100), dev)
    assert not inc.csr.segmented  # opt-in
    inc.csr.configure_kernel(True)
    inc.csc.configure_kernel(True)
    assert inc.csr.segmented and not inc.csc.segmented


@pytest.mark.parametrize("d", [192, 256, 320, 512])
@pytest.mark.parametrize("weighted", [False, True])
def test_spmm_interleaved_column_passes_are_bitwise_the_pass_loop(dev, d, weighted):
    """HGD_TUNE_SPMM_PASS_INTERLEAVE: a row wider than one column pass as ONE launch whose
    workgroups walk the passes of a row block back to back on one XCD — the same sums in the
    same order as one launch per pass, so bitwise equal; over a row range, with row scales, and
    against the float64 oracle."""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    lib = nat.load()
    rng = np.random.default_rng(d + 3 * weighted)
    R, C = 3001, 517
    r, c = random_coo(rng, R, C, 40000)
    vals = rng.standard_normal(len(r)).astype(np.float32) if weighted else None
    inc = _build(r, c, vals, (R, C), dev)
    X = torch.from_numpy(rng.standard_normal((C, d)).astype(np.float32)).to(dev)
    scale = torch.from_numpy(rng.random(R).astype(np.float32)).to(dev)
    outs = []
    try:
        for inter in (0, 1):
            nat.check(lib.hgd_set_tuning(17, inter), "interleave")
            Y = torch.full((R, d), float("nan"), device=dev)
            spmm_csr(inc.csr, X, val=inc.val, row_scale=scale, out=Y, row_begin=37, row_end=2900)
            outs.append(Y)
    finally:
        nat.check(lib.hgd_set_tuning(17, 0), "interleave off")
    assert torch.equal(outs[0][37:2900], outs[1][37:2900])
    assert bool(outs[1][:37].isnan().all()) and bool(outs[1][2900:].isnan().all())
    rowptr, col, v, _ = O.csr_from_coo(r, c, R, vals)
    Xn = X.cpu().numpy()
    sn = scale.cpu().numpy()
    ref = O.spmm_csr(rowptr, col, Xn, v, sn)
    mag = O.spmm_csr(rowptr, col, Xn, v, sn, absolute=True)
    assert_close(outs[1][37:2900].cpu().numpy(), ref[37:2900], mag[37:2900],
                 what=f"interleaved d={d}")


def _blocked_case(dev, seed, R=2001, C=613, nnz=30000, weighted=True, sorted_cols=True):
    rng = np.random.default_rng(seed)
    r, c = random_coo(rng, R, C, nnz)
    vals = rng.standard_normal(len(r)).astype(np.float32) if weighted else None
    # the CSC of this incidence: rows = items (C), sources = users (R), rows' columns ascending
    inc = _build(r, c, vals, (R, C), dev, split_threshold=0)
    return rng, r, c, vals, inc


@pytest.mark.parametrize("n_blocks", [1, 2, 3, 7, 64])
def test_spmm_col_blocks_is_the_block_major_copy(dev, n_blocks):
    """hgd_spmm_col_blocks: all rows' nonzeros of source block 0, then of block 1, … (block k =
    columns [⌊n_cols·k/P⌋, ⌊n_cols·(k+1)/P⌋)), each row's in its original order — bit-exact
    against a numpy restatement, rows with no nonzeros included; blk_perm maps back."""
    _, r, c, _, inc = _blocked_case(dev, 40 + n_blocks, nnz=9000)
    csc = inc.csc
    assert csc.cols_ascending and not inc.csr.cols_ascending
    start, bcol, perm = (t.cpu().numpy() for t in csc.col_blocks(n_blocks))
    rp = csc.rowptr.cpu().numpy()
    col = csc.col.cpu().numpy()
    R = csc.n_rows
    cuts = np.array([csc.n_cols * k // n_blocks for k in range(n_blocks + 1)])
    blk = np.searchsorted(cuts, col, side="right") - 1  # block of every nonzero
    row = np.repeat(np.arange(R), np.diff(rp))
    order = np.lexsort((np.arange(len(col)), row, blk))  # block, then row, then position
    np.testing.assert_array_equal(perm, order)
    np.testing.assert_array_equal(bcol, col[order])
    cnt = np.zeros(n_blocks * R, np.int64)
    np.add.at(cnt, blk * R + row, 1)
    np.testing.assert_array_equal(start, np.concatenate([[0], np.cumsum(cnt)]))
    assert csc.col_blocks(n_blocks) is csc.col_blocks(n_blocks)  # cached per block count


@pytest.mark.parametrize("d", [7, 16, 64, 128, 256])
@pytest.mark.parametrize("n_blocks", [2, 3, 5])
@pytest.mark.parametrize("epi", [None, "leaky_relu"])
def test_spmm_blocked_matches_the_oracle(dev, monkeypatch, d, n_blocks, epi):
    """The source-blocked hop (hgd_spmm_blocked through spmm_csr, forced by HGD_SPMM_BLOCKS)
    over the CSC of an incidence: blockwise partial sums, so a different fp32 association —
    element-wise within 1e-5·Σ|terms| of the float64 oracle, over a row range, with row scales,
    per-nonzero weights and the activation applied once after the last block; rows outside the
    range untouched."""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_blocks
    monkeypatch.setenv("HGD_SPMM_BLOCKS", str(n_blocks))
    rng, r, c, vals, inc = _blocked_case(dev, d * 13 + n_blocks)
    assert spmm_blocks(inc.csc, d) == n_blocks
    R, C = 2001, 613
    X = torch.from_numpy(rng.standard_normal((R, d)).astype(np.float32)).to(dev)
    q = torch.from_numpy(rng.random(C).astype(np.float32)).to(dev)
    code = {None: nat.EPI_NONE, "leaky_relu": nat.EPI_LEAKY_RELU}[epi]
    Y = torch.full((C, d), float("nan"), device=dev)
    spmm_csr(inc.csc, X, val=inc.val_t, row_scale=q, out=Y, row_begin=11, row_end=600,
             epilogue=code, slope=0.2)
    assert bool(Y[:11].isnan().all()) and bool(Y[600:].isnan().all())
    rowptr, col, v, _ = O.csr_from_coo(c, r, C, vals)
    Xn, qn = X.cpu().numpy(), q.cpu().numpy()
    ref = O.spmm_csr(rowptr, col, Xn, v, qn, epi=epi, slope=0.2)
    mag = O.spmm_csr(rowptr, col, Xn, v, qn, absolute=True)
    assert_close(Y[11:600].cpu().numpy(), ref[11:600], mag[11:600],
                 what=f"blocked d={d} P={n_blocks} epi={epi}")


@pytest.mark.parametrize("d", [16, 64, 256])
def test_spmm_one_block_is_bitwise_the_plain_hop(dev, monkeypatch, d):
    """With one block the block-major copy IS the structure and hgd_spmm_blocked walks
    [rowptr[r], rowptr[r+1]) exactly as hgd_spmm: bitwise equal."""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    from hypergraph_diffusion_for_recommendation_amd.incidence import _stream
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "0")  # the plain hop, whatever the environment says
    rng, r, c, vals, inc = _blocked_case(dev, 77 + d)
    csc = inc.csc
    X = torch.from_numpy(rng.standard_normal((2001, d)).astype(np.float32)).to(dev)
    q = torch.from_numpy(rng.random(613).astype(np.float32)).to(dev)
    plain = spmm_csr(csc, X, val=inc.val_t, row_scale=q)
    start, bcol, perm = csc.col_blocks(1)
    assert torch.equal(start, csc.rowptr) and torch.equal(bcol, csc.col)
    bval = csc.blocked_values(1, inc.val_t)
    assert csc.blocked_values(1, inc.val_t) is bval  # cached while the tensor lives unmodified
    Y = torch.empty_like(plain)
    nat.check(nat.load().hgd_spmm_blocked(
        start.data_ptr(), bcol.data_ptr(), bval.data_ptr(), q.data_ptr(), csc.n_rows,
        csc.n_cols, 0, csc.n_rows, X.data_ptr(), d, Y.data_ptr(), d, d, 0, 0.0, 1,
        _stream(X.device)), "hgd_spmm_blocked")
    assert torch.equal(Y, plain)
    v2 = inc.val_t.clone()
    b1 = csc.blocked_values(1, v2)
    v2.mul_(2.0)  # modified in place: gathered again
    b2 = csc.blocked_values(1, v2)
    assert b2 is not b1 and torch.equal(b2, 2.0 * bval)
    with torch.inference_mode():  # no version counter: gathered every call, still right
        v3 = inc.val_t * 3.0
        assert torch.equal(csc.blocked_values(1, v3), 3.0 * bval)


def test_spmm_blocked_two_hop_fwd_bwd(dev, monkeypatch):
    """hgconv2 fwd + bwd with the hops into items blocked (HGD_SPMM_BLOCKS=4) against the
    float64 oracle of the two-hop and its backward, and the blocked backward of the symmetric
    operator bitwise its blocked forward (the same hops)."""
    from hypergraph_diffusion_for_recommendation_amd import hgconv2
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_blocks
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "4")
    rng = np.random.default_rng(123)
    U, I, d = 3000, 400, 64
    r, c = random_coo(rng, U, I, 40000)
    inc = _build(r, c, None, (U, I), dev, split_threshold=0)
    assert spmm_blocks(inc.csc, d) == 4 and spmm_blocks(inc.csr, d) == 0
    X = torch.from_numpy(rng.standard_normal((U, d)).astype(np.float32)).to(dev)
    W = torch.from_numpy(rng.standard_normal((U, d)).astype(np.float32)).to(dev)
    Xr = X.clone().requires_grad_(True)
    Y = hgconv2(inc, Xr)
    (dX,) = torch.autograd.grad(Y, Xr, W)
    assert torch.equal(dX, hgconv2(inc, W))
    Xn = X.cpu().numpy()
    ref = O.two_hop(r, c, None, (U, I), Xn, P="sym", Q="mean", R="sym")
    mag = O.two_hop(r, c, None, (U, I), np.abs(Xn), P="sym", Q="mean", R="sym")
    assert_close(Y.detach().cpu().numpy(), ref, mag, what="blocked hgconv2")


@pytest.mark.parametrize("d", [16, 64, 128, 256])
@pytest.mark.parametrize("n_blocks", [2, 5])
def test_spmm_blocked_segmented_walk_is_bitwise_the_row_walk(dev, monkeypatch, d, n_blocks):
    """HGD_TUNE_SPMM_BLOCKED_SEG: each source block's short rows walked by the segmented kernel
    sum the same nonzeros in the same order as a lane group per row — bitwise equal, over a row
    range with weights, row scales and the activation."""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    lib = nat.load()
    monkeypatch.setenv("HGD_SPMM_BLOCKS", str(n_blocks))
    rng, r, c, vals, inc = _blocked_case(dev, 500 + d + n_blocks)
    X = torch.from_numpy(rng.standard_normal((2001, d)).astype(np.float32)).to(dev)
    q = torch.from_numpy(rng.random(613).astype(np.float32)).to(dev)
    outs = []
    try:
        for seg in (0, 1):
            nat.check(lib.hgd_set_tuning(18, seg), "blocked seg")
            Y = torch.full((613, d), float("nan"), device=dev)
            spmm_csr(inc.csc, X, val=inc.val_t, row_scale=q, out=Y, row_begin=5, row_end=601,
                     epilogue=nat.EPI_LEAKY_RELU, slope=0.2)
            outs.append(Y)
    finally:
        nat.check(lib.hgd_set_tuning(18, 0), "blocked seg off")
    assert torch.equal(outs[0][5:601], outs[1][5:601])
    assert bool(outs[1][:5].isnan().all()) and bool(outs[1][601:].isnan().all())


def test_spmm_blocked_two_hop_replays_in_a_hip_graph(dev, monkeypatch):
    """bench.py --graph on's pattern with the blocked hop into items: eager warm-up steps (they
    build the block-major copy and the blocked weights), then fwd + autograd bwd captured in one
    HIP graph; every replay is bitwise the eager step."""
    from hypergraph_diffusion_for_recommendation_amd import hgconv2
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "4")
    rng = np.random.default_rng(321)
    U, I, d = 5000, 700, 64
    r, c = random_coo(rng, U, I, 60000)
    inc = _build(r, c, None, (U, I), dev, split_threshold=0)
    X = torch.from_numpy(rng.standard_normal((U, d)).astype(np.float32)).to(dev)
    dY = torch.from_numpy(rng.standard_normal((U, d)).astype(np.float32)).to(dev)
    X.requires_grad_(True)

    def step():
        Y = hgconv2(inc, X)
        (dX,) = torch.autograd.grad(Y, X, dY)
        return Y, dX

    Y0, dX0 = step()
    Y0 = Y0.detach()  # an eager output holding its autograd graph would break the capture
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream(dev).wait_stream(side)
    gc.collect()
    graph = torch.cuda.CUDAGraph()
    # thread-local, as bench.py: autograd's device thread runs the backward during the capture
    with torch.cuda.graph(graph, capture_error_mode="thread_local"):
        Yg, dXg = step()
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize(dev)
        assert torch.equal(Yg, Y0) and torch.equal(dXg, dX0)


def test_spmm_blocks_zero_keeps_the_plain_hop(dev, monkeypatch):
    """``spmm_csr(..., blocks=0)`` (the sharded hop's uncached exchange slots) runs hgd_spmm even
    where the rule (here forced by HGD_SPMM_BLOCKS) would block: bitwise the plain hop."""
    from hypergraph_diffusion_for_recommendation_amd import spmm_csr
    rng, r, c, vals, inc = _blocked_case(dev, 909)
    X = torch.from_numpy(rng.standard_normal((2001, 64)).astype(np.float32)).to(dev)
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "0")
    plain = spmm_csr(inc.csc, X, val=inc.val_t)
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "3")
    blocked = spmm_csr(inc.csc, X, val=inc.val_t)
    kept = spmm_csr(inc.csc, X, val=inc.val_t, blocks=0)
    assert torch.equal(kept, plain) and not torch.equal(blocked, plain)
