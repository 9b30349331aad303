"""CPU: the oracle against its committed golden vectors, hand-derived known answers and the
torch-CPU library calls the reference makes (oracle/ref_cpu.py)."""
import os

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import hgd_oracle as O
from oracle import ref_cpu
from tests._util import assert_close

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


def test_golden_regenerates_exactly():
    """make_golden.py is deterministic and the committed vectors are what it produces."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("mg", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    rng = np.random.default_rng(2024)
    fresh = {"toy_hgconv2": mg.toy_hgconv2(), "hgcn_conv": mg.hgcn_fixture(rng),
             "edhnn": mg.edhnn_fixture(rng), "dropedge": mg.dropedge_fixture(rng),
             "structure": mg.structure_fixture(rng), "hgconv2": mg.hgconv2_fixture(),
             "hccf": mg.hccf_fixture(rng)}
    for name, arrs in fresh.items():
        gold = load(name)
        assert set(gold) == set(arrs), name
        for k, v in arrs.items():
            np.testing.assert_array_equal(np.asarray(v), gold[k], err_msg=f"{name}.{k}")


def test_toy_known_answer():
    g = load("toy_hgconv2")
    s = 1.0 / (2.0 * np.sqrt(2.0))
    T = np.array([[0.5, s, 0.0], [s, 0.5, s], [0.0, s, 0.5]])
    np.testing.assert_allclose(g["Y"], T @ g["X"].astype(np.float64), rtol=0, atol=1e-15)


def test_normalize_graph_mat_known_answer():
    """2 users, 1 item, both connected: degrees (1,1,2) → entries 1/√2 (data/graph.py:11-25)."""
    A = O.bipartite_adjacency([0, 1], [0, 0], 2, 1)
    N = O.normalize_graph_mat(A).toarray()
    r = np.float32(1.0) / np.sqrt(np.float32(2.0))
    exp = np.array([[0, 0, r], [0, 0, r], [r, r, 0]], dtype=np.float32)
    np.testing.assert_allclose(N, exp, rtol=1e-7)
    assert N.dtype == np.float32
    # empty node: inf → 0
    A2 = sp.csr_matrix(np.array([[0, 1, 0], [1, 0, 0], [0, 0, 0]], dtype=np.float32))
    assert np.isfinite(O.normalize_graph_mat(A2).toarray()).all()


def test_duplicates_summed_in_bipartite_adjacency():
    A = O.bipartite_adjacency([0, 0, 1], [0, 0, 1], 2, 2).toarray()
    assert A[0, 2] == 2.0 and A[2, 0] == 2.0 and A[1, 3] == 1.0


def test_mean_pair_row_stochastic():
    """Means of a constant signal are that constant on every non-isolated vertex."""
    g = load("edhnn")
    X = np.ones((int(g["N"]), 3))
    Y = O.equivset_mean_2hop(X, g["V"], g["E"], int(g["N"]))
    has = np.bincount(g["V"], minlength=int(g["N"])) > 0
    np.testing.assert_allclose(Y[has], 1.0, rtol=1e-14)
    assert (Y[~has] == 0).all()


def test_hgconv2_adjoint():
    g = load("hgconv2")
    rng = np.random.default_rng(0)
    X2 = rng.standard_normal(g["X"].shape)
    a = np.sum(g["Y"] * X2)
    b = np.sum(g["X"] * O.two_hop(g["rows"], g["cols"], None, tuple(g["shape"]), X2, "sym",
                                   "mean", "sym"))
    assert abs(a - b) < 1e-9 * (abs(a) + abs(b))


def test_oracle_vs_torch_sparse_mm():
    g = load("hgcn_conv")
    idx, vals = g["indices"], g["values"]
    N = int(g["n_users"] + g["n_items"])
    adj = ref_cpu.coo_tensor(idx[0], idx[1], vals, (N, N))
    Xt = torch.from_numpy(g["X"]).requires_grad_(True)
    Yt = ref_cpu.hgcn_conv(adj, Xt, act=True, slope=0.5)
    (dXt,) = torch.autograd.grad(Yt, Xt, torch.from_numpy(g["dY"]))
    mag = O.two_hop(idx[0], idx[1], np.abs(vals), (N, N), np.abs(g["X"]))
    assert_close(Yt.detach().numpy(), g["Y"], mag, what="HGCNConv fwd")
    dmag = O.two_hop(idx[0], idx[1], np.abs(vals), (N, N), np.abs(g["dY"]))
    assert_close(dXt.numpy(), g["dX"], dmag, what="HGCNConv bwd")


def test_scatter_mean_semantics():
    src = np.array([[1.0], [2.0], [4.0]])
    idx = np.array([0, 0, 2])
    out = O.scatter_mean(src, idx)
    np.testing.assert_array_equal(out, [[1.5], [0.0], [4.0]])
    out = O.scatter_mean(src, idx, dim_size=5)
    assert out.shape == (5, 1)
    t = ref_cpu.scatter_mean(torch.tensor(src, dtype=torch.float32), torch.tensor(idx))
    np.testing.assert_allclose(t.numpy(), [[1.5], [0.0], [4.0]])


def test_structure_fixture_consistency():
    g = load("structure")
    # CSR reproduces the COO as a multiset per row, in input order
    for r in range(len(g["rowptr"]) - 1):
        sel = np.nonzero(g["rows"] == r)[0]
        np.testing.assert_array_equal(g["col"][g["rowptr"][r]:g["rowptr"][r + 1]], g["cols"][sel])
    # CSC rows ascending inside every column
    for c in range(len(g["colptr"]) - 1):
        seg = g["rows_t"][g["colptr"][c]:g["colptr"][c + 1]]
        assert np.all(np.diff(seg) >= 0)


def test_dropedge_fixture_matches_reference_expression():
    g = load("dropedge")
    t_idx = torch.from_numpy(g["indices"])[:, torch.from_numpy(g["mask"])]
    t_val = torch.from_numpy(g["values"])[torch.from_numpy(g["mask"])] / float(g["keep"])
    np.testing.assert_array_equal(t_idx.numpy(), g["new_indices"])
    np.testing.assert_array_equal(t_val.numpy().view(np.uint32), g["new_values"].view(np.uint32))


def test_nonzero_order_matches_torch():
    g = load("edhnn")
    nz = torch.nonzero(torch.from_numpy(g["dense"]) > 0)
    np.testing.assert_array_equal(nz[:, 0].numpy(), g["V"])
    np.testing.assert_array_equal(nz[:, 1].numpy(), g["E"])


@pytest.mark.parametrize("zipf", [None, 1.0])
def test_synthetic_generator_dedup_sorted(zipf):
    r, c = O.synthetic_incidence(1000, 200, 20000, seed=0, zipf=zipf)
    key = r * 200 + c
    assert np.all(np.diff(key) > 0)
    assert r.max() < 1000 and c.max() < 200


@pytest.mark.parametrize("K", [1, 3, 10, 40])
def test_find_k_largest_closed_form(K):
    """The literal find_k_largest equals the closed form (seed ∪ stream ordering), incl. ties
    and the duplicated first-K entries."""
    rng = np.random.default_rng(K)
    for trial in range(30):
        n = int(rng.integers(K, 200))
        c = rng.integers(-5, 6, size=n).astype(np.float32)  # heavy ties
        if trial % 3 == 0:
            c[: min(K, n)] += 10  # top items inside the seed window → duplicates
        ids, sc = O.find_k_largest(K, c)
        ids2, sc2 = O.topk_closed_form(K, c)
        assert ids == ids2 and np.allclose(sc, sc2), (trial, ids, ids2)


def test_find_k_largest_duplicates_seed_items():
    ids, sc = O.find_k_largest(3, np.array([5.0, 4.0, 3.0, 10.0, 1.0]))
    assert ids == [3, 0, 0] and sc == [10.0, 5.0, 5.0]


@pytest.mark.parametrize("act,slope,ln", [(None, 0.0, True), ("leaky_relu", 0.2, True),
                                          ("relu", 0.0, False), ("leaky_relu", 0.5, False)])
def test_row_epilogue_backward_matches_torch_autograd(act, slope, ln):
    """The LN / LeakyReLU / blend gradient restatement against torch autograd in float64."""
    import torch
    rng = np.random.default_rng(5)
    Z = rng.standard_normal((40, 24))
    dY = rng.standard_normal((40, 24))
    g = rng.random(24) + 0.5
    b = rng.standard_normal(24)
    R1 = rng.standard_normal((40, 24))
    Y, _ = O.row_epilogue(Z, act, slope, ln, g, b, 1e-5, 0.7, R1, 0.4)
    Zt = torch.tensor(Z, requires_grad=True)
    gt = torch.tensor(g, requires_grad=True)
    bt = torch.tensor(b, requires_grad=True)
    a = Zt
    if act == "leaky_relu":
        a = torch.nn.functional.leaky_relu(Zt, slope)
    elif act == "relu":
        a = torch.relu(Zt)
    if ln:
        a = torch.nn.functional.layer_norm(a, (24,), gt, bt, 1e-5)
    Yt = 0.7 * a + 0.4 * torch.tensor(R1)
    np.testing.assert_allclose(Y, Yt.detach().numpy(), rtol=1e-12, atol=1e-12)
    Yt.backward(torch.tensor(dY))
    dZ, dg, db = O.row_epilogue_backward(Z, dY, act, slope, ln, g, 1e-5, 0.7)
    np.testing.assert_allclose(dZ, Zt.grad.numpy(), rtol=1e-10, atol=1e-12)
    if ln:
        np.testing.assert_allclose(dg, gt.grad.numpy(), rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(db, bt.grad.numpy(), rtol=1e-10, atol=1e-12)


def test_contrast_loss_restatements_agree():
    """numpy restatement vs the reference's torch calls (oracle/ref_cpu.contrast_loss), float64."""
    import torch
    from oracle import ref_cpu
    rng = np.random.default_rng(4)
    E1 = rng.standard_normal((50, 16))
    E2 = rng.standard_normal((50, 16))
    E1[3] = 0.0  # a zero row: normalize(0 + 1e-8) stays finite
    nodes = rng.integers(0, 50, size=20)
    a = O.contrast_loss(E1, E2, nodes, 0.2)
    b = ref_cpu.contrast_loss(torch.tensor(E1), torch.tensor(E2), torch.tensor(nodes), 0.2)
    assert abs(a - b.item()) <= 1e-12 * max(1.0, abs(a))


def test_ranking_evaluation_known_answer():
    """ranking_evaluation (util/evaluation.py:169-196) on a hand-checked case: a duplicated
    list entry counts once for hits and twice for DCG; unseen test items count in |test|."""
    origin = {1: {10: 1, 11: 1}, 2: {12: 1, 99: 1, 13: 1}}
    res = {1: [(10, .9), (10, .9), (5, .3)], 2: [(13, .5), (12, .4), (7, .1)]}
    got = O.ranking_evaluation(origin, res, [1, 3])
    # top 3: hits 1 + 2 of 5 test items; recall (1/2 + 2/3) / 2; NDCG: user 1 DCG = IDCG,
    # user 2 (1 + 1/log2 3) / (1 + 1/log2 3 + 1/2)
    assert got == ['Top 1\n', 'Hit Ratio:0.4\n', 'Precision:1.0\n', 'Recall:0.41667\n',
                   'NDCG:1.0\n', 'Top 3\n', 'Hit Ratio:0.6\n', 'Precision:0.5\n',
                   'Recall:0.58333\n', 'NDCG:0.88268\n']


def test_dropout_keep_mask_restatement():
    """oracle.dropout_keep_mask (the library dropout's RNG, hgd_dropout_apply): the numpy form
    equals a scalar Python restatement of the grouped draw (two lowbias32 rounds per group of
    four elements, a third for the second pair of 16-bit halves), keeps about keep·n elements;
    successive seeds give uncorrelated masks."""
    import numpy as np
    from oracle import hgd_oracle as O
    M = 0xFFFFFFFF

    def lb(x):
        x ^= x >> 16
        x = (x * 0x7FEB352D) & M
        x ^= x >> 15
        x = (x * 0x846CA68B) & M
        return x ^ (x >> 16)

    seed, keep = 0x123456789ABCDEF, 0.7
    thr = int(np.float32(keep) * np.float32(65536.0) + np.float32(0.5))
    assert thr == 45875
    got = O.dropout_keep_mask(seed, 301, keep)
    assert got.shape == (301,)
    for i in range(301):
        h1 = lb(lb(((i >> 2) + (seed & M)) & M) ^ (seed >> 32))
        h2 = lb(h1 ^ 0x9E3779B9)
        half = [h1 & 0xFFFF, h1 >> 16, h2 & 0xFFFF, h2 >> 16][i & 3]
        assert got[i] == (half < thr)
    assert O.dropout_keep_mask(seed, 1000, 1.0).all()
    a = O.dropout_keep_mask(7, 1_000_000, 0.5)
    b = O.dropout_keep_mask(8, 1_000_000, 0.5)
    assert abs(a.mean() - 0.5) < 0.003
    assert abs((a == b).mean() - 0.5) < 0.003
