"""GPU parity against the committed golden vectors (tests/golden/*.npz), through the C ABI."""
import os

import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O
from tests._util import assert_close

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


def test_golden_toy_hgconv2(dev):
    from hypergraph_diffusion_for_recommendation_amd import Incidence, hgconv2
    g = load("toy_hgconv2")
    inc = Incidence.from_coo(torch.from_numpy(np.stack([g["rows"], g["cols"]])), None,
                             tuple(g["shape"]), device=dev)
    Y = hgconv2(inc, torch.from_numpy(g["X"]).to(dev)).cpu().numpy()
    mag = O.two_hop(g["rows"], g["cols"], None, tuple(g["shape"]), np.abs(g["X"]), "sym", "mean",
                    "sym")
    assert_close(Y, g["Y"], mag, what="toy")


def test_golden_hgconv2_fwd_bwd(dev):
    from hypergraph_diffusion_for_recommendation_amd import Incidence, hgconv2
    g = load("hgconv2")
    shape = tuple(g["shape"])
    inc = Incidence.from_coo(torch.from_numpy(np.stack([g["rows"], g["cols"]])), None, shape,
                             device=dev)
    X = torch.from_numpy(g["X"]).to(dev).requires_grad_(True)
    Y = hgconv2(inc, X)
    (dX,) = torch.autograd.grad(Y, X, torch.from_numpy(g["dY"]).to(dev))
    mag = O.two_hop(g["rows"], g["cols"], None, shape, np.abs(g["X"]), "sym", "mean", "sym")
    dmag = O.two_hop(g["rows"], g["cols"], None, shape, np.abs(g["dY"]), "sym", "mean", "sym")
    assert_close(Y.detach().cpu().numpy(), g["Y"], mag, what="hgconv2 Y")
    assert_close(dX.cpu().numpy(), g["dX"], dmag, what="hgconv2 dX")


def test_golden_hgcn_conv(dev):
    """HGCNConv act=True on norm_adj from torch sparse COO (the reference's own input)."""
    from hypergraph_diffusion_for_recommendation_amd.layers import GCNLayer, HGCNConv
    g = load("hgcn_conv")
    N = int(g["n_users"] + g["n_items"])
    adj = torch.sparse_coo_tensor(torch.from_numpy(g["indices"]), torch.from_numpy(g["values"]),
                                  (N, N)).to(dev)
    X = torch.from_numpy(g["X"]).to(dev).requires_grad_(True)
    Y = HGCNConv(leaky=0.5)(adj, X, act=True)
    (dX,) = torch.autograd.grad(Y, X, torch.from_numpy(g["dY"]).to(dev))
    idx, vals = g["indices"], g["values"]
    mag = O.two_hop(idx[0], idx[1], np.abs(vals), (N, N), np.abs(g["X"]))
    dmag = O.two_hop(idx[0], idx[1], np.abs(vals), (N, N), np.abs(g["dY"]))
    assert_close(Y.detach().cpu().numpy(), g["Y"], mag, what="HGCNConv Y")
    assert_close(dX.cpu().numpy(), g["dX"], dmag * 0.5 + dmag * 0.5, what="HGCNConv dX")
    G = GCNLayer(0.5)(adj, torch.from_numpy(g["X"]).to(dev)).cpu().numpy()
    assert_close(G, g["G"], O.spmm_coo(idx[0], idx[1], np.abs(vals), N, np.abs(g["X"])),
                 what="GCNLayer")


def test_golden_edhnn(dev):
    from hypergraph_diffusion_for_recommendation_amd import Incidence, mean2hop
    from hypergraph_diffusion_for_recommendation_amd.incidence import dense_threshold
    g = load("edhnn")
    N = int(g["N"])
    rowptr, cols = dense_threshold(torch.from_numpy(g["dense"]).to(dev), 0.0)
    V = np.repeat(np.arange(N), np.diff(rowptr.cpu().numpy()))
    np.testing.assert_array_equal(V, g["V"])
    np.testing.assert_array_equal(cols.cpu().numpy(), g["E"])
    inc = Incidence.from_index_lists(torch.from_numpy(g["V"]), torch.from_numpy(g["E"]), N,
                                     device=dev)
    Y = mean2hop(inc, torch.from_numpy(g["X"]).to(dev)).cpu().numpy()
    assert_close(Y, g["Y"], O.equivset_mean_2hop(np.abs(g["X"]), g["V"], g["E"], N), what="edhnn")


def test_golden_dropedge(dev):
    from hypergraph_diffusion_for_recommendation_amd.incidence import drop_edges
    g = load("dropedge")
    idx, v = drop_edges(torch.from_numpy(g["indices"]).to(dev),
                        torch.from_numpy(g["values"]).to(dev),
                        torch.from_numpy(g["mask"]).to(dev), float(g["keep"]))
    np.testing.assert_array_equal(idx.cpu().numpy(), g["new_indices"])
    np.testing.assert_array_equal(v.cpu().numpy().view(np.uint32), g["new_values"].view(np.uint32))


def test_golden_structure(dev):
    from hypergraph_diffusion_for_recommendation_amd import Incidence
    g = load("structure")
    inc = Incidence.from_coo(torch.from_numpy(np.stack([g["rows"], g["cols"]])),
                             torch.from_numpy(g["vals"]), (30, 20), device=dev,
                             split_threshold=12, split_chunk=4)
    np.testing.assert_array_equal(inc.csr.rowptr.cpu().numpy(), g["rowptr"])
    np.testing.assert_array_equal(inc.csr.col.cpu().numpy(), g["col"])
    np.testing.assert_array_equal(inc.val.cpu().numpy(), g["val"])
    np.testing.assert_array_equal(inc.csc.rowptr.cpu().numpy(), g["colptr"])
    np.testing.assert_array_equal(inc.csc.col.cpu().numpy(), g["rows_t"])
    np.testing.assert_array_equal(inc.val_t.cpu().numpy(), g["val_t"])
    if len(g["heavy"]):
        hr, hc, ch = inc.csr._plan_arrays
        np.testing.assert_array_equal(hr.cpu().numpy(), g["heavy"])
        np.testing.assert_array_equal(hc.cpu().numpy(), g["heavy_cptr"])
        np.testing.assert_array_equal(ch.cpu().numpy(), g["chunk_heavy"])
