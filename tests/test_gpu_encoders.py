"""GPU: the encoder callers against the golden HCCF vectors and float64 CPU restatements of
LocalAwareEncoder and HCCF_diffusion's encoder (eval mode: dropout off, keep_rate = 1). Bound:
every row within 1e-5 of its scale (tests/_ref64.py check_rows; the train-mode forward and
backward at the configs' shapes are in test_gpu_config_parity.py)."""
import copy
import os
from types import SimpleNamespace

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import hgd_oracle as O
from oracle import ref_cpu
from tests import _ref64 as R
from tests._util import random_coo

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")

HCCF_KW = dict(lrate=0.001, lr_decay=0.9, max_epoch=1, batch_size=32, reg=0.01,
               embedding_size=16, hyper_dim=8, drop_rate=0.5, p=0.5, n_layers=2)


def test_hccf_encoder_golden(dev):
    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFEncoder
    g = dict(np.load(os.path.join(GOLDEN, "hccf.npz"), allow_pickle=False))
    U, I = int(g["n_users"]), int(g["n_items"])
    A = sp.coo_matrix((g["values"], (g["indices"][0], g["indices"][1])), shape=(U + I, U + I))
    data = SimpleNamespace(n_users=U, n_items=I, norm_adj=A.tocsr())
    enc = HCCFEncoder(HCCF_KW, data, device=dev).eval()
    with torch.no_grad():
        for k in ("E_u", "E_i", "W_u", "W_i"):
            name = {"E_u": "user_emb", "E_i": "item_emb", "W_u": "user_w", "W_i": "item_w"}[k]
            enc.embedding_dict[name].copy_(torch.from_numpy(g[k]))
        ue, ie, gcns, hyps = enc(keep_rate=1)
    for name, got, ref in (("user_emb", ue, g["user_emb"]), ("item_emb", ie, g["item_emb"]),
                           ("gcn0", gcns[0], g["gcn0"]), ("gcn1", gcns[1], g["gcn1"]),
                           ("hyp0", hyps[0], g["hyp0"]), ("hyp1", hyps[1], g["hyp1"])):
        R.check_rows(got, torch.from_numpy(ref), name)


def test_hccf_encoder_trains(dev):
    """One BPR step through keep_rate < 1 (drop-edge per layer) backpropagates to every
    parameter."""
    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFEncoder
    rng = np.random.default_rng(0)
    u, i = random_coo(rng, 50, 40, 300)
    A = O.normalize_graph_mat(O.bipartite_adjacency(u, i, 50, 40))
    data = SimpleNamespace(n_users=50, n_items=40, norm_adj=A)
    torch.manual_seed(0)
    enc = HCCFEncoder(HCCF_KW, data, device=dev)
    ue, ie, _, _ = enc(keep_rate=0.7)
    # numerically stable BPR-style term (log(sigmoid(s)) underflows to -inf for s < -88)
    loss = -torch.nn.functional.logsigmoid((ue[:10] * ie[:10]).sum(-1)).mean()
    loss.backward()
    for name, p in enc.embedding_dict.items():
        assert p.grad is not None and torch.isfinite(p.grad).all(), name


def test_local_aware_encoder_eval(dev):
    from hypergraph_diffusion_for_recommendation_amd.encoders import LocalAwareEncoder
    rng = np.random.default_rng(1)
    U, I, d = 60, 45, 16
    u, i = random_coo(rng, U, I, 400)
    ui = O.bipartite_adjacency(u, i, U, I)
    A = O.normalize_graph_mat(ui)
    data = SimpleNamespace(n_users=U, n_items=I, norm_adj=A, ui_adj=ui)
    torch.manual_seed(0)
    enc = LocalAwareEncoder(data, d, d, 3, 0.3, 0.2, device=dev).eval()
    ego = torch.randn(U + I, d)
    adj = enc.sparse_norm_adj
    with torch.no_grad():
        ue, ie = enc(ego.to(dev), adj)
    # float64 CPU restatement of HGNN_HD4.py:390-405 with the same parameters
    ec = copy.deepcopy(enc).cpu().double().eval()
    dense = torch.tensor(ui.todense(), dtype=torch.float32)
    nz = torch.nonzero(dense > 0)
    V, E = nz[:, 0], nz[:, 1]
    idx, vals = O.coo_of(A)
    adj_c = ref_cpu.coo_tensor(idx[0], idx[1], vals, A.shape).double()
    x = ego.double()
    with torch.no_grad():
        for k in range(3):
            if k != 2:
                blk = ec.edhnn_layers[k]
                h = torch.relu(blk.lin_in(x))
                h = ref_cpu.equivset_conv(h, V, E, h, blk.conv.W1, None, blk.conv.W, 0.0, "mean")
                x = torch.relu(h) + ego.double()
            else:
                x = ec.lns[0](ref_cpu.hgcn_conv(adj_c, x, act=False)) + ego.double()
    R.check_rows(torch.cat([ue, ie]), x, "LocalAwareEncoder")


def test_hccf_diffusion_encoder_eval(dev):
    """HCCF_diffusion's encoder (HCCF_diffusion.py:131-215) in eval mode against a CPU
    restatement with the reference's ops: torch.sparse.mm GCN hop, nonzero(H > 0) of the learned
    hypergraph E·W with the n + K offset on E, scatter means (index_reduce), Linear(LN(·))."""
    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFDiffusionEncoder
    rng = np.random.default_rng(2)
    U, I = 70, 55
    u, i = random_coo(rng, U, I, 500)
    A = O.normalize_graph_mat(O.bipartite_adjacency(u, i, U, I))
    data = SimpleNamespace(n_users=U, n_items=I, norm_adj=A)
    torch.manual_seed(0)
    enc = HCCFDiffusionEncoder(HCCF_KW, data, device=dev).eval()
    with torch.no_grad():
        ue, ie, gcns, hyps = enc(keep_rate=1)
    ec = copy.deepcopy(enc).cpu().double().eval()
    e = {k: v.detach().cpu() for k, v in ec.embedding_dict.items()}
    idx, vals = O.coo_of(A)
    adj_c = ref_cpu.coo_tensor(idx[0], idx[1], vals, A.shape).double()
    K = e["user_w"].shape[1]
    blk = ec.edhnnlayer

    def edhnn(x, H, n_nodes):
        nz = torch.nonzero(H > 0)
        V, E = nz[:, 0], nz[:, 1] + n_nodes
        h = torch.relu(blk.lin_in(x))
        h = ref_cpu.equivset_conv(h, V, E, h, blk.conv.W1, None, blk.conv.W, 0.0, "mean")
        return torch.relu(h)

    with torch.no_grad():
        hidden = [torch.cat([e["user_emb"], e["item_emb"]], 0)]
        huu, hii = e["user_emb"] @ e["user_w"], e["item_emb"] @ e["item_w"]
        for layer in range(HCCF_KW["n_layers"]):
            gcn = torch.sparse.mm(adj_c, hidden[-1])
            hyp = torch.cat([edhnn(hidden[-1][:U], huu, U + K), edhnn(hidden[-1][U:], hii, I + K)])
            R.check_rows(gcns[layer], gcn, f"gcn[{layer}]")
            R.check_rows(hyps[layer], hyp, f"hyper[{layer}]")
            hidden.append(gcn + hyp)
        emb = sum(hidden)
    R.check_rows(torch.cat([ue, ie]), emb, "HCCFDiffusionEncoder")
