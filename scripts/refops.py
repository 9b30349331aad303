"""Baselines and inputs for the component benches in scripts/ — NOT the parity oracle.

The benches time this library against "the reference's own ops": the torch / numpy / Python
calls the reference makes, run here on the same box. They are restated in this module so that
scripts/ never imports oracle/ (which stays test infrastructure for tests/, smoke() and
bench.py's cpu_baseline leg). Paths are relative to /root/reference/HD_SELFRec.
"""
from __future__ import annotations

import re

import numpy as np
import scipy.sparse as sp
import torch
import torch.nn.functional as F


# ---- inputs -------------------------------------------------------------------------------
def synthetic_incidence(n_users, n_items, nnz, seed=0):
    """SURVEY.md §8d generator: PCG64(seed) uniform users and items, deduplicated, row-major."""
    rng = np.random.Generator(np.random.PCG64(seed))
    u = rng.integers(0, n_users, size=nnz, dtype=np.int64)
    i = rng.integers(0, n_items, size=nnz, dtype=np.int64)
    key = np.unique(u * n_items + i)
    return key // n_items, key % n_items


def bipartite_adjacency(user_idx, item_idx, n_users, n_items):
    """ui_adj = tmp + tmp.T, tmp = csr((1, (u, i + n_users))) (data/ui_graph.py:70-84)."""
    n = n_users + n_items
    user_idx = np.asarray(user_idx)
    item_idx = np.asarray(item_idx)
    tmp = sp.csr_matrix((np.ones_like(user_idx, dtype=np.float32), (user_idx, item_idx + n_users)),
                        shape=(n, n), dtype=np.float32)
    return tmp + tmp.T


def normalize_graph_mat(adj):
    """Graph.normalize_graph_mat (data/graph.py:11-25)."""
    rowsum = np.array(adj.sum(1))
    with np.errstate(divide="ignore"):
        if adj.shape[0] == adj.shape[1]:
            d = np.power(rowsum, -0.5).flatten()
            d[np.isinf(d)] = 0.0
            D = sp.diags(d)
            return D.dot(adj).dot(D)
        d = np.power(rowsum, -1).flatten()
        d[np.isinf(d)] = 0.0
        return sp.diags(d).dot(adj)


def coo_of(mat):
    """convert_sparse_mat_to_tensor's (indices, values) (base/torch_interface.py:8-12)."""
    coo = mat.tocoo()
    return np.stack([coo.row.astype(np.int64), coo.col.astype(np.int64)]), coo.data.astype(np.float32)


# ---- the reference's ops ------------------------------------------------------------------
def hgcn_conv(adj, X, act=True, slope=0.5):
    """HGCNConv.forward (HGNN_HD4.py:455-462)."""
    Y = torch.sparse.mm(adj, torch.sparse.mm(adj.t(), X))
    return F.leaky_relu(Y, slope) if act else Y


def contrast_loss(embeds1, embeds2, nodes, temp):
    """contrastLoss (util/loss_torch.py:103-110)."""
    embeds1 = F.normalize(embeds1 + 1e-8, p=2)
    embeds2 = F.normalize(embeds2 + 1e-8, p=2)
    p1, p2 = embeds1[nodes], embeds2[nodes]
    nume = torch.exp(torch.sum(p1 * p2, dim=-1) / temp)
    deno = torch.exp(p1 @ p2.T / temp).sum(-1) + 1e-8
    return -torch.log(nume / deno).mean()


def load_data_set(path):
    """FileIO.load_data_set (data/loader.py:24-38)."""
    data = []
    with open(path) as f:
        next(f)
        for line in f:
            items = re.split("\t" if "\t" in line else ",", line.strip())
            data.append([int(items[0]), int(items[1]), 1.0])
    return data


def remap_ids(pairs):
    """Interaction.__generate_set's first-appearance dicts (data/ui_graph.py:43-56)."""
    user, item = {}, {}
    for u, i in pairs:
        if u not in user:
            user[u] = len(user)
        if i not in item:
            item[i] = len(item)
    return user, item


def find_k_largest(K, candidates):
    """util/algorithm.py:143-173 as the evaluation loop runs it per user (numba absent here:
    the vectorised equivalent of its output — first K of the seed ∪ stream ordering)."""
    c = np.asarray(candidates)
    n = len(c)
    sc = np.concatenate([c[:K], c])
    seed = np.concatenate([np.ones(K, np.int64), np.zeros(n, np.int64)])
    idx = np.concatenate([np.arange(K), np.arange(n)])
    order = np.lexsort((idx, -seed, -sc.astype(np.float64)))[:K]
    return idx[order].tolist(), sc[order].tolist()


topk_closed_form = find_k_largest


# ---- HCCF with the reference's torch ops (HCCF.py:136-226, loss_torch.py:5-9,103-110) -------
def bpr_loss(user_emb, pos_item_emb, neg_item_emb):
    """util/loss_torch.py:5-9."""
    pos_score = torch.mul(user_emb, pos_item_emb).sum(dim=1)
    neg_score = torch.mul(user_emb, neg_item_emb).sum(dim=1)
    return torch.mean(-torch.log(10e-6 + torch.sigmoid(pos_score - neg_score)))


def sp_adj_drop_edge(adj, keep_rate):
    """SpAdjDropEdge.forward (HCCF.py:213-226): CPU torch.rand mask, device compaction."""
    if keep_rate == 1.0:
        return adj
    vals = adj._values()
    idxs = adj._indices()
    mask = ((torch.rand(vals.size()) + keep_rate).floor()).type(torch.bool)
    return torch.sparse_coo_tensor(idxs[:, mask.to(idxs.device)],
                                   vals[mask.to(vals.device)] / keep_rate, adj.shape)


class HCCFEncoderRef(torch.nn.Module):
    """HCCFEncoder (HCCF.py:136-191) with the reference's ops: torch.sparse.mm GCN hop on the
    edge-dropped norm_adj, torch.mm learned-hypergraph hops. Same parameter names as
    encoders.HCCFEncoder, so a state_dict moves between them."""

    def __init__(self, n_users, n_items, latent, hyper_dim, n_layers, drop_rate, sparse_adj):
        super().__init__()
        self.n_users, self.n_layers = n_users, n_layers
        self.adj = sparse_adj
        init = torch.nn.init.xavier_uniform_
        dev = sparse_adj.device
        self.embedding_dict = torch.nn.ParameterDict({
            'user_emb': torch.nn.Parameter(init(torch.empty(n_users, latent)).to(dev)),
            'item_emb': torch.nn.Parameter(init(torch.empty(n_items, latent)).to(dev)),
            'user_w': torch.nn.Parameter(init(torch.empty(latent, hyper_dim)).to(dev)),
            'item_w': torch.nn.Parameter(init(torch.empty(latent, hyper_dim)).to(dev)),
        })
        self.drop_out = torch.nn.Dropout(drop_rate)

    def forward(self, keep_rate=0.5):
        nu = self.n_users
        e = self.embedding_dict
        hidden = [torch.cat([e['user_emb'], e['item_emb']], 0)]
        gcn_hidden, hgnn_hidden = [], []
        hyper_uu = e['user_emb'] @ e['user_w']
        hyper_ii = e['item_emb'] @ e['item_w']
        for _ in range(self.n_layers):
            gcn = torch.sparse.mm(sp_adj_drop_edge(self.adj, keep_rate), hidden[-1])
            hu = self.drop_out(hyper_uu)
            hi = self.drop_out(hyper_ii)
            hyper_u = torch.mm(hu, torch.mm(hu.T, hidden[-1][:nu]))
            hyper_i = torch.mm(hi, torch.mm(hi.T, hidden[-1][nu:]))
            gcn_hidden.append(gcn)
            hgnn_hidden.append(torch.cat([hyper_u, hyper_i], 0))
            hidden.append(gcn + hgnn_hidden[-1])
        emb = sum(hidden)
        return emb[:nu], emb[nu:], gcn_hidden, hgnn_hidden
