"""CPU oracle for the hypergraph-propagation hot path — TEST INFRASTRUCTURE ONLY.

This module is a plain numpy restatement of the reference's algorithm for the path named by
BASELINE.json ``north_star``. Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import it, and only as the checker; the product path
(``hypergraph_diffusion_for_recommendation_amd``) never calls it and fails loudly without its
HIP library.

Parity status: **parity unpinned by the reference itself.** The reference ships no tests, golden
vectors or fixtures for this path, and importing/running the reference in
this container was denied by the environment, so no reference outputs exist.
The restatement is pinned instead by (i) hand-derived known-answer cases, (ii) cross-checks
against the torch-CPU library calls the reference itself makes (``oracle/ref_cpu.py``:
``torch.sparse.mm``, ``index_reduce_('mean')`` for torch_scatter's mean), and (iii) algebraic
properties (adjointness, row-stochastic means).

Floating point is float64 here; integer/index results (orders, masks, row pointers) are exact.
Every function cites the reference file:line it restates (relative to
/root/reference/HD_SELFRec).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp


# ---------------------------------------------------------------------------------------------
# Graph construction — data/ui_graph.py, data/graph.py, base/torch_interface.py
# ---------------------------------------------------------------------------------------------
def load_data_set(path):
    """FileIO.load_data_set (data/loader.py:24-38): skip the header line; a line containing a
    tab splits on tabs, otherwise on commas, after strip(); int() of fields 0 and 1; weight 1.
    Python's own exceptions propagate where the reference's would."""
    import re
    data = []
    with open(path) as f:
        next(f)
        for line in f:
            sep = "\t" if "\t" in line else ","
            items = re.split(sep, line.strip())
            data.append([int(items[0]), int(items[1]), 1.0])
    return data


def remap_ids(pairs):
    """Id maps in first-appearance order of the training file (data/ui_graph.py:43-68)."""
    user, item = {}, {}
    for u, i in pairs:
        if u not in user:
            user[u] = len(user)
        if i not in item:
            item[i] = len(item)
    return user, item


def bipartite_adjacency(user_idx, item_idx, n_users, n_items):
    """ui_adj = [[0, R], [Rᵀ, 0]] as float32 CSR, duplicates summed
    (Interaction.__create_sparse_bipartite_adjacency, data/ui_graph.py:70-84)."""
    n = n_users + n_items
    user_idx = np.asarray(user_idx)
    item_idx = np.asarray(item_idx)
    ratings = np.ones_like(user_idx, dtype=np.float32)
    tmp = sp.csr_matrix((ratings, (user_idx, item_idx + n_users)), shape=(n, n),
                        dtype=np.float32)
    return tmp + tmp.T


def normalize_graph_mat(adj):
    """D^-1/2·A·D^-1/2 for square, D^-1·A otherwise, inf→0 (Graph.normalize_graph_mat,
    data/graph.py:11-25). Float32 like the reference (rowsum of a float32 matrix)."""
    shape = adj.get_shape()
    rowsum = np.array(adj.sum(1))
    with np.errstate(divide="ignore"):
        if shape[0] == shape[1]:
            d_inv = np.power(rowsum, -0.5).flatten()
            d_inv[np.isinf(d_inv)] = 0.0
            d = sp.diags(d_inv)
            return d.dot(adj).dot(d)
        d_inv = np.power(rowsum, -1).flatten()
        d_inv[np.isinf(d_inv)] = 0.0
        return sp.diags(d_inv).dot(adj)


def normalize_graph_mat_hyper(H):
    """D_v^-1/2·H·D_e^-1·Hᵀ·D_v^-1/2 (Graph.normalize_graph_mat_hyper, data/graph.py:28-42) —
    the operator the benchmark's hgconv2 applies without forming it."""
    colsum = np.array(H.sum(0))
    rowsum = np.array(H.sum(1))
    with np.errstate(divide="ignore"):
        de = np.power(colsum, -1.0).flatten()
        de[np.isinf(de)] = 0.0
        dv = np.power(rowsum, -0.5).flatten()
        dv[np.isinf(dv)] = 0.0
    Dv, De = sp.diags(dv), sp.diags(de)
    return Dv.dot(H).dot(De).dot(H.T).dot(Dv)


def coo_of(mat):
    """(indices int64 [2,nnz], values float32) in ``tocoo()`` order
    (TorchGraphInterface.convert_sparse_mat_to_tensor, base/torch_interface.py:8-12)."""
    coo = mat.tocoo()
    idx = np.stack([coo.row.astype(np.int64), coo.col.astype(np.int64)])
    return idx, coo.data.astype(np.float32)


# ---------------------------------------------------------------------------------------------
# Structure (integer, bit-exact)
# ---------------------------------------------------------------------------------------------
def csr_from_coo(rows, cols, n_rows, vals=None):
    """Stable row ordering of a COO (entries keep their order inside a row), row pointer."""
    rows = np.asarray(rows, dtype=np.int64)
    cols = np.asarray(cols, dtype=np.int64)
    perm = np.argsort(rows, kind="stable")
    rowptr = np.zeros(n_rows + 1, dtype=np.int64)
    np.add.at(rowptr, rows + 1, 1)
    rowptr = np.cumsum(rowptr)
    v = None if vals is None else np.asarray(vals)[perm]
    return rowptr, cols[perm].astype(np.int32), v, perm


def transpose_csr(rowptr, col, n_cols, vals=None):
    """CSC of a CSR via a stable counting sort on the column id: inside every column the rows
    stay ascending (the order ``adj.t()`` + coalesce produces for a row-sorted COO)."""
    n_rows = len(rowptr) - 1
    rows = np.repeat(np.arange(n_rows, dtype=np.int64), np.diff(rowptr))
    perm = np.argsort(col, kind="stable")
    colptr = np.zeros(n_cols + 1, dtype=np.int64)
    np.add.at(colptr, np.asarray(col, dtype=np.int64) + 1, 1)
    colptr = np.cumsum(colptr)
    v = None if vals is None else np.asarray(vals)[perm]
    return colptr, rows[perm].astype(np.int32), v, perm


def split_plan(rowptr, threshold, chunk):
    """Rows with degree > threshold, their chunk ranges and each chunk's owner
    (the deterministic long-row split of hgd_spmm; not a reference concept)."""
    deg = np.diff(rowptr)
    heavy = np.nonzero(deg > threshold)[0].astype(np.int32)
    nch = (deg[heavy] + chunk - 1) // chunk
    cptr = np.concatenate([[0], np.cumsum(nch)]).astype(np.int64)
    chunk_heavy = np.repeat(np.arange(len(heavy), dtype=np.int32), nch)
    return heavy, cptr, chunk_heavy


def dropedge(indices, values, mask, keep_rate):
    """SpAdjDropEdge.forward (model/graph/HCCF.py:217-226): keep entries where mask is set,
    in order, values divided by keepRate in float32. ``mask`` is
    ``((torch.rand(nnz) + keepRate).floor()).type(torch.bool)`` drawn by the caller."""
    mask = np.asarray(mask, dtype=bool)
    new_idx = np.asarray(indices)[:, mask]
    new_vals = (np.asarray(values, dtype=np.float32)[mask] / np.float32(keep_rate)).astype(
        np.float32)
    return new_idx, new_vals


def nonzero_threshold(dense, thresh=0.0):
    """torch.nonzero(H > thresh) row-major (EquivSetGNN.generate_V_E,
    model/layers/layers2/EquivSetGNN2.py:105-133): V = rows, E = cols."""
    r, c = np.nonzero(np.asarray(dense) > thresh)
    return r.astype(np.int64), c.astype(np.int64)


# ---------------------------------------------------------------------------------------------
# Propagation (float64)
# ---------------------------------------------------------------------------------------------
def spmm_coo(rows, cols, vals, n_rows, X):
    """Y = A·X for COO A (torch.sparse.mm(adj, X), HCCF.py:199); float64, duplicates summed."""
    X = np.asarray(X, dtype=np.float64)
    Y = np.zeros((n_rows, X.shape[1]), dtype=np.float64)
    w = np.ones(len(rows)) if vals is None else np.asarray(vals, dtype=np.float64)
    np.add.at(Y, np.asarray(rows), w[:, None] * X[np.asarray(cols)])
    return Y


def spmm_csr(rowptr, col, X, val=None, row_scale=None, epi=None, slope=0.0, absolute=False):
    """The hgd_spmm contract in float64: Y[r] = epi(s[r]·Σ val[e]·X[col[e]]).
    ``absolute=True`` returns Σ|s·val·X| (the magnitude the fp32 tolerance is scaled by)."""
    X = np.asarray(X, dtype=np.float64)
    n_rows = len(rowptr) - 1
    rows = np.repeat(np.arange(n_rows), np.diff(rowptr))
    w = np.ones(len(col)) if val is None else np.asarray(val, dtype=np.float64)
    s = np.ones(n_rows) if row_scale is None else np.asarray(row_scale, dtype=np.float64)
    terms = w[:, None] * X[np.asarray(col, dtype=np.int64)]
    if absolute:
        terms = np.abs(terms)
    Y = np.zeros((n_rows, X.shape[1]))
    np.add.at(Y, rows, terms)
    Y *= (np.abs(s) if absolute else s)[:, None]
    if not absolute:
        Y = epilogue(Y, epi, slope)
    return Y


def epilogue(Y, epi, slope):
    """nn.LeakyReLU(negative_slope) / nn.ReLU (HGCNConv act=True, HGNN_HD4.py:459-460)."""
    if epi == "leaky_relu":
        return np.where(Y > 0, Y, Y * slope)
    if epi == "relu":
        return np.where(Y > 0, Y, 0.0)
    return Y


def degree_scale(deg, power):
    """deg^power with 0 → 0 (np.power(.., -p) then inf→0, data/graph.py:15-16)."""
    deg = np.asarray(deg, dtype=np.float64)
    out = np.zeros_like(deg)
    nz = deg != 0
    out[nz] = np.power(deg[nz], power)
    return out


def scatter_mean(src, index, dim_size=None):
    """torch_scatter.scatter(src, index, dim=-2, reduce='mean') (pytorch-scatter 2.1.0,
    selfrec.yml:181): out size dim_size or max(index)+1, sum / clamp(count, min=1)."""
    src = np.asarray(src, dtype=np.float64)
    index = np.asarray(index, dtype=np.int64)
    n = dim_size if dim_size is not None else (int(index.max()) + 1 if len(index) else 0)
    out = np.zeros((n, src.shape[1]))
    np.add.at(out, index, src)
    cnt = np.bincount(index, minlength=n).astype(np.float64)
    return out / np.maximum(cnt, 1.0)[:, None]


def equivset_mean_2hop(X, V, E, N):
    """EquivSetConv.forward core with W1 = Identity, W2 = the Xev slice (mlp2_layers = 0),
    alpha = 0 (layers2/EquivSetConv2.py:85-97; args HGNN_HD4.py:371-388):
    Xe = scatter_mean(X[V], E); Xv = scatter_mean(Xe[E], V, dim_size=N)."""
    X = np.asarray(X, dtype=np.float64)
    Xe = scatter_mean(X[V], E)
    return scatter_mean(Xe[E], V, dim_size=N)


def two_hop(rows, cols, vals, shape, X, P=None, Q=None, R=None, epi=None, slope=0.0):
    """epi(P·A·Q·Aᵀ·R·X) for COO A with named diagonal scales (None/'mean'/'sym'/'wmean'/
    'wsym'); HGCNConv is P=Q=R=None (HGNN_HD4.py:455-462), hgconv2 is P=R='sym', Q='mean'
    (data/graph.py:28-42), the ED-HNN mean pair is P=Q='mean' (EquivSetConv2.py:88-93)."""
    n_r, n_c = shape
    rows = np.asarray(rows, dtype=np.int64)
    cols = np.asarray(cols, dtype=np.int64)
    w = np.ones(len(rows)) if vals is None else np.asarray(vals, dtype=np.float64)
    Ps = _scale(rows, w, n_r, P)
    Qs = _scale(cols, w, n_c, Q)
    Rs = _scale(rows, w, n_r, R)
    X = np.asarray(X, dtype=np.float64) * Rs[:, None]
    M = spmm_coo(cols, rows, w, n_c, X) * Qs[:, None]
    Y = spmm_coo(rows, cols, w, n_r, M) * Ps[:, None]
    return epilogue(Y, epi, slope)


def two_hop_backward(rows, cols, vals, shape, Y_out, dY, P=None, Q=None, R=None, epi=None,
                     slope=0.0):
    """dX of :func:`two_hop`: dZ = dY·epi'(Z); dX = R·A·Q·Aᵀ·P·dZ."""
    n_r, n_c = shape
    rows = np.asarray(rows, dtype=np.int64)
    cols = np.asarray(cols, dtype=np.int64)
    w = np.ones(len(rows)) if vals is None else np.asarray(vals, dtype=np.float64)
    dZ = np.asarray(dY, dtype=np.float64)
    if epi == "leaky_relu":
        dZ = np.where(np.asarray(Y_out) > 0, dZ, dZ * slope)
    elif epi == "relu":
        dZ = np.where(np.asarray(Y_out) > 0, dZ, 0.0)
    Ps = _scale(rows, w, n_r, P)
    Qs = _scale(cols, w, n_c, Q)
    Rs = _scale(rows, w, n_r, R)
    dM = spmm_coo(cols, rows, w, n_c, dZ * Ps[:, None]) * Qs[:, None]
    return spmm_coo(rows, cols, w, n_r, dM) * Rs[:, None]


def _scale(idx, w, n, kind):
    if kind is None:
        return np.ones(n)
    weighted = kind.startswith("w")
    base = kind[1:] if weighted else kind
    deg = np.zeros(n)
    np.add.at(deg, idx, w if weighted else 1.0)
    return degree_scale(deg, {"mean": -1.0, "sym": -0.5}[base])


def hgconv2(H, X):
    """D_v^-1/2·H·D_e^-1·Hᵀ·D_v^-1/2·X for a scipy incidence H [V,E] (data/graph.py:28-42)."""
    H = H.tocoo()
    return two_hop(H.row, H.col, None, H.shape, X, P="sym", Q="mean", R="sym")


def layer_norm(X, weight=None, bias=None, eps=1e-5):
    """nn.LayerNorm(d) over the last dim (MLP InputNorm, model/layers/MLP.py:65-71)."""
    X = np.asarray(X, dtype=np.float64)
    mu = X.mean(-1, keepdims=True)
    var = X.var(-1, keepdims=True)
    Y = (X - mu) / np.sqrt(var + eps)
    if weight is not None:
        Y = Y * weight
    if bias is not None:
        Y = Y + bias
    return Y


def row_epilogue(Z, act=None, slope=0.0, ln=False, gamma=None, beta=None, eps=1e-5,
                 out_scale=1.0, res1=None, s1=1.0, res2=None, s2=1.0):
    """The torch op chain after an HGCNConv two-hop that hgd_spmm_fused runs in its store:
    ``Xe = LN0(leaky(Z)) + Xve`` (model/layers/EquivSetConv.py:86-92, HGNN_HD3.py:705-712) and
    ``(1-α)·(LN1(leaky(Z')) + Xev) + α·X0`` (EquivSetConv.py:100-104), or the restart blend
    ``(1-α)·Xv + α·X0`` of layers2/EquivSetConv2.py:96. Returns (Y, a) with a = act(Z)."""
    a = epilogue(np.asarray(Z, dtype=np.float64), act, slope)
    b = layer_norm(a, gamma, beta, eps) if ln else a
    Y = out_scale * b
    if res1 is not None:
        Y = Y + s1 * np.asarray(res1, dtype=np.float64)
    if res2 is not None:
        Y = Y + s2 * np.asarray(res2, dtype=np.float64)
    return Y, a


def row_epilogue_backward(Z, dY, act=None, slope=0.0, ln=False, gamma=None, eps=1e-5,
                          out_scale=1.0):
    """Gradient of :func:`row_epilogue` w.r.t. Z, γ and β (the autograd of nn.LayerNorm and
    nn.LeakyReLU as torch defines them): returns (dZ, dgamma, dbeta)."""
    Z = np.asarray(Z, dtype=np.float64)
    a = epilogue(Z, act, slope)
    dy = out_scale * np.asarray(dY, dtype=np.float64)
    dgamma = dbeta = None
    if ln:
        d = a.shape[-1]
        mu = a.mean(-1, keepdims=True)
        rstd = 1.0 / np.sqrt(a.var(-1, keepdims=True) + eps)
        ah = (a - mu) * rstd
        g = np.ones(d) if gamma is None else np.asarray(gamma, dtype=np.float64)
        gh = dy * g
        da = rstd * (gh - gh.mean(-1, keepdims=True) - ah * (gh * ah).mean(-1, keepdims=True))
        dgamma = (dy * ah).sum(0)
        dbeta = dy.sum(0)
    else:
        da = dy
    if act == "leaky_relu":
        da = np.where(Z > 0, da, da * slope)
    elif act == "relu":
        da = np.where(Z > 0, da, 0.0)
    return da, dgamma, dbeta


def contrast_loss(E1, E2, nodes, temp):
    """contrastLoss, util/loss_torch.py:103-110: InfoNCE between the batch rows of two
    row-normalised tables (F.normalize(x + 1e-8), eps 1e-12), float64."""
    def normalize(X):
        X = np.asarray(X, dtype=np.float64) + 1e-8
        n = np.sqrt((X * X).sum(-1, keepdims=True))
        return X / np.maximum(n, 1e-12)
    nodes = np.asarray(nodes, dtype=np.int64)
    P1 = normalize(E1)[nodes]
    P2 = normalize(E2)[nodes]
    nume = np.exp((P1 * P2).sum(-1) / temp)
    deno = np.exp(P1 @ P2.T / temp).sum(-1) + 1e-8
    return float(-np.log(nume / deno).mean())


def linear(X, W, b=None):
    """nn.Linear: X·Wᵀ + b."""
    Y = np.asarray(X, dtype=np.float64) @ np.asarray(W, dtype=np.float64).T
    return Y if b is None else Y + b


def equivset_conv(X, V, E, X0, alpha, ln_w, ln_b, lin_w, lin_b):
    """EquivSetConv2.forward with the HGNN_HD4 configuration (W1 = Identity, W2 = slice,
    W = MLP('ln', InputNorm, 1 layer) = Linear(LayerNorm(·))), layers2/EquivSetConv2.py:85-100,
    model/layers/MLP.py:65-72,109-117."""
    N = X.shape[0]
    Xv = equivset_mean_2hop(X, V, E, N)
    Xv = (1 - alpha) * Xv + alpha * np.asarray(X0, dtype=np.float64)
    return linear(layer_norm(Xv, ln_w, ln_b), lin_w, lin_b)


# ---------------------------------------------------------------------------------------------
# HCCF encoder (dense learned hypergraph) — model/graph/HCCF.py:173-211
# ---------------------------------------------------------------------------------------------
def hccf_forward(norm_adj_rows, norm_adj_cols, norm_adj_vals, N, E_u, E_i, W_u, W_i, n_layers):
    """HCCFEncoder.forward with keep_rate = 1 and dropout off (HCCF.py:173-191): per layer
    gcn = Â·h, hyper_u = H_u·(H_uᵀ·h_u) with H_u = E_u·W_u (same for items); h += gcn + hyper."""
    E_u = np.asarray(E_u, dtype=np.float64)
    E_i = np.asarray(E_i, dtype=np.float64)
    Hu = E_u @ np.asarray(W_u, dtype=np.float64)
    Hi = E_i @ np.asarray(W_i, dtype=np.float64)
    U = E_u.shape[0]
    h = np.concatenate([E_u, E_i], 0)
    hidden = [h]
    gcns, hyps = [], []
    for _ in range(n_layers):
        g = spmm_coo(norm_adj_rows, norm_adj_cols, norm_adj_vals, N, hidden[-1])
        hu = Hu @ (Hu.T @ hidden[-1][:U])
        hi = Hi @ (Hi.T @ hidden[-1][U:])
        hyp = np.concatenate([hu, hi], 0)
        gcns.append(g)
        hyps.append(hyp)
        hidden.append(g + hyp)
    emb = sum(hidden)
    return emb[:U], emb[U:], gcns, hyps


# ---------------------------------------------------------------------------------------------
# Synthetic graphs (SURVEY.md §8d generator)
# ---------------------------------------------------------------------------------------------
def synthetic_incidence(n_users, n_items, nnz, seed=0, zipf=None):
    """U×I binary incidence: PCG64(seed) uniform users and items (or Zipf(zipf) items,
    truncated to I), deduplicated, row-major sorted. Returns (rows, cols) int64."""
    rng = np.random.Generator(np.random.PCG64(seed))
    u = rng.integers(0, n_users, size=nnz, dtype=np.int64)
    if zipf is None:
        i = rng.integers(0, n_items, size=nnz, dtype=np.int64)
    else:
        ranks = np.arange(1, n_items + 1, dtype=np.float64)
        p = ranks ** (-float(zipf))
        p /= p.sum()
        i = rng.choice(n_items, size=nnz, p=p).astype(np.int64)
    key = np.unique(u * n_items + i)
    return key // n_items, key % n_items


# ---------------------------------------------------------------------------------------------
# Evaluation top-K — base/graph_recommender.py:61-92, util/algorithm.py:143-173
# ---------------------------------------------------------------------------------------------
def find_k_largest(K, candidates):
    """Literal restatement of the numba find_k_largest (util/algorithm.py:143-173), including
    its re-scan of the first K candidates (so a top item among them is listed twice)."""
    cand = list(candidates)
    n = [(iid, s) for iid, s in enumerate(cand[:K])]
    n.sort(key=lambda d: d[1], reverse=True)
    scores = [x[1] for x in n]
    ids = [x[0] for x in n]
    for iid, score in enumerate(cand):
        ind = K
        l, r = 0, K - 1
        if scores[r] < score:
            while r >= l:
                mid = int((r - l) / 2) + l
                if scores[mid] >= score:
                    l = mid + 1
                elif scores[mid] < score:
                    r = mid - 1
                if r < l:
                    ind = r
                    break
        if ind < K - 2:
            scores[ind + 2:] = scores[ind + 1:-1]
            ids[ind + 2:] = ids[ind + 1:-1]
        if ind < K - 1:
            scores[ind + 1] = score
            ids[ind + 1] = iid
    return ids, scores


def topk_closed_form(K, candidates):
    """The same result as :func:`find_k_largest`: the first K of {(c_j, j): j < K} (seed) ∪
    {(c_i, i)} ordered by score desc, seed first, index asc (vectorised, for large rows)."""
    c = np.asarray(candidates)
    n = len(c)
    sc = np.concatenate([c[:K], c])
    seed = np.concatenate([np.ones(K, np.int64), np.zeros(n, np.int64)])
    idx = np.concatenate([np.arange(K), np.arange(n)])
    order = np.lexsort((idx, -seed, -sc.astype(np.float64)))[:K]
    return idx[order].tolist(), sc[order].tolist()


def masked_scores(user_emb, item_emb, users, rated, mask_value=-10e8):
    """score = user_emb[u]·item_embᵀ with every rated item set to -10e8
    (GraphRecommender.test, base/graph_recommender.py:73-80); float64 scores."""
    S = np.asarray(user_emb, np.float64)[users] @ np.asarray(item_emb, np.float64).T
    for r, u in enumerate(users):
        S[r, list(rated[u])] = mask_value
    return S


# ---------------------------------------------------------------------------------------------
# Ranking metrics — util/evaluation.py:8-97 (Metric) and :169-196 (ranking_evaluation)
# ---------------------------------------------------------------------------------------------
def ranking_evaluation(origin, res, N):
    """Literal restatement of ranking_evaluation (util/evaluation.py:169-196) over
    origin = {user: {item: rating}} and res = {user: [(item, score), ...]}: per N the
    'Top N', 'Hit Ratio', 'Precision', 'Recall', 'NDCG' strings, with Metric.hits (:8-15),
    hit_ratio (:17-29), precision (:49-52), recall (:54-58) and NDCG (:84-97) in their loop
    order (plain ``+=`` sums, math.log(n+2, 2) discounts, round(·, 5))."""
    import math

    measure = []
    for n in N:
        predicted = {user: res[user][:n] for user in res}
        if len(origin) != len(predicted):
            raise ValueError("The Lengths of test set and predicted set do not match!")
        hits = {}
        for user in origin:                                   # Metric.hits
            items = list(origin[user].keys())
            pred = [item[0] for item in predicted[user]]
            hits[user] = len(set(items).intersection(set(pred)))
        total_num = 0                                         # Metric.hit_ratio
        for user in origin:
            total_num += len(list(origin[user].keys()))
        hit_num = 0
        for user in hits:
            hit_num += hits[user]
        hr = round(hit_num / total_num, 5)
        prec = 0                                              # Metric.precision
        for u in hits:
            prec += hits[u]
        prec = round(prec / (len(hits) * n), 5)
        recall_list = [hits[u] / len(origin[u]) for u in hits]  # Metric.recall
        s = 0
        for v in recall_list:
            s += v
        recall = round(s / len(recall_list), 5)
        sum_ndcg = 0                                          # Metric.NDCG
        for user in predicted:
            dcg = 0
            idcg = 0
            for k, item in enumerate(predicted[user]):
                if item[0] in origin[user]:
                    dcg += 1.0 / math.log(k + 2, 2)
            for k, item in enumerate(list(origin[user].keys())[:n]):
                idcg += 1.0 / math.log(k + 2, 2)
            sum_ndcg += dcg / idcg
        ndcg = round(sum_ndcg / len(predicted), 5)
        measure.append('Top ' + str(n) + '\n')
        measure += ['Hit Ratio:' + str(hr) + '\n', 'Precision:' + str(prec) + '\n',
                    'Recall:' + str(recall) + '\n', 'NDCG:' + str(ndcg) + '\n']
    return measure


# ---------------------------------------------------------------------------------------------
# Pairwise sampler — util/sampler.py:237-264
# ---------------------------------------------------------------------------------------------
def next_batch_pairwise(data, batch_size, n_negs=1):
    """Restatement of next_batch_pairwise (util/sampler.py:237-264) on Python's ``random``:
    in-place shuffle of data.training_data, then per record n_negs random.choice draws over
    list(data.item.keys()), redrawn while in data.training_set_u[user]. Yields dense-id lists."""
    from random import choice, shuffle

    training_data = data.training_data
    shuffle(training_data)
    ptr = 0
    data_size = len(training_data)
    while ptr < data_size:
        batch_end = ptr + batch_size if ptr + batch_size < data_size else data_size
        users = [training_data[idx][0] for idx in range(ptr, batch_end)]
        items = [training_data[idx][1] for idx in range(ptr, batch_end)]
        ptr = batch_end
        u_idx, i_idx, j_idx = [], [], []
        item_list = list(data.item.keys())
        for i, user in enumerate(users):
            i_idx.append(data.item[items[i]])
            u_idx.append(data.user[user])
            for _ in range(n_negs):
                neg_item = choice(item_list)
                while neg_item in data.training_set_u[user]:
                    neg_item = choice(item_list)
                j_idx.append(data.item[neg_item])
        yield u_idx, i_idx, j_idx


def dropout_keep_mask(seed, n, keep):
    """The keep-mask of the library's device dropout (hgd_dropout_apply and the row GEMM's
    dropout epilogue, hgd_gemm_rows_desc.drop_*: the build's own counter-based RNG for the
    ED-HNN block's nn.Dropout, layers2/EquivSetGNN2.py:91-101; the reference draws torch's
    CUDA philox stream, which no test can share, so the parity tests rebuild these masks here
    and feed them to the float64 reference). Elements 4c .. 4c + 3 (c < 2^30) share one draw:
    h1 = lowbias32(lowbias32(c + lo32(seed)) ^ hi32(seed)), h2 = lowbias32(h1 ^ 0x9E3779B9);
    element 4c + s takes the s-th 16-bit half of (h1, h2), low half first, and is kept iff that
    half is below thr = floor(keep·2^16 + 1/2) computed in float32 (device_util.h
    dropout_keep4). Bit-exact restatement for testing."""
    m32 = np.uint32(0xFFFFFFFF)

    def lowbias32(x):
        x = x ^ (x >> np.uint32(16))
        x = (x * np.uint32(0x7FEB352D)) & m32
        x = x ^ (x >> np.uint32(15))
        x = (x * np.uint32(0x846CA68B)) & m32
        return x ^ (x >> np.uint32(16))

    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    lo, hi = np.uint32(seed & 0xFFFFFFFF), np.uint32(seed >> 32)
    thr = np.uint32(np.float32(keep) * np.float32(65536.0) + np.float32(0.5))
    groups = (int(n) + 3) // 4
    with np.errstate(over="ignore"):
        c = np.arange(groups, dtype=np.uint32)
        h1 = lowbias32(lowbias32((c + lo) & m32) ^ hi)
        h2 = lowbias32(h1 ^ np.uint32(0x9E3779B9))
    halves = np.stack([h1 & np.uint32(0xFFFF), h1 >> np.uint32(16),
                       h2 & np.uint32(0xFFFF), h2 >> np.uint32(16)], axis=1).reshape(-1)
    return (halves < thr)[:int(n)]


def device_keep_mask(seed, n, keep):
    """The keep-mask of the library's device drop-edge draw (hgd_bernoulli_mask /
    hgd_bernoulli_mask_dev: the build's own counter-based RNG for ``SpAdjDropEdge(device_rng=
    True)``; the reference draws ``torch.rand`` on the CPU, HCCF.py:223, which the default path
    reproduces bit for bit instead). u = top 24 bits of splitmix64(seed ^ splitmix64(i)) / 2^24,
    kept iff floor(u + keep) != 0 in float32 — the same Bernoulli(keep) decision rule as
    HCCF.py:223 on a different uniform stream. Bit-exact restatement for testing."""
    m64 = np.uint64(0xFFFFFFFFFFFFFFFF)

    def splitmix64(x):
        with np.errstate(over="ignore"):
            x = (x + np.uint64(0x9E3779B97F4A7C15)) & m64
            x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & m64
            x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & m64
            return x ^ (x >> np.uint64(31))

    i = np.arange(n, dtype=np.uint64)
    h = splitmix64(np.uint64(seed) ^ splitmix64(i))
    u = (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return np.floor(u + np.float32(keep)) != 0
