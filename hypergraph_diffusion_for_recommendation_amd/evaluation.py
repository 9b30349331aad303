"""Batched scoring + top-K recommendation lists.

Replaces the per-user loop of ``GraphRecommender.test()`` (base/graph_recommender.py:61-92 in the
reference): for each test user ``predict(u)`` = ``user_emb[u] @ item_emb.T`` copied to the host,
rated items set to -10e8, then numba ``find_k_largest`` (util/algorithm.py:143-173). Here users
are scored in batches with one library GEMM (rocBLAS via torch.mm), the rated items are masked
by ``hgd_mask_scores`` and the lists come from ``hgd_topk_rows``, which reproduces
find_k_largest's ordering exactly — including its duplicated entries for top items among the
first K candidates. Only the [n_users, K] result crosses to the host.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as nat
from .incidence import CSR

MASK_VALUE = -10e8  # base/graph_recommender.py:80


def rated_csr(interaction_mat, device) -> CSR:
    """Rated items per user (the training interactions, ``data.user_rated``) as a device CSR
    from the reference's ``data.interaction_mat`` (scipy [n_users, n_items])."""
    m = interaction_mat.tocsr()
    rowptr = torch.from_numpy(m.indptr.astype(np.int64)).to(device)
    col = torch.from_numpy(m.indices.astype(np.int32)).to(device)
    return CSR(rowptr, col, m.shape[0], m.shape[1], split_threshold=0)


def topk_rows(scores: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """find_k_largest(k, row) for every row of a device fp32 score matrix."""
    if scores.dim() != 2 or scores.dtype != torch.float32 or scores.device.type != "cuda":
        raise TypeError("topk_rows: expects a 2-D float32 device tensor")
    if scores.stride(1) != 1:
        scores = scores.contiguous()
    n, m = scores.shape
    ids = torch.empty((n, k), dtype=torch.int32, device=scores.device)
    vals = torch.empty((n, k), dtype=torch.float32, device=scores.device)
    nat.check(nat.load().hgd_topk_rows(scores.data_ptr(), n, m, scores.stride(0), int(k),
                                       ids.data_ptr(), vals.data_ptr(),
                                       torch.cuda.current_stream(scores.device).cuda_stream),
              "hgd_topk_rows")
    return ids, vals


def mask_scores(scores: torch.Tensor, rated: CSR, users: torch.Tensor,
                value: float = MASK_VALUE) -> torch.Tensor:
    """In place: scores[r, rated items of users[r]] = value."""
    row_map = users.to(device=scores.device, dtype=torch.int32).contiguous()
    nat.check(nat.load().hgd_mask_scores(
        scores.data_ptr(), scores.shape[0], scores.stride(0), rated.rowptr.data_ptr(),
        rated.col.data_ptr() if rated.nnz else None, row_map.data_ptr(), float(value),
        torch.cuda.current_stream(scores.device).cuda_stream), "hgd_mask_scores")
    return scores


SCORE_BUFFER_BYTES = 4 << 30  # default user batch: as many score rows as fit in 4 GiB


@torch.no_grad()
def rank_users(user_emb: torch.Tensor, item_emb: torch.Tensor, users: torch.Tensor, rated: CSR,
               k: int, batch: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Top-k (ids, scores) for each user id in ``users``: ``user_emb[u] @ item_emb.T``, rated
    items masked to -10e8, find_k_largest ordering. Returns device int32 / fp32 [len(users), k].

    ``batch`` users are scored per GEMM (default: a 4 GiB score buffer; the [B, d]·[d, I]
    product writes at 1.6 TB/s for B = 4,096 and 2.4 TB/s for B = 8,192 at the Yelp shape)."""
    users = users.to(device=user_emb.device, dtype=torch.int64)
    n = users.numel()
    if batch is None:
        batch = max(1024, SCORE_BUFFER_BYTES // (4 * max(1, item_emb.shape[0])))
    out_ids = torch.empty((n, k), dtype=torch.int32, device=user_emb.device)
    out_sc = torch.empty((n, k), dtype=torch.float32, device=user_emb.device)
    it = item_emb.t().contiguous()
    for b0 in range(0, n, batch):
        ub = users[b0:b0 + batch]
        S = torch.mm(user_emb.index_select(0, ub), it)  # library GEMM (rocBLAS / hipBLASLt)
        mask_scores(S, rated, ub)
        ids, sc = topk_rows(S, k)
        out_ids[b0:b0 + batch] = ids
        out_sc[b0:b0 + batch] = sc
    return out_ids, out_sc


def test_rec_list(data, user_emb: torch.Tensor, item_emb: torch.Tensor, max_N: int,
                  batch: Optional[int] = None) -> Dict:
    """Drop-in for ``GraphRecommender.test()``: ``{user: [(item_name, score), ...]}`` over
    ``data.test_set`` in its iteration order, ready for the reference's ``evaluate()``."""
    users = list(data.test_set)
    if not users:
        return {}
    uid = torch.tensor([data.user[u] for u in users], dtype=torch.int64)
    rated = rated_csr(data.interaction_mat, user_emb.device)
    ids, sc = rank_users(user_emb, item_emb, uid, rated, max_N, batch)
    ids, sc = ids.cpu().numpy(), sc.cpu().numpy()
    rec = {}
    for r, u in enumerate(users):
        rec[u] = [(data.id2item[int(i)], float(s)) for i, s in zip(ids[r], sc[r])]
    return rec
