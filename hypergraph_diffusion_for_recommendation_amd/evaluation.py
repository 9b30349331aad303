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

import ctypes
import math
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
                                       nat.stream_handle(scores.device)),
              "hgd_topk_rows")
    return ids, vals


def mask_scores(scores: torch.Tensor, rated: CSR, users: torch.Tensor,
                value: float = MASK_VALUE) -> torch.Tensor:
    """In place: scores[r, rated items of users[r]] = value."""
    row_map = users.to(device=scores.device, dtype=torch.int32).contiguous()
    nat.check(nat.load().hgd_mask_scores(
        scores.data_ptr(), scores.shape[0], scores.stride(0), rated.rowptr.data_ptr(),
        rated.col.data_ptr() if rated.nnz else None, row_map.data_ptr(), float(value),
        nat.stream_handle(scores.device)), "hgd_mask_scores")
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


def ndcg_discount(k: int) -> List[float]:
    """1.0/math.log(n+2, 2) for n < k, as Metric.NDCG computes it (util/evaluation.py:92-95)."""
    return [1.0 / math.log(n + 2, 2) for n in range(k)]


class TestLists:
    """The test set of ``ranking_evaluation`` (``origin`` = data.test_set, util/evaluation.py:169)
    on the device: per test user (in the dict's order) the internal ids of its test items that
    exist in the training maps (sorted; items never seen in training can never be recommended,
    so they are never hits) and the full count ``len(origin[user])`` (the recall / hit-ratio /
    IDCG denominators count them)."""

    def __init__(self, origin: Dict, item_map: Dict, device):
        self.users = list(origin)
        counts = np.empty(len(self.users), dtype=np.int64)
        rowptr = np.zeros(len(self.users) + 1, dtype=np.int64)
        cols: List[np.ndarray] = []
        for r, u in enumerate(self.users):
            items = origin[u]
            counts[r] = len(items)
            ids = np.fromiter((item_map[i] for i in items if i in item_map), dtype=np.int64)
            ids.sort()
            cols.append(ids)
            rowptr[r + 1] = rowptr[r] + ids.size
        self.counts = counts
        self.rowptr = torch.from_numpy(rowptr).to(device)
        flat = np.concatenate(cols) if cols else np.zeros(0, dtype=np.int64)
        self.cols = torch.from_numpy(flat.astype(np.int32)).to(device)


@torch.no_grad()
def rank_metrics(ids: torch.Tensor, tests: TestLists, cutoffs: Sequence[int],
                 discount: Optional[torch.Tensor] = None) -> Tuple[np.ndarray, np.ndarray]:
    """hgd_rank_metrics: per test user and cut-off N, the distinct hits among ids[:, :N] and the
    DCG in position order (float64, bit-identical to Metric.NDCG's loop). ids: device int32
    [n_users, k] of internal item ids, rows in ``tests.users`` order."""
    if ids.dim() != 2 or ids.dtype != torch.int32 or ids.device.type != "cuda":
        raise TypeError("rank_metrics: ids must be a 2-D int32 device tensor")
    if ids.shape[0] != len(tests.users):
        raise ValueError(f"rank_metrics: {ids.shape[0]} lists for {len(tests.users)} test users")
    if ids.stride(1) != 1:
        ids = ids.contiguous()
    k = int(ids.shape[1])
    cut = [int(c) for c in cutoffs]
    if discount is None:
        discount = torch.tensor(ndcg_discount(k), dtype=torch.float64, device=ids.device)
    n = ids.shape[0]
    hits = torch.empty((n, len(cut)), dtype=torch.int32, device=ids.device)
    dcg = torch.empty((n, len(cut)), dtype=torch.float64, device=ids.device)
    carr = (ctypes.c_int32 * len(cut))(*cut)
    nat.check(nat.load().hgd_rank_metrics(
        ids.data_ptr(), n, ids.stride(0), k, tests.rowptr.data_ptr(),
        tests.cols.data_ptr() if tests.cols.numel() else None, carr, len(cut),
        discount.data_ptr(), hits.data_ptr(), dcg.data_ptr(),
        nat.stream_handle(ids.device)), "hgd_rank_metrics")
    return hits.cpu().numpy(), dcg.cpu().numpy()


def _seq_sum(values: np.ndarray) -> float:
    """Left-to-right float64 sum, as the reference's ``sum(list)`` / ``+=`` loops round it:
    ``np.cumsum`` accumulates sequentially (``np.sum`` is pairwise and Python >= 3.12's ``sum``
    compensated — both would round differently)."""
    return float(np.cumsum(np.asarray(values, dtype=np.float64))[-1]) if len(values) else 0.0


def ranking_evaluation(tests: TestLists, ids: torch.Tensor, N: Sequence[int]) -> List[str]:
    """Drop-in for ``ranking_evaluation(data.test_set, rec_list, N)`` (util/evaluation.py:169-196)
    when rec_list came from ``rank_users`` for ``tests.users``: the same list of strings
    ('Top N', 'Hit Ratio:…', 'Precision:…', 'Recall:…', 'NDCG:…' per N), the same float64
    arithmetic in the same order, from the device per-user hits / DCG."""
    N = [int(n) for n in N]
    order = sorted(set(N))
    hits, dcg = rank_metrics(ids, tests, order)
    disc = ndcg_discount(max(order))
    idcg_prefix = [0.0]  # IDCG of a c-item test list: the first min(N, c) discounts, in order
    for v in disc:
        idcg_prefix.append(idcg_prefix[-1] + v)
    idcg_prefix = np.asarray(idcg_prefix, dtype=np.float64)
    counts = tests.counts.astype(np.int64)
    total_num = int(counts.sum())  # Metric.hit_ratio (:17-29), integer
    n_users = len(counts)
    measure: List[str] = []
    for n in N:
        c = order.index(n)
        h = hits[:, c].astype(np.int64)
        hit_num = int(h.sum())
        hr = round(hit_num / total_num, 5)
        prec = round(hit_num / (n_users * n), 5)                                  # :49-52
        recall = round(_seq_sum(h / counts) / n_users, 5)                         # :54-58
        ndcg = round(_seq_sum(dcg[:, c] / idcg_prefix[np.minimum(counts, n)]) / n_users,
                     5)                                                           # :84-97
        measure.append('Top ' + str(n) + '\n')
        measure += ['Hit Ratio:' + str(hr) + '\n', 'Precision:' + str(prec) + '\n',
                    'Recall:' + str(recall) + '\n', 'NDCG:' + str(ndcg) + '\n']
    return measure


def evaluate_test_users(data, user_emb: torch.Tensor, item_emb: torch.Tensor,
                        topN: Sequence[int], tests: Optional[TestLists] = None,
                        rated: Optional[CSR] = None,
                        batch: Optional[int] = None) -> Tuple[List[str], torch.Tensor,
                                                              torch.Tensor]:
    """GraphRecommender.test() + ranking_evaluation (base/graph_recommender.py:61-92, 130-133)
    on the device up to the per-user counts: scores, masking, find_k_largest lists and the
    metric inputs. Returns (measure strings, ids, scores); ids / scores are the device
    [n_test_users, max(topN)] lists in data.test_set order (internal item ids)."""
    if tests is None:
        tests = TestLists(data.test_set, data.item, user_emb.device)
    if rated is None:
        rated = rated_csr(data.interaction_mat, user_emb.device)
    if not tests.users:
        raise ValueError("evaluate_test_users: empty test set")
    uid = torch.tensor([data.user[u] for u in tests.users], dtype=torch.int64)
    ids, sc = rank_users(user_emb, item_emb, uid, rated, max(int(n) for n in topN), batch)
    return ranking_evaluation(tests, ids, topN), ids, sc


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
