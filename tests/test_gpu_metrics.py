"""GPU: ranking metrics (hgd_rank_metrics + evaluation.ranking_evaluation) bit-exact with the
reference's ranking_evaluation (util/evaluation.py:169-196) restated in oracle/hgd_oracle.py —
the same strings, from the same float64 arithmetic in the same order."""
import math
from types import SimpleNamespace

import numpy as np
import pytest
import scipy.sparse as sp
import torch

from oracle import hgd_oracle as O

pytestmark = pytest.mark.gpu


def _random_case(rng, n_users, n_items, k, unseen=True):
    """origin {user: {item: 1.0}} with ragged test lists (some items unseen in training), ids
    [n_users, k] with find_k_largest-style duplicates and frequent hits."""
    users = [int(u) for u in rng.permutation(10 * n_users)[:n_users] + 1000]
    item_names = [int(x) for x in rng.permutation(5 * n_items)[:n_items] + 7]
    item_map = {name: i for i, name in enumerate(item_names)}
    origin = {}
    ids = np.empty((n_users, k), dtype=np.int32)
    for r, u in enumerate(users):
        n_test = int(rng.integers(1, 3 * k))
        test = rng.choice(n_items, size=min(n_test, n_items), replace=False)
        d = {item_names[t]: 1.0 for t in test}
        if unseen and r % 3 == 0:
            d[10 ** 9 + r] = 1.0   # a test item the training maps never saw
        origin[u] = d
        # half the list from the test items (hits), the rest random, then seed duplicates
        pool = np.concatenate([test, rng.integers(0, n_items, size=k)])
        row = rng.permutation(pool)[:k]
        if r % 2 == 0 and k >= 4:
            row[k // 2] = row[0]       # a duplicated entry (find_k_largest's seed copy)
            row[k - 1] = row[1]
        ids[r] = row
    return users, item_names, item_map, origin, ids


@pytest.mark.parametrize("n_users,k,topN", [(1, 1, [1]), (37, 10, [10]), (500, 20, [10, 20]),
                                            (300, 40, [5, 10, 20, 40]), (64, 256, [1, 100, 256])])
def test_ranking_evaluation_bit_exact(dev, n_users, k, topN):
    from hypergraph_diffusion_for_recommendation_amd.evaluation import (TestLists,
                                                                         rank_metrics,
                                                                         ranking_evaluation)
    rng = np.random.default_rng(n_users * 7 + k)
    users, names, item_map, origin, ids = _random_case(rng, n_users, 400, k)
    tests = TestLists(origin, item_map, dev)
    d_ids = torch.from_numpy(ids).to(dev)
    got = ranking_evaluation(tests, d_ids, topN)
    res = {u: [(names[i], 0.0) for i in ids[r]] for r, u in enumerate(users)}
    assert got == O.ranking_evaluation(origin, res, topN)
    # per-user values (before any rounding) equal the reference loops exactly
    hits, dcg = rank_metrics(d_ids, tests, sorted(set(topN)))
    for c, n in enumerate(sorted(set(topN))):
        for r, u in enumerate(users):
            pred = [names[i] for i in ids[r][:n]]
            assert hits[r, c] == len(set(origin[u]) & set(pred))
            ref = 0
            for p, name in enumerate(pred):
                if name in origin[u]:
                    ref += 1.0 / math.log(p + 2, 2)
            assert dcg[r, c] == ref


def test_rank_metrics_edges(dev):
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd.evaluation import TestLists, rank_metrics
    origin = {1: {5: 1.0}, 2: {99: 1.0}, 3: {6: 1.0, 7: 1.0}}
    item_map = {5: 0, 6: 1, 7: 2}
    tests = TestLists(origin, item_map, dev)
    ids = torch.tensor([[0, 0, 1], [1, 2, 0], [-1, 2, 2]], dtype=torch.int32, device=dev)
    hits, dcg = rank_metrics(ids, tests, [1, 3])
    assert hits.tolist() == [[1, 1], [0, 0], [0, 1]]
    disc = [1.0 / math.log(n + 2, 2) for n in range(3)]
    assert dcg[0].tolist() == [disc[0], disc[0] + disc[1]]   # a duplicated hit counts twice
    assert dcg[2].tolist() == [0.0, disc[1] + disc[2]]
    with pytest.raises(nat.HGDNativeError):
        rank_metrics(ids, tests, [3, 1])          # cut-offs must ascend
    with pytest.raises(nat.HGDNativeError):
        rank_metrics(ids, tests, [4])             # and stay within k
    # empty test user list: nothing to launch
    empty = TestLists({}, item_map, dev)
    h, d = rank_metrics(torch.zeros((0, 3), dtype=torch.int32, device=dev), empty, [1])
    assert h.shape == (0, 1) and d.shape == (0, 1)


def test_evaluate_test_users_matches_reference_pipeline(dev):
    """GraphRecommender.test() (score, mask rated -10e8, find_k_largest, names) + ranking_evaluation,
    restated on the host, against evaluate_test_users on the device."""
    from hypergraph_diffusion_for_recommendation_amd.evaluation import evaluate_test_users
    rng = np.random.default_rng(11)
    U, I, d = 120, 300, 16
    R = sp.random(U, I, density=0.05, random_state=4, format="csr", dtype=np.float32)
    R.data[:] = 1.0
    user = {u + 500: u for u in range(U)}
    item = {i * 3 + 1: i for i in range(I)}
    id2item = {v: k for k, v in item.items()}
    test_set = {}
    for u in rng.permutation(U)[:90]:
        n = int(rng.integers(1, 15))
        picks = rng.choice(I, size=n, replace=False)
        test_set[int(u) + 500] = {id2item[int(p)]: 1.0 for p in picks}
    data = SimpleNamespace(test_set=test_set, user=user, item=item, id2item=id2item,
                           interaction_mat=R)
    # small-integer embeddings: exact fp32 scores, so the GPU GEMM and numpy agree bitwise and
    # ties are frequent (the find_k_largest duplicates and tie order matter)
    ue = rng.integers(-2, 3, size=(U, d)).astype(np.float32)
    ie = rng.integers(-2, 3, size=(I, d)).astype(np.float32)
    topN = [10, 20]
    measure, ids, _ = evaluate_test_users(data, torch.from_numpy(ue).to(dev),
                                          torch.from_numpy(ie).to(dev), topN)
    rated = [set(R.indices[R.indptr[u]:R.indptr[u + 1]].tolist()) for u in range(U)]
    res = {}
    for u in test_set:
        S = O.masked_scores(ue, ie, [user[u]], rated)[0]
        rid, rsc = O.find_k_largest(max(topN), S)
        res[u] = [(id2item[i], s) for i, s in zip(rid, rsc)]
    assert measure == O.ranking_evaluation(test_set, res, topN)
