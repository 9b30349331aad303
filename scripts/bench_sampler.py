"""Pairwise sampler epoch time: the reference's Python loop (restated in oracle/, identical
output) vs sampler.next_batch_pairwise (libhgd host code), Yelp2018-like shape."""
import json
import random
import sys
import time
from collections import defaultdict
from types import SimpleNamespace

import numpy as np

sys.path.insert(0, ".")
from oracle import hgd_oracle as O  # noqa: E402
from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise  # noqa: E402


def make(n_records, n_users, n_items, seed=0):
    rng = np.random.default_rng(seed)
    users = rng.integers(0, n_users, n_records)
    items = rng.zipf(1.2, n_records) % n_items
    td = [[int(u), int(i), 1.0] for u, i in zip(users, items)]
    user, item, tsu = {}, {}, defaultdict(dict)
    for u, i, r in td:
        user.setdefault(u, len(user))
        item.setdefault(i, len(item))
        tsu[u][i] = r
    return SimpleNamespace(training_data=td, user=user, item=item, training_set_u=tsu)


def main():
    n, U, I = 1_170_000, 31_668, 38_048
    out = {"shape": f"{n} records, {U} users, {I} items, batch 4096, 1 negative"}
    d = make(n, U, I)
    random.seed(0)
    t = time.perf_counter()
    for _ in O.next_batch_pairwise(d, 4096):
        pass
    out["reference_python_s"] = round(time.perf_counter() - t, 3)
    d = make(n, U, I)
    random.seed(0)
    list(next_batch_pairwise(d, 4096))  # first epoch builds the dense state
    times = []
    for _ in range(3):
        t = time.perf_counter()
        for _ in next_batch_pairwise(d, 4096):
            pass
        times.append(time.perf_counter() - t)
    out["native_s"] = round(min(times), 4)
    out["speedup"] = round(out["reference_python_s"] / out["native_s"], 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
