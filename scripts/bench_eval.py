#!/usr/bin/env python3
"""Time the batched scoring + top-K evaluation (evaluation.rank_users) for every user of a
dataset-shaped graph, beside the reference's per-user CPU formulation (score row, mask rated
items, find_k_largest ordering via the closed form (scripts/refops); numba is not installed, so the
CPU figure is a numpy port, timed on a user sample and scaled). One JSON line per variant."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=31_668)
    ap.add_argument("--items", type=int, default=38_048)
    ap.add_argument("--edges", type=int, default=1_170_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--k", type=int, default=40)
    ap.add_argument("--cpu-sample", type=int, default=200)
    args = ap.parse_args()
    import numpy as np
    import scipy.sparse as sp
    import torch

    from hypergraph_diffusion_for_recommendation_amd.evaluation import rank_users, rated_csr
    import refops as O

    u, i = O.synthetic_incidence(args.users, args.items, args.edges, seed=0)
    R = sp.csr_matrix((np.ones(len(u), np.float32), (u, i)), shape=(args.users, args.items))
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    ue = torch.randn(args.users, args.dim, device=dev, generator=g)
    ie = torch.randn(args.items, args.dim, device=dev, generator=g)
    rated = rated_csr(R, dev)
    users = torch.arange(args.users)
    rank_users(ue, ie, users, rated, args.k)  # warm-up
    ts = []
    for _ in range(5):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ids, sc = rank_users(ue, ie, users, rated, args.k)
        ids.cpu()
        ts.append(time.perf_counter() - t0)
    gpu_s = sorted(ts)[2]
    print(json.dumps({"variant": "gpu_rank_users", "users": args.users, "items": args.items,
                      "k": args.k, "seconds_all_users": round(gpu_s, 5),
                      "users_per_s": round(args.users / gpu_s, 1)}))
    uec, iec = ue.cpu().numpy(), ie.cpu().numpy()
    n = min(args.cpu_sample, args.users)
    t0 = time.perf_counter()
    for uu in range(n):
        cand = (uec[uu] @ iec.T).astype(np.float32)
        cand[R.indices[R.indptr[uu]:R.indptr[uu + 1]]] = -10e8
        O.topk_closed_form(args.k, cand)
    cpu_s = (time.perf_counter() - t0) / n * args.users
    print(json.dumps({"variant": "cpu_port_per_user", "users": args.users, "items": args.items,
                      "k": args.k, "seconds_all_users": round(cpu_s, 3),
                      "users_per_s": round(args.users / cpu_s, 1),
                      "sample_users": n, "threads": torch.get_num_threads()}))


if __name__ == "__main__":
    main()
