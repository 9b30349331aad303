#!/usr/bin/env python3
"""Per-step cost of HCCF's edge dropout + GCN hop (SpAdjDropEdge → GCNLayer, HCCF.py:182) on a
dataset-shaped normalised bipartite graph, for: the reference's CPU path (scripts/refops-style
torch CPU ops), the GPU with the reference's CPU mask + from-scratch rebuild, the sort-free
rebuild, and the device mask. Prints one JSON line per variant."""
import argparse
import json
import os
import statistics
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--keep", type=float, default=0.7)
    args = ap.parse_args()
    import numpy as np
    import torch

    from hypergraph_diffusion_for_recommendation_amd import Incidence
    from hypergraph_diffusion_for_recommendation_amd.encoders import sparse_tensor_of
    from hypergraph_diffusion_for_recommendation_amd.layers import GCNLayer, SpAdjDropEdge
    import refops as O

    u, i = O.synthetic_incidence(args.users, args.items, args.edges, seed=0)
    A = O.normalize_graph_mat(O.bipartite_adjacency(u, i, args.users, args.items))
    N = A.shape[0]
    dev = torch.device("cuda")
    adj = sparse_tensor_of(A, dev)
    X = torch.randn(N, args.dim, device=dev)
    gcn = GCNLayer(0.5)

    def run(fn, reps):
        ts = []
        for _ in range(reps + 2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts[2:]) * 1e3

    results = {}
    drop = SpAdjDropEdge()
    results["gpu_sortfree_cpu_mask"] = run(lambda: gcn(drop(adj, args.keep), X), args.reps)
    parent = adj._hgd_incidence
    perm = parent.perm_t
    parent.perm_t = None  # forces the from-scratch rebuild (index narrow, sort, plan count)
    results["gpu_rebuild_cpu_mask"] = run(lambda: gcn(drop(adj, args.keep), X), args.reps)
    parent.perm_t = perm
    ddrop = SpAdjDropEdge(device_rng=True)
    results["gpu_sortfree_device_mask"] = run(lambda: gcn(ddrop(adj, args.keep), X), args.reps)
    results["gpu_hop_only"] = run(lambda: gcn(adj, X), args.reps)
    # reference CPU path: HCCF.py:217-226 + torch.sparse.mm (HCCF.py:199)
    adj_c = torch.sparse_coo_tensor(adj._indices().cpu(), adj._values().cpu(), adj.shape)
    Xc = X.cpu()

    def ref_step():
        vals = adj_c._values()
        idxs = adj_c._indices()
        mask = ((torch.rand(vals.size()) + args.keep).floor()).type(torch.bool)
        a2 = torch.sparse_coo_tensor(idxs[:, mask], vals[mask] / args.keep, adj_c.shape)
        return torch.sparse.mm(a2, Xc)

    results["cpu_reference"] = run(ref_step, max(3, args.reps // 5))
    for k, v in results.items():
        print(json.dumps({"variant": k, "ms_per_step": round(v, 4), "nnz": parent.nnz,
                          "N": N, "d": args.dim, "cpu_threads": torch.get_num_threads()}))


if __name__ == "__main__":
    main()
