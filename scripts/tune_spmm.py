#!/usr/bin/env python3
"""A/B the hgd_spmm tuning variants (unroll × cache policy) on the bench graph, interleaved in
one process (guide §5.4 rule 24). Prints median ms per hop kind and variant.

    python scripts/tune_spmm.py [--users 10000000 --items 1000000 --edges 100000000 --rounds 5]
"""
import argparse
import itertools
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=100_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--zipf", type=float, default=None)
    ap.add_argument("--unrolls", default="4,8,16")
    ap.add_argument("--policies", default="0,1,2,3,4,5,6,7")
    ap.add_argument("--segmented", default="0,1", help="user-hop kernel variants to A/B")
    args = ap.parse_args()

    import torch

    import bench
    from hypergraph_diffusion_for_recommendation_amd import Incidence, _native
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_csr

    dev = torch.device("cuda:0")
    idx = bench.make_graph(args.users, args.items, args.edges, 0, args.zipf, dev)
    inc = Incidence.from_coo(idx, None, (args.users, args.items), device=dev, validate=False,
                             rows_sorted=True)
    del idx
    X = torch.randn(args.users, args.dim, device=dev)
    vcsc = inc.edge_values("csc", "sym")
    q = inc.scale("col", "mean")
    p = inc.scale("row", "sym")
    M = torch.randn(args.items, args.dim, device=dev)
    Yi = torch.empty(args.items, args.dim, device=dev)
    Yu = torch.empty(args.users, args.dim, device=dev)
    lib = _native.load()
    variants = list(itertools.product([int(u) for u in args.unrolls.split(",")],
                                      [int(x) for x in args.policies.split(",")],
                                      [int(x) for x in args.segmented.split(",")]))
    res = {v: {"items": [], "users": []} for v in variants}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for _ in range(args.rounds):
        for u, pol, seg in variants:
            inc.csr.configure_kernel(segmented=bool(seg))
            _native.check(lib.hgd_set_tuning(1, u), "unroll")
            _native.check(lib.hgd_set_tuning(2, pol), "policy")
            ev[0].record()
            spmm_csr(inc.csc, X, val=vcsc, row_scale=q, out=Yi)
            ev[1].record()
            spmm_csr(inc.csr, M, row_scale=p, out=Yu)
            ev[2].record()
            torch.cuda.synchronize()
            res[(u, pol, seg)]["items"].append(ev[0].elapsed_time(ev[1]))
            res[(u, pol, seg)]["users"].append(ev[1].elapsed_time(ev[2]))
    print(f"graph {args.users}x{args.items}x{inc.nnz} d={args.dim} zipf={args.zipf}")
    print("unroll policy seg  items_ms(med/min)  users_ms(med/min)  sum")
    rows = []
    for v in variants:
        it, us = res[v]["items"], res[v]["users"]
        rows.append((statistics.median(it) + statistics.median(us), v, it, us))
    for s, v, it, us in sorted(rows):
        print(f"{v[0]:6d} {v[1]:6d} {v[2]:3d}  {statistics.median(it):7.4f}/{min(it):7.4f}  "
              f"{statistics.median(us):7.4f}/{min(us):7.4f}  {s:7.4f}")


if __name__ == "__main__":
    main()
