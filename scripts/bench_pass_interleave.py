#!/usr/bin/env python3
"""A/B of HGD_TUNE_SPMM_PASS_INTERLEAVE at the bench graph: a row wider than one column pass
(d = 256 → four 64-column passes) as one launch per pass (0) or as one launch whose workgroups
walk a row block's passes back to back on one XCD (1). Both hops of hgconv2 (into items: CSC,
into users: CSR), interleaved rounds in one process (guide §5.4 rule 24), median ms per hop and
the algorithmic rate (SURVEY §8d bytes); the outputs are compared bitwise.

    python scripts/bench_pass_interleave.py [--dim 256 --rounds 7]
"""
import argparse
import json
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
    ap.add_argument("--dim", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=7)
    args = ap.parse_args()

    import torch

    import bench
    from hypergraph_diffusion_for_recommendation_amd import Incidence, _native
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_csr

    dev = torch.device("cuda:0")
    U, I, d = args.users, args.items, args.dim
    idx = bench.make_graph(U, I, args.edges, 0, None, dev)
    inc = Incidence.from_coo(idx, None, (U, I), device=dev, validate=False, rows_sorted=True)
    del idx
    nnz = inc.nnz
    X = torch.randn(U, d, device=dev)
    M = torch.randn(I, d, device=dev)
    vcsc = inc.edge_values("csc", "sym")
    q = inc.scale("col", "mean")
    p = inc.scale("row", "sym")
    lib = _native.load()
    bytes_items = nnz * (4 + 4 * d) + I * (4 * d + 4) + (I + 1) * 4
    bytes_users = nnz * (4 + 4 * d) + U * (4 * d + 4) + (U + 1) * 4
    times = {v: {"items": [], "users": []} for v in (0, 1)}
    outs = {}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    try:
        for rnd in range(args.rounds + 1):
            for v in (0, 1):
                _native.check(lib.hgd_set_tuning(17, v), "interleave")
                Yi = torch.empty(I, d, device=dev)
                Yu = torch.empty(U, d, device=dev)
                ev[0].record()
                spmm_csr(inc.csc, X, val=vcsc, row_scale=q, out=Yi)
                ev[1].record()
                spmm_csr(inc.csr, M, row_scale=p, out=Yu)
                ev[2].record()
                torch.cuda.synchronize()
                if rnd:  # round 0 warms up
                    times[v]["items"].append(ev[0].elapsed_time(ev[1]))
                    times[v]["users"].append(ev[1].elapsed_time(ev[2]))
                else:
                    outs[v] = (Yi, Yu)
    finally:
        _native.check(lib.hgd_set_tuning(17, 0), "interleave off")
    res = {"dim": d, "nnz": nnz, "rounds": args.rounds,
           "bitwise_equal": bool(torch.equal(outs[0][0], outs[1][0]) and
                                 torch.equal(outs[0][1], outs[1][1]))}
    for v in (0, 1):
        mi = statistics.median(times[v]["items"])
        mu = statistics.median(times[v]["users"])
        res[f"interleave_{v}"] = {"items_ms": round(mi, 4), "users_ms": round(mu, 4),
                                  "items_GBps": round(bytes_items / mi / 1e6, 1),
                                  "users_GBps": round(bytes_users / mu / 1e6, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
