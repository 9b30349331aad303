#!/usr/bin/env python3
"""Does blocking the into-items hop by USER range pay on MI355X? The hop Hᵀ·X gathers 256-B rows
of the 2.56 GB user table at random (5.9–6.4 TB/s, the random-gather ceiling), while the
into-users hop, whose 256 MB item table the 256 MB Infinity Cache (MALL) mostly holds, runs at
7.5 TB/s. Here the item hop is split into P phases, phase k summing only the neighbours in user
block k (a CSC of H's rows [u_k, u_k+1)), so each phase gathers from a U/P-row slice of X that
the MALL can hold; the phases accumulate into Y (Y = s·acc_k + Y). The price is P−1 extra
read+write passes over Y. Round 6 first emulated this with one sub-CSC per block and the fused
residual epilogue; it now times the library's hgd_spmm_blocked (one launch per block over the
block-major copy of the CSC, hgd_spmm_col_blocks, selected through HGD_SPMM_BLOCKS) against
hgd_spmm in interleaved rounds and reports the worst relative difference (a different fp32
summation order, so not bitwise).

    python scripts/bench_mall_blocked.py [--dim 64 --rounds 5]
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
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--blocks", default="2,4,8,10,16")
    ap.add_argument("--hop", choices=("items", "users"), default="items",
                    help="items: Hᵀ·X over the CSC (gathers the user table); users: H·M over the "
                         "CSR (gathers the item table)")
    ap.add_argument("--ld", type=int, default=0,
                    help="row stride of X (0 = dim): a column slice of a wider table, as the "
                         "sharded hop's 32-column slices of a d = 64 table")
    ap.add_argument("--unroll", type=int, default=8,
                    help="HGD_TUNE_SPMM_UNROLL for every variant (gathers in flight per lane)")
    ap.add_argument("--policy", type=int, default=8,
                    help="HGD_TUNE_SPMM_POLICY for every variant (8 = the default)")
    ap.add_argument("--seg", type=int, default=0,
                    help="HGD_TUNE_SPMM_BLOCKED_SEG for the blocked variants (1 = segmented walk)")
    ap.add_argument("--pass-cols", type=int, default=0,
                    help="HGD_TUNE_SPMM_PASS_COLS for every variant (0 = the default passes)")
    args = ap.parse_args()

    import torch

    import bench
    from hypergraph_diffusion_for_recommendation_amd import Incidence
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_csr

    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    nat.check(nat.load().hgd_set_tuning(3, args.pass_cols), "pass cols")
    nat.check(nat.load().hgd_set_tuning(2, args.policy), "policy")
    nat.check(nat.load().hgd_set_tuning(1, args.unroll), "unroll")
    nat.check(nat.load().hgd_set_tuning(18, args.seg), "blocked seg")
    dev = torch.device("cuda:0")
    U, I, d = args.users, args.items, args.dim
    idx = bench.make_graph(U, I, args.edges, 0, None, dev)
    inc = Incidence.from_coo(idx, None, (U, I), device=dev, validate=False, rows_sorted=True)
    del idx
    nnz = inc.nnz
    if args.hop == "items":
        S, R = inc.csc, I
        X = torch.randn(U, max(d, args.ld), device=dev)[:, :d]
        q = inc.scale("col", "mean")
        w_full = inc.edge_values("csc", "sym")
    else:
        # make_graph's COO is sorted by (user, item): every CSR row's columns ascend
        S, R = inc.csr, U
        rows = torch.repeat_interleave(torch.arange(U, device=dev), S.degrees())
        same = rows[1:] == rows[:-1]
        assert bool((S.col[1:][same] >= S.col[:-1][same]).all()), "CSR columns not ascending"
        del rows, same
        S.cols_ascending = True
        X = torch.randn(I, d, device=dev)
        q = inc.scale("row", "sym")
        w_full = None
    blocks = [int(p) for p in args.blocks.split(",")]
    for P in blocks:  # block-major copies built outside the timed rounds
        S.col_blocks(P)
        S.blocked_values(P, w_full)

    def run(P):
        # HGD_SPMM_BLOCKS=0: hgd_spmm; =P: hgd_spmm_blocked over P source ranges (spmm_blocks)
        os.environ["HGD_SPMM_BLOCKS"] = str(P)
        return spmm_csr(S, X, val=w_full, row_scale=q)

    ref = run(0)
    res = {"dim": d, "hop": args.hop, "pass_cols": args.pass_cols, "policy": args.policy, "unroll": args.unroll, "seg": args.seg, "ld": args.ld, "nnz": nnz,
           "bytes_algorithmic": nnz * (4 + 4 * d) + R * (4 * d + 4) + (R + 1) * 4, "variants": {}}
    times = {"plain": []}
    times.update({P: [] for P in blocks})
    diffs = {}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for rnd in range(args.rounds + 1):
        for key in ["plain"] + blocks:
            ev[0].record()
            Y = run(0 if key == "plain" else key)
            ev[1].record()
            torch.cuda.synchronize()
            if rnd:
                times[key].append(ev[0].elapsed_time(ev[1]))
            elif key != "plain":
                diffs[key] = float((Y - ref).abs().max() / ref.abs().max())
    for key, ts in times.items():
        ms = statistics.median(ts)
        res["variants"][str(key)] = {"ms": round(ms, 4),
                                     "GBps_algorithmic": round(res["bytes_algorithmic"] / ms / 1e6,
                                                               1),
                                     "max_rel_diff_vs_plain": diffs.get(key, 0.0)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
