#!/usr/bin/env python3
"""Prices the peer transport's data path on ONE MI355X at the N = 8 shard shape (VERDICT r3
next 3; SURVEY.md §8e "ring vs mesh"):

* hop 1 of one 32-column slice (CSC hop into the 1 M item rows of a 1.25 M-user shard with
  12.5 M nonzeros, as sharded.ShardedIncidence.two_hop runs it) writing into
    - a plain torch allocation (the RCCL transport's Ms),
    - an hgd_p2p send slot in uncached memory (the default segments),
    - an hgd_p2p send slot in plain device memory (HGD_TUNE_P2P_CACHED = 1);
* k_reduce + k_gather of one slice exchange ([1 M, 32] floats = 128 MB) at the 1/N block sizes
  of N = 2, 4, 8, every "peer" slot a separate local allocation (hgd_p2p_price_local), uncached
  and cached.

Local HBM stands in for the peers: the kernels' own cost, not xGMI's. Prints one JSON object.
    python scripts/bench_p2p_price.py [--reps 20]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=1_250_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=12_500_000)
    ap.add_argument("--width", type=int, default=32)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    import bench
    from hypergraph_diffusion_for_recommendation_amd import Incidence
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_csr
    from hypergraph_diffusion_for_recommendation_amd.sharded import P2PExchange

    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    lib = nat.load()
    U, I, w = a.users, a.items, a.width
    idx = bench.make_graph(U, I, a.edges, 0, None, dev)
    inc = Incidence.from_coo(idx, None, (U, I), device=dev, validate=False, rows_sorted=True)
    del idx
    X = torch.randn(U, 64, device=dev)
    val_t = inc.edge_values("csc", "sym")
    q = inc.scale("col", "mean")
    Xs = X[:, 0:w]

    def time_hop(out):
        for _ in range(3):
            spmm_csr(inc.csc, Xs, val=val_t, row_scale=q, out=out)
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            spmm_csr(inc.csc, Xs, val=val_t, row_scale=q, out=out)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts)

    res = {"shape": {"users": U, "items": I, "nnz": inc.nnz, "slice_width": w,
                     "slice_bytes": I * w * 4}}
    hop = {"plain_torch_buffer": time_hop(torch.empty(I, w, device=dev))}
    for cached in (0, 1):
        nat.check(lib.hgd_set_tuning(11, cached), "hgd_set_tuning")  # P2P_CACHED
        ex = P2PExchange(I * w, 2, dev)
        hop["p2p_slot_" + ("cached" if cached else "uncached")] = time_hop(ex.slot(0, I, w))
        ex.close()
    nat.check(lib.hgd_set_tuning(11, 0), "hgd_set_tuning")
    # algorithmic bytes of the hop (SURVEY §8d B_hop at width w): nnz·(4 + 4w) + I·(4w + 4) + ...
    b_hop = inc.nnz * (4 + 4 * w) + I * (4 * w + 4) + (I + 1) * 4
    res["hop1_slice_ms"] = {k: round(v, 4) for k, v in hop.items()}
    res["hop1_slice_TBps"] = {k: round(b_hop / (v * 1e-3) / 1e12, 3) for k, v in hop.items()}
    res["hop1_algorithmic_bytes"] = b_hop
    st = torch.cuda.current_stream(dev).cuda_stream
    ex_rows = []
    for n in (2, 4, 8):
        for cached in (0, 1):
            mr, mg = ctypes.c_float(), ctypes.c_float()
            nat.check(lib.hgd_p2p_price_local(n, I * w, cached, a.reps, ctypes.byref(mr),
                                              ctypes.byref(mg), st), "hgd_p2p_price_local")
            blk = I * w * 4 / n
            ex_rows.append({
                "nranks": n, "memory": "cached" if cached else "uncached",
                "reduce_ms": round(mr.value, 4), "gather_ms": round(mg.value, 4),
                # reduce reads n blocks and writes 2 (reduced slot + out); gather reads and
                # writes n - 1 blocks
                "reduce_TBps": round((n + 2) * blk / (mr.value * 1e-3) / 1e12, 3),
                "gather_TBps": round(2 * (n - 1) * blk / (mg.value * 1e-3) / 1e12, 3)
                if mg.value > 0 else None})
    res["exchange_kernels_local"] = ex_rows
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
