#!/usr/bin/env python3
"""HCCF's drop-edge hop (HCCF.py:199) on a SKEWED catalogue — the plugin epoch's set
(bench_plugin_epoch.py: 31,668 uniform users × 38,048 items with Zipf(1.2) popularity, 1.17 M
interactions) — under several long-row split plans (threshold, chunk): event-timed medians of
the masked view's forward (CSR) and backward (CSC) hops at d = 64, with the degree profile.
Prints one JSON line."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import numpy as np
    import torch

    import refops as R
    from hypergraph_diffusion_for_recommendation_amd.incidence import Incidence, spmm_csr
    dev = torch.device("cuda")
    nu, ni, n, d, keep = 31_668, 38_048, 1_170_000, 64, 0.5
    rng = np.random.default_rng(0)
    u = rng.integers(0, nu, n)
    i = rng.zipf(1.2, n) % ni
    key = np.unique(u * ni + i)
    u, i = key // ni, key % ni
    A = R.normalize_graph_mat(R.bipartite_adjacency(u, i, nu, ni)).tocoo()
    deg = np.bincount(A.row, minlength=A.shape[0])
    out = {"nnz": int(A.nnz), "rows": int(A.shape[0]), "max_degree": int(deg.max()),
           "rows_over": {str(t): int((deg > t).sum()) for t in (128, 256, 512, 1024, 2048)},
           "nnz_in_rows_over": {str(t): int(deg[deg > t].sum()) for t in (256, 512, 2048)}}
    idx = torch.from_numpy(np.stack([A.row, A.col]).astype("int64"))
    val = torch.from_numpy(A.data.astype("float32"))
    X = torch.randn(A.shape[1], d, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)

    def timed(fn, reps=100):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return round(statistics.median(ts), 1)

    plans = {}
    ref = None
    for thr, chunk in ((None, None), (2048, 512), (1024, 256), (512, 256), (512, 128),
                       (256, 128), (256, 64), (128, 64)):
        inc = Incidence.from_coo(idx, val, A.shape, device=dev, split_threshold=thr,
                                 split_chunk=chunk)
        mask = (torch.rand(inc.nnz, device=dev, generator=torch.Generator(device=dev)
                           .manual_seed(1)) < keep).to(torch.uint8)
        view = inc.masked(mask, keep)
        child = inc.drop(mask, keep)
        name = "auto" if thr is None else f"{thr}/{chunk}"
        rec = {"csr_heavy": inc.csr.n_heavy, "masked_fwd_us": timed(lambda: spmm_csr(view.csr, X, view.val)),
               "masked_bwd_us": timed(lambda: spmm_csr(view.csc, X, view.val_t)),
               "compacted_fwd_us": timed(lambda: spmm_csr(child.csr, X, child.val)),
               "full_fwd_us": timed(lambda: spmm_csr(inc.csr, X, inc.val))}
        y = spmm_csr(view.csr, X, view.val)
        if ref is None:
            ref = spmm_csr(child.csr, X, child.val).double()
        rec["max_rel_vs_first_compacted"] = float(((y.double() - ref).abs().max(1).values
                                                   / ref.abs().max(1).values.clamp_min(1e-30)
                                                   ).max())
        plans[name] = rec
        del inc, view, child
    out["plans"] = plans
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
