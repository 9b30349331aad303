#!/usr/bin/env python3
"""One ED-HNN block variant for K steps (for rocprofv3 per-variant kernel stats).
usage: edhnn_one.py --form mean|spmm --fused 0|1 [--graph 0|1] --steps K"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--form", default="mean")
    ap.add_argument("--fused", type=int, default=1)
    ap.add_argument("--graph", type=int, default=0)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--users", type=int, default=31_668)
    ap.add_argument("--items", type=int, default=38_048)
    ap.add_argument("--edges", type=int, default=1_170_000)
    args = ap.parse_args()
    import numpy as np
    import scipy.sparse as sp
    import torch
    from hypergraph_diffusion_for_recommendation_amd import edhnn_spmm
    from hypergraph_diffusion_for_recommendation_amd.encoders import sparse_tensor_of
    from hypergraph_diffusion_for_recommendation_amd.layers import EquivSetGNN
    import refops as O
    from bench_edhnn import ARGS
    u, i = O.synthetic_incidence(args.users, args.items, args.edges, seed=0)
    ui = O.bipartite_adjacency(u, i, args.users, args.items)
    A = O.normalize_graph_mat(ui)
    N = A.shape[0]
    dev = torch.device("cuda")
    d = 64
    cfg = dict(ARGS, MLP_hidden=d)
    X = torch.randn(N, d, device=dev)
    dY = torch.randn(N, d, device=dev)
    if args.form == "spmm":
        adj = sparse_tensor_of(A, dev)
        m = edhnn_spmm.EquivSetGNN(d, cfg).to(dev).train()
        call = lambda xx: m(xx, adj, N)  # noqa: E731
    else:
        H = sparse_tensor_of(sp.csr_matrix((np.ones(ui.nnz, np.float32), ui.indices, ui.indptr),
                                           shape=ui.shape), dev)
        m = EquivSetGNN(d, cfg, H).to(dev).train()
        call = lambda xx: m(xx, H, N)  # noqa: E731
    m.conv.fused_epilogue = bool(args.fused)
    xs = X.detach().clone().requires_grad_(True)

    def body():
        xs.grad = None
        call(xs).backward(dY)

    step = body
    if args.graph:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                body()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            call(xs).backward(dY)
        step = g.replay
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps * 1e3
    print(f"form={args.form} fused={args.fused} graph={args.graph} ms/step={dt:.4f}", flush=True)


if __name__ == "__main__":
    main()
