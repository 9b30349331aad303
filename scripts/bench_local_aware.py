#!/usr/bin/env python3
"""HGNN_HD4's local encoder (LocalAwareEncoder, HGNN_HD4.py:390-405; BASELINE configs[3]:
Amazon-Book-shaped "hypergraph diffusion", d = 128) fwd + bwd on one MI355X, train mode: the
ED-HNN block(s) over ui_adj and the last LN(HGCNConv) + residual layer over norm_adj, with a
fixed random upstream gradient. Variants: eager, and the same step replayed from one captured
HIP graph (static input / gradient). Prints one JSON line per variant."""
import argparse
import json
import os
import statistics
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=52_643)
    ap.add_argument("--items", type=int, default=91_599)
    ap.add_argument("--edges", type=int, default=2_240_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="eager,graph")
    args = ap.parse_args()
    import torch

    import refops as R
    from hypergraph_diffusion_for_recommendation_amd.encoders import LocalAwareEncoder

    dev = torch.device("cuda")
    U, I, d = args.users, args.items, args.dim
    u, i = R.synthetic_incidence(U, I, args.edges, seed=0)
    ui = R.bipartite_adjacency(u, i, U, I).tocsr()
    data = types.SimpleNamespace(n_users=U, n_items=I, ui_adj=ui,
                                 norm_adj=R.normalize_graph_mat(ui).tocsr())
    torch.manual_seed(0)
    enc = LocalAwareEncoder(data, d, d, args.layers, 0.3, 0.2, device=dev).train()
    g = torch.Generator(device=dev).manual_seed(1)
    ego = torch.randn(U + I, d, device=dev, generator=g).requires_grad_(True)
    gout = torch.randn(U + I, d, device=dev, generator=g)

    def step():
        # a training step's gradients start empty (optimizer.zero_grad(set_to_none=True)):
        # no accumulation into last step's .grad
        enc.zero_grad(set_to_none=True)
        ego.grad = None
        ue, ie = enc(ego, enc.sparse_norm_adj)
        torch.autograd.backward([ue, ie], [gout[:U], gout[U:]])

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts)

    out = []
    want = args.variants.split(",")
    if "eager" in want:
        out.append(("eager", timed(step)))
    if "graph" in want:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                step()
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            step()
        out.append(("graph", timed(graph.replay)))
    for name, ms in out:
        print(json.dumps({"variant": name, "ms_per_step": round(ms, 3), "users": U, "items": I,
                          "interactions": len(u), "d": d, "layers": args.layers}), flush=True)


if __name__ == "__main__":
    main()
