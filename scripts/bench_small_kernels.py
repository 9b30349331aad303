#!/usr/bin/env python3
"""The small-shape dense kernels of the Yelp-shaped carriers, each launched --reps times in
isolation so a ``rocprofv3 --kernel-trace --stats`` run gives their device durations:

* HGNNLayer (HCCF.py:201-211, K = hyper_dim = 32, d = 64, n = 31,668 users): the dense two-hop
  H·(Hᵀ·X) forward and backward through functional.dense_two_hop (split-K Hᵀ·X, row GEMMs);
* Linear (MLP.py:109-117 / lin_in, EquivSetGNN2.py:93-94) at the ED-HNN node count 69,716 × 64:
  forward with ReLU, backward-data, backward-weight;
* InfoNCE (util/loss_torch.py:103-110) at B = 4,096 batch rows of 31,668 × 64 tables.

Prints one JSON line per case with the host-side wall time per call (HIP events around
--reps calls); the per-kernel durations come from the rocprof summary."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--cases", default="hgnn,linear,infonce")
    args = ap.parse_args()
    import torch

    from hypergraph_diffusion_for_recommendation_amd import functional as F
    from hypergraph_diffusion_for_recommendation_amd.layers import Linear

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)

    def timed(name, fn, **info):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        e1.synchronize()
        print(json.dumps({"case": name, "us_per_call": round(e0.elapsed_time(e1) * 1e3 / args.reps, 2),
                          **info}), flush=True)

    cases = args.cases.split(",")
    if "hgnn" in cases:
        n, K, d = 31_668, 32, 64
        H = torch.randn(n, K, device=dev, generator=g).requires_grad_(True)
        X = torch.randn(n, d, device=dev, generator=g).requires_grad_(True)
        dY = torch.randn(n, d, device=dev, generator=g)

        def hgnn():
            Y = F.dense_two_hop(H, X)
            torch.autograd.backward(Y, dY)

        timed("hgnn_fwd_bwd", hgnn, n=n, K=K, d=d)
    if "linear" in cases:
        n, d = 69_716, 64
        lin = Linear(d, d).to(dev)
        Xl = torch.randn(n, d, device=dev, generator=g).requires_grad_(True)
        dYl = torch.randn(n, d, device=dev, generator=g)

        def linear():
            Y = lin(Xl, relu=True)
            torch.autograd.backward(Y, dYl)

        timed("linear_fwd_bwd", linear, n=n, d=d)
    if "infonce" in cases:
        n, d, B = 31_668, 64, 4096
        E1 = torch.randn(n, d, device=dev, generator=g).requires_grad_(True)
        E2 = torch.randn(n, d, device=dev, generator=g).requires_grad_(True)
        nodes = torch.randperm(n, device=dev, generator=g)[:B]

        def nce():
            loss = F.contrast_loss(E1, E2, nodes, 0.2)
            loss.backward()

        timed("infonce_fwd_bwd", nce, n=n, d=d, B=B)


if __name__ == "__main__":
    main()
