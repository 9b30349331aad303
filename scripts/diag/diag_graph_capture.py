#!/usr/bin/env python3
"""Round 6 diagnostic: hgconv2 fwd + autograd bwd captured in one HIP graph (bench.py --graph on's
pattern) on a small random incidence, with HGD_SPMM_BLOCKS = --blocks (0 = plain hops) and the
functional op or the sharded one (--op). Prints one JSON line: replay bitwise equal to eager.

    python scripts/diag/diag_graph_capture.py --blocks 4 --op functional
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=0)
    ap.add_argument("--op", choices=("functional", "sharded", "torch"), default="functional")
    ap.add_argument("--users", type=int, default=5000)
    ap.add_argument("--items", type=int, default=700)
    ap.add_argument("--edges", type=int, default=60000)
    ap.add_argument("--split", type=int, default=0, help="split_threshold (-1 = auto)")
    ap.add_argument("--what", choices=("fwdbwd", "fwd", "hop"), default="fwdbwd",
                    help="captured: fwd + autograd bwd, the forward only, or one plain hop")
    ap.add_argument("--detach", type=int, default=1,
                    help="1: drop the eager output's autograd graph before the capture")
    ap.add_argument("--mode", choices=("global", "thread_local", "relaxed"), default="global",
                    help="torch.cuda.graph capture_error_mode")
    args = ap.parse_args()
    os.environ["HGD_SPMM_BLOCKS"] = str(args.blocks)
    import numpy as np
    import torch

    from hypergraph_diffusion_for_recommendation_amd import Incidence, hgconv2
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(321)
    U, I, d = args.users, args.items, 64
    key = np.unique(rng.integers(0, U, args.edges) * I + rng.integers(0, I, args.edges))
    idx = torch.from_numpy(np.stack([key // I, key % I]))
    kw = {} if args.split < 0 else {"split_threshold": args.split}
    inc = Incidence.from_coo(idx, None, (U, I), device=dev, **kw)
    X = torch.from_numpy(rng.standard_normal((U, d)).astype(np.float32)).to(dev)
    dY = torch.from_numpy(rng.standard_normal((U, d)).astype(np.float32)).to(dev)
    Mfix = torch.from_numpy(rng.standard_normal((I, d)).astype(np.float32)).to(dev)
    X.requires_grad_(True)
    if args.op == "sharded":
        from hypergraph_diffusion_for_recommendation_amd.sharded import (ShardedIncidence,
                                                                          sharded_two_hop)
        sh = ShardedIncidence(inc)

        def conv(x):
            return sharded_two_hop(sh, x)
    elif args.op == "torch":  # no libhgd at all: torch ops with autograd
        W = torch.from_numpy(rng.standard_normal((d, d)).astype(np.float32)).to(dev)

        def conv(x):
            return torch.tanh(x @ W) * 2.0
    else:
        def conv(x):
            return hgconv2(inc, x)

    def step():
        if args.what == "hop":
            from hypergraph_diffusion_for_recommendation_amd import spmm_csr
            Y = spmm_csr(inc.csr, Mfix)
            return Y, Y
        if args.what == "fwd":
            with torch.no_grad():
                Y = conv(X)
            return Y, Y
        Y = conv(X)
        (dX,) = torch.autograd.grad(Y, X, dY)
        return Y, dX

    Y0, dX0 = step()
    if args.detach:
        Y0 = Y0.detach()
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(2):
            step()
    torch.cuda.current_stream(dev).wait_stream(side)
    import gc
    gc.collect()
    print("capturing", flush=True)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, capture_error_mode=args.mode):
        Yg, dXg = step()
    print("captured", flush=True)
    ok = True
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize(dev)
        ok = ok and torch.equal(Yg, Y0.detach()) and torch.equal(dXg, dX0)
    print(json.dumps({"blocks": args.blocks, "op": args.op, "split": args.split,
                      "what": args.what, "mode": args.mode, "detach": args.detach,
                      "replay_bitwise": bool(ok)}), flush=True)


if __name__ == "__main__":
    main()
