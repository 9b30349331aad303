#!/usr/bin/env python3
"""Fused InfoNCE (hgd_infonce_*) vs the reference's contrastLoss (util/loss_torch.py:103-110) on
the same GPU, fwd+bwd per call, at HCCF shapes: [N, d] tables, batch B. Prints one JSON line per
case (device time from HIP events, median)."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    import torch

    from hypergraph_diffusion_for_recommendation_amd.functional import contrast_loss
    import refops as ref_cpu
    dev = torch.device("cuda")
    for N, d, B in ((31_668, 64, 2048), (1_000_000, 64, 2048), (10_000_000, 64, 4096)):
        E1 = torch.randn(N, d, device=dev, requires_grad=True)
        E2 = torch.randn(N, d, device=dev, requires_grad=True)
        nodes = torch.randint(0, N, (B,), device=dev)
        for name, fn in (("hgd_fused", contrast_loss), ("reference_ops", ref_cpu.contrast_loss)):
            def step():
                E1.grad = E2.grad = None
                fn(E1, E2, nodes, 0.2).backward()
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            ts = []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                step()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            print(json.dumps({"case": name, "N": N, "d": d, "B": B,
                              "ms_fwd_bwd": round(statistics.median(ts), 4)}), flush=True)


if __name__ == "__main__":
    main()
