#!/usr/bin/env python3
"""Host-side (Python) cost of one eager hgconv2 fwd+bwd step at the ML-1M shape: wall time per
step with and without a device sync, and a cProfile of 200 steps (top functions by own time)."""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from hypergraph_diffusion_for_recommendation_amd import Incidence, hgconv2
    from oracle import hgd_oracle as O
    dev = torch.device("cuda")
    rows, cols = O.synthetic_incidence(6040, 3706, 750_000, seed=0)
    inc = Incidence.from_coo(torch.from_numpy(np.stack([rows, cols])), None, (6040, 3706),
                             device=dev)
    X = torch.randn(6040, 64, device=dev, requires_grad=True)
    dY = torch.randn(6040, 64, device=dev)

    def step():
        Y = hgconv2(inc, X)
        torch.autograd.grad(Y, X, dY)

    for _ in range(20):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host issue {1e3 * (t1 - t0) / 200:.3f} ms/step, wall {1e3 * (t2 - t0) / 200:.3f} ms/step",
          flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
