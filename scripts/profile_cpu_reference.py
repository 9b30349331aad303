"""Why the CPU baseline does not scale with host threads (VERDICT r05 'Next' 4): times the
reference's torch.sparse.mm fwd+bwd (oracle/ref_cpu.py, HCCF.py:199 on the data/graph.py:28-42
normalisation) and one bare torch.sparse.mm at 1 and N threads, and prints torch.profiler's
per-op table of one fwd+bwd. A 1M x 1M x 10M-edge uniform graph at d = 64 (a tenth of the
headline graph, the size of bench.py's CPU sample).

    python scripts/profile_cpu_reference.py [--threads 8]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import ref_cpu  # noqa: E402  (checker / CPU baseline only)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=len(os.sched_getaffinity(0)))
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=64)
    a = ap.parse_args()
    U, I, E, d = a.users, a.items, a.edges, a.dim
    rng = np.random.default_rng(0)
    key = np.unique(rng.integers(0, U, E) * I + rng.integers(0, I, E))
    idx = torch.from_numpy(np.stack([key // I, key % I]))
    H = torch.sparse_coo_tensor(idx, torch.ones(idx.shape[1]), (U, I))
    X = torch.randn(U, d) * 0.01
    dY = torch.randn(U, d)
    print(f"host: os.cpu_count()={os.cpu_count()} affinity={len(os.sched_getaffinity(0))} "
          f"torch threads={torch.get_num_threads()}; graph {U}x{I}, {idx.shape[1]} edges, d={d}")
    ref_cpu.hgconv2_fwd_bwd(H, X, dY)
    Ht = H.t()
    for th in (1, a.threads):
        torch.set_num_threads(th)
        t0 = time.perf_counter()
        ref_cpu.hgconv2_fwd_bwd(H, X, dY)
        t1 = time.perf_counter()
        torch.sparse.mm(Ht, X)
        t2 = time.perf_counter()
        X.mul(2.0)
        t3 = time.perf_counter()
        print(f"threads {th:3d}: fwd+bwd {t1 - t0:7.3f} s | one torch.sparse.mm (aten::addmm, "
              f"sparse COO x dense) {t2 - t1:6.3f} s | dense X*2 {1e3 * (t3 - t2):6.1f} ms")
    torch.set_num_threads(a.threads)
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as p:
        ref_cpu.hgconv2_fwd_bwd(H, X, dY)
    print(f"torch.profiler, one fwd+bwd at {a.threads} threads:")
    print(p.key_averages().table(sort_by="self_cpu_time_total", row_limit=12))


if __name__ == "__main__":
    main()
