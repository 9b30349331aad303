#!/usr/bin/env python3
"""The reference's drop-edge keep-mask stream (HCCF.py:223: floor(torch.rand(nnz) + keep)) drawn
by hgd_torch_cpu_keep_mask at 1..16 host threads (GF(2) jump-ahead split, csrc/torch_rng.cpp):
median ms per draw and bit-identity with torch.rand at every thread count. One JSON line per
thread count.
    python scripts/bench_cpu_mask.py [--n 2473226 --reps 30]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_473_226)  # Yelp-shaped norm_adj nonzeros
    ap.add_argument("--keep", type=float, default=0.5)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--threads", default="1,2,4,8,16")
    a = ap.parse_args()
    import torch

    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd.layers import _draw_keep_mask
    lib = nat.load()
    torch.manual_seed(0)
    torch.rand(17)
    st = torch.get_rng_state()
    ref = ((torch.rand(a.n) + a.keep).floor()).type(torch.bool)
    ref_next = torch.rand(8)
    for T in (int(t) for t in a.threads.split(",")):
        nat.check(lib.hgd_set_tuning(12, T), "hgd_set_tuning")
        m, kept, end = _draw_keep_mask(st.clone(), a.n, a.keep)
        torch.set_rng_state(end)
        ok = bool(torch.equal(m.bool(), ref)) and kept == int(ref.sum()) and bool(
            torch.equal(torch.rand(8), ref_next))
        ts = []
        for _ in range(a.reps):
            s = st.clone()
            t0 = time.perf_counter()
            _draw_keep_mask(s, a.n, a.keep)
            ts.append((time.perf_counter() - t0) * 1e3)
        print(json.dumps({"threads": T, "n": a.n, "ms_median": round(statistics.median(ts), 3),
                          "ms_min": round(min(ts), 3), "bit_identical_to_torch_rand": ok}),
              flush=True)
    nat.check(lib.hgd_set_tuning(12, 0), "hgd_set_tuning")


if __name__ == "__main__":
    main()
