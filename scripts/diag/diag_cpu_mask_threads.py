#!/usr/bin/env python3
"""Host cost of the reference's drop-edge draw (HCCF.py:223, torch.rand on the CPU generator)
as hgd_torch_cpu_keep_mask_threads splits it: one HCCF step's three Yelp-shaped masks (3 ×
2,473,226 draws) into one pinned buffer, by thread count, and the same thread counts at the
smallest split length (the per-thread MT19937 jump alone, nearly no draws). Medians in µs; one
JSON line."""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    lib = nat.load()
    n = 3 * 2_473_226
    mask = torch.empty(n, dtype=torch.uint8, pin_memory=torch.cuda.is_available())
    mask.fill_(0)
    kept = ctypes.c_int64()
    st0 = torch.get_rng_state()

    def run(count, threads, reps=15):
        ts = []
        for _ in range(reps):
            st = st0.clone()
            t = time.perf_counter()
            nat.check(lib.hgd_torch_cpu_keep_mask_threads(st.data_ptr(), st.numel(), count, 0.5,
                                                          mask.data_ptr(), ctypes.byref(kept),
                                                          threads), "keep_mask")
            ts.append(time.perf_counter() - t)
        return round(statistics.median(ts[2:]) * 1e6, 1)

    out = {"n": n, "step_draw_us": {}, "jump_only_us": {}}
    for th in (1, 2, 4, 8, 12, 16, 24, 32):
        out["step_draw_us"][str(th)] = run(n, th)
        out["jump_only_us"][str(th)] = run(th * 64 * 624, th)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
