#!/usr/bin/env python3
"""Worst row ratios (error / row scale against float64, tests/_ref64.check_rows) of the HCCF
config-parity step, ours against the reference's own torch calls evaluated in float32, per tensor,
over LastFM seeds 10-19 on both drop-edge paths (compacted children / masked views). Prints one
JSON line per case; nothing is asserted (the test is
tests/test_gpu_config_parity.py::test_hccf_lastfm_seeds_no_worse_than_reference_fp32)."""
import io
import json
import os
import sys
from contextlib import redirect_stdout

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    from tests import _ref64 as R
    from tests import test_gpu_config_parity as T
    rows = R.check_rows
    R.check_rows = lambda g, r, what, tol=None: rows(g, r, what, 1.0)
    dev = torch.device("cuda")
    seeds = [int(s) for s in sys.argv[1:]] or list(range(10, 20))
    for seed in seeds:
        for cs in (False, True):
            with redirect_stdout(io.StringIO()):
                ratios = T._hccf_case(dev, T.LASTFM, 32, 1, seed=seed, capture_safe=cs,
                                      fp32_record=True)
            worst_k = max(ratios, key=lambda k: ratios[k][0] / max(R.TOL, ratios[k][1]))
            print(json.dumps({
                "seed": seed, "path": "view" if cs else "compacted",
                "worst_ours": max(a for a, _ in ratios.values()),
                "worst_ref_fp32": max(b for _, b in ratios.values()),
                "tightest_tensor": worst_k, "ours": ratios[worst_k][0],
                "ref_fp32": ratios[worst_k][1],
                "over_1e-5": {k: [a, b] for k, (a, b) in ratios.items() if max(a, b) > R.TOL},
            }), flush=True)


if __name__ == "__main__":
    main()
