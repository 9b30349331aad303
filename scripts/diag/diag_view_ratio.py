#!/usr/bin/env python3
"""Worst row ratios (error / row scale, tests/_ref64.check_rows) of the HCCF config-parity step
with compacted drop-edge children vs masked views, over a few seeds: is a view-path excess over
the 1e-5 bound the path's or the seed's? Prints one line per case; the bound is not enforced."""
import io
import os
import sys
from contextlib import redirect_stdout

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    from tests import _ref64 as R
    from tests import test_gpu_config_parity as T
    R.TOL = 1.0  # report, do not assert
    rows, wgrad = R.check_rows, R.check_weight_grad
    R.check_rows = lambda g, r, what, tol=None: rows(g, r, what, 1.0)
    R.check_weight_grad = lambda g, r, e, what, tol=None: wgrad(g, r, e, what, 1.0)
    dev = torch.device("cuda")
    for name, shape, d, L, seeds in (("LASTFM", T.LASTFM, 32, 1, (10, 11, 12, 13)),
                                     ("YELP", T.YELP, 64, 3, (20, 21))):
        for seed in seeds:
            for cs in (False, True):
                buf = io.StringIO()
                with redirect_stdout(buf):
                    T._hccf_case(dev, shape, d, L, seed=seed, capture_safe=cs)
                line = [x for x in buf.getvalue().splitlines() if "worst row ratio" in x][-1]
                print(f"{name} seed {seed} {'view' if cs else 'compacted'}: {line}", flush=True)


if __name__ == "__main__":
    main()
