#!/usr/bin/env python3
"""Microbenchmark of the skinny Linear kernels (hgd_linear_*) against the library GEMMs torch
uses for the same products, at ED-HNN shapes: rows × d → d. Prints one JSON line per case with
device times from HIP events (median of --reps) and the achieved HBM rate on the algorithmic
bytes (inputs read once, outputs written once). Each timing brackets --inner back-to-back
launches (kernel time without the per-launch host gap); HGD_ROWGEMM_BLOCKS sets the row-GEMM
workgroup cap (hgd_set_tuning key 4) for a sweep."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[69_716, 2_200_000])
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--inner", type=int, default=20)
    ap.add_argument("--cases", nargs="*", default=None,
                    help="only these case names (e.g. fwd_hgd bwd_weight_hgd), for profiling")
    args = ap.parse_args()
    import torch

    from hypergraph_diffusion_for_recommendation_amd import _native as nat

    lib = nat.load()
    dev = torch.device("cuda")
    d = args.dim

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.inner):
                fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / args.inner)
        return statistics.median(ts)

    for n in args.rows:
        X = torch.randn(n, d, device=dev)
        W = torch.randn(d, d, device=dev)
        b = torch.randn(d, device=dev)
        dY = torch.randn(n, d, device=dev)
        Y = torch.empty(n, d, device=dev)
        dX = torch.empty(n, d, device=dev)
        dW = torch.empty(d, d, device=dev)
        db = torch.empty(d, device=dev)
        wsb = lib.hgd_linear_backward_weight_workspace_size(n, d, d)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        st = torch.cuda.current_stream().cuda_stream
        seed = torch.tensor([12345], dtype=torch.int64, device=dev)
        drop = nat.GemmRowsDesc()
        drop.A, drop.lda, drop.B, drop.bsk, drop.bsn = X.data_ptr(), d, W.data_ptr(), 1, d
        drop.bias, drop.relu, drop.Y, drop.ldy, drop.rows, drop.K, drop.N = (
            b.data_ptr(), 1, Y.data_ptr(), d, n, d, d)
        drop.drop_seed, drop.drop_keep, drop.drop_scale = seed.data_ptr(), 0.5, 2.0
        drop_arr = (nat.GemmRowsDesc * 1)(drop)
        R = torch.randn(n, d, device=dev)
        Y2 = torch.empty(n, d, device=dev)
        dres = nat.GemmRowsDesc.from_buffer_copy(drop)
        dres.res, dres.ldres, dres.Y2, dres.ldy2 = R.data_ptr(), d, Y2.data_ptr(), d
        dres_arr = (nat.GemmRowsDesc * 1)(dres)
        cases = {
            "fwd_drop_hgd": lambda: lib.hgd_gemm_rows(drop_arr, 1, st),
            "fwd_drop_res_hgd": lambda: lib.hgd_gemm_rows(dres_arr, 1, st),
            "fwd_hgd": lambda: lib.hgd_linear_forward(X.data_ptr(), d, n, d, W.data_ptr(), d, d,
                                                      b.data_ptr(), 1, Y.data_ptr(), d, st),
            "fwd_torch": lambda: torch.relu(torch.nn.functional.linear(X, W, b)),
            "bwd_data_hgd": lambda: lib.hgd_linear_backward_data(
                dY.data_ptr(), d, Y.data_ptr(), d, n, d, W.data_ptr(), d, d, dX.data_ptr(), d,
                st),
            "bwd_data_torch": lambda: torch.mm(dY * (Y > 0), W),
            "bwd_weight_hgd": lambda: lib.hgd_linear_backward_weight(
                dY.data_ptr(), d, None, 0, X.data_ptr(), d, n, d, d, dW.data_ptr(),
                db.data_ptr(), ws.data_ptr(), wsb, st),
            "bwd_weight_torch": lambda: (torch.mm(dY.t(), X), dY.sum(0)),
            # the ED-HNN weight gradient: dY masked by the forward's ReLU output
            "bwd_weight_mask_hgd": lambda: lib.hgd_linear_backward_weight(
                dY.data_ptr(), d, Y.data_ptr(), d, X.data_ptr(), d, n, d, d, dW.data_ptr(),
                db.data_ptr(), ws.data_ptr(), wsb, st),
            # the HBM reference point: one read and one write of the same bytes as the forward
            "copy_torch": lambda: Y.copy_(X),
        }
        algo = {"fwd": 2 * n * d * 4, "fwd_drop": 2 * n * d * 4, "fwd_drop_res": 4 * n * d * 4, "bwd_data": 3 * n * d * 4, "bwd_weight": 2 * n * d * 4, "bwd_weight_mask": 3 * n * d * 4,
                "copy": 2 * n * d * 4}
        for name, fn in cases.items():
            if args.cases and name not in args.cases:
                continue
            us = timed(fn)
            kind = name.rsplit("_", 1)[0]
            print(json.dumps({"case": name, "rows": n, "d": d, "us": round(us, 2),
                              "rowgemm_blocks": os.environ.get("HGD_ROWGEMM_BLOCKS", "512"),
                              "splitk_rows": os.environ.get("HGD_SPLITK_ROWS", "auto"),
                              "alg_GBps": round(algo[kind] / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
