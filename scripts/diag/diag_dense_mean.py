"""Diagnostic: the pieces of dense_mean_two_hop_pair's backward at (nu, ni, K, d) against torch
float64, for each GEMM form (exact / split-bf16 row GEMM / split-bf16 split-K)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch

from hypergraph_diffusion_for_recommendation_amd import _native as nat
from hypergraph_diffusion_for_recommendation_amd import functional as F

lib = nat.load()
dev = torch.device("cuda")


def rel(a, b):
    return float((a.double() - b).abs().max() / (b.abs().max() + 1e-30))


for cfg in [(0, 0, 1), (0, 0, 0), (1, 0, 0), (0, 128, 1)]:
    ex, cols, sk = cfg
    lib.hgd_set_tuning(6, ex)
    lib.hgd_set_tuning(7, cols)
    lib.hgd_set_tuning(8, sk)
    for nu, ni, K, d in [(1024, 64, 128, 16), (3000, 2500, 32, 64)]:
        g = torch.Generator(device=dev).manual_seed(nu + ni)
        Hu = torch.randn(nu, K, device=dev, generator=g)
        B = (Hu > 0).double()
        X = torch.randn(nu, d, device=dev, generator=g)
        sc = torch.rand(nu, device=dev, generator=g)
        cnt = torch.empty((1, K), device=dev)
        C = F._bin_tn([(Hu, X, 0)], K, d, dev, cnt, None)
        r1 = rel(C[0], B.t() @ X.double())
        C2 = F._bin_tn([(Hu, X, 0)], K, d, dev, None, sc)
        r2 = rel(C2[0], B.t() @ (X.double() * sc.double()[:, None]))
        M = torch.randn(1, K, d, device=dev, generator=g)
        Y = torch.empty(nu, d, device=dev)
        F._bin_rows([(Hu, 0)], M, cnt, Y, None)
        r3 = rel(Y, B @ (M[0].double() / cnt[0].double().clamp(min=1)[:, None]))
        rinv = torch.empty(nu, device=dev)
        F._bin_rows([(Hu, 0)], M, cnt, Y, rinv)
        ref = B @ (M[0].double() / cnt[0].double().clamp(min=1)[:, None])
        ref = ref / B.sum(1).clamp(min=1)[:, None]
        r4 = rel(Y, ref)
        print(f"exact={ex} cols={cols} x3splitk={sk} nu={nu} K={K} d={d}: tn {r1:.2e} tn_rowscale "
              f"{r2:.2e} rows {r3:.2e} rows_inv {r4:.2e}", flush=True)
