"""Diagnostic: hgd_gemm_rows (the staged split-bf16 kernel by default) against float64 over the
K / N / row-count grid and the epilogue flags; prints the worst relative error and which rows
are off."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch

from hypergraph_diffusion_for_recommendation_amd import _native as nat
from hypergraph_diffusion_for_recommendation_amd import functional as F

lib = nat.load()
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(0)
bad = 0
for K in (32, 64, 128):
    for N in (16, 32, 64, 128):
        for rows in (1000, 4099, 70001):
            for mode in ("plain", "bin", "bin_inv", "bias_relu"):
                A = torch.randn(rows, K, device=dev, generator=g)
                B = torch.randn(K, N, device=dev, generator=g)
                bias = torch.randn(N, device=dev, generator=g)
                Y = torch.zeros(rows, N, device=dev)
                d = F._rows_desc(A, B, N, 1, K, N, Y)
                Ad = A.double()
                if mode.startswith("bin"):
                    d.binarize_a = 1
                    Ad = (A > 0).double()
                rinv = None
                if mode == "bin_inv":
                    rinv = torch.empty(rows, device=dev)
                    d.row_inv = rinv.data_ptr()
                if mode == "bias_relu":
                    d.bias, d.relu = bias.data_ptr(), 1
                F._gemm_rows([d], dev)
                torch.cuda.synchronize()
                ref = Ad @ B.double()
                if mode == "bin_inv":
                    ref = ref / Ad.sum(1).clamp(min=1)[:, None]
                if mode == "bias_relu":
                    ref = (ref + bias.double()).clamp(min=0)
                err = (Y.double() - ref).abs().amax(1) / (ref.abs().amax(1) + 1e-30)
                worst = float(err.max())
                if worst > 1e-5:
                    bad += 1
                    rowsbad = torch.nonzero(err > 1e-5).flatten()
                    print(f"BAD K={K} N={N} rows={rows} {mode}: worst {worst:.3e}, "
                          f"{rowsbad.numel()} rows, first {rowsbad[:8].tolist()}", flush=True)
print("bad cases:", bad, flush=True)
