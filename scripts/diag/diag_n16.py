"""Diagnostic for the staged row GEMM at N = 16: error structure on a small case."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch

from hypergraph_diffusion_for_recommendation_amd import _native as nat
from hypergraph_diffusion_for_recommendation_amd import functional as F

lib = nat.load()
dev = torch.device("cuda")
torch.set_printoptions(precision=3, linewidth=200, sci_mode=False)
for K, rows in ((128, 64), (64, 64), (128, 16)):
    A = torch.zeros(rows, K, device=dev)
    B = torch.zeros(K, 16, device=dev)
    # A = identity-like: row r has a single 1 at column r % K; B[k, n] = 100 k + n
    for r in range(rows):
        A[r, r % K] = 1.0
    B = (100 * torch.arange(K, device=dev, dtype=torch.float32)[:, None]
         + torch.arange(16, device=dev, dtype=torch.float32)[None, :])
    Y = torch.zeros(rows, 16, device=dev)
    d = F._rows_desc(A, B, 16, 1, K, 16, Y)
    F._gemm_rows([d], dev)
    torch.cuda.synchronize()
    ref = A @ B
    bad = (Y - ref).abs().amax(1) > 1e-3
    print(f"K={K} rows={rows}: bad rows {int(bad.sum())}", flush=True)
    print("got rows 0..5:\n", Y[:6], flush=True)
    print("ref rows 0..5:\n", ref[:6], flush=True)
