"""Probe: library GEMM for the scoring product [B, d] x [d, I] (rocBLAS vs hipBLASLt), and the
top-k kernel alone, at the Yelp shape."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from hypergraph_diffusion_for_recommendation_amd.evaluation import topk_rows

dev = torch.device("cuda")
I, d = 38048, 64
for B in (4096, 8192, 26000):
    u = torch.randn(B, d, device=dev)
    it = torch.randn(d, I, device=dev)
    for lib in ("default", "hipblaslt", "rocblas"):
        try:
            if lib != "default":
                torch.backends.cuda.preferred_blas_library(lib)
        except Exception as e:
            print(lib, "unavailable", e); continue
        for _ in range(3):
            S = torch.mm(u, it)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            S = torch.mm(u, it)
        e1.record(); e1.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"B={B} {lib}: {ms:.3f} ms, write {B*I*4/ms/1e6:.0f} GB/s, {2*B*I*d/ms/1e9:.1f} TF/s", flush=True)
    topk_rows(S, 40)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        topk_rows(S, 40)
    e1.record(); e1.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"B={B} topk: {ms:.3f} ms, {B*I*4/ms/1e6:.0f} GB/s per sweep", flush=True)
