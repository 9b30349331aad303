#!/usr/bin/env python3
"""Which arithmetic does this torch build's device Adam use, op by op? Each foreach op of
torch.optim.Adam's multi-tensor step (torch/optim/adam.py _multi_tensor_adam, non-capturable)
runs on random data and is compared with candidate formulas (fused multiply-adds emulated in
float64, then rounded once to float32); prints the mismatch count of every candidate. The
hgd_adam_step variant bits follow from the zero rows (csrc/adam.hip)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(7)
    n = 1 << 20
    f32, f64 = torch.float32, torch.float64

    def r(scale=1.0):
        return torch.randn(n, device=dev, generator=g) * scale

    def fma(a, b, c):  # a·b + c rounded once (double holds a·b exactly)
        return (a.to(f64) * b.to(f64) + c.to(f64)).to(f32)

    out = {}
    m, gr = r(1e-2), r(1e-1)
    w = 1 - 0.9
    t = [m.clone()]
    torch._foreach_lerp_(t, [gr], w)
    wf = torch.tensor(w, dtype=f32, device=dev)
    cands = {"m+w*(g-m)": m + wf * (gr - m), "fma(w,g-m,m)": fma(wf, gr - m, m),
             "fma(w,g,m-w*m)": fma(wf, gr, m - wf * m), "m*(1-w)+w*g": m * (1 - wf) + wf * gr}
    out["lerp"] = {k: int((v != t[0]).sum()) for k, v in cands.items()}

    v = r(1e-3).abs()
    val = 1 - 0.999
    t = [v.clone()]
    torch._foreach_addcmul_(t, [gr], [gr], val)
    vf = torch.tensor(val, dtype=f32, device=dev)
    cands = {"v+val*(g*g)": v + vf * (gr * gr), "fma(val,g*g,v)": fma(vf, gr * gr, v),
             "v+(val*g)*g": v + (vf * gr) * gr, "fma(val*g,g,v)": fma(vf * gr, gr, v)}
    out["addcmul"] = {k: int((c != t[0]).sum()) for k, c in cands.items()}

    t = torch._foreach_sqrt([v])
    cands = {"sqrt_rn": torch.sqrt(v.to(f64)).to(f32), "torch.sqrt": torch.sqrt(v)}
    out["sqrt"] = {k: int((c != t[0]).sum()) for k, c in cands.items()}

    d = torch.sqrt(v) + 1e-8
    c2 = (1 - 0.999 ** 7) ** 0.5
    t = [d.clone()]
    torch._foreach_div_(t, [c2])
    cf = torch.tensor(c2, dtype=f32, device=dev)
    cands = {"d/c_rn": (d.to(f64) / cf.to(f64)).to(f32), "d/c torch": d / cf,
             "d*(1/c)": d * (1 / cf)}
    out["div_scalar"] = {k: int((c != t[0]).sum()) for k, c in cands.items()}

    p = r()
    step = -(1e-3 / (1 - 0.9 ** 7))
    t = [p.clone()]
    torch._foreach_addcdiv_(t, [m], [d], [step])
    sf = torch.tensor(step, dtype=f32, device=dev)
    q = (m.to(f64) / d.to(f64)).to(f32)
    cands = {"p+s*(m/d)": p + sf * q, "fma(s,m/d,p)": fma(sf, q, p),
             "p+(s*m)/d": p + (sf * m) / d, "fma(s*m... )": fma(sf * m, 1 / d, p)}
    out["addcdiv"] = {k: int((c != t[0]).sum()) for k, c in cands.items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
