#!/usr/bin/env python3
"""Is a capturable Adam bitwise the reference's Adam (torch.optim.Adam(lr=float), HCCF.py:33) on
HCCF's parameters? (VERDICT r4 "next" 5.) A Yelp-shaped HCCFEncoder (3 layers, d = 64) takes
``--steps`` capture-safe eager steps with the reference's Adam; every other optimizer gets the
SAME gradients (copied from the reference trajectory) on its own copy of the same start, and is
compared with the reference's parameters after each step, bit for bit. One JSON line per
optimizer: the first step whose parameters differ and the largest difference at the end.

    python scripts/diag/diag_adam_bitwise.py [--steps 50]
"""
import argparse
import copy
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    import torch

    import refops as R
    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFEncoder
    from hypergraph_diffusion_for_recommendation_amd.optim import ReferenceAdam
    from hypergraph_diffusion_for_recommendation_amd.functional import (bpr_loss_rows,
                                                                         contrast_loss_layers,
                                                                         unique_long_n_group)
    dev = torch.device("cuda")
    nu, ni, E, d = 31_668, 38_048, 1_237_259, 64
    u, i = R.synthetic_incidence(nu, ni, E, seed=0)
    A = R.normalize_graph_mat(R.bipartite_adjacency(u, i, nu, ni))
    data = types.SimpleNamespace(n_users=nu, n_items=ni, norm_adj=A)
    conf = dict(lrate=0.001, lr_decay=0.7, max_epoch=1, batch_size=4096, reg=0.1,
                embedding_size=d, hyper_dim=32, drop_rate=0.5, p=0.1, n_layers=3)
    torch.manual_seed(0)
    model = HCCFEncoder(conf, data, dev)
    model.edgeDropper.capture_safe = True
    g = torch.Generator(device=dev).manual_seed(0)
    lr = conf["lrate"]
    ref_opt = torch.optim.Adam(model.parameters(), lr=lr)
    start = [p.detach().clone() for p in model.parameters()]

    def lr_t():
        return torch.tensor(lr, dtype=torch.float32, device=dev)

    variants = {
        "capturable_foreach": lambda ps: torch.optim.Adam(ps, lr=lr_t(), capturable=True,
                                                          foreach=True),
        "capturable_single_tensor": lambda ps: torch.optim.Adam(ps, lr=lr_t(), capturable=True,
                                                                foreach=False),
        "capturable_fused": lambda ps: torch.optim.Adam(ps, lr=lr_t(), capturable=True,
                                                        fused=True),
        "capturable_foreach_float_lr": lambda ps: torch.optim.Adam(ps, lr=lr, capturable=True,
                                                                   foreach=True),
        "fused_float_lr": lambda ps: torch.optim.Adam(ps, lr=lr, fused=True),
        # the reference's Adam as one capturable libhgd kernel (optim.ReferenceAdam)
        "hgd_reference_adam": lambda ps: ReferenceAdam(ps, lr=lr),
    }
    others = {}
    for name, make in variants.items():
        ps = [torch.nn.Parameter(s.clone()) for s in start]
        others[name] = (ps, make(ps), None)
    for k in range(args.steps):
        uid = torch.randint(0, nu, (4096,), device=dev, generator=g)
        pid = torch.randint(0, ni, (4096,), device=dev, generator=g)
        nid = torch.randint(0, ni, (4096,), device=dev, generator=g)
        ue, ie, gcn, hyp = model(keep_rate=0.5)
        bpr, anc, pos = bpr_loss_rows(ue, ie, uid, pid, nid)
        (un, uc), (pn, pc) = unique_long_n_group([anc, pos], [nu, ni])
        ssl = contrast_loss_layers([t.detach() for t in gcn], hyp, nu, un, pn, 0.2, uc, pc)
        loss = bpr + 1e-4 * ssl
        ref_opt.zero_grad()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 4)
        loss.backward()
        grads = [p.grad.detach().clone() for p in model.parameters()]
        ref_opt.step()
        for name, (ps, opt, first) in list(others.items()):
            for p, gr in zip(ps, grads):
                p.grad = gr.clone()
            opt.step()
            same = all(torch.equal(p.detach(), q.detach()) for p, q in zip(ps, model.parameters()))
            if not same and first is None:
                others[name] = (ps, opt, k)
    for name, (ps, opt, first) in others.items():
        diff = max(float((p.detach() - q.detach()).abs().max())
                   for p, q in zip(ps, model.parameters()))
        print(json.dumps({"optimizer": name, "steps": args.steps, "bitwise_equal": first is None,
                          "first_differing_step": first, "max_abs_diff_at_end": diff}),
              flush=True)


if __name__ == "__main__":
    main()
