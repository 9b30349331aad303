#!/usr/bin/env python3
"""Which Python lines launch the torch-native kernels of the HCCF step (adds, fills, copies,
dropout and its backward, reductions)? One eager, capture-safe step of the Yelp-shaped HCCFEncoder
(the profile_graph_step_host.py body) under torch.profiler with shapes and stacks; prints one
JSON line per aten op that reached the device: count, input shapes and the innermost repository
frames that called it."""
import collections
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import torch
    from torch.profiler import ProfilerActivity, profile

    import refops as R
    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFEncoder
    from hypergraph_diffusion_for_recommendation_amd.functional import (bpr_loss_rows,
                                                                         contrast_loss_layers,
                                                                         unique_long_n_group)
    from hypergraph_diffusion_for_recommendation_amd.optim import ReferenceAdam
    dev = torch.device("cuda")
    nu, ni = 31_668, 38_048
    u, i = R.synthetic_incidence(nu, ni, 1_237_259, seed=0)
    A = R.normalize_graph_mat(R.bipartite_adjacency(u, i, nu, ni))
    data = types.SimpleNamespace(n_users=nu, n_items=ni, norm_adj=A)
    conf = dict(lrate=0.001, lr_decay=0.7, max_epoch=1, batch_size=4096, reg=0.1,
                embedding_size=64, hyper_dim=32, drop_rate=0.5, p=0.1, n_layers=3)
    torch.manual_seed(0)
    model = HCCFEncoder(conf, data, dev)
    model.edgeDropper.capture_safe = True
    opt = ReferenceAdam(model.parameters(), lr=1e-3)
    g = torch.Generator(device=dev).manual_seed(0)
    batch = tuple(torch.randint(0, n, (4096,), device=dev, generator=g) for n in (nu, ni, ni))

    def body(uid, pid, nid):
        ue, ie, gcn, hyp = model(keep_rate=0.5)
        bpr, anc, pos = bpr_loss_rows(ue, ie, uid, pid, nid)
        (un, uc), (pn, pc) = unique_long_n_group([anc, pos], [nu, ni])
        ssl = contrast_loss_layers([t.detach() for t in gcn], hyp, nu, un, pn, 0.2, uc, pc)
        loss = bpr + 1e-4 * ssl
        opt.zero_grad()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 4)
        loss.backward()
        opt.step()
        return loss

    for _ in range(3):
        body(*batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                 with_stack=True) as prof:
        body(*batch)
        torch.cuda.synchronize()
    groups = collections.defaultdict(lambda: {"count": 0, "device_us": 0.0})
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.device_time_total <= 0:
            continue
        if any(c.name.startswith("aten::") for c in [ev.cpu_parent] if c is not None):
            continue  # count the outermost aten op only
        frames = [f for f in (ev.stack or []) if "hypergraph_diffusion" in f or "diag_step" in f
                  or "torch/nn/utils" in f or "torch/optim" in f or "autograd" in f][:3]
        up = ev.cpu_parent  # the backward node (autograd engine frames carry no Python stack)
        while up is not None and up.name.startswith("aten::"):
            up = up.cpu_parent
        if up is not None:
            frames.insert(0, up.name[:90])
        key = (ev.name, str(ev.input_shapes)[:120], " | ".join(frames))
        groups[key]["count"] += 1
        groups[key]["device_us"] += ev.device_time_total
    for (name, shapes, frames), v in sorted(groups.items(), key=lambda kv: -kv[1]["device_us"]):
        print(json.dumps({"op": name, "count": v["count"], "device_us": round(v["device_us"], 1),
                          "shapes": shapes, "frames": frames}), flush=True)


if __name__ == "__main__":
    main()
