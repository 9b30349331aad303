#!/usr/bin/env python3
"""Host-side time of one HCCF step (bench_hccf's hgd_device_mask variant): phase timers without
syncs, and torch.profiler CPU self-time by op."""
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import torch
    import refops as R
    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFEncoder
    from hypergraph_diffusion_for_recommendation_amd.functional import contrast_loss, unique_long
    dev = torch.device("cuda")
    nu, ni, E, d, L, B = 31_668, 38_048, 1_237_259, 64, 3, 4096
    u, i = R.synthetic_incidence(nu, ni, E, seed=0)
    A = R.normalize_graph_mat(R.bipartite_adjacency(u, i, nu, ni))
    data = types.SimpleNamespace(n_users=nu, n_items=ni, norm_adj=A)
    conf = dict(lrate=0.001, lr_decay=0.7, max_epoch=1, batch_size=B, reg=0.1,
                embedding_size=d, hyper_dim=32, drop_rate=0.5, p=0.1, n_layers=L)
    torch.manual_seed(0)
    model = HCCFEncoder(conf, data, dev)
    model.edgeDropper.device_rng = True
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    g = torch.Generator(device=dev).manual_seed(0)
    uid = torch.randint(0, nu, (B,), device=dev, generator=g)
    pid = torch.randint(0, ni, (B,), device=dev, generator=g)
    nid = torch.randint(0, ni, (B,), device=dev, generator=g)
    T = {}

    def tick(name, t0):
        t = time.perf_counter()
        T[name] = T.get(name, 0.0) + (t - t0)
        return t

    def step():
        t = time.perf_counter()
        ue, ie, gcn, hyp = model(keep_rate=0.5)
        t = tick("forward", t)
        anc, pos, neg = ue[uid], ie[pid], ie[nid]
        ssl = 0
        for layer in range(L):
            e1, e2 = gcn[layer].detach(), hyp[layer]
            t = tick("misc", t)
            na, np_ = unique_long(anc), unique_long(pos)
            t = tick("unique", t)
            ssl = ssl + contrast_loss(e1[:nu], e2[:nu], na, 0.2) \
                + contrast_loss(e1[nu:], e2[nu:], np_, 0.2)
            t = tick("contrast", t)
        loss = R.bpr_loss(anc, pos, neg) + 1e-4 * ssl
        opt.zero_grad()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 4)
        t = tick("loss+clip", t)
        loss.backward()
        t = tick("backward", t)
        opt.step()
        tick("adam", t)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    T.clear()
    n = 30
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n * 1e3
    print(f"wall ms/step {wall:.3f}")
    for k, v in T.items():
        print(f"  host {k:10s} {v / n * 1e3:7.3f} ms")
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        for _ in range(10):
            step()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=35))


if __name__ == "__main__":
    main()
