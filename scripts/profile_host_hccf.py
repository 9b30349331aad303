#!/usr/bin/env python3
"""cProfile of eager HCCF training steps at the Yelp shape — the plugins' eager default
(encoders.HCCFEncoder with masked drop-edge views on the reference's CPU mask stream, fused BPR,
the grouped unique and InfoNCE with device counts, the reference's Adam): where the host time of
the eager path goes."""
import cProfile
import os
import pstats
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import torch

    import refops as R
    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFEncoder
    from hypergraph_diffusion_for_recommendation_amd.functional import (bpr_loss_rows,
                                                                         contrast_loss_layers,
                                                                         unique_long_n_group)
    dev = torch.device("cuda")
    nu, ni = 31_668, 38_048
    u, i = R.synthetic_incidence(nu, ni, 1_237_259, seed=0)
    A = R.normalize_graph_mat(R.bipartite_adjacency(u, i, nu, ni))
    data = types.SimpleNamespace(n_users=nu, n_items=ni, norm_adj=A)
    conf = dict(lrate=0.001, lr_decay=0.7, max_epoch=1, batch_size=4096, reg=0.1,
                embedding_size=64, hyper_dim=32, drop_rate=0.5, p=0.1, n_layers=3)
    torch.manual_seed(0)
    model = HCCFEncoder(conf, data, dev)
    model.edgeDropper.capture_safe = True  # the plugins' default (device_rng off)
    opt = torch.optim.Adam(model.parameters(), lr=0.001)
    g = torch.Generator(device=dev).manual_seed(0)
    uid, pid, nid = (torch.randint(0, n, (4096,), device=dev, generator=g) for n in (nu, ni, ni))

    def step():
        ue, ie, gcn, hyp = model(keep_rate=0.5)
        bpr, anc, pos = bpr_loss_rows(ue, ie, uid, pid, nid)
        (un, uc), (pn, pc) = unique_long_n_group([anc, pos], [nu, ni])
        ssl = contrast_loss_layers([t.detach() for t in gcn], hyp, nu, un, pn, 0.2, uc, pc)
        loss = bpr + 1e-4 * ssl
        opt.zero_grad()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 4)
        loss.backward()
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    print(f"eager step {1e3 * (time.perf_counter() - t0) / 20:.3f} ms", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
    st.sort_stats("cumulative").print_stats(40)


if __name__ == "__main__":
    main()
