#!/usr/bin/env python3
"""The HCCF step's dense hypergraph products (HGNNLayer, HCCF.py:201-211: M = Hᵀ·h by split-K,
H·M by the row GEMM, and their gradients) under the library's dense-product tunings: for each
(HGD_TUNE_SPLITK_ROWS, HGD_TUNE_X3_SPLITK, HGD_TUNE_GEMM_EXACT) setting the Yelp-shaped step
(the profile_graph_step_host.py body: 3 layers, d = 64, K = 32, batch 4,096, the reference's
Adam in the graph) is captured afresh and its replays event-timed (median µs), with the
largest parameter difference from the default setting's step as a numerics check. One JSON
line per setting."""
import json
import os
import statistics
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, ROOT + "/scripts")


def main():
    import torch

    import refops as R
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFEncoder
    from hypergraph_diffusion_for_recommendation_amd.functional import (bpr_loss_rows,
                                                                         contrast_loss_layers,
                                                                         unique_long_n_group)
    from hypergraph_diffusion_for_recommendation_amd.graphs import CapturedStep
    from hypergraph_diffusion_for_recommendation_amd.optim import ReferenceAdam
    lib = nat.load()
    dev = torch.device("cuda")
    nu, ni = 31_668, 38_048
    u, i = R.synthetic_incidence(nu, ni, 1_237_259, seed=0)
    A = R.normalize_graph_mat(R.bipartite_adjacency(u, i, nu, ni))
    data = types.SimpleNamespace(n_users=nu, n_items=ni, norm_adj=A)
    conf = dict(lrate=0.001, lr_decay=0.7, max_epoch=1, batch_size=4096, reg=0.1,
                embedding_size=64, hyper_dim=32, drop_rate=0.5, p=0.1, n_layers=3)
    g = torch.Generator(device=dev).manual_seed(0)
    batches = [tuple(torch.randint(0, n, (4096,), device=dev, generator=g) for n in (nu, ni, ni))
               for _ in range(4)]
    settings = [(0, 2, 0), (512, 2, 0), (1024, 2, 0), (2048, 2, 0), (4096, 2, 0), (8192, 2, 0),
                (0, 0, 0), (0, 1, 0), (1024, 0, 0), (2048, 0, 0), (0, 2, 1)]
    ref_params = None
    for rows, x3, exact in settings:
        for key, val in ((5, rows), (8, x3), (6, exact)):
            nat.check(lib.hgd_set_tuning(key, val), "hgd_set_tuning")
        torch.manual_seed(0)
        model = HCCFEncoder(conf, data, dev)
        model.edgeDropper.capture_safe = True
        model.edgeDropper.device_rng = True  # device masks: the same every setting, no host draw
        opt = ReferenceAdam(model.parameters(), lr=1e-3)
        capturing = [False]

        def body(uid, pid, nid):
            ue, ie, gcn, hyp = model(keep_rate=0.5)
            bpr, anc, pos = bpr_loss_rows(ue, ie, uid, pid, nid)
            (un, uc), (pn, pc) = unique_long_n_group([anc, pos], [nu, ni])
            ssl = contrast_loss_layers([t.detach() for t in gcn], hyp, nu, un, pn, 0.2, uc, pc)
            loss = bpr + 1e-4 * ssl
            opt.zero_grad()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 4)
            loss.backward()
            if capturing[0]:
                opt.launch()
            else:
                opt.step()
            return loss

        body(*batches[0])
        capturing[0] = True
        cap = CapturedStep(body, batches[1], before_replay=opt.prepare)
        capturing[0] = False
        ts = []
        for k in range(40):
            b = batches[k % len(batches)]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            opt.prepare()
            for dst, src in zip(cap.static, b):
                dst.copy_(src)
            e0.record()
            cap.graph.replay()
            e1.record()
            e1.synchronize()
            if k >= 5:
                ts.append(e0.elapsed_time(e1) * 1e3)
        params = [p.detach().clone() for p in model.parameters()]
        if ref_params is None:
            ref_params = params
        diff = max(float((a - b).abs().max()) for a, b in zip(params, ref_params))
        print(json.dumps({"splitk_rows": rows, "x3_splitk": x3, "gemm_exact": exact,
                          "replay_us": round(statistics.median(ts), 1),
                          "max_param_diff_vs_default": diff}), flush=True)
        del cap, model, opt
        torch.cuda.synchronize()
    for key, val in ((5, 0), (8, 2), (6, 0)):
        nat.check(lib.hgd_set_tuning(key, val), "hgd_set_tuning")


if __name__ == "__main__":
    main()
