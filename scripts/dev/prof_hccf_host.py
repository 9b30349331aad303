"""Host-side profile (cProfile) of the HCCF training step of scripts/bench_hccf.py (device mask):
where the Python / launch time of a step goes."""
import cProfile
import os
import pstats
import sys
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
    nu, ni = 31_668, 38_048
    u, i = R.synthetic_incidence(nu, ni, 1_237_259, seed=0)
    A = R.normalize_graph_mat(R.bipartite_adjacency(u, i, nu, ni))
    data = types.SimpleNamespace(n_users=nu, n_items=ni, norm_adj=A)
    conf = dict(lrate=0.001, lr_decay=0.7, max_epoch=1, batch_size=4096, reg=0.1,
                embedding_size=64, hyper_dim=32, drop_rate=0.5, p=0.1, n_layers=3)
    torch.manual_seed(0)
    model = HCCFEncoder(conf, data, dev)
    model.edgeDropper.device_rng = True
    opt = torch.optim.Adam(model.parameters(), lr=0.001)
    g = torch.Generator(device=dev).manual_seed(0)
    b = [torch.randint(0, n, (4096,), device=dev, generator=g) for n in (nu, ni, ni)]

    def step():
        ue, ie, gcn, hyp = model(keep_rate=0.5)
        anc, pos, neg = ue[b[0]], ie[b[1]], ie[b[2]]
        un, pn = unique_long(anc), unique_long(pos)
        ssl = 0
        for layer in range(3):
            e1, e2 = gcn[layer].detach(), hyp[layer]
            ssl = ssl + contrast_loss(e1[:nu], e2[:nu], un, 0.2) + contrast_loss(e1[nu:], e2[nu:], pn, 0.2)
        loss = R.bpr_loss(anc, pos, neg) + 1e-4 * ssl
        opt.zero_grad()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 4)
        loss.backward()
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
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
