#!/usr/bin/env python3
"""Forward + backward of the KG carriers' encoders at the Yelp2018 shape of BASELINE configs[2]
(31,668 × 38,048, 1.24 M interactions, 3 layers, d = 64), training mode, edge-dropped
``norm_adj`` (keep 0.5) drawn per step:

* self_aware / self_aware_ref — encoders.SelfAwareEncoder (HGNN_cp.py:368-411 with the
  UGformer off, KHGRec's setting): per layer LN(leaky(A·(Aᵀ·x))) + res as one fused two-hop;
  against the reference's torch calls on the same GPU (torch.sparse.mm pair, F.leaky_relu,
  F.layer_norm, add).
* hd / hd_ref — encoders.SelfAwareEncoderHD (HD.py:398-487): ED-HNN blocks on the norm_adj
  pattern; against the reference's torch calls (V/E of the pattern, index_reduce means as
  torch_scatter's, F.linear / F.layer_norm / dropout). The reference's V/E extraction
  (``nonzero(hypergraph > 0)`` per call) is not timed on its side.

Prints one JSON line per variant (event-timed median of --reps steps)."""
import argparse
import json
import os
import statistics
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=31_668)
    ap.add_argument("--items", type=int, default=38_048)
    ap.add_argument("--edges", type=int, default=1_237_259)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--layers", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import torch.nn.functional as F

    import refops as R
    from hypergraph_diffusion_for_recommendation_amd.encoders import (SelfAwareEncoder,
                                                                      SelfAwareEncoderHD)
    from hypergraph_diffusion_for_recommendation_amd.layers import SpAdjDropEdge

    dev = torch.device("cuda")
    nu, ni, d, L = args.users, args.items, args.dim, args.layers
    u, i = R.synthetic_incidence(nu, ni, args.edges, seed=0)
    A = R.normalize_graph_mat(R.bipartite_adjacency(u, i, nu, ni))
    data = types.SimpleNamespace(n_users=nu, n_items=ni, norm_adj=A, ui_adj=None)
    keep = 0.5
    torch.manual_seed(0)
    ego = torch.nn.Parameter(torch.randn(nu + ni, d, device=dev) * 0.1)
    dY = torch.randn(nu + ni, d, device=dev)

    sa = SelfAwareEncoder(data, d, d, L, 0.1, 0.1, device=dev, use_self_att=False).train()
    hd = SelfAwareEncoderHD(data, d, d, L, 0.1, 0.1, device=dev).train()
    adj = hd.sparse_norm_adj.detach().clone().coalesce()
    dropper = SpAdjDropEdge()
    dropper.device_rng = True

    def step_sa():
        ue, ie = sa(ego, dropper(hd.sparse_norm_adj, keep))
        torch.autograd.backward([ue, ie], [dY[:nu], dY[nu:]])

    def step_sa_ref():
        a = R.sp_adj_drop_edge(adj, keep)
        x = ego
        for k in range(L):
            z = torch.sparse.mm(a, torch.sparse.mm(a.t(), x))
            if k != L - 1:
                z = F.leaky_relu(z, 0.1)
            ln = sa.lns[k]
            x = F.layer_norm(z, (d,), ln.weight, ln.bias, ln.eps) + ego
        torch.autograd.backward([x[:nu], x[nu:]], [dY[:nu], dY[nu:]])

    def step_hd():
        ue, ie = hd(ego)
        torch.autograd.backward([ue, ie], [dY[:nu], dY[nu:]])

    V, E = adj._indices()[0], adj._indices()[1]  # values are all > 0: the whole pattern

    def ref_block(blk, x):
        x = blk.dropout(x)
        x = F.relu(F.linear(x, blk.lin_in.weight, blk.lin_in.bias))
        x = blk.dropout(x)
        xe = torch.zeros(int(E.max()) + 1, d, device=dev).index_reduce_(
            0, E, x[V], "mean", include_self=False)
        xv = torch.zeros_like(x).index_reduce_(0, V, xe[E], "mean", include_self=False)
        mlp = blk.conv.W
        ln, lin = mlp.normalizations[0], mlp.lins[0]
        h = F.layer_norm(xv, (d,), ln.weight, ln.bias, ln.eps)
        return blk.dropout(F.relu(F.linear(h, lin.weight, lin.bias)))

    def step_hd_ref():
        x = ego
        for k in range(L):
            x = ref_block(hd.edhnn_layers[0 if k != L - 1 else 1], x) + ego
        torch.autograd.backward([x[:nu], x[nu:]], [dY[:nu], dY[nu:]])

    def timed(step):
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            step()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts)

    for name, fn in (("self_aware", step_sa), ("self_aware_ref", step_sa_ref),
                     ("hd", step_hd), ("hd_ref", step_hd_ref)):
        ms = timed(fn)
        print(json.dumps({"variant": name, "ms_fwd_bwd": round(ms, 3), "users": nu,
                          "items": ni, "edges": len(u), "d": d, "layers": L}), flush=True)


if __name__ == "__main__":
    main()
