#!/usr/bin/env python3
"""Per-step fwd+bwd cost of one ED-HNN block on a dataset-shaped
normalised bipartite graph, for both forms:

* ``spmm``  — edhnn_spmm.EquivSetGNN (model/layers/EquivSetConv.py:86-107 + EquivSetGNN.py:85-101):
              two HGCNConv two-hops over norm_adj with LayerNorm + residual + restart blend;
* ``mean``  — layers.EquivSetGNN (layers2/EquivSetConv2.py:85-100, HGNN_HD4's W2 = slice):
              the V/E scatter-mean pair + restart blend over the binary interaction hypergraph;

each with the fused row epilogue (hgd_spmm_fused) and with the reference's separate torch ops
(``fused_epilogue = False``), plus the reference's CPU path for the SpMM form (torch.sparse.mm +
nn.LayerNorm on the host, scripts/refops.hgcn_conv) on the same graph. Training mode (dropout
on), synthetic graph and random weights. Prints one JSON line per variant.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ARGS = {  # LocalAwareEncoder.init_edhnn_config, HGNN_HD4.py:371-388 (hidden = emb_size)
    'MLP_hidden': 64, 'MLP1_num_layers': 0, 'MLP2_num_layers': 0, 'MLP3_num_layers': 1,
    'MLP_num_layers': 0, 'restart_alpha': 0.5, 'aggregate': 'mean', 'dropout': 0.5,
    'normalization': 'ln', 'input_norm': True, 'All_num_layers': 1, 'activation': 'relu',
    'input_dropout': 0.6, 'AllSet_input_norm': True}


def make_reference_step(m, form, A, ui, N, d, dev, X, dY):
    """One fwd+bwd of the block with the reference's torch ops on the device: torch.sparse.mm
    hops (model/layers/EquivSetConv.py:86-107) or torch_scatter-style means (sum / count,
    layers2/EquivSetConv2.py:88-93), F.layer_norm / F.linear / F.dropout."""
    import torch
    import torch.nn.functional as F
    import refops as O

    c = m.conv
    p_drop = m.dropout.p
    alpha = c.alpha
    lin_in = (m.lin_in.weight, m.lin_in.bias)
    Wn, Wl = c.W.normalizations[0], c.W.lins[0]

    def tail(Xv, x0):
        Xb = (1 - alpha) * Xv + alpha * x0
        Xb = F.layer_norm(Xb, (d,), Wn.weight, Wn.bias, Wn.eps)
        y = torch.relu(F.linear(Xb, Wl.weight, Wl.bias))
        return F.dropout(y, p_drop, True)

    if form == "spmm":
        idx, vals = O.coo_of(A)
        adj = torch.sparse_coo_tensor(torch.from_numpy(idx), torch.from_numpy(vals),
                                      A.shape).coalesce().to(dev)
        ln0, ln1 = c.lns[0], c.lns[1]

        def hop(x):
            return F.leaky_relu(torch.sparse.mm(adj, torch.sparse.mm(adj.t(), x)), 0.2)

        def step():
            xx = X.detach().requires_grad_(True)
            h = F.dropout(xx, p_drop, True)
            h = torch.relu(F.linear(h, *lin_in))
            x0 = h
            h = F.dropout(h, p_drop, True)
            Xe = F.layer_norm(hop(h), (d,), ln0.weight, ln0.bias, ln0.eps) + h
            Xv = F.layer_norm(hop(Xe), (d,), ln1.weight, ln1.bias, ln1.eps) + Xe
            tail(Xv, x0).backward(dY)
        return step

    coo = ui.tocoo()
    V = torch.from_numpy(coo.row.astype("int64")).to(dev)
    E = torch.from_numpy(coo.col.astype("int64")).to(dev)
    ones = torch.ones(len(V), device=dev)
    cnt_e = torch.zeros(N, device=dev).index_add_(0, E, ones).clamp_(min=1)[:, None]
    cnt_v = torch.zeros(N, device=dev).index_add_(0, V, ones).clamp_(min=1)[:, None]

    def step():
        xx = X.detach().requires_grad_(True)
        h = F.dropout(xx, p_drop, True)
        h = torch.relu(F.linear(h, *lin_in))
        x0 = h
        h = F.dropout(h, p_drop, True)
        Xe = torch.zeros(N, d, device=dev).index_add(0, E, h[V]) / cnt_e
        Xv = torch.zeros(N, d, device=dev).index_add(0, V, Xe[E]) / cnt_v
        tail(Xv, x0).backward(dY)
    return step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--users", type=int, default=31_668)
    ap.add_argument("--items", type=int, default=38_048)
    ap.add_argument("--edges", type=int, default=1_170_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--cpu-reps", type=int, default=3)
    ap.add_argument("--tag", default="yelp")
    ap.add_argument("--variants",
                    default="gpu_fused,gpu_fused_graph,gpu_unfused,gpu_reference_ops,cpu_reference_ops",
                    help="comma list of variants to run")
    args = ap.parse_args()
    import numpy as np
    import scipy.sparse as sp
    import torch

    from hypergraph_diffusion_for_recommendation_amd import edhnn_spmm
    from hypergraph_diffusion_for_recommendation_amd.encoders import sparse_tensor_of
    from hypergraph_diffusion_for_recommendation_amd.layers import EquivSetGNN
    import refops as O
    import refops as ref_cpu

    u, i = O.synthetic_incidence(args.users, args.items, args.edges, seed=0)
    ui = O.bipartite_adjacency(u, i, args.users, args.items)
    A = O.normalize_graph_mat(ui)
    N = A.shape[0]
    dev = torch.device("cuda")
    adj = sparse_tensor_of(A, dev)
    H = sparse_tensor_of(sp.csr_matrix((np.ones(ui.nnz, np.float32), ui.indices, ui.indptr),
                                       shape=ui.shape), dev)
    d = args.dim
    cfg = dict(ARGS, MLP_hidden=d)
    X = torch.randn(N, d, device=dev)
    dY = torch.randn(N, d, device=dev)

    def gpu_time(step, reps):
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(reps):
            e0.record()
            step()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        return statistics.median(ts)

    out = []
    for form in ("spmm", "mean"):
        torch.manual_seed(0)
        if form == "spmm":
            m = edhnn_spmm.EquivSetGNN(d, cfg).to(dev).train()
            call = lambda xx: m(xx, adj, N)  # noqa: E731
        else:
            m = EquivSetGNN(d, cfg, H).to(dev).train()
            call = lambda xx: m(xx, H, N)  # noqa: E731
        want = set(args.variants.split(","))
        for fused in (True, False):
            if ("gpu_fused" if fused else "gpu_unfused") not in want:
                continue
            m.conv.fused_epilogue = fused

            def step():
                xx = X.detach().requires_grad_(True)
                y = call(xx)
                y.backward(dY)

            ms = gpu_time(step, args.reps)
            out.append({"form": form, "variant": "gpu_fused" if fused else "gpu_unfused",
                        "ms_per_step": round(ms, 4)})
        # the reference's own op chain on the same GPU (torch.sparse.mm / index_add means,
        # nn.functional LayerNorm / Linear / dropout), same parameters
        if "gpu_fused_graph" in want:
            # the same fused step captured once in a HIP graph (static X / dY; dropout masks are
            # drawn from the graph-safe philox state, fresh every replay)
            m.conv.fused_epilogue = True
            xs = X.detach().clone().requires_grad_(True)

            def body():
                m.zero_grad(set_to_none=False)
                xs.grad = None
                call(xs).backward(dY)

            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(3):
                    body()
            torch.cuda.current_stream().wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                call(xs).backward(dY)
            ms = gpu_time(graph.replay, args.reps)
            out.append({"form": form, "variant": "gpu_fused_graph", "ms_per_step": round(ms, 4)})
        if "gpu_reference_ops" in want:
            ref_step = make_reference_step(m, form, A, ui, N, d, dev, X, dY)
            out.append({"form": form, "variant": "gpu_reference_ops",
                        "ms_per_step": round(gpu_time(ref_step, args.reps), 4)})
        if form == "spmm" and "cpu_reference_ops" in want:
            # the reference's CPU path: same parameters, torch.sparse.mm + host ops
            mc = edhnn_spmm.EquivSetGNN(d, cfg).train()
            mc.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
            idx, vals = O.coo_of(A)
            adj_c = torch.sparse_coo_tensor(torch.from_numpy(idx), torch.from_numpy(vals),
                                            A.shape).coalesce()
            Xc, dYc = X.cpu(), dY.cpu()
            c = mc.conv

            def cpu_step():
                xx = Xc.detach().requires_grad_(True)
                h = mc.dropout(xx)
                h = torch.relu(mc.lin_in(h))
                x0 = h
                h = mc.dropout(h)
                Xve = c.W1(h)
                Xe = c.lns[0](ref_cpu.hgcn_conv(adj_c, Xve, act=True, slope=0.2)) + Xve
                Xev = Xe
                Xv = c.lns[1](ref_cpu.hgcn_conv(adj_c, Xev, act=True, slope=0.2)) + Xev
                y = mc.dropout(mc.act(c.W((1 - c.alpha) * Xv + c.alpha * x0)))
                y.backward(dYc)

            cpu_step()
            ts = []
            for _ in range(args.cpu_reps):
                t0 = time.perf_counter()
                cpu_step()
                ts.append((time.perf_counter() - t0) * 1e3)
            out.append({"form": form, "variant": "cpu_reference_ops",
                        "ms_per_step": round(statistics.median(ts), 3),
                        "threads": torch.get_num_threads()})
    for r in out:
        r.update({"graph": args.tag, "n_nodes": N, "nnz_adj": int(A.nnz), "d": d})
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
