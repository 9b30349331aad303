#!/usr/bin/env python3
"""One HCCF training step (BASELINE configs[2]: Yelp2018-shaped, 3 layers, d = 64, InfoNCE SSL;
HCCF.py:56-106) on one MI355X: forward (edge-dropped GCN hop + learned-hypergraph hops per
layer), BPR + per-layer contrastLoss on users and items, backward, clip_grad_norm_ (where the
reference calls it) and Adam. Variants:

* hgd_cpu_mask     — encoders.HCCFEncoder: hops, drop-edge compaction / sort-free rebuild,
                     HGNNLayer and InfoNCE on this library; the drop-edge mask drawn by the
                     reference's CPU torch.rand (bit-identical masks for a seed);
* hgd_device_mask  — the same with SpAdjDropEdge(device_rng=True);
* hgd_graph        — the device-mask step replayed from one HIP graph (graphs.CapturedStep:
                     capture-safe drop-edge, device-side InfoNCE node counts, capturable Adam);
* hgd_graph_cpu_mask — the same replay with the masks of the reference's CPU torch.rand stream,
                     drawn on the host before each replay (SpAdjDropEdge.refill);
* hgd_graph_ref_adam — the hgd_graph_cpu_mask replay holding only the forward + backward, the
                     reference's Adam (torch.optim.Adam(lr=float)) stepping eagerly after it;
* hgd_graph_kernel_adam — the same replay with the reference's Adam as one captured kernel
                     (optim.ReferenceAdam: bitwise torch's Adam), the plugins' graph default;
* hgd_capture_safe_eager — the graph variant's ops (device mask), launched eagerly;
* hgd_cs_eager_cpu_mask — eager, capture-safe drop-edge views (the reference's CPU mask stream
                     through the per-call slots), device-side InfoNCE counts, fused BPR, the
                     reference's unfused Adam: no host read inside the step;
* reference_ops    — scripts/refops.HCCFEncoderRef + the reference's losses (torch.sparse.mm,
                     torch.mm, F.normalize …) on the same GPU, same parameters.

Synthetic graph (SURVEY.md §8d generator), random batches drawn on the device (the reference's
Python sampler is outside the path). Prints one JSON line per variant."""
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
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--variants", default="hgd_cpu_mask,hgd_device_mask,hgd_graph,reference_ops")
    args = ap.parse_args()
    import torch

    import refops as R
    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFEncoder
    from hypergraph_diffusion_for_recommendation_amd.functional import (bpr_loss_rows,
                                                                         contrast_loss,
                                                                         contrast_loss_layers,
                                                                         unique_long,
                                                                         unique_long_n,
                                                                         unique_long_n_group)
    from hypergraph_diffusion_for_recommendation_amd.graphs import CapturedStep

    dev = torch.device("cuda")
    u, i = R.synthetic_incidence(args.users, args.items, args.edges, seed=0)
    A = R.normalize_graph_mat(R.bipartite_adjacency(u, i, args.users, args.items))
    nu, ni = args.users, args.items
    data = types.SimpleNamespace(n_users=nu, n_items=ni, norm_adj=A)
    conf = dict(lrate=0.001, lr_decay=0.7, max_epoch=1, batch_size=args.batch, reg=0.1,
                embedding_size=args.dim, hyper_dim=32, drop_rate=0.5, p=0.1,
                n_layers=args.layers)
    temp, cl_rate, keep = 0.2, 1e-4, 0.5
    g = torch.Generator(device=dev).manual_seed(0)
    batches = [(torch.randint(0, nu, (args.batch,), device=dev, generator=g),
                torch.randint(0, ni, (args.batch,), device=dev, generator=g),
                torch.randint(0, ni, (args.batch,), device=dev, generator=g)) for _ in range(8)]

    def make_step(model, loss_fn, unique, hoist=True, graph=False, counted=None, host_fed=None,
                  fused_adam=None, adam_after_replay=False, kernel_adam=False):
        # adam_after_replay: the graph holds the forward + backward only; the reference's Adam
        # (torch.optim.Adam(lr=float), non-capturable) steps eagerly after each replay
        counted = graph if counted is None else counted
        fused_adam = (counted and not adam_after_replay) if fused_adam is None else fused_adam
        if kernel_adam:  # the reference's Adam as one capturable kernel (optim.ReferenceAdam)
            from hypergraph_diffusion_for_recommendation_amd.optim import ReferenceAdam
            opt = ReferenceAdam(model.parameters(), lr=conf["lrate"])
        elif fused_adam:
            lr = torch.tensor(conf["lrate"], dtype=torch.float32, device=dev)
            opt = torch.optim.Adam(model.parameters(), lr=lr, capturable=True, fused=True)
        else:
            opt = torch.optim.Adam(model.parameters(), lr=conf["lrate"])
        state = {"k": 0, "cap": None, "capturing": False}

        def body(uid, pid, nid):
            ue, ie, gcn, hyp = model(keep_rate=keep)
            if counted:  # the plugin's fused BPR on the encoder table (functional.bpr_loss_rows)
                bpr, anc, pos = bpr_loss_rows(ue, ie, uid, pid, nid)
            else:
                anc, pos, neg = ue[uid], ie[pid], ie[nid]
                bpr = R.bpr_loss(anc, pos, neg)
            ssl = 0
            # the reference recomputes torch.unique(·.long()) per layer; ours hoists it (same value)
            if counted:  # both node lists in one launch per kernel (the plugin's ssl_loss)
                un = tuple(unique_long_n_group([anc, pos], [nu, ni]))
            else:
                un = (unique(anc, nu), unique(pos, ni)) if hoist else None
            if counted:  # (nodes, device count) pairs: every layer's both halves in one op
                ssl = contrast_loss_layers([t.detach() for t in gcn], hyp, nu, un[0][0],
                                           un[1][0], temp, un[0][1], un[1][1])
            for layer in range(0 if counted else args.layers):
                e1, e2 = gcn[layer].detach(), hyp[layer]
                nu_nodes, np_nodes = un if hoist else (unique(anc, nu), unique(pos, ni))
                ssl = ssl + loss_fn(e1[:nu], e2[:nu], nu_nodes, temp) \
                    + loss_fn(e1[nu:], e2[nu:], np_nodes, temp)
            loss = bpr + cl_rate * ssl
            opt.zero_grad()
            torch.nn.utils.clip_grad_norm_(model.parameters(), 4)  # before backward, as HCCF.py:95
            loss.backward()
            if kernel_adam and state["capturing"]:
                opt.launch()  # the graph's half; opt.prepare() runs before each replay
            elif not adam_after_replay:
                opt.step()
            return loss

        def step():
            uid, pid, nid = batches[state["k"] % len(batches)]
            state["k"] += 1
            if not graph:
                out = body(uid, pid, nid)
                if adam_after_replay:
                    opt.step()
                return out
            if state["cap"] is None:
                if state["k"] == 1:
                    out = body(uid, pid, nid)  # one eager step: optimizer state, handles
                    if adam_after_replay:
                        opt.step()
                    return out
                if host_fed is not None:  # the reference's CPU mask stream, drawn per replay
                    host_fed.host_fed(True)

                def before():
                    if host_fed is not None:
                        host_fed.refill()
                    if kernel_adam:
                        opt.prepare()
                state["capturing"] = True
                state["cap"] = CapturedStep(body, (uid, pid, nid), before_replay=before)
                state["capturing"] = False
            out = state["cap"](uid, pid, nid)
            if adam_after_replay:
                opt.step()
            return out
        return step

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

    torch.manual_seed(0)
    ours = HCCFEncoder(conf, data, dev)
    ref = R.HCCFEncoderRef(nu, ni, args.dim, 32, args.layers, conf["drop_rate"],
                           ours.sparse_norm_adj.detach().clone().coalesce())
    ref.load_state_dict(ours.state_dict(), strict=False)
    out = []
    want = args.variants.split(",")
    if "hgd_cpu_mask" in want:
        out.append(("hgd_cpu_mask", timed(make_step(ours, contrast_loss, lambda t, n: unique_long(t)))))
    if "hgd_device_mask" in want:
        ours.edgeDropper.device_rng = True
        out.append(("hgd_device_mask", timed(make_step(ours, contrast_loss, lambda t, n: unique_long(t)))))
    if "hgd_graph" in want:
        torch.manual_seed(0)
        g_model = HCCFEncoder(conf, data, dev)
        g_model.load_state_dict(ours.state_dict())
        g_model.edgeDropper.device_rng = True
        g_model.edgeDropper.capture_safe = True
        out.append(("hgd_graph", timed(make_step(g_model, contrast_loss, unique_long_n,
                                                 graph=True))))
    if "hgd_graph_cpu_mask" in want:  # graph replay, masks from the reference's CPU stream
        torch.manual_seed(0)
        c_model = HCCFEncoder(conf, data, dev)
        c_model.load_state_dict(ours.state_dict())
        c_model.edgeDropper.device_rng = False
        c_model.edgeDropper.capture_safe = True
        out.append(("hgd_graph_cpu_mask", timed(make_step(c_model, contrast_loss, unique_long_n,
                                                          graph=True,
                                                          host_fed=c_model.edgeDropper))))
    if "hgd_graph_ref_adam" in want:  # replayed fwd + bwd on the reference's CPU mask stream,
        torch.manual_seed(0)             # the reference's Adam eagerly after each replay
        a_model = HCCFEncoder(conf, data, dev)
        a_model.load_state_dict(ours.state_dict())
        a_model.edgeDropper.device_rng = False
        a_model.edgeDropper.capture_safe = True
        out.append(("hgd_graph_ref_adam", timed(make_step(a_model, contrast_loss, unique_long_n,
                                                          graph=True,
                                                          host_fed=a_model.edgeDropper,
                                                          adam_after_replay=True))))
    if "hgd_graph_kernel_adam" in want:  # replayed step incl. the reference's Adam as one
        torch.manual_seed(0)               # captured kernel (the plugins' graph default)
        k_model = HCCFEncoder(conf, data, dev)
        k_model.load_state_dict(ours.state_dict())
        k_model.edgeDropper.device_rng = False
        k_model.edgeDropper.capture_safe = True
        out.append(("hgd_graph_kernel_adam", timed(make_step(k_model, contrast_loss,
                                                             unique_long_n, graph=True,
                                                             host_fed=k_model.edgeDropper,
                                                             kernel_adam=True))))
    if "hgd_capture_safe_eager" in want:  # the graph variant's ops, launched eagerly
        torch.manual_seed(0)
        e_model = HCCFEncoder(conf, data, dev)
        e_model.load_state_dict(ours.state_dict())
        e_model.edgeDropper.device_rng = True
        e_model.edgeDropper.capture_safe = True
        out.append(("hgd_capture_safe_eager", timed(make_step(e_model, contrast_loss,
                                                              unique_long_n, counted=True))))
    if "hgd_cs_eager_cpu_mask" in want:  # eager, capture-safe ops on the reference's CPU mask
        torch.manual_seed(0)                # stream, the reference's (unfused) Adam
        f_model = HCCFEncoder(conf, data, dev)
        f_model.load_state_dict(ours.state_dict())
        f_model.edgeDropper.device_rng = False
        f_model.edgeDropper.capture_safe = True
        out.append(("hgd_cs_eager_cpu_mask", timed(make_step(f_model, contrast_loss,
                                                             unique_long_n, counted=True,
                                                             fused_adam=False))))
    if "reference_ops" in want:
        out.append(("reference_ops", timed(make_step(ref, R.contrast_loss, lambda t, n: torch.unique(t.long()), hoist=False))))
    for name, ms in out:
        print(json.dumps({"variant": name, "ms_per_step": round(ms, 3), "users": nu,
                          "items": ni, "edges": len(u), "d": args.dim, "layers": args.layers,
                          "batch": args.batch}), flush=True)


if __name__ == "__main__":
    main()
