#!/usr/bin/env python3
"""Is the second-epoch divergence of the HCCF plugin on a skewed catalogue the reference's own
dynamics? (VERDICT r4 "what's weak" 2; profiles/r04_hccf/eager_views/zipf_two_epoch_divergence.txt)

Same set-up, batches and modes as scripts/diag/diag_epoch_nan.py (bench_plugin_epoch's Zipf-1.2
Yelp-shaped files, epoch 1 on the reference's CPU drop-edge stream, epoch 2 on device-drawn
masks): the trajectory is the one that diverged. From batch ``--start`` of epoch 2 on, every step
is teacher-forced: from the parameters the plugin holds before the step and with the step's own
drop-edge structures and dropout masks (recorded, not re-drawn), the reference's torch calls
(tests/_ref64.py: HCCF.py:61-97, 173-191, util/loss_torch.py) give the batch loss and every
parameter gradient in float64 — and in float32, for the reference's own rounding — which are
compared with what the plugin computed and its optimizer then applied. One JSON line per step:
loss relative error, worst gradient row ratio (tests/_ref64.check_rows) against float64 and the
reference-fp32's own, and the tables' magnitudes. Ends at the IndexError (or the epoch's end).

    python scripts/diag/diag_zipf_teacher_forced.py [--start 200]
"""
import argparse
import json
import os
import random
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=200)
    ap.add_argument("--stop", type=int, default=10_000)
    ap.add_argument("--users", type=int, default=31_668)
    ap.add_argument("--items", type=int, default=38_048)
    ap.add_argument("--train", type=int, default=1_170_000)
    ap.add_argument("--test", type=int, default=390_000)
    ap.add_argument("--orders", type=int, default=0,
                    help="at every step where ours exceeds max(1e-5, the reference-fp32 "
                         "deviation): the reference's fp32 calls again with each drop-edge COO's "
                         "entries in this many other orders, and the worst rows named")
    ap.add_argument("--analyze", type=int, default=4,
                    help="decompose the first N steps over the bound (forward outputs, the BPR "
                         "and InfoNCE gradients apart, a bitwise re-run of the step)")
    args = ap.parse_args()
    import torch

    import bench_plugin_epoch as E
    from hypergraph_diffusion_for_recommendation_amd.plugins import HCCF
    from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
    from hypergraph_diffusion_for_recommendation_amd.selfrec import (FileIO, ModelConf,
                                                                     default_args)
    from tests import _ref64 as R

    tmp = tempfile.mkdtemp(prefix="hgd_zipf_tf_")
    os.chdir(tmp)
    d = os.path.join(tmp, "dataset", "yelp_synth")
    E.write_files(d, args.users, args.items, args.train, args.test)
    with open("HCCF.conf", "w") as f:
        f.write(E.CONF)
    conf = ModelConf("HCCF.conf")
    kw = default_args(model="HCCF", dataset="yelp_synth", max_epoch=1, batch_size=4096,
                      embedding_size=64, hyper_dim=32, n_layers=3, lrate=0.001, drop_rate=0.5,
                      p=0.1, cl_rate=1e-4, temp=0.2, reg=0.1, item_ranking="10,20")
    train = FileIO.load_data_set(d + "/train.txt")
    test = FileIO.load_data_set(d + "/test.txt")
    torch.manual_seed(0)
    rec = HCCF(conf, train, test, None, **kw)
    enc = rec.model
    nu, ni, L = rec.data.n_users, rec.data.n_items, rec.nLayers
    N = nu + ni
    dropper = enc.edgeDropper
    keep_h = 1 - enc.drop_rate

    class DropoutRecorder(torch.nn.Module):
        """The encoder's own nn.Dropout and its exact keep-mask: the same draw applied to ones
        (the device generator's state restored in between), so the mask is known where the
        input is 0 too — reading it off the output (y != 0) would drop those elements, and an
        exact-zero input element still passes its gradient through a kept mask entry."""

        def __init__(self, inner):
            super().__init__()
            self.inner, self.masks = inner, []
            self.zero_inputs = 0

        def forward(self, x):
            if not self.training:
                return self.inner(x)
            st = torch.cuda.get_rng_state(x.device)
            m = self.inner(torch.ones_like(x)) != 0
            torch.cuda.set_rng_state(st, x.device)
            y = self.inner(x)
            assert torch.equal(y != 0, m & (x != 0)), "dropout replay drew another mask"
            self.zero_inputs += int((x == 0).sum())
            self.masks.append(m.cpu())
            return y

    class ChildRecorder(R.DropRecorder):
        """R.DropRecorder that also keeps each output's device Incidence (the compacted child
        the hops run over) for the hop-level checks of analyze()."""

        def __init__(self, inner):
            super().__init__(inner)
            self.incs = []

        def forward(self, adj, keep):
            out = super().forward(adj, keep)
            self.incs.append(getattr(out, "_hgd_incidence", None))
            return out

    enc.drop_out = DropoutRecorder(enc.drop_out)
    enc.edgeDropper = ChildRecorder(dropper)
    captured = {}
    ssl_loss = rec.ssl_loss

    def ssl_capture(anchor_emb, pos_emb, *a, **k):  # the plugin's own anchor / positive rows
        captured["anc"], captured["pos"] = anchor_emb.detach(), pos_emb.detach()
        return ssl_loss(anchor_emb, pos_emb, *a, **k)

    rec.ssl_loss = ssl_capture
    print(json.dumps({"n_users": nu, "n_items": ni, "start": args.start}), flush=True)

    def permuted(di, dv, dtype, seed):
        """The same dropped matrix with its entries listed in another order (an uncoalesced COO:
        torch.sparse.mm's CPU kernel sums each row in storage order, so this is the reference's
        own calls on the same matrix with a different, equally valid fp32 summation order)."""
        ii = torch.as_tensor(np.asarray(di), dtype=torch.int64)
        vv = torch.as_tensor(np.asarray(dv)).to(dtype)
        p = torch.randperm(ii.shape[1], generator=torch.Generator().manual_seed(seed))
        return torch.sparse_coo_tensor(ii[:, p], vv[p], (N, N))

    def reference(P, dtype, drops, masks, u, i, j, parts=False, order_seed=None):
        if order_seed is None:
            adjs = [R.sparse(di, dv, (N, N), dtype) for di, dv in drops]
        else:
            adjs = [permuted(di, dv, dtype, order_seed * 97 + k)
                    for k, (di, dv) in enumerate(drops)]
        ueR, ieR, gR, hR = R.hccf_encoder(P, adjs, [m.to(dtype) for m in masks], keep_h, nu, L)
        anc, pos, neg = ueR[u], ieR[i], ieR[j]
        nodes = []
        for ref_rows, ours in ((anc, captured["anc"]), (pos, captured["pos"])):
            mine = torch.unique(ref_rows.long())
            theirs = torch.unique(ours.cpu().long())
            if not torch.equal(mine, theirs):
                # .long() of a value within rounding of an integer: take the plugin's list (as
                # _ref64.ReluMasks does for a ReLU at 0) after checking that is the only cause
                diff = (ref_rows.long() != ours.cpu().long())
                gap = (ref_rows[diff] - ref_rows[diff].round()).abs().max()
                nodes.append((theirs, float(gap)))
            else:
                nodes.append((mine, None))
        ssl = 0
        for layer in range(L):
            e1, e2 = gR[layer].detach(), hR[layer]
            ssl = ssl + R.contrast_loss(e1[:nu], e2[:nu], nodes[0][0], rec.temp) \
                + R.contrast_loss(e1[nu:], e2[nu:], nodes[1][0], rec.temp)
        bpr = R.bpr_loss(anc, pos, neg)
        loss = bpr + ssl * rec.ss_rate
        names = list(P)
        if parts:  # the encoder's outputs and the two losses' gradients apart
            gb = dict(zip(names, torch.autograd.grad(bpr, [P[n] for n in names],
                                                     retain_graph=True)))
            gs = dict(zip(names, torch.autograd.grad(ssl * rec.ss_rate, [P[n] for n in names])))
            return (ueR, ieR, gR, hR), gb, gs
        grads = dict(zip(names, torch.autograd.grad(loss, [P[n] for n in names])))
        mags = {"user_emb": float(ueR.abs().max()), "item_emb": float(ieR.abs().max()),
                f"hyper[{L - 1}]": float(hR[-1].abs().max())}
        return float(loss), grads, [g for _, g in nodes], mags

    from hypergraph_diffusion_for_recommendation_amd.functional import bpr_loss_rows
    adj_idx = enc.sparse_norm_adj._indices()
    node_deg = torch.bincount(adj_idx[0], minlength=N).cpu()

    def worst_row(got, ref):
        g = got.detach().cpu().double()
        r = ref.detach().cpu().double()
        if g.dim() == 1:
            g, r = g[None], r[None]
        err = (g - r).abs().amax(1)
        scale = r.abs().amax(1)
        ratio = torch.where(scale == 0, err, err / scale.clamp_min(1e-300))
        k = int(ratio.argmax())
        return {"ratio": float(ratio[k]), "row": k, "err": float(err[k]),
                "scale": float(scale[k]), "rows_over_1e-5": int((ratio > 1e-5).sum())}

    def analyze(b, u, i, j, before, pre_rng, drops, masks):
        """Re-runs the bad step from its start: the same parameters and RNG states (so the same
        drop-edge and dropout draws), the forward outputs and the BPR / InfoNCE gradients apart
        against float64, and whether the re-run's total gradient is bitwise the step's."""
        params = dict(enc.named_parameters())
        step_grads = {n: p.grad.detach().clone() for n, p in params.items()}
        # each layer's compacted child, both orientations, against the recorded COO in float64
        from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_csr
        hops = {}
        gX = torch.Generator(device=rec.device).manual_seed(b)
        for layer, ch in enumerate(list(enc.edgeDropper.incs[:L])):
            if ch is None:
                continue
            di, dv = drops[layer]
            A64 = torch.sparse_coo_tensor(di, dv.double(), (N, N)).coalesce()
            X = torch.randn(N, 64, device=rec.device, generator=gX)
            Yr = spmm_csr(ch.csr, X, ch.val)
            Yc = spmm_csr(ch.csc, X, ch.val_t)
            Xh = X.cpu().double()
            hops[f"layer{layer}"] = {
                "csr": worst_row(Yr, torch.sparse.mm(A64, Xh)),
                "csc": worst_row(Yc, torch.sparse.mm(A64.t().coalesce(), Xh)),
                "n_heavy_csr": ch.csr.n_heavy, "n_heavy_csc": ch.csc.n_heavy,
                "nnz": ch.nnz}
        post = {n: p.detach().clone() for n, p in params.items()}
        post_rng = (torch.get_rng_state(), torch.cuda.get_rng_state())
        with torch.no_grad():
            for n, p in params.items():
                p.copy_(before[n].to(device=p.device, dtype=p.dtype))
        torch.set_rng_state(pre_rng[0])
        torch.cuda.set_rng_state(pre_rng[1])
        enc.drop_out.masks.clear()
        enc.edgeDropper.outputs.clear()
        enc.zero_grad(set_to_none=True)
        ue, ie, gcn, hyp = enc(keep_rate=1 - rec.dropRate)
        same_draws = (all(torch.equal(a[0], b_[0]) and torch.equal(a[1], b_[1])
                          for a, b_ in zip(enc.edgeDropper.outputs[:L], drops)) and
                      all(torch.equal(a, b_) for a, b_ in zip(enc.drop_out.masks[:2 * L], masks)))
        bpr, anc, pos = bpr_loss_rows(ue, ie, u, i, j)
        names = list(params)
        gb = dict(zip(names, torch.autograd.grad(bpr, [params[n] for n in names],
                                                 retain_graph=True, allow_unused=True)))
        ssl = rec.ssl_loss(anc, pos, gcn, hyp)
        gs = dict(zip(names, torch.autograd.grad(ssl, [params[n] for n in names],
                                                 allow_unused=True)))
        P64 = {n: v.clone().requires_grad_(True) for n, v in before.items()}
        (ueR, ieR, gR, hR), gbR, gsR = reference(P64, torch.float64, drops, masks, u.cpu(),
                                                 i.cpu(), j.cpu(), parts=True)
        rep = {"batch": b, "analysis": True, "same_draws_on_rerun": same_draws, "hops": hops,
               "forward": {"user_emb": worst_row(ue, ueR), "item_emb": worst_row(ie, ieR)}}
        for layer in range(L):
            rep["forward"][f"gcn[{layer}]"] = worst_row(gcn[layer], gR[layer])
            rep["forward"][f"hyper[{layer}]"] = worst_row(hyp[layer], hR[layer])
        rep["bpr_grad"] = {n: worst_row(gb[n] if gb[n] is not None else torch.zeros_like(
            params[n]), gbR[n]) for n in names}
        rep["ssl_grad"] = {n: worst_row(gs[n] if gs[n] is not None else torch.zeros_like(
            params[n]), gsR[n]) for n in names}
        rerun = {n: (gb[n] if gb[n] is not None else 0) + (gs[n] if gs[n] is not None else 0)
                 for n in names}
        # the same step with the encoder's ops swapped for torch's, one more at a time: which op
        # carries the error (A: as run; B: the layer loop unfused; C: + torch HGNN products;
        # D: + torch E·W; E: + torch.sparse.mm GCN hops — only the BPR / InfoNCE kernels left)
        from hypergraph_diffusion_for_recommendation_amd import encoders as ENC
        saved_ops = (ENC.dense_two_hop_pair, ENC.linear, type(enc.gcnlayer).forward)
        ref_tot = {n: gbR[n] + gsR[n] for n in names}
        configs = {}
        for cfg in "ABCDE":
            with torch.no_grad():
                for n, p in params.items():
                    p.copy_(before[n].to(device=p.device, dtype=p.dtype))
            torch.set_rng_state(pre_rng[0])
            torch.cuda.set_rng_state(pre_rng[1])
            enc.fused_layers = cfg == "A"
            if cfg >= "C":
                ENC.dense_two_hop_pair = lambda Hu, Hi, X, nu_: torch.cat(
                    [Hu @ (Hu.T @ X[:nu_]), Hi @ (Hi.T @ X[nu_:])], 0)
            if cfg >= "D":
                ENC.linear = lambda X, W, bias=None, **k: X @ W.t()
            if cfg >= "E":
                type(enc.gcnlayer).forward = lambda self_, adj, x: torch.sparse.mm(adj, x)
            try:
                ue2, ie2, gcn2, hyp2 = enc(keep_rate=1 - rec.dropRate)
                b2, a2, p2 = bpr_loss_rows(ue2, ie2, u, i, j)
                tot = b2 + rec.ssl_loss(a2, p2, gcn2, hyp2)
                g2 = dict(zip(names, torch.autograd.grad(tot, [params[n] for n in names])))
                configs[cfg] = {n[15:]: worst_row(g2[n], ref_tot[n]) for n in names}
            except Exception as e:  # noqa: BLE001
                configs[cfg] = {"error": repr(e)[:200]}
            finally:
                ENC.dense_two_hop_pair, ENC.linear = saved_ops[0], saved_ops[1]
                type(enc.gcnlayer).forward = saved_ops[2]
                enc.fused_layers = True
        rep["op_swaps"] = configs
        rep["rerun_total_equals_step"] = {n: bool(torch.equal(rerun[n], step_grads[n]))
                                          for n in names}
        rep["rerun_vs_step_max_abs"] = {n: float((rerun[n] - step_grads[n]).abs().max())
                                        for n in names}
        # the worst rows of the step's own gradient: how often in the batch, graph degree
        uc, ic, jc = u.cpu(), i.cpu(), j.cpu()
        for n, off, ids in (("embedding_dict.item_emb", nu, (ic, jc)),
                            ("embedding_dict.user_emb", 0, (uc,))):
            gR_tot = gbR[n] + gsR[n]
            w = worst_row(step_grads[n], gR_tot)
            k = w["row"]
            w.update({"times_in_batch": [int((t == k).sum()) for t in ids],
                      "node_degree": int(node_deg[off + k]),
                      "max_degree": int(node_deg[off:off + (ni if off else nu)].max())})
            rep[f"step_worst_{n[15:]}"] = w
        print(json.dumps(rep), flush=True)
        with torch.no_grad():
            for n, p in params.items():
                p.copy_(post[n])
                p.grad = step_grads[n]
        torch.set_rng_state(post_rng[0])
        torch.cuda.set_rng_state(post_rng[1])

    random.seed(1)
    worst_all = 0.0
    analyzed = 0
    for ep, mode in enumerate(("cpu", "device")):
        dropper.device_rng = mode == "device"
        dropper.capture_safe = False
        for b, (u, i, j) in enumerate(next_batch_pairwise(rec.data, rec.batchSize, device=rec.device)):
            forced = ep == 1 and args.start <= b < args.stop
            enc.drop_out.masks.clear()
            enc.edgeDropper.outputs.clear()
            enc.edgeDropper.incs.clear()
            before = ({n: p.detach().cpu().double() for n, p in enc.named_parameters()}
                      if forced else None)
            pre_rng = (torch.get_rng_state(), torch.cuda.get_rng_state()) if forced else None
            try:
                got = float(rec.train_step(u, i, j).detach())
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"epoch": ep, "batch": b, "mode": mode,
                                  "raised": repr(e)[:300]}), flush=True)
                print(json.dumps({"summary": "stopped at the exception", "worst_ratio_over_bound":
                                  worst_all}), flush=True)
                return 0
            if not forced:
                if b % 50 == 0:
                    print(json.dumps({"epoch": ep, "batch": b, "mode": mode, "loss": got}),
                          flush=True)
                continue
            drops = list(enc.edgeDropper.outputs[:L])
            masks = list(enc.drop_out.masks[:2 * L])
            assert len(drops) == L and len(masks) == 2 * L, (len(drops), len(masks))
            uc, ic, jc = u.cpu(), i.cpu(), j.cpu()
            P64 = {n: v.clone().requires_grad_(True) for n, v in before.items()}
            P32 = {n: v.float().requires_grad_(True) for n, v in before.items()}
            l64, g64, gaps, mags = reference(P64, torch.float64, drops, masks, uc, ic, jc)
            l32, g32, _, _ = reference(P32, torch.float32, drops, masks, uc, ic, jc)
            params = dict(enc.named_parameters())
            rows, over = {}, 0.0
            for n in g64:
                own = R.check_rows(g32[n], g64[n], f"ref32 {n}", tol=1e9)
                ours = R.check_rows(params[n].grad, g64[n], f"{n}", tol=1e9)
                rows[n] = [ours, own]
                over = max(over, ours / max(R.TOL, own))
            loss_rel = abs(got - l64) / abs(l64)
            loss_rel32 = abs(l32 - l64) / abs(l64)
            over = max(over, loss_rel / max(R.TOL, loss_rel32))
            worst_all = max(worst_all, over)
            orders = None
            if args.orders and over > 1.0:
                # the excess tensors: the reference's fp32 deviation under other entry orders,
                # and where the worst rows of ours sit (which node, its degree, its batch count)
                orders = {}
                for n, (ours, own) in rows.items():
                    if ours <= max(R.TOL, own):
                        continue
                    devs = []
                    for o in range(args.orders):
                        Po = {k: v.float().requires_grad_(True) for k, v in before.items()}
                        _, go, _, _ = reference(Po, torch.float32, drops, masks, uc, ic, jc,
                                                order_seed=1000 * b + o)
                        devs.append(R.check_rows(go[n], g64[n], f"ref32 order {o} {n}",
                                                 tol=1e9))
                    off = nu if "item" in n else 0
                    w = worst_row(params[n].grad, g64[n])
                    w32 = worst_row(g32[n], g64[n])
                    k = w["row"]
                    ids = (ic, jc) if "item" in n else (uc,)
                    orders[n] = {"ours": ours, "ref32": own, "ref32_other_orders": devs,
                                 "max_ref32_any_order": max([own] + devs),
                                 "ours_over_max_ref32_any_order": ours / max([own] + devs),
                                 "worst_row": k, "ref32_worst_row": w32["row"],
                                 "node_degree": int(node_deg[off + k]),
                                 "times_in_batch": [int((t == k).sum()) for t in ids]}
            print(json.dumps({"epoch": ep, "batch": b, "mode": mode, "loss": got,
                              "dropout_zero_inputs_so_far": enc.drop_out.zero_inputs,
                              "loss_ref64": l64, "loss_rel": loss_rel, "loss_rel_ref32": loss_rel32,
                              "grad_row_ratio": rows, "ratio_over_bound": over,
                              "within_bound": over <= 1.0, "node_list_gaps": gaps,
                              "max_abs_ref64": mags, "orders": orders}), flush=True)
            if over > 10.0 and analyzed < args.analyze:
                analyzed += 1
                analyze(b, u, i, j, before, pre_rng, drops, masks)
    print(json.dumps({"summary": "epochs finished", "worst_ratio_over_bound": worst_all}),
          flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
